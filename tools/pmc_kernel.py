#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per dispatch of the kernels whose name contains a pattern.
usage: pmc_kernel.py <counter_collection.csv> [pattern] -> JSON {counter: mean per dispatch, ...}"""
import collections
import csv
import json
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "corr_pyramid"
vals = collections.defaultdict(list)
names = set()
for r in csv.DictReader(open(path)):
    if pat in r["Kernel_Name"]:
        names.add(r["Kernel_Name"][:80])
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({"kernels": sorted(names), "dispatches": max((len(v) for v in vals.values()), default=0),
                  **{k: sum(v) / len(v) for k, v in sorted(vals.items())}}, indent=1))
