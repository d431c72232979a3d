#!/usr/bin/env python3
"""Average per-dispatch value of each PMC counter, per (kernel, grid), for kernels whose name contains
a pattern, from a rocprofv3 --pmc counter_collection.csv.  FETCH_SIZE / WRITE_SIZE are in KiB
(gfx950: FETCH_SIZE counts 64-B requests for 128-B reads -> x2, see MI355X_MICROARCH.md).
usage: pmc_kernel_avg.py <counter_collection.csv> <pattern>"""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if sys.argv[2] not in n:
        continue
    key = (n.replace("void ", "")[:70], r.get("Grid_Size", r.get("Grid_Size_X", "")))
    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())}, "dispatches", max(len(v) for v in cs.values()))
