#!/usr/bin/env python3
"""HBM bytes per dispatch by kernel from two rocprofv3 counter passes (--pmc FETCH_SIZE, --pmc
WRITE_SIZE) over the same program: gfx950 corrections as bench.live_traffic (both counters in KiB,
FETCH_SIZE doubled).  Kernels whose name contains 'rmd' only.
usage: pmc_traffic_by_kernel.py <fetch counter_collection.csv> <write counter_collection.csv> -> JSON lines"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") == counter and "rmd" in r["Kernel_Name"]:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def short(name):
    m = re.search(r"(\w+_kernel\w*|prep_\w+|corr_pyramid_\w+|\w+)(<[^(]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:90]


f = per_kernel(sys.argv[1], "FETCH_SIZE")
w = per_kernel(sys.argv[2], "WRITE_SIZE")
for k in sorted(set(f) | set(w)):
    rd = 2.0 * sum(f.get(k, [0])) / max(1, len(f.get(k, [])))
    wr = sum(w.get(k, [0])) / max(1, len(w.get(k, [])))
    print(json.dumps({"kernel": short(k), "dispatches": len(f.get(k, [])), "read_mb": round(rd / 1e6, 2),
                      "write_mb": round(wr / 1e6, 2), "total_mb": round((rd + wr) / 1e6, 2)}))
