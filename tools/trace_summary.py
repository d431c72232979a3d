#!/usr/bin/env python3
"""Median kernel duration per (kernel, grid) from a rocprofv3 kernel_trace.csv, for kernels whose
name contains a pattern.  usage: trace_summary.py <kernel_trace.csv> <pattern>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2]
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if pat in n:
        key = (n.replace("void ", "")[:60], r.get("Grid_Size_X", ""), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""),
               r.get("Workgroup_Size_X", ""))
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    v.sort()
    print(f"{k}  n={len(v)}  median_us={v[len(v) // 2]:.2f}  min_us={v[0]:.2f}")
