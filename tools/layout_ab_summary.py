#!/usr/bin/env python3
"""Per-layout medians of the lookup kernel's trace duration and PMC counters from tools/_gpu_layout_ab.sh
(rocprofv3 csv output under <dir>/{kt,fetch,sq,ta}); the kernel's LAY template argument tells the
layouts apart.  usage: layout_ab_summary.py <dir> -> JSON on stdout"""
import csv
import glob
import json
import os
import statistics
import sys


def lay(name):
    if "corr_lookup_kernel" not in name:
        return None
    return "tiles" if "Li4ELi3ELi1E" in name or ", 4, 3, 1>" in name else "rows"


def main():
    d = sys.argv[1]
    out = {"tiles": {}, "rows": {}}
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        durs = {"tiles": [], "rows": []}
        for r in csv.DictReader(open(f)):
            k = lay(r["Kernel_Name"])
            if k:
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in durs.items():
            if v:
                out[k]["trace_median_us"] = statistics.median(v)
                out[k]["trace_launches"] = len(v)
    for sub in ("fetch", "sq", "ta"):
        for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
            vals = {}
            for r in csv.DictReader(open(f)):
                k = lay(r["Kernel_Name"])
                if k:
                    vals.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
            for (k, c), v in vals.items():
                m = statistics.median(v)
                out[k][c] = m * 2048.0 if c == "FETCH_SIZE" else m      # KiB x2 (gfx950 wide-read correction)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
