#!/usr/bin/env python3
"""Summarise rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE PMC passes of bench.py into
profiles/pmc_<round>.json (per-launch HBM bytes of the GEMM and lookup kernels).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE
counts exactly half the bytes of wide coalesced streaming reads, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane stores.
usage: pmc_summary.py <prof_dir> <out.json> <precision>
"""
import csv
import glob
import json
import os
import sys


def per_kernel(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        key = "gemm" if "corr_pyramid_" in name else \
              "lookup" if "corr_lookup_kernel" in name else "prep" if "prep_" in name else None
        if key:
            vals.setdefault(key, []).append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    d, out, precision = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = per_kernel(glob.glob(os.path.join(d, "*fetch*counter_collection.csv"))[0], "FETCH_SIZE")
    write = per_kernel(glob.glob(os.path.join(d, "*write*counter_collection.csv"))[0], "WRITE_SIZE")
    stats = {}
    for r in csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_stats.csv"))[0])):
        stats[r["Name"][:120]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    res = {}
    for k in ("gemm", "lookup", "prep"):
        if k in fetch and k in write:
            res[k] = {"fetch_bytes": 2.0 * fetch[k], "write_bytes": write[k],
                      "hbm_bytes_per_launch": 2.0 * fetch[k] + write[k]}
    entry = {"gemm_hbm_bytes_per_launch": res.get("gemm", {}).get("hbm_bytes_per_launch"),
             "lookup_hbm_bytes_per_launch": res.get("lookup", {}).get("hbm_bytes_per_launch"),
             "detail": res, "kernel_stats": stats,
             "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes"}
    allres = {}
    if os.path.exists(out):
        allres = json.load(open(out))
    allres[precision] = entry
    json.dump(allres, open(out, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
