#!/usr/bin/env python3
"""Per-dispatch SQ/GRBM counters of one kernel from a rocprofv3 `--pmc ... --kernel-trace` run, with the
derived effective clock and MFMA-busy fraction (MI355X_MICROARCH.md 'DVFS give-back' and the
cycle-constants row of SQ_VALU_MFMA_BUSY_CYCLES):

  clock_ghz  = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (cycles the matrix pipes
               were busy over the cycles the chip was busy, averaged over every SIMD)

usage: pmc_clock.py <rocprofv3 output dir> <kernel-name pattern> [label] -> one JSON line
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, pat = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else pat
    vals = collections.defaultdict(dict)       # dispatch -> counter -> value
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if pat in r["Kernel_Name"]:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                vals[key][r["Counter_Name"]] = vals[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    durs = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if pat in r["Kernel_Name"]:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                durs[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    keys = [k for k in vals if k in durs] or list(vals)
    if not keys:
        print(json.dumps({"label": label, "error": "no dispatch of " + pat}))
        return
    # drop the first dispatch (cold caches, first-launch clock ramp) when there are several
    if len(keys) > 2:
        keys = sorted(keys, key=lambda k: int(k))[1:]
    counters = sorted({c for k in keys for c in vals[k]})
    avg = {c: sum(vals[k].get(c, 0.0) for k in keys) / len(keys) for c in counters}
    res = {"label": label, "dispatches": len(keys), **{c: round(v, 1) for c, v in avg.items()}}
    if all(k in durs for k in keys):
        dur = sorted(durs[k] for k in keys)
        res["duration_ms_median"] = round(dur[len(dur) // 2] * 1e3, 4)
        res["duration_ms_mean"] = round(sum(dur) / len(dur) * 1e3, 4)
        if "GRBM_GUI_ACTIVE" in avg:
            res["clock_ghz"] = round(avg["GRBM_GUI_ACTIVE"] / 8 / (sum(dur) / len(dur)) / 1e9, 3)
    if "GRBM_GUI_ACTIVE" in avg and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        res["mfma_busy"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * avg["GRBM_GUI_ACTIVE"] / 8), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
