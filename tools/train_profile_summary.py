#!/usr/bin/env python3
"""Per-step kernel time of the cfg5 training step (tools/train_probe.py under rocprofv3 --kernel-trace):
the kernels after the last idle gap of > 0.5 s (the timed steps), grouped into the rmd hot-path kernels
(by kernel) and everything else (MIOpen convolutions, rocBLAS/hipBLASLt GEMMs, torch elementwise, ...).
usage: train_profile_summary.py <kernel_trace.csv> <steps> -> JSON on stdout"""
import csv
import json
import sys


def group(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    if n.startswith("rmd::") or "_ZN3rmd" in n:
        return "rmd", n.split("(")[0].replace("rmd::", "")[:70]
    for key, label in (("miopen", "MIOpen"), ("igemm", "MIOpen"), ("naive_conv", "MIOpen"), ("batchnorm", "MIOpen"),
                       ("Cijk", "rocBLAS/hipBLASLt GEMM"), ("elementwise", "torch elementwise"),
                       ("reduce", "torch reduce"), ("multi_tensor", "optimizer (multi-tensor)"),
                       ("grid_sampler", "torch grid_sample"), ("upsample", "torch upsample")):
        if key.lower() in n.lower():
            return "other", label
    return "other", "other: " + n.split("(")[0][:50]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows]
    cut = 0
    for i in range(1, len(rows)):
        if starts[i] - int(rows[i - 1]["End_Timestamp"]) > 500_000_000:   # ns
            cut = i
    timed = rows[cut:]
    tot, rmd, other = 0.0, {}, {}
    for r in timed:
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / steps
        tot += t
        g, k = group(r["Kernel_Name"])
        d = rmd if g == "rmd" else other
        d[k] = d.get(k, 0.0) + t
    span = (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e6 / steps
    other = dict(sorted(other.items(), key=lambda kv: -kv[1]))
    out = {"kernels_after_gap": len(timed), "ms_per_step_span": span, "ms_per_step_kernels": tot,
           "rmd_ms_per_step": sum(rmd.values()), "rmd_share_of_kernel_time": sum(rmd.values()) / tot,
           "rmd_kernels_ms": dict(sorted(rmd.items(), key=lambda kv: -kv[1])),
           "other_ms_top": dict(list(other.items())[:15])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
