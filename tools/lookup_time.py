#!/usr/bin/env python3
"""Per-lookup time of rmd_corr_lookup at cfg2 (B=8, 55x128, C=256, 4 levels, r=4) on bench.py's synthetic
coordinates for the bf16 (tiles layout) and fp32 (row layout) pyramids, HIP events around each of 12
lookups x reps; run once per library build (RMD_LIBRARY=...) on one box for an A/B.  Prints one JSON
line with a checksum of one output (equal across builds = same results).
usage: python3 tools/lookup_time.py [reps] [precision ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    precs = sys.argv[2:] or ["bf16", "fp32"]
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, "cuda")
    res = {"lib": os.path.basename(os.environ.get("RMD_LIBRARY", "librmd.so"))}
    for p in precs:
        pyr = ops.corr_pyramid(f1, f2, 4, p)
        for i in range(12):
            ops.corr_lookup(pyr, coords[i], 4)
        ts = []
        for _ in range(reps):
            ev = []
            for i in range(12):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ops.corr_lookup(pyr, coords[i], 4)
                b.record()
                ev.append((a, b))
            torch.cuda.synchronize()
            ts += [a.elapsed_time(b) for a, b in ev]
        ts.sort()
        out = ops.corr_lookup(pyr, coords[7], 4)
        res[p] = {"median_us": ts[len(ts) // 2] * 1e3, "min_us": ts[0] * 1e3,
                  "checksum": float(out.double().abs().sum()), "nan": bool(torch.isnan(out).any())}
        del pyr, out
    print(json.dumps(res))


if __name__ == "__main__":
    main()
