#!/usr/bin/env python3
"""Per-lookup time of the on-the-fly lookup (rmd_corr_otf_lookup) at cfg2 (B=8, 55x128, C=256, 4 levels,
r=4) on bench.py's synthetic coordinates, HIP events around each of 12 lookups x reps; run it once per
library build (RMD_LIBRARY=...) on one box for an A/B.  Prints one JSON line.
usage: python3 tools/otf_time.py [reps] [precision ...]; OTF_SHAPE=B,H,W overrides the map (4K: 2,270,480)"""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    precs = sys.argv[2:] or ["bf16", "fp32"]
    b, h, w = (int(v) for v in os.environ.get("OTF_SHAPE", "8,55,128").split(","))
    f1, f2, coords = bench.synthetic(b, 256, h, w, 12, 1234, "cuda")
    res = {"lib": os.environ.get("RMD_LIBRARY", "librmd.so"), "shape": [b, 256, h, w]}
    for p in precs:
        st = ops.otf_prepare(f1, f2, 4, p, scale=1.0)
        for i in range(12):
            ops.otf_lookup(st, coords[i], 4)
        ts = []
        for _ in range(reps):
            ev = []
            for i in range(12):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ops.otf_lookup(st, coords[i], 4)
                b.record()
                ev.append((a, b))
            torch.cuda.synchronize()
            ts += [a.elapsed_time(b) for a, b in ev]
        ts.sort()
        out = ops.otf_lookup(st, coords[5], 4)
        chk = float(out.float().abs().sum())
        res[p] = {"median_us": ts[len(ts) // 2] * 1e3, "min_us": ts[0] * 1e3, "checksum": chk,
                  "frac_140MB_of_8TBps": 140.0e6 / (ts[len(ts) // 2] * 1e-3) / 8e12}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
