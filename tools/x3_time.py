#!/usr/bin/env python3
"""GEMM-only time of the fp32-mode correlation pyramid (corr_pyramid_x3) at cfg2 (B=8, 55x128, C=256,
4 levels): HIP events around the rmd_corr_pyramid_prepared launch (ops.corr_pyramid(events=...)), reps
launches; run once per library build (RMD_LIBRARY=...) on one box for an A/B.  Prints one JSON line with
a checksum of the pyramid (equal across builds = same results).
usage: python3 tools/x3_time.py [reps] [precision]"""
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
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    f1, f2, _ = bench.synthetic(8, 256, 55, 128, 1, 1234, "cuda")
    fill = os.environ.get("X3_FILL", "")          # power check: 'zero' operands (DVFS give-back)
    if fill == "zero":
        f1.zero_()
        f2.zero_()
    res = {"lib": os.path.basename(os.environ.get("RMD_LIBRARY", "librmd.so")), "precision": prec}
    ts = []
    pyr = None
    for i in range(reps + 3):
        ev = []
        del pyr
        pyr = ops.corr_pyramid(f1, f2, 4, prec, events=ev)
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(ev[0][0].elapsed_time(ev[0][1]))
    ts.sort()
    data = pyr.data if hasattr(pyr, "data") else pyr
    if data.dtype == torch.uint8:                 # RMD_S24 bytes
        from rmd import library
        data = library.s24_decode(data)
    res.update({"median_ms": ts[len(ts) // 2], "min_ms": ts[0],
                "checksum": float(data.double().abs().sum()), "nan": bool(torch.isnan(data).any())})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
