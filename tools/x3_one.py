#!/usr/bin/env python3
"""Run the cfg2 correlation GEMM a few times with the current RMD_* diag knobs (for PMC passes).
usage: x3_one.py [precision]   (fp32 = the x3 kernel, default; bf16 = corr_pyramid_w8)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RMD_LIBRARY", os.path.join(ROOT, "raft-meets-dicl_amd", "rmd", "librmd_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402

f1, f2, _ = bench.synthetic(8, 256, 55, 128, 1, 1234, torch.device("cuda", 0))
for _ in range(6):
    ops.corr_pyramid(f1, f2, 4, sys.argv[1] if len(sys.argv) > 1 else "fp32")
torch.cuda.synchronize()
