#!/usr/bin/env python3
"""Run ONE corr_pyramid variant (env RMD_GEMM_WAVES / RMD_ABLATE) at cfg2 and check ABL=0 results
against the default kernel on sampled queries.  Diagnostic only; one variant per process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402

dev = torch.device("cuda", 0)
f1, f2, co = bench.synthetic(8, 256, 55, 128, 12, 1234, dev)
pyr = ops.corr_pyramid(f1, f2, 4, "bf16")
out = ops.corr_lookup(pyr, co[3], 4)
torch.cuda.synchronize()
print("variant", os.environ.get("RMD_GEMM_WAVES"), os.environ.get("RMD_ABLATE"), "ok", float(out.abs().mean()))
