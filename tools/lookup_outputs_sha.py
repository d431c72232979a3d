#!/usr/bin/env python3
"""sha256 of all 12 bench-step lookup outputs (cfg2, bf16 and fp32 pyramids) for the library in
RMD_LIBRARY: equal digests across A/B builds = bitwise-equal results.  usage: python3 tools/lookup_outputs_sha.py"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402

f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, "cuda")
res = {"lib": os.path.basename(os.environ.get("RMD_LIBRARY", "librmd.so"))}
for p in ("bf16", "fp32"):
    pyr = ops.corr_pyramid(f1, f2, 4, p)
    h = hashlib.sha256()
    for i in range(12):
        h.update(ops.corr_lookup(pyr, coords[i], 4).cpu().numpy().tobytes())
    # a masked level and far-off coordinates too
    h.update(ops.corr_lookup(pyr, coords[5] * 3.0 - 40.0, 4, mask_costs=[1]).cpu().numpy().tobytes())
    res[p] = h.hexdigest()[:16]
print(json.dumps(res))
