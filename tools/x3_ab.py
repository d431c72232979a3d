#!/usr/bin/env python3
"""A/B timing of the fp32-mode (split-bf16, x3) correlation GEMM at cfg2 (diagnostic build).
RMD_X3_PP=1 (ping-pong phases, product) vs 0 (free-running waves); RMD_X3_QMAX = largest number of
query-tile quarters the persistent schedule may use (1 = one workgroup per block, the round-2 launch);
HIP events around the GEMM launch."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RMD_LIBRARY", os.path.join(ROOT, "raft-meets-dicl_amd", "rmd", "librmd_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402

dev = torch.device("cuda", 0)
f1, f2, _ = bench.synthetic(8, 256, 55, 128, 1, 1234, dev)
res, ref = {}, None
VARIANTS = {"1": ("1", "0", "8"), "0": ("0", "0", "8"), "pp_nostore": ("1", "1", "8"), "pp_epilogue_only": ("1", "2", "8"),
            "q1": ("1", "0", "1"), "q1_nostore": ("1", "1", "1"), "q2": ("1", "0", "2")}
for rnd in range(4):
    for v, (pp, abl, qs) in VARIANTS.items():
        os.environ["RMD_X3_QMAX"] = qs
        os.environ["RMD_X3_PP"] = pp
        os.environ["RMD_ABLATE"] = abl
        ev = []
        for _ in range(2):
            ops.corr_pyramid(f1, f2, 4, "fp32")
        for _ in range(10):
            pyr = ops.corr_pyramid(f1, f2, 4, "fp32", events=ev)
        torch.cuda.synchronize()
        res.setdefault(v, []).extend(a.elapsed_time(b) for a, b in ev)
        if ref is None:
            ref = pyr.data.clone()
        elif rnd == 0 and abl == "0":
            res["mismatch_" + v] = int((pyr.data != ref).sum())
out = {k: (sorted(v)[len(v) // 2] if isinstance(v, list) else v) for k, v in res.items()}
print(json.dumps({"pp_median_ms": out["1"], "free_median_ms": out["0"], "pp_nostore_ms": out["pp_nostore"],
                  "pp_epilogue_only_ms": out["pp_epilogue_only"], "q1_ms": out["q1"], "q1_nostore_ms": out["q1_nostore"],
                  "q2_ms": out["q2"], **{k: v for k, v in out.items() if k.startswith("mis")}}))
