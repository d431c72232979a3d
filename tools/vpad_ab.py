#!/usr/bin/env python3
"""A/B of the vmcnt padding of the GEMM tile loops (rmd_common.h vmcnt_pad_n) at cfg2 (diagnostic
build): RMD_W8_VPAD / RMD_X3_PAD = 1 (product) vs 0 (previous loop form, whose first k-steps wait for
the previous epilogue's store acknowledgements).  HIP events around the GEMM launch, interleaved
rounds, median; results compared bitwise with the product variant."""
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

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
f1, f2, _ = bench.synthetic(8, 256, 55, 128, 1, 1234, torch.device("cuda", 0))
res, ref, same = {}, {}, {}
for rnd in range(rounds):
    for prec, knob in (("bf16", "RMD_W8_VPAD"), ("fp32", "RMD_X3_PAD")):
        for v in ("1", "0"):
            os.environ[knob] = v
            ev = []
            for _ in range(2):
                ops.corr_pyramid(f1, f2, 4, prec)
            for _ in range(10):
                pyr = ops.corr_pyramid(f1, f2, 4, prec, events=ev)
            torch.cuda.synchronize()
            res.setdefault(f"{prec}_pad{v}", []).extend(a.elapsed_time(b) for a, b in ev)
            if rnd == 0:
                if v == "1":
                    ref[prec] = pyr.data.clone()
                else:
                    same[prec] = bool(torch.equal(pyr.data, ref[prec]))
            del pyr
print(json.dumps({"median_ms": {k: sorted(x)[len(x) // 2] for k, x in res.items()},
                  "min_ms": {k: min(x) for k, x in res.items()}, "bitwise_equal": same, "rounds": rounds}))
