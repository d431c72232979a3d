#!/usr/bin/env python3
"""Diagnostic ablations of the cfg2 hot-path kernels (MI355X only; not part of the product).

Times, in one process with HIP events on the launch stream:
  * HBM write / copy baselines (torch fill_ / copy_ of ~1.1 GB),
  * rmd_corr_pyramid with RMD_ABLATE = 0 (normal), 1 (stores to a trash slot), 2 (no MFMA),
  * rmd_corr_lookup  with RMD_ABLATE = 0, 1 (no output traffic), 2 (no pyramid loads), and
    all levels masked (stores of zeros only).
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    from rmd import ops
    dev = torch.device("cuda", 0)
    res = {}
    big = torch.empty(int(1.1e9) // 4, dtype=torch.float32, device=dev)
    t = timeit(lambda: big.fill_(1.0))
    res["fill_1.1GB_ms"] = t
    res["fill_TBps"] = big.numel() * 4 / t / 1e9
    src = torch.empty(int(0.55e9) // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    t = timeit(lambda: dst.copy_(src))
    res["copy_0.55GB_TBps"] = 2 * src.numel() * 4 / t / 1e9
    del big, src, dst
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, dev)
    for waves in ("8", "4"):
        os.environ["RMD_GEMM_WAVES"] = waves
        for abl in (0, 1, 2):
            os.environ["RMD_ABLATE"] = str(abl)
            res[f"corr_pyramid_w{waves}_abl{abl}_ms"] = timeit(lambda: ops.corr_pyramid(f1, f2, 4, "bf16"))
    os.environ["RMD_ABLATE"] = "0"
    os.environ.pop("RMD_GEMM_WAVES")
    os.environ["RMD_FORCE_TILED_GEMM"] = "1"
    res["corr_pyramid_tiled_bf16_ms"] = timeit(lambda: ops.corr_pyramid(f1, f2, 4, "bf16"))
    os.environ.pop("RMD_FORCE_TILED_GEMM")
    res["corr_pyramid_fp32_ms"] = timeit(lambda: ops.corr_pyramid(f1, f2, 4, "fp32"), reps=3, warm=1)
    pyr = ops.corr_pyramid(f1, f2, 4, "bf16")
    for abl in (0, 1, 2):
        os.environ["RMD_ABLATE"] = str(abl)
        res[f"lookup_abl{abl}_ms"] = timeit(lambda: ops.corr_lookup(pyr, coords[5], 4))
    os.environ["RMD_ABLATE"] = "0"
    res["lookup_all_masked_ms"] = timeit(lambda: ops.corr_lookup(pyr, coords[5], 4, mask_costs=[3, 4, 5, 6]))
    res["lookup_zero_flow_ms"] = timeit(lambda: ops.corr_lookup(pyr, coords[0] * 0 + bench.synthetic(8, 1, 55, 128, 1, 0, dev)[2][0] * 0, 4))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
