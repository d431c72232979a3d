#!/usr/bin/env python3
"""The bench.py headline step (operand prep + correlation GEMM + 12 lookups at cfg2) for a rocprofv3
--pmc pass: bench.py's live `roofline.traffic` runs this under `rocprofv3 --pmc FETCH_SIZE` and
`--pmc WRITE_SIZE` as a child process (rank 0, single-GPU runs) and averages the counters per launch
of the GEMM and lookup kernels (tools/pmc_summary.py does the same for hand-run passes).

usage: python3 tools/pmc_probe.py [--precision bf16] [--steps 3] [--batch 8]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=436)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--channels", type=int, default=256)
    ap.add_argument("--iters", type=int, default=12)
    a = ap.parse_args()
    import torch
    import bench
    from rmd import ops
    h, w = bench.padded(a.height, a.width)
    f1, f2, coords = bench.synthetic(a.batch, a.channels, h // 8, w // 8, a.iters, 1234, "cuda")
    for _ in range(a.steps):
        pyr = ops.corr_pyramid(f1, f2, 4, a.precision)
        for it in range(a.iters):
            ops.corr_lookup(pyr, coords[it], 4)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
