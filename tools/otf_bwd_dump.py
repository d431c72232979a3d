#!/usr/bin/env python3
"""Gradients of a raft_fs on-the-fly block (cfg2 shape, 12 lookups, bench.py's synthetic inputs) written
to an .npz, to compare two library builds bitwise (RMD_LIBRARY=...).  usage: otf_bwd_dump.py out.npz [precision]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rmd  # noqa: E402


def main():
    prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, "cuda")
    g = torch.Generator(device="cpu").manual_seed(7)
    gouts = [torch.randn(8, 324, 55, 128, generator=g).cuda() for _ in range(12)]
    t1, t2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    cb = rmd.raft_fs.CorrBlock(t1, t2, 4, 4, precision=prec, method="otf")
    loss = sum((cb(coords[i]) * gouts[i]).sum() for i in range(12))
    g1, g2 = torch.autograd.grad(loss, (t1, t2))
    np.savez(sys.argv[1], g1=g1.cpu().numpy(), g2=g2.cpu().numpy())


if __name__ == "__main__":
    main()
