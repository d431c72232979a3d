#!/usr/bin/env python3
"""Golden vectors for the backward of raft_fs.CorrBlock (test infrastructure).

Runs the reference's own raft_fs.CorrBlock (src/models/impls/raft_fs.py:13-87) from /root/reference in
the build container, with feature maps that require gradients, and stores the gradients of a seeded
upstream gradient w.r.t. both feature maps (autograd through its avg_pool2d chain, grid_sample and
matmul).  Coordinates are detached, as every caller does (raft_fs.py:149).  Two cases: 4 levels r=4
with level 5 masked, and 3 levels r=3 on a ragged map.

Usage:  python tests/golden/gen_golden_fs_backward.py   (writes tests/golden/corr_fs_bwd_*.npz)
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import _coords, _import_reference  # noqa: E402


def main():
    import torch
    ref = _import_reference()
    t = torch.from_numpy
    rng = np.random.default_rng(2024)
    for name, (b, c, h, w, levels, r, sigma, mask) in {
        "corr_fs_bwd_b2_c32_24x40": (2, 32, 24, 40, 4, 4, 3.0, (5,)),
        "corr_fs_bwd_b1_c48_21x35_l3r3": (1, 48, 21, 35, 3, 3, 2.0, ()),
    }.items():
        f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
        f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
        co = _coords(rng, b, h, w, sigma, oob=False)
        tf1, tf2 = t(f1).requires_grad_(True), t(f2).requires_grad_(True)
        cb = ref["raft_fs"].CorrBlock(tf1, tf2, num_levels=levels, radius=r)
        out = cb(t(co), list(mask))
        g = rng.standard_normal(out.shape, dtype=np.float32)
        d1, d2 = torch.autograd.grad(out, (tf1, tf2), t(g))
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, fmap1=f1, fmap2=f2, coords=co, grad_out=g,
                            grad_fmap1=d1.numpy(), grad_fmap2=d2.numpy(), levels=np.int32(levels),
                            radius=np.int32(r), mask_costs=np.asarray(mask, dtype=np.int32))
        print(f"{name}.npz  {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
