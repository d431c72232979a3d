#!/usr/bin/env python3
"""Golden vectors for non-finite lookup coordinates, made by RUNNING the reference (test
infrastructure only; see gen_golden.py for the import stubs).

The reference's lookup is ``F.grid_sample`` (bilinear, zero padding, align_corners=True) on
coords / 2^i + delta (raft.CorrBlock.__call__, src/models/impls/raft.py:49-95; raft_fs.CorrBlock,
src/models/impls/raft_fs.py:13-87).  On the CPU a NaN or +-inf coordinate yields NaN for every
tap of the window (0 * NaN weight), while a huge finite one (1e30) yields zeros; these fixtures pin
that for rmd_corr_lookup and rmd_corr_otf_lookup.

Usage:  python tests/golden/gen_golden_nonfinite.py   (writes corr*_nonfinite.npz)
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import OUT, _coords, _import_reference  # noqa: E402


def main():
    import torch
    ref = _import_reference()
    rng = np.random.default_rng(4321)
    b, c, h, w, levels, radius = 2, 16, 16, 24, 4, 4
    f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    co = _coords(rng, b, h, w, 2.0)
    nan, inf = np.float32(np.nan), np.float32(np.inf)
    special = [((nan, 3.0)), ((5.0, nan)), ((nan, nan)), ((inf, 4.0)), ((-inf, 4.0)), ((6.0, inf)),
               ((6.0, -inf)), ((1e30, 2.0)), ((-1e30, -1e30)), ((nan, -500.0)), ((-500.0, nan)),
               ((3.0e6, 7.0)), ((2.5, -3.0e6))]
    for k, (x, y) in enumerate(special):
        bb, p = k % b, 7 * k + 3
        co[bb, 0].flat[p] = x
        co[bb, 1].flat[p] = y
    t = torch.from_numpy
    out = ref["raft"].CorrBlock(t(f1), t(f2), num_levels=levels, radius=radius)(t(co), [])
    out_fs = ref["raft_fs"].CorrBlock(t(f1), t(f2), num_levels=levels, radius=radius)(t(co), [])
    for name, o in (("corr_b2_c16_16x24_nonfinite", out), ("corr_fs_b2_c16_16x24_nonfinite", out_fs)):
        path = os.path.join(OUT, name + ".npz")
        np.savez_compressed(path, fmap1=f1, fmap2=f2, coords=co, out=o.detach().numpy(),
                            levels=np.int32(levels), radius=np.int32(radius), mask_costs=np.zeros(0, np.int32))
        print(f"{name}.npz  {os.path.getsize(path) / 1e6:.2f} MB  NaN entries {int(np.isnan(o.numpy()).sum())}")


if __name__ == "__main__":
    main()
