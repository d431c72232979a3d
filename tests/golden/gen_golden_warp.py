#!/usr/bin/env python3
"""Golden vectors for backward warping and the warped DICL volume, produced by RUNNING the reference.

Test infrastructure only; same import recipe as gen_golden.py.  Functions exercised (reference file:line):
  * common.warp.warp_backwards                     src/models/common/warp.py:5-33
  * impls.dicl.FlowLevel.forward -> compute_cost   src/models/impls/dicl.py:171-238 (coarse flow
    upsampled and detached, feat2 warped, integer volume with occlusion mask = the MatchingNet input)
Usage:  python tests/golden/gen_golden_warp.py        (writes tests/golden/warp_*.npz)
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from detinit import det_init  # noqa: E402
from gen_golden import OUT, _import_reference  # noqa: E402


def main():
    import torch
    import torch.nn.functional as F
    ref = _import_reference()
    from src.models.common import warp as ref_warp
    torch.manual_seed(0)
    rng = np.random.default_rng(2468)
    t = torch.from_numpy

    def save(name, **arrays):
        path = os.path.join(OUT, name + ".npz")
        np.savez_compressed(path, **arrays)
        print(f"{name}.npz  {os.path.getsize(path) / 1e6:.2f} MB  keys={sorted(arrays)}")

    # ---- warp_backwards: random flows plus border / out-of-bounds / integer cases -----------------
    b, c, h, w = 2, 8, 10, 12
    img2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    flow = (2.5 * rng.standard_normal((b, 2, h, w))).astype(np.float32)
    flow[0, :, 0, 0] = (0.0, 0.0)                       # corner, zero flow: valid
    flow[0, :, 0, 1] = (w - 2.0, h - 1.0)               # lands exactly on (w-1, h-1): valid
    flow[0, :, 1, 1] = (-1.5, 0.25)                     # half a pixel outside: invalid
    flow[0, :, 2, 2] = (3.0, 4.0)                       # integer displacement
    flow[1, :, 5, 5] = (100.0, -100.0)                  # far outside
    flow[1, :, 9, 11] = (1e-7, 0.0)                     # just past the last column (mask tolerance eps)
    timg = t(img2).requires_grad_(True)
    est, mask = ref_warp.warp_backwards(timg, t(flow))
    g = rng.standard_normal(est.shape, dtype=np.float32)
    (dimg,) = torch.autograd.grad(est, timg, t(g))
    save("warp_b2_c8_10x12", img2=img2, flow=flow, est=est.detach().numpy(), mask=mask.numpy(),
         grad_out=g, grad_img2=dimg.numpy())

    # ---- DICL level with a coarse flow: warp + masked integer volume (MatchingNet input) ----------
    b, c, h, w = 2, 16, 10, 12
    lvl = det_init(ref["dicl"].FlowLevel(c, 3, (3, 3))).eval()
    cap = {}
    lvl.mnet.register_forward_hook(lambda m, i, o: cap.update(mvol=i[0]))
    f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    f2[1, :, 4:6, 2:5] = 0.0                            # zero feature vectors: occlusion holes after warping
    coarse = (1.5 * rng.standard_normal((b, 2, h // 2, w // 2))).astype(np.float32)
    tf1, tf2 = t(f1).requires_grad_(True), t(f2).requires_grad_(True)
    lvl(None, tf1, tf2, t(coarse), ctx=False)
    flow_up = (2.0 * F.interpolate(t(coarse), (h, w), mode="bilinear", align_corners=True)).numpy()
    gm = rng.standard_normal(cap["mvol"].shape, dtype=np.float32)
    d1, d2 = torch.autograd.grad(cap["mvol"], (tf1, tf2), t(gm))
    save("warp_dicl_cost_b2_c16_10x12", fmap1=f1, fmap2=f2, flow_coarse=coarse, flow_up=flow_up,
         maxdisp=np.int32([3, 3]), mvol=cap["mvol"].detach().numpy(), grad_mvol=gm,
         grad_fmap1=d1.numpy(), grad_fmap2=d2.numpy())


if __name__ == "__main__":
    main()
