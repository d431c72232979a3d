"""Drop-in for common.warp.warp_backwards — src/models/common/warp.py:5-33.

One rmd_warp_backwards launch (bilinear sample at grid + flow, zero padding, validity mask) instead of
the reference's two grid_samples over img2 and a ones tensor, compare and multiply.  Returns
(est1 * mask, mask) like the reference; the bool mask is one (B, 1, h, w) plane expanded to
(B, C, h, w) (its values are identical across channels in the reference too).  Gradient flows to
img2 only (the reference's callers detach the flow, impls/dicl.py:178).
"""

import torch

from .ops import _same_device


def warp_backwards(img2, flow, eps=1e-5):
    """warp img2 back to img1 based on flow -> (est1 * mask, mask) (torch.ops.rmd.warp_backwards)."""
    _same_device(img2, flow)
    out, mask = torch.ops.rmd.warp_backwards(img2, flow, float(eps))
    return out.to(img2.dtype), mask.expand(img2.shape)
