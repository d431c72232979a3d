"""Drop-in for common.warp.warp_backwards — src/models/common/warp.py:5-33.

One rmd_warp_backwards launch (bilinear sample at grid + flow, zero padding, validity mask) instead of
the reference's two grid_samples over img2 and a ones tensor, compare and multiply.  Returns
(est1 * mask, mask) like the reference; the bool mask is one (B, 1, h, w) plane expanded to
(B, C, h, w) (its values are identical across channels in the reference too).  Gradient flows to
img2 only (the reference's callers detach the flow, impls/dicl.py:178).
"""

import torch

from . import _lib
from .ops import _ptr, _require_gpu, _stream


class _Warp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img2, flow, eps):
        _require_gpu(img2, flow)
        b, c, h, w = img2.shape
        if tuple(flow.shape) != (b, 2, h, w):
            raise ValueError(f"warp_backwards: flow {tuple(flow.shape)} must be (B, 2, h, w) for img2 {tuple(img2.shape)}")
        ic = img2.detach().float().contiguous()
        fc = flow.detach().float().contiguous()
        out = torch.empty_like(ic)
        mask = torch.empty((b, 1, h, w), dtype=torch.uint8, device=ic.device)
        with torch.cuda.device(ic.device):
            _lib.check(_lib.lib().rmd_warp_backwards(_ptr(ic), _ptr(fc), b, c, h, w, float(eps), _ptr(out), _ptr(mask),
                                                     _stream(ic)), "rmd_warp_backwards")
        ctx.save_for_backward(fc)
        ctx.meta = (b, c, h, w, float(eps), img2.dtype)
        ctx.mark_non_differentiable(mask)
        return out.to(img2.dtype), mask.bool().expand(b, c, h, w)

    @staticmethod
    def backward(ctx, grad, _gmask):
        (fc,) = ctx.saved_tensors
        b, c, h, w, eps, dtype = ctx.meta
        g = grad.float().contiguous()
        gi = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            _lib.check(_lib.lib().rmd_warp_backwards_backward(_ptr(g), _ptr(fc), b, c, h, w, eps, _ptr(gi), _stream(g)),
                       "rmd_warp_backwards_backward")
        return gi.to(dtype), None, None


def warp_backwards(img2, flow, eps=1e-5):
    """warp img2 back to img1 based on flow -> (est1 * mask, mask)."""
    return _Warp.apply(img2, flow, eps)
