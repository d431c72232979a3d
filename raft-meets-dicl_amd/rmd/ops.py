"""Torch-facing wrappers over the C ABI (include/rmd.h): device checks, allocation, streams.

Outputs and workspaces come from torch's caching allocator; the C launchers only enqueue kernels
on torch's current HIP stream.  Every function requires GPU tensors and raises otherwise.
"""

import ctypes

import torch

from . import _lib
from ._lib import RMD_BF16, RMD_F16, RMD_F32

# precision modes: (GEMM compute type, pyramid storage type)
PRECISIONS = {
    "fp32": (RMD_F32, RMD_F32),       # exact f32 MFMA, f32 pyramid: the parity mode (default)
    "bf16": (RMD_BF16, RMD_F16),      # bf16 MFMA operands, f32 accumulate, fp16 pyramid: perf mode
    "bf16-f32": (RMD_BF16, RMD_F32),  # bf16 operands, f32 pyramid
    "fp32-f16": (RMD_F32, RMD_F16),   # exact f32 GEMM, fp16 pyramid
}
_default_precision = "fp32"


def set_default_precision(name):
    global _default_precision
    if name not in PRECISIONS:
        raise ValueError(f"unknown precision '{name}', expected one of {sorted(PRECISIONS)}")
    _default_precision = name


def get_default_precision():
    return _default_precision


def _require_gpu(*tensors):
    for t in tensors:
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise RuntimeError("rmd: HIP kernels need GPU tensors (no CPU fallback exists)")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


_STORAGE_DTYPE = {RMD_F32: torch.float32, RMD_F16: torch.float16}


class Pyramid:
    """Correlation pyramid in the tiled, query-minor HBM layout of include/rmd.h."""

    def __init__(self, data, desc, channels):
        self.data = data
        self.desc = desc
        self.channels = channels

    @property
    def levels(self):
        return self.desc.levels

    def level_shape(self, i):
        return self.desc.level_h[i], self.desc.level_w[i]

    def unpack(self, i):
        """Level i in the reference layout (B, H, W, 1, H_i, W_i) as float32 — for tests/debugging."""
        d = self.desc
        b, h, w = d.batch, d.height, d.width
        th, tw, ty, tx = d.tile_h[i], d.tile_w[i], d.tiles_y[i], d.tiles_x[i]
        hl, wl = d.level_h[i], d.level_w[i]
        n = h * w
        off = d.level_offset[i]
        x = self.data[off: off + b * ty * tx * n * th * tw].view(b, ty, tx, n, th, tw)
        x = x.permute(0, 3, 1, 4, 2, 5).reshape(b, n, ty * th, tx * tw)[:, :, :hl, :wl]
        return x.float().reshape(b, h, w, 1, hl, wl)


def corr_pyramid(fmap1, fmap2, levels=4, precision=None):
    """raft.CorrBlock.__init__ (raft.py:18-47) on the GPU -> Pyramid."""
    _require_gpu(fmap1, fmap2)
    if fmap1.shape != fmap2.shape or fmap1.dim() != 4:
        raise ValueError(f"fmap1/fmap2 must be equal (B,C,H,W) shapes, got {tuple(fmap1.shape)} / {tuple(fmap2.shape)}")
    compute, storage = PRECISIONS[precision or _default_precision]
    f1 = fmap1.detach().float().contiguous()
    f2 = fmap2.detach().float().contiguous()
    b, c, h, w = f1.shape
    d = _lib.describe(b, h, w, levels, storage)
    lib = _lib.lib()
    ws_bytes = lib.rmd_corr_pyramid_workspace_bytes(ctypes.byref(d), c, compute)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=f1.device)
    data = torch.empty(d.total_elements, dtype=_STORAGE_DTYPE[storage], device=f1.device)
    with torch.cuda.device(f1.device):
        _lib.check(lib.rmd_corr_pyramid(_ptr(f1), _ptr(f2), c, ctypes.byref(d), compute, _ptr(data), _ptr(ws),
                                        _lib.stream_ptr(f1.device)), "rmd_corr_pyramid")
    return Pyramid(data, d, c)


def corr_lookup(pyr, coords, radius, mask_costs=()):
    """raft.CorrBlock.__call__ (raft.py:49-95) on the GPU -> (B, L*(2r+1)^2, H, W) float32."""
    _require_gpu(pyr.data, coords)
    d = pyr.desc
    if tuple(coords.shape) != (d.batch, 2, d.height, d.width):
        raise ValueError(f"coords must be (B,2,H,W)=({d.batch},2,{d.height},{d.width}), got {tuple(coords.shape)}")
    co = coords.detach().float().contiguous()
    mask = 0
    for m in mask_costs:
        if 0 <= m - 3 < d.levels:
            mask |= 1 << (m - 3)
    dd = (2 * radius + 1) ** 2
    out = torch.empty((d.batch, d.levels * dd, d.height, d.width), dtype=torch.float32, device=co.device)
    with torch.cuda.device(co.device):
        _lib.check(_lib.lib().rmd_corr_lookup(_ptr(pyr.data), ctypes.byref(d), _ptr(co), radius, mask, _ptr(out),
                                              _lib.stream_ptr(co.device)), "rmd_corr_lookup")
    return out
