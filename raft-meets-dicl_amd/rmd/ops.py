"""Torch-facing wrappers over the C ABI (include/rmd.h): device checks, allocation, streams.

Outputs and workspaces come from torch's caching allocator; the C launchers only enqueue kernels
on torch's current HIP stream.  Every function requires GPU tensors and raises otherwise.
"""

import ctypes

import torch

from . import _lib
from ._lib import RMD_BF16, RMD_BF16X3, RMD_F16, RMD_F32

# precision modes: (GEMM compute type, pyramid storage type)
PRECISIONS = {
    "fp32": (RMD_BF16X3, RMD_F32),    # fp32-accurate split-bf16 MFMA (3 products), f32 pyramid: parity mode (default)
    "fp32-exact": (RMD_F32, RMD_F32), # exact f32 MFMA (v_mfma_f32_32x32x2_f32), f32 pyramid
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

    def __init__(self, data, desc, channels, scale):
        self.data = data
        self.desc = desc
        self.channels = channels
        self.scale = scale

    @property
    def levels(self):
        return self.desc.levels

    def level_shape(self, i):
        return self.desc.level_h[i], self.desc.level_w[i]

    def unpack(self, i):
        """Level i in the reference layout (B, H, W, 1, H_i, W_i) as float32 — for tests/debugging."""
        d = self.desc
        b, h, w = d.batch, d.height, d.width
        cw, nc = d.tile_w[i], d.tiles_x[i]
        hl, wl = d.level_h[i], d.level_w[i]
        n = h * w
        off = d.level_offset[i]
        x = self.data[off: off + b * hl * nc * n * cw].view(b, hl, nc, n, cw)
        x = x.permute(0, 3, 1, 2, 4).reshape(b, n, hl, nc * cw)[..., :wl]
        return x.float().reshape(b, h, w, 1, hl, wl)


def corr_pyramid(fmap1, fmap2, levels=4, precision=None, events=None, scale=None):
    """raft.CorrBlock.__init__ (raft.py:18-47) on the GPU -> Pyramid.

    ``scale`` multiplies the products: None = 1/sqrt(C) (raft.py:33), 1.0 = raft_fs.CorrBlock.

    ``events`` (optional list) receives (start, end) HIP events bracketing the GEMM launch alone
    (the operand prep runs before the start event) — bench.py's roofline timing.
    """
    _require_gpu(fmap1, fmap2)
    if fmap1.shape != fmap2.shape or fmap1.dim() != 4:
        raise ValueError(f"fmap1/fmap2 must be equal (B,C,H,W) shapes, got {tuple(fmap1.shape)} / {tuple(fmap2.shape)}")
    compute, storage = PRECISIONS[precision or _default_precision]
    f1 = fmap1.detach().float().contiguous()
    f2 = fmap2.detach().float().contiguous()
    b, c, h, w = f1.shape
    scale = 1.0 / float(c) ** 0.5 if scale is None else float(scale)
    d = _lib.describe(b, h, w, levels, storage)
    lib = _lib.lib()
    ws_bytes = lib.rmd_corr_pyramid_workspace_bytes(ctypes.byref(d), c, compute)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=f1.device)
    data = torch.empty(d.total_elements, dtype=_STORAGE_DTYPE[storage], device=f1.device)
    with torch.cuda.device(f1.device):
        stream = _lib.stream_ptr(f1.device)
        _lib.check(lib.rmd_corr_prepare(_ptr(f1), _ptr(f2), c, scale, ctypes.byref(d), compute, _ptr(ws), stream),
                   "rmd_corr_prepare")
        if events is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _lib.check(lib.rmd_corr_pyramid_prepared(c, scale, ctypes.byref(d), compute, _ptr(data), _ptr(ws), stream),
                   "rmd_corr_pyramid_prepared")
        if events is not None:
            e1.record()
            events.append((e0, e1))
    return Pyramid(data, d, c, scale)


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


# ---- on-the-fly lookup (raft_fs semantics without the volume) -------------------------------------

class OtfState:
    """Operand rows of rmd_corr_otf_prepare (query rows * scale, pooled target rows of every level)."""

    def __init__(self, ws, b, c, h, w, levels, compute):
        self.ws, self.b, self.c, self.h, self.w, self.levels, self.compute = ws, b, c, h, w, levels, compute


def otf_prepare(fmap1, fmap2, levels, precision=None, scale=1.0):
    _require_gpu(fmap1, fmap2)
    if fmap1.shape != fmap2.shape or fmap1.dim() != 4:
        raise ValueError(f"fmap1/fmap2 must be equal (B,C,H,W) shapes, got {tuple(fmap1.shape)} / {tuple(fmap2.shape)}")
    compute = PRECISIONS[precision or _default_precision][0]
    if compute == RMD_BF16X3:           # the on-the-fly kernels take exact f32 or bf16 operands
        compute = RMD_F32
    f1 = fmap1.detach().float().contiguous()
    f2 = fmap2.detach().float().contiguous()
    b, c, h, w = f1.shape
    lib = _lib.lib()
    nbytes = lib.rmd_corr_otf_workspace_bytes(b, c, h, w, levels, compute)
    if nbytes == 0:
        raise ValueError(f"otf: unsupported sizes {tuple(f1.shape)} with {levels} levels")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=f1.device)
    with torch.cuda.device(f1.device):
        _lib.check(lib.rmd_corr_otf_prepare(_ptr(f1), _ptr(f2), b, c, h, w, levels, float(scale), compute, _ptr(ws),
                                            _lib.stream_ptr(f1.device)), "rmd_corr_otf_prepare")
    return OtfState(ws, b, c, h, w, levels, compute)


def otf_lookup(st, coords, radius, mask_costs=()):
    _require_gpu(st.ws, coords)
    if tuple(coords.shape) != (st.b, 2, st.h, st.w):
        raise ValueError(f"coords must be (B,2,H,W)=({st.b},2,{st.h},{st.w}), got {tuple(coords.shape)}")
    co = coords.detach().float().contiguous()
    dd = (2 * radius + 1) ** 2
    out = torch.empty((st.b, st.levels * dd, st.h, st.w), dtype=torch.float32, device=co.device)
    with torch.cuda.device(co.device):
        _lib.check(_lib.lib().rmd_corr_otf_lookup(_ptr(st.ws), st.b, st.c, st.h, st.w, st.levels, st.compute, _ptr(co),
                                                  radius, _mask_bits(mask_costs, st.levels), _ptr(out),
                                                  _lib.stream_ptr(co.device)), "rmd_corr_otf_lookup")
    return out


# ---- RAFT correlation autograd (training) -------------------------------------------------------
#
# The pyramid Function returns a scalar "token" that every lookup of the same CorrBlock takes as an
# input, so autograd runs all lookup backwards before the pyramid backward.  Each lookup backward
# accumulates into ONE dense fp32 gradient G (B, T, N), query-minor, shared through _CorrState (include/rmd.h,
# rmd_corr_lookup_backward); the pyramid backward then turns G into d fmap1 / d fmap2 with two
# library GEMMs (hipBLASLt; fp32 modes: three split-bf16 products each with fp32 accumulation,
# fp32-exact: plain fp32) and the native pool / unpool kernels.

class _CorrState:
    def __init__(self, pyr, f1, f2, precision):
        self.pyr = pyr
        self.f1 = f1
        self.f2 = f2
        self.precision = precision
        self.grad = None          # dense G, allocated by the first lookup backward


def _mask_bits(mask_costs, levels):
    mask = 0
    for m in mask_costs:
        if 0 <= m - 3 < levels:
            mask |= 1 << (m - 3)
    return mask


class _CorrPyramidFn(torch.autograd.Function):
    """Autograd node of raft.CorrBlock.__init__ (raft.py:18-47)."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, state):
        ctx.state = state
        return fmap1.new_zeros(())

    @staticmethod
    def backward(ctx, _gtoken):
        st = ctx.state
        f1, f2 = st.f1, st.f2
        b, c, h, w = f1.shape
        n = h * w
        levels = st.pyr.levels
        if st.grad is None:
            return torch.zeros_like(f1), torch.zeros_like(f2), None
        lib = _lib.lib()
        t = lib.rmd_corr_grad_targets(h, w, levels)
        scale = st.pyr.scale
        pooled = torch.empty((b, c, t), dtype=torch.float32, device=f1.device)
        g2 = torch.empty_like(f2)
        with torch.cuda.device(f1.device):
            stream = _stream(f1)
            _lib.check(lib.rmd_corr_pool_targets(_ptr(f2), b, c, h, w, levels, scale, _ptr(pooled), stream),
                       "rmd_corr_pool_targets")
            G = st.grad.view(b, t, n)
            f1m = f1.view(b, c, n)
            if PRECISIONS[st.precision][0] == RMD_F32:
                g1 = torch.bmm(pooled, G)                                   # (B, C, N)   exact fp32
                dpool = torch.bmm(f1m, G.transpose(1, 2))                   # (B, C, T)
            else:
                Gs = _split(G)                                              # G split once, used twice
                g1 = _bmm_split(_split(pooled), Gs, st.precision)
                dpool = _bmm_split(_split(f1m), Gs, st.precision, transpose_b=True)
            _lib.check(lib.rmd_corr_unpool_targets(_ptr(dpool), b, c, h, w, levels, scale, _ptr(g2), stream),
                       "rmd_corr_unpool_targets")
        st.grad = None
        return g1.view(b, c, h, w), g2, None


def _split(x):
    """x (fp32) -> (hi, lo) bf16 with x ~= hi + lo (rmd_split_bf16)."""
    x = x.contiguous()
    hi = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    lo = torch.empty_like(hi)
    _lib.check(_lib.lib().rmd_split_bf16(_ptr(x), x.numel(), _ptr(hi), _ptr(lo), _stream(x)), "rmd_split_bf16")
    return hi, lo


def _bmm_split(a, b, precision, transpose_b=False):
    """a (B, M, K) @ b (B, K, N) [or b^T for b (B, N, K)], operands given split (_split), with fp32
    output from bf16 library GEMMs (hipBLASLt, fp32 accumulation): hi.hi + hi.lo + lo.hi for the
    fp32 modes, hi.hi for bf16."""
    ah, al = a
    bh, bl = b
    if transpose_b:
        bh, bl = bh.transpose(1, 2), bl.transpose(1, 2)
    out = torch.bmm(ah, bh, out_dtype=torch.float32)
    if PRECISIONS[precision][0] != RMD_BF16:
        out += torch.bmm(ah, bl, out_dtype=torch.float32)
        out += torch.bmm(al, bh, out_dtype=torch.float32)
    return out


class _CorrLookupFn(torch.autograd.Function):
    """Autograd node of raft.CorrBlock.__call__ (raft.py:49-95); coords carry no gradient (raft.py:402)."""

    @staticmethod
    def forward(ctx, token, coords, state, radius, mask_costs):
        out = corr_lookup(state.pyr, coords, radius, mask_costs)
        ctx.state = state
        ctx.radius = radius
        ctx.mask = _mask_bits(mask_costs, state.pyr.levels)
        ctx.save_for_backward(coords.detach().float().contiguous())
        return out

    @staticmethod
    def backward(ctx, gout):
        (co,) = ctx.saved_tensors
        st = ctx.state
        d = st.pyr.desc
        lib = _lib.lib()
        if st.grad is None:
            t = lib.rmd_corr_grad_targets(d.height, d.width, d.levels)
            st.grad = torch.zeros(d.batch * d.height * d.width * t, dtype=torch.float32, device=co.device)
        g = gout.float().contiguous()
        with torch.cuda.device(co.device):
            _lib.check(lib.rmd_corr_lookup_backward(_ptr(g), ctx_desc(st), _ptr(co), ctx.radius, ctx.mask,
                                                    _ptr(st.grad), _stream(co)), "rmd_corr_lookup_backward")
        return gout.new_zeros(()), None, None, None, None


def ctx_desc(st):
    return ctypes.byref(st.pyr.desc)


def corr_block_autograd(fmap1, fmap2, levels, precision, scale=None):
    """Pyramid + autograd token for a CorrBlock whose feature maps require gradients."""
    _require_gpu(fmap1, fmap2)
    precision = precision or _default_precision
    pyr = corr_pyramid(fmap1, fmap2, levels, precision, scale=scale)
    st = _CorrState(pyr, fmap1.detach().float().contiguous(), fmap2.detach().float().contiguous(), precision)
    token = _CorrPyramidFn.apply(fmap1, fmap2, st)
    return pyr, st, token


def corr_lookup_autograd(token, state, coords, radius, mask_costs=()):
    return _CorrLookupFn.apply(token, coords, state, radius, tuple(mask_costs))


# ---- DICL cost volumes and DAP ------------------------------------------------------------------

def _stream(t):
    return _lib.stream_ptr(t.device)


class _DiclStack(torch.autograd.Function):
    """stack = [f1 expanded | bilinear(f2, coords/2^level + delta)] — corr/dicl.py:26-54."""

    @staticmethod
    def forward(ctx, f1, f2, coords, radius, level, norm_hw, extra_delta):
        _require_gpu(f1, f2, coords)
        f1c = f1.detach().float().contiguous()
        f2c = f2.detach().float().contiguous()
        co = coords.detach().float().contiguous()
        b, c, h, w = f1c.shape
        hl, wl = f2c.shape[-2:]
        if f2c.shape[:2] != (b, c) or tuple(co.shape) != (b, 2, h, w):
            raise ValueError("dicl_stack: fmap2 must be (B,C,hl,wl) and coords (B,2,h,w) matching fmap1")
        nh, nw = norm_hw if norm_hw is not None else (h, w)
        d = 2 * radius + 1
        out = torch.empty((b, d, d, 2 * c + (2 if extra_delta else 0), h, w), dtype=torch.float32,
                          device=f1c.device)
        with torch.cuda.device(f1c.device):
            _lib.check(_lib.lib().rmd_dicl_stack(_ptr(f1c), _ptr(f2c), _ptr(co), b, c, h, w, hl, wl, radius, level,
                                                 nh, nw, int(bool(extra_delta)), _ptr(out), _stream(f1c)),
                       "rmd_dicl_stack")
        ctx.save_for_backward(co)
        ctx.meta = (b, c, h, w, hl, wl, radius, level, nh, nw, int(bool(extra_delta)))
        return out

    @staticmethod
    def backward(ctx, grad):
        (co,) = ctx.saved_tensors
        b, c, h, w, hl, wl, radius, level, nh, nw, extra = ctx.meta
        g = grad.float().contiguous()
        g1 = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
        g2 = torch.empty((b, c, hl, wl), dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            _lib.check(_lib.lib().rmd_dicl_stack_backward(_ptr(g), _ptr(co), b, c, h, w, hl, wl, radius, level, nh,
                                                          nw, extra, _ptr(g1), _ptr(g2), _stream(g)),
                       "rmd_dicl_stack_backward")
        return g1, g2, None, None, None, None, None


def dicl_stack(fmap1, fmap2, coords, radius, level=0, norm_hw=None, extra_delta=False):
    """(B,C,h,w), (B,C,hl,wl), (B,2,h,w) -> (B, 2r+1, 2r+1, 2C[+2], h, w) MatchingNet input."""
    return _DiclStack.apply(fmap1, fmap2, coords, radius, level, norm_hw, extra_delta)


class _DiclStackInt(torch.autograd.Function):
    """Integer-displacement matching volume with occlusion mask — impls/dicl.py:212-238."""

    @staticmethod
    def forward(ctx, f1, f2, ru, rv):
        _require_gpu(f1, f2)
        f1c = f1.detach().float().contiguous()
        f2c = f2.detach().float().contiguous()
        b, c, h, w = f1c.shape
        if tuple(f2c.shape) != (b, c, h, w):
            raise ValueError("dicl_stack_int: fmap1 and fmap2 must have equal (B,C,h,w) shapes")
        lib = _lib.lib()
        ws = torch.empty(lib.rmd_dicl_stack_int_workspace_bytes(b, h, w), dtype=torch.uint8, device=f1c.device)
        out = torch.empty((b, 2 * ru + 1, 2 * rv + 1, 2 * c, h, w), dtype=torch.float32, device=f1c.device)
        with torch.cuda.device(f1c.device):
            _lib.check(lib.rmd_dicl_stack_int(_ptr(f1c), _ptr(f2c), b, c, h, w, ru, rv, _ptr(out), _ptr(ws),
                                              _stream(f1c)), "rmd_dicl_stack_int")
        ctx.save_for_backward(f2c)
        ctx.meta = (b, c, h, w, ru, rv)
        return out

    @staticmethod
    def backward(ctx, grad):
        (f2c,) = ctx.saved_tensors
        b, c, h, w, ru, rv = ctx.meta
        g = grad.float().contiguous()
        lib = _lib.lib()
        ws = torch.empty(lib.rmd_dicl_stack_int_workspace_bytes(b, h, w), dtype=torch.uint8, device=g.device)
        g1 = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
        g2 = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            _lib.check(lib.rmd_dicl_stack_int_backward(_ptr(g), _ptr(f2c), b, c, h, w, ru, rv, _ptr(g1), _ptr(g2),
                                                       _ptr(ws), _stream(g)), "rmd_dicl_stack_int_backward")
        return g1, g2, None, None


def dicl_stack_int(fmap1, fmap2, ru, rv):
    return _DiclStackInt.apply(fmap1, fmap2, ru, rv)


class _DiclStackIntWarped(torch.autograd.Function):
    """Integer volume on feat2 warped back by a (detached) flow — impls/dicl.py:178-181 + 212-238."""

    @staticmethod
    def forward(ctx, f1, f2, flow, ru, rv):
        _require_gpu(f1, f2, flow)
        f1c = f1.detach().float().contiguous()
        f2c = f2.detach().float().contiguous()
        fc = flow.detach().float().contiguous()
        b, c, h, w = f1c.shape
        if tuple(f2c.shape) != (b, c, h, w) or tuple(fc.shape) != (b, 2, h, w):
            raise ValueError("dicl_stack_int_warped: need fmap1, fmap2 (B,C,h,w) and flow (B,2,h,w)")
        lib = _lib.lib()
        ws = torch.empty(lib.rmd_dicl_stack_int_warped_workspace_bytes(b, c, h, w), dtype=torch.uint8,
                         device=f1c.device)
        out = torch.empty((b, 2 * ru + 1, 2 * rv + 1, 2 * c, h, w), dtype=torch.float32, device=f1c.device)
        with torch.cuda.device(f1c.device):
            _lib.check(lib.rmd_dicl_stack_int_warped(_ptr(f1c), _ptr(f2c), _ptr(fc), b, c, h, w, ru, rv, _ptr(out),
                                                     _ptr(ws), _stream(f1c)), "rmd_dicl_stack_int_warped")
        ctx.save_for_backward(f2c, fc)
        ctx.meta = (b, c, h, w, ru, rv)
        return out

    @staticmethod
    def backward(ctx, grad):
        f2c, fc = ctx.saved_tensors
        b, c, h, w, ru, rv = ctx.meta
        g = grad.float().contiguous()
        lib = _lib.lib()
        ws = torch.empty(lib.rmd_dicl_stack_int_warped_workspace_bytes(b, c, h, w), dtype=torch.uint8, device=g.device)
        g1 = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
        g2 = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            _lib.check(lib.rmd_dicl_stack_int_warped_backward(_ptr(g), _ptr(f2c), _ptr(fc), b, c, h, w, ru, rv,
                                                              _ptr(g1), _ptr(g2), _ptr(ws), _stream(g)),
                       "rmd_dicl_stack_int_warped_backward")
        return g1, g2, None, None, None


def dicl_stack_int_warped(fmap1, fmap2, flow, ru, rv):
    """Masked integer volume of (fmap1, warp_backwards(fmap2, flow)) in one fused pass pair."""
    return _DiclStackIntWarped.apply(fmap1, fmap2, flow, ru, rv)


class _Dap(torch.autograd.Function):
    """out[b,o,p] = sum_i W[o,i] x[b,i,p] — blocks/dicl.py:143-150 (1x1 conv, no bias)."""

    @staticmethod
    def forward(ctx, x, weight):
        _require_gpu(x, weight)
        b, dd = x.shape[0], weight.shape[0]
        if x.numel() % (b * dd) or weight.numel() != dd * dd:
            raise ValueError(f"dap: x {tuple(x.shape)} does not hold {dd} displacement channels per batch")
        xc = x.detach().float().contiguous()
        wc = weight.detach().float().reshape(dd, dd).contiguous()
        n = xc.numel() // (b * dd)
        out = torch.empty_like(xc)
        with torch.cuda.device(xc.device):
            _lib.check(_lib.lib().rmd_dap(_ptr(xc), _ptr(wc), b, dd, n, 0, _ptr(out), _stream(xc)), "rmd_dap")
        ctx.save_for_backward(xc, wc)
        ctx.wshape = weight.shape
        return out

    @staticmethod
    def backward(ctx, grad):
        xc, wc = ctx.saved_tensors
        b, dd = xc.shape[0], wc.shape[0]
        n = xc.numel() // (b * dd)
        g = grad.float().contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(g)
            with torch.cuda.device(g.device):
                _lib.check(_lib.lib().rmd_dap(_ptr(g), _ptr(wc), b, dd, n, 1, _ptr(gx), _stream(g)), "rmd_dap^T")
        gw = None
        if ctx.needs_input_grad[1]:
            # plain library GEMM (hipBLASLt): dW = sum_b g_b x_b^T
            gw = torch.matmul(g.view(b, dd, n), xc.view(b, dd, n).transpose(1, 2)).sum(0).reshape(ctx.wshape)
        return gx, gw


def dap(x, weight):
    """x (B, D, ...) -> W x over the displacement dim; weight (D, D[, 1, 1])."""
    return _Dap.apply(x, weight)


# ---- per-iteration flow heads (rmd_up8, rmd_softargmax) -----------------------------------------

class _Up8(torch.autograd.Function):
    """Convex 8x upsampling after Up8Network's convolutions — raft.py:319-331."""

    @staticmethod
    def forward(ctx, mask, flow, temperature):
        _require_gpu(mask, flow)
        b, c, h, w = flow.shape
        if c != 2 or tuple(mask.shape) != (b, 576, h, w):
            raise ValueError(f"up8: need flow (B,2,h,w) and mask (B,576,h,w), got {tuple(flow.shape)}, "
                             f"{tuple(mask.shape)}")
        mc = mask.detach().float().contiguous()
        fc = flow.detach().float().contiguous()
        out = torch.empty((b, 2, 8 * h, 8 * w), dtype=torch.float32, device=fc.device)
        with torch.cuda.device(fc.device):
            _lib.check(_lib.lib().rmd_up8(_ptr(mc), _ptr(fc), b, h, w, float(temperature), _ptr(out), _stream(fc)),
                       "rmd_up8")
        ctx.save_for_backward(mc, fc)
        ctx.temperature = float(temperature)
        ctx.dtypes = (mask.dtype, flow.dtype)
        return out

    @staticmethod
    def backward(ctx, grad):
        mc, fc = ctx.saved_tensors
        b, _, h, w = fc.shape
        g = grad.float().contiguous()
        lib = _lib.lib()
        ws = torch.empty(lib.rmd_up8_workspace_bytes(b, h, w), dtype=torch.uint8, device=g.device)
        gm = torch.empty_like(mc)
        gf = torch.empty_like(fc)
        with torch.cuda.device(g.device):
            _lib.check(lib.rmd_up8_backward(_ptr(mc), _ptr(fc), _ptr(g), b, h, w, ctx.temperature, _ptr(gm), _ptr(gf),
                                            _ptr(ws), _stream(g)), "rmd_up8_backward")
        return gm.to(ctx.dtypes[0]), gf.to(ctx.dtypes[1]), None


def up8(mask, flow, temperature=4.0):
    """mask (B, 576, h, w) logits, flow (B, 2, h, w) -> convex-upsampled flow (B, 2, 8h, 8w)."""
    return _Up8.apply(mask, flow, temperature)


class _SoftArgMax(torch.autograd.Function):
    """Soft-argmax over each level's (2r+1)^2 costs — raft.py:112-135, corr/dot.py:83-90."""

    @staticmethod
    def forward(ctx, cost, levels, radius, temperature):
        _require_gpu(cost)
        b, ctot = cost.shape[:2]
        n = cost[0, 0].numel()
        dd = (2 * radius + 1) ** 2
        if ctot < levels * dd:
            raise ValueError(f"softargmax: {ctot} channels < {levels} levels x {dd} displacements")
        cc = cost.detach().float().contiguous()
        flows = torch.empty((levels, b, 2) + tuple(cost.shape[2:]), dtype=torch.float32, device=cc.device)
        with torch.cuda.device(cc.device):
            _lib.check(_lib.lib().rmd_softargmax(_ptr(cc), b, ctot, n, levels, radius, float(temperature), _ptr(flows),
                                                 _stream(cc)), "rmd_softargmax")
        ctx.save_for_backward(cc)
        ctx.meta = (levels, radius, float(temperature), cost.dtype)
        return flows

    @staticmethod
    def backward(ctx, gflows):
        (cc,) = ctx.saved_tensors
        levels, radius, temperature, dtype = ctx.meta
        b, ctot = cc.shape[:2]
        n = cc[0, 0].numel()
        g = gflows.float().contiguous()
        gc = torch.zeros_like(cc) if ctot > levels * (2 * radius + 1) ** 2 else torch.empty_like(cc)
        with torch.cuda.device(g.device):
            _lib.check(_lib.lib().rmd_softargmax_backward(_ptr(cc), _ptr(g), b, ctot, n, levels, radius, temperature,
                                                          _ptr(gc), _stream(g)), "rmd_softargmax_backward")
        return gc.to(dtype), None, None, None


def softargmax(cost, levels, radius, temperature=1.0):
    """cost (B, >= L*(2r+1)^2, h, w) -> list of L flows (B, 2, h, w), level l scaled by 2^l."""
    return list(_SoftArgMax.apply(cost, levels, radius, temperature).unbind(0))
