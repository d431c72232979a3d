"""Torch-facing wrappers over the C ABI (include/rmd.h): device checks, allocation, streams.

Outputs and workspaces come from torch's caching allocator; the C launchers only enqueue kernels
on torch's current HIP stream.  GPU tensors run the HIP kernels (and raise if librmd.so is missing);
CPU tensors dispatch to the operators' CPU kernels (rmd/cpu.py, the reference's ATen algorithm).
The token-linked autograd functions of the RAFT correlation and of the on-the-fly lookup are
GPU-only: on the CPU the operators' own ATen graph carries the gradient.
"""

import ctypes

import torch

from . import _lib, config, library
from ._lib import RMD_BF16, RMD_BF16X3, RMD_F16, RMD_F32, RMD_S24

# precision modes: (GEMM compute type, pyramid storage type)
PRECISIONS = {
    "fp32": (RMD_BF16X3, RMD_S24),    # fp32-accurate split-bf16 MFMA (3 products), 24-bit pyramid: parity mode (default)
    "fp32-f32": (RMD_BF16X3, RMD_F32),# the same GEMM, f32 pyramid
    "fp32-s24": (RMD_BF16X3, RMD_S24),# the same GEMM, 24-bit pyramid
    "fp32-exact": (RMD_F32, RMD_F32), # exact f32 MFMA (v_mfma_f32_32x32x2_f32), f32 pyramid
    "bf16": (RMD_BF16, RMD_F16),      # bf16 MFMA operands, f32 accumulate, fp16 pyramid: perf mode
    "bf16-f32": (RMD_BF16, RMD_F32),  # bf16 operands, f32 pyramid
    "fp32-f16": (RMD_F32, RMD_F16),   # exact f32 GEMM, fp16 pyramid
}


def set_default_precision(name):
    """Process-wide precision of blocks built with precision=None (rmd.config 'corr-precision')."""
    if name not in PRECISIONS:
        raise ValueError(f"unknown precision '{name}', expected one of {sorted(PRECISIONS)}")
    config.configure(precision=name)


def get_default_precision():
    return config.current().precision


def _require_gpu(*tensors):
    for t in tensors:
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise RuntimeError("rmd: HIP kernels need GPU tensors")


def _same_device(*tensors):
    """All inputs on one device: GPU tensors run the HIP kernels, CPU tensors the CPU kernels."""
    dev = None
    for t in tensors:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"rmd: expected a tensor, got {type(t).__name__}")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"rmd: tensors on different devices ({dev} / {t.device})")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class Pyramid:
    """Correlation pyramid in the tiled, query-minor HBM layout of include/rmd.h.  ``data`` is 1-D in the
    row layout, (n, 8) in the tiles layout (rmd.library.pyramid_view) and uint8 (n, 3) with RMD_S24 storage."""

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
        th, tw, ty, tx = d.tile_h[i], d.tile_w[i], d.tiles_y[i], d.tiles_x[i]
        hl, wl = d.level_h[i], d.level_w[i]
        s = d.query_slots
        off = d.level_offset[i]
        flat = library.s24_decode(self.data) if d.storage == RMD_S24 else self.data.reshape(-1)
        x = flat[off: off + b * ty * tx * s * th * tw].view(b, ty, tx, s, th, tw)
        x = x.permute(0, 3, 1, 4, 2, 5).reshape(b, s, ty * th, tx * tw)[..., :hl, :wl]
        if d.layout == _lib.RMD_LAYOUT_TILES:
            x = x.index_select(1, torch.as_tensor(tiles_slots(h, w), device=x.device))
        return x.float().reshape(b, h, w, 1, hl, wl)


def tiles_slots(h, w):
    """Query slot of every pixel (raster order) in the tiles layout (include/rmd.h RMD_LAYOUT_TILES)."""
    y1, x1 = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    qx, hp = (w + 15) // 16, h // 2
    s = ((y1 // 2) * qx + x1 // 16) * 32 + ((x1 % 16) // 4) * 8 + (y1 % 2) * 4 + x1 % 4
    s = torch.where(y1 < 2 * hp, s, hp * qx * 32 + x1)
    return s.reshape(-1)


def corr_pyramid(fmap1, fmap2, levels=4, precision=None, events=None, scale=None):
    """raft.CorrBlock.__init__ (raft.py:18-47) on the GPU -> Pyramid (torch.ops.rmd.corr_pyramid).

    ``scale`` multiplies the products: None = 1/sqrt(C) (raft.py:33), 1.0 = raft_fs.CorrBlock.

    ``events`` (optional list) receives (start, end) HIP events bracketing the GEMM launch alone
    (the operand prep runs before the start event) — bench.py's roofline timing; that call runs the
    same two C-ABI halves (rmd_corr_prepare, rmd_corr_pyramid_prepared) directly.
    """
    _same_device(fmap1, fmap2)
    if fmap1.shape != fmap2.shape or fmap1.dim() != 4:
        raise ValueError(f"fmap1/fmap2 must be equal (B,C,H,W) shapes, got {tuple(fmap1.shape)} / {tuple(fmap2.shape)}")
    compute, storage = PRECISIONS[precision or get_default_precision()]
    b, c, h, w = fmap1.shape
    scale = 1.0 / float(c) ** 0.5 if scale is None else float(scale)
    if events is None:
        data = torch.ops.rmd.corr_pyramid(fmap1, fmap2, levels, compute, storage, scale)
        # the storage the GEMM wrote (S24 is the x3 GEMM's alone: other GEMMs of the call store F32)
        d = library.describe(b, h, w, levels, library.pyramid_storage(data), library.pyramid_layout(data))
        return Pyramid(data, d, c, scale)
    _require_gpu(fmap1, fmap2)
    d = library.describe_for(b, h, w, levels, storage, c, compute)
    f1 = fmap1.detach().float().contiguous()
    f2 = fmap2.detach().float().contiguous()
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_corr_pyramid_workspace_bytes(ctypes.byref(d), c, compute), dtype=torch.uint8,
                     device=f1.device)
    data = library.new_pyramid(f1, d)
    with torch.cuda.device(f1.device):
        stream = _lib.stream_ptr(f1.device)
        _lib.check(lib.rmd_corr_prepare(_ptr(f1), _ptr(f2), c, scale, ctypes.byref(d), compute, _ptr(ws), stream),
                   "rmd_corr_prepare")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.check(lib.rmd_corr_pyramid_prepared(c, scale, ctypes.byref(d), compute, _ptr(data), _ptr(ws), stream),
                   "rmd_corr_pyramid_prepared")
        e1.record()
        events.append((e0, e1))
    return Pyramid(data, d, c, scale)


def corr_lookup(pyr, coords, radius, mask_costs=()):
    """raft.CorrBlock.__call__ (raft.py:49-95) -> (B, L*(2r+1)^2, H, W) float32."""
    _same_device(pyr.data, coords)
    d = pyr.desc
    if tuple(coords.shape) != (d.batch, 2, d.height, d.width):
        raise ValueError(f"coords must be (B,2,H,W)=({d.batch},2,{d.height},{d.width}), got {tuple(coords.shape)}")
    return torch.ops.rmd.corr_lookup(pyr.data, coords, d.levels, radius, _mask_bits(mask_costs, d.levels))


# ---- on-the-fly lookup (raft_fs semantics without the volume) -------------------------------------

class OtfState:
    """Operand rows of rmd_corr_otf_prepare (query rows * scale, pooled target rows of every level)."""

    def __init__(self, ws, b, c, h, w, levels, compute):
        self.ws, self.b, self.c, self.h, self.w, self.levels, self.compute = ws, b, c, h, w, levels, compute


def otf_prepare(fmap1, fmap2, levels, precision=None, scale=1.0):
    _same_device(fmap1, fmap2)
    if fmap1.shape != fmap2.shape or fmap1.dim() != 4:
        raise ValueError(f"fmap1/fmap2 must be equal (B,C,H,W) shapes, got {tuple(fmap1.shape)} / {tuple(fmap2.shape)}")
    compute = PRECISIONS[precision or get_default_precision()][0]     # fp32: split bf16, fp32-exact: f32
    b, c, h, w = fmap1.shape
    ws = torch.ops.rmd.corr_otf_prepare(fmap1, fmap2, levels, compute, float(scale))
    return OtfState(ws, b, c, h, w, levels, compute)


def otf_lookup(st, coords, radius, mask_costs=()):
    _same_device(st.ws, coords)
    if tuple(coords.shape) != (st.b, 2, st.h, st.w):
        raise ValueError(f"coords must be (B,2,H,W)=({st.b},2,{st.h},{st.w}), got {tuple(coords.shape)}")
    return torch.ops.rmd.corr_otf_lookup(st.ws, coords, st.c, st.levels, st.compute, radius,
                                         _mask_bits(mask_costs, st.levels))


# ---- on-the-fly lookup autograd (training without the volume) ----------------------------------
#
# Same token scheme as the volume path below: every lookup's backward turns its grad_out into a record
# of patch weights (rmd_corr_otf_record, O(L*N*(2r+2)^2) floats, no volume), and the prepare's
# backward — which autograd runs after all of them — computes d fmap1 / d fmap2 from all records in one
# pass (rmd_corr_otf_backward: the union target box of a query tile swept once for every iteration).

class _OtfState:
    def __init__(self, otf, f1, f2, scale):
        self.otf = otf
        self.f1 = f1
        self.f2 = f2
        self.scale = scale
        self.records = []
        self.radius = None


class _OtfPrepareFn(torch.autograd.Function):
    """Autograd node of raft_fs.CorrBlock.__init__ (raft_fs.py:16-31) on the on-the-fly path."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, state):
        ctx.state = state
        return fmap1.new_zeros(())

    @staticmethod
    def backward(ctx, _gtoken):
        st = ctx.state
        o = st.otf
        if not st.records:
            return torch.zeros_like(st.f1), torch.zeros_like(st.f2), None
        lib = _lib.lib()
        nbytes = lib.rmd_corr_otf_backward_workspace_bytes(o.b, o.c, o.h, o.w, o.levels, o.compute)
        if nbytes == 0:
            raise ValueError(f"otf backward: unsupported sizes (C={o.c} must be <= 256)")
        ws = torch.empty(nbytes, dtype=torch.uint8, device=st.f1.device)
        g1 = torch.empty_like(st.f1)
        g2 = torch.empty_like(st.f2)
        recs = (ctypes.c_void_p * len(st.records))(*[r.data_ptr() for r in st.records])
        with torch.cuda.device(st.f1.device):
            _lib.check(lib.rmd_corr_otf_backward(_ptr(st.f1), _ptr(st.f2), _ptr(o.ws), o.b, o.c, o.h, o.w, o.levels,
                                                 float(st.scale), o.compute, st.radius, len(st.records), recs,
                                                 _ptr(g1), _ptr(g2), _ptr(ws), _stream(st.f1)),
                       "rmd_corr_otf_backward")
        st.records = []
        return g1, g2, None


class _OtfLookupFn(torch.autograd.Function):
    """Autograd node of raft_fs.CorrBlock.__call__ (raft_fs.py:33-87) on the on-the-fly path; coords carry
    no gradient (raft.py:402)."""

    @staticmethod
    def forward(ctx, token, coords, state, radius, mask_costs):
        out = otf_lookup(state.otf, coords, radius, mask_costs)
        ctx.state = state
        ctx.radius = radius
        ctx.mask = _mask_bits(mask_costs, state.otf.levels)
        ctx.save_for_backward(coords.detach().float().contiguous())
        return out

    @staticmethod
    def backward(ctx, gout):
        (co,) = ctx.saved_tensors
        st = ctx.state
        o = st.otf
        if st.radius is not None and st.radius != ctx.radius:
            raise ValueError("otf backward: all lookups of one block must use the same radius")
        st.radius = ctx.radius
        lib = _lib.lib()
        rec = torch.empty(lib.rmd_corr_otf_record_bytes(o.b, o.h, o.w, o.levels, ctx.radius), dtype=torch.uint8,
                          device=co.device)
        g = gout.float().contiguous()
        with torch.cuda.device(co.device):
            _lib.check(lib.rmd_corr_otf_record(_ptr(g), _ptr(co), o.b, o.h, o.w, o.levels, ctx.radius, ctx.mask,
                                               _ptr(rec), _stream(co)), "rmd_corr_otf_record")
        st.records.append(rec)
        return gout.new_zeros(()), None, None, None, None


def otf_block_autograd(fmap1, fmap2, levels, precision, scale=1.0):
    """On-the-fly operands + autograd token for a block whose feature maps require gradients."""
    _require_gpu(fmap1, fmap2)
    otf = otf_prepare(fmap1, fmap2, levels, precision, scale=scale)
    st = _OtfState(otf, fmap1.detach().float().contiguous(), fmap2.detach().float().contiguous(), scale)
    token = _OtfPrepareFn.apply(fmap1, fmap2, st)
    return otf, st, token


def otf_lookup_autograd(token, state, coords, radius, mask_costs=()):
    return _OtfLookupFn.apply(token, coords, state, radius, tuple(mask_costs))


# ---- RAFT correlation autograd (training) -------------------------------------------------------
#
# The pyramid Function returns a scalar "token" that every lookup of the same CorrBlock takes as an
# input, so autograd runs all lookup backwards before the pyramid backward.  Each lookup backward
# only hands its grad_out and coordinates to the shared _CorrState; the pyramid backward writes ONE
# dense fp32 gradient G over the T' padded targets, in the pyramid's chunked query-minor order
# (8-target chunks, include/rmd.h), from all of them in one pass (rmd_corr_grad_build: the sums of
# one rmd_corr_lookup_backward per lookup into a zeroed G, in the same order, without the zero fill
# and the per-lookup read-modify-write passes), then turns G into d fmap1 / d fmap2 with two MFMA
# GEMMs that read G in its blocked order (rmd_corr_grad_gemm layouts 3 / 2, no transpose pass;
# split-bf16 products in the fp32 modes, bf16 products with fp32 accumulation in the bf16 modes) and
# the native pool / unpool kernels (G, pool and unpool in fp32 in every mode).

# False: one rmd_corr_lookup_backward per lookup into a zeroed G (the round-4 path; A/B only)
GRAD_BUILD = True
# bf16 modes: G written as bfloat16 by the build and read by the bf16-B grad GEMMs (bit-identical to
# the fp32 G, whose GEMM rounds it to bfloat16 on load; half the G traffic).  False: fp32 G (A/B only)
GRAD_BF16 = True
# The pending lookup gradients are fp32 (B, L (2r+1)^2, H, W) tensors kept alive until the pyramid
# backward (cfg2 b8, r = 4: 73 MB each, 0.88 GB for 12 lookups).  Past this many bytes they are folded
# into an fp32 G early (the build accumulates in lookup order, so G is the same sums) and released.
GRAD_PENDING_BYTES = 1 << 30


class _CorrState:
    def __init__(self, pyr, f1, f2, precision):
        self.pyr = pyr
        self.f1 = f1
        self.f2 = f2
        self.precision = precision
        self.grad = None          # dense G (GRAD_BUILD False: allocated by the first lookup backward)
        self.pending = []         # (grad_out, coords, radius, level mask) per lookup backward, in order


def _mask_bits(mask_costs, levels):
    mask = 0
    for m in mask_costs:
        if 0 <= m - 3 < levels:
            mask |= 1 << (m - 3)
    return mask


def _build_grad(st, bf16=False):
    """G from the pending lookup gradients (rmd_corr_grad_build), consecutive equal radii per launch,
    added to the fp32 G of an earlier flush if there is one; bf16: one launch writes a bfloat16 G (the
    caller checked one radius, <= 16 lookups, no earlier flush)."""
    d = st.pyr.desc
    lib = _lib.lib()
    t = lib.rmd_corr_grad_targets(d.height, d.width, d.levels)
    pend, st.pending = st.pending, []
    dev = pend[0][0].device
    G = st.grad
    if G is None:
        G = torch.empty(d.batch * d.height * d.width * t, dtype=torch.bfloat16 if bf16 else torch.float32,
                        device=dev)
    i = 0
    acc0 = 1 if st.grad is not None else 0
    with torch.cuda.device(dev):
        stream = _stream(G)
        while i < len(pend):
            j = i
            while j < len(pend) and pend[j][2] == pend[i][2]:
                j += 1
            grp = pend[i:j]
            gouts = (ctypes.c_void_p * len(grp))(*[x[0].data_ptr() for x in grp])
            cos = (ctypes.c_void_p * len(grp))(*[x[1].data_ptr() for x in grp])
            masks = (ctypes.c_uint * len(grp))(*[x[3] for x in grp])
            _lib.check(lib.rmd_corr_grad_build_ex(gouts, cos, masks, len(grp), ctypes.byref(d), grp[0][2],
                                                  1 if i > 0 else acc0, 1 if bf16 else 0, _ptr(G), stream),
                       "rmd_corr_grad_build")
            i = j
    return G


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
        bf16_mode = PRECISIONS[st.precision][0] == RMD_BF16
        if st.pending:
            one_launch = len(st.pending) <= 16 and len({x[2] for x in st.pending}) == 1 and st.grad is None
            st.grad = _build_grad(st, bf16=GRAD_BF16 and bf16_mode and one_launch)
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
            G = st.grad                 # (B, T'/8, N, 8): element (t', p) at ((t'/8) N + p) 8 + t' % 8
            g1 = torch.empty((b, c, n), dtype=torch.float32, device=f1.device)
            dpool = torch.empty((b, c, t), dtype=torch.float32, device=f1.device)
            ws = torch.empty(max(lib.rmd_corr_grad_gemm_workspace_bytes(b, c, t, n),
                                 lib.rmd_corr_grad_gemm_workspace_bytes(b, c, n, t), 1),
                             dtype=torch.uint8, device=f1.device)
            # grad_fmap1 = P G (K = T', layout 3: G blocked along k), dP = fmap1 G^T (K = N, layout 2: G
            # blocked along n): MFMA GEMMs (corr_grad.hip) in the block's compute — split-bf16 (fp32
            # accuracy) for the fp32 modes, one bf16 product for the bf16 modes
            gc = RMD_BF16 if bf16_mode else RMD_BF16X3
            if G.dtype == torch.bfloat16:
                # bfloat16 G (bf16 modes): the same products as the fp32-G GEMM, half the bytes
                _lib.check(lib.rmd_corr_grad_gemm_bf16g(_ptr(pooled), t, _ptr(G), n, b, c, t, n, 3, _ptr(g1),
                                                        _ptr(ws), stream), "rmd_corr_grad_gemm_bf16g")
                _lib.check(lib.rmd_corr_grad_gemm_bf16g(_ptr(f1), n, _ptr(G), n, b, c, n, t, 2, _ptr(dpool),
                                                        _ptr(ws), stream), "rmd_corr_grad_gemm_bf16g")
            else:
                _lib.check(lib.rmd_corr_grad_gemm(_ptr(pooled), t, _ptr(G), n, b, c, t, n, 3, gc, _ptr(g1),
                                                  _ptr(ws), stream), "rmd_corr_grad_gemm")
                _lib.check(lib.rmd_corr_grad_gemm(_ptr(f1), n, _ptr(G), n, b, c, n, t, 2, gc, _ptr(dpool),
                                                  _ptr(ws), stream), "rmd_corr_grad_gemm")
            _lib.check(lib.rmd_corr_unpool_targets(_ptr(dpool), b, c, h, w, levels, scale, _ptr(g2), stream),
                       "rmd_corr_unpool_targets")
        st.grad = None
        return g1.view(b, c, h, w), g2, None


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
        g = gout.float().contiguous()
        if GRAD_BUILD:
            # G is written from every lookup's gradient at once by the pyramid backward
            st.pending.append((g, co, ctx.radius, ctx.mask))
            if sum(x[0].numel() for x in st.pending) * 4 > GRAD_PENDING_BYTES:
                st.grad = _build_grad(st)         # fp32 G, accumulated from here on
            return gout.new_zeros(()), None, None, None, None
        d = st.pyr.desc
        lib = _lib.lib()
        if st.grad is None:
            t = lib.rmd_corr_grad_targets(d.height, d.width, d.levels)
            st.grad = torch.zeros(d.batch * d.height * d.width * t, dtype=torch.float32, device=co.device)
        with torch.cuda.device(co.device):
            _lib.check(lib.rmd_corr_lookup_backward(_ptr(g), ctx_desc(st), _ptr(co), ctx.radius, ctx.mask,
                                                    _ptr(st.grad), _stream(co)), "rmd_corr_lookup_backward")
        return gout.new_zeros(()), None, None, None, None


def ctx_desc(st):
    return ctypes.byref(st.pyr.desc)


def corr_block_autograd(fmap1, fmap2, levels, precision, scale=None):
    """Pyramid + autograd token for a CorrBlock whose feature maps require gradients."""
    _require_gpu(fmap1, fmap2)
    precision = precision or get_default_precision()
    pyr = corr_pyramid(fmap1, fmap2, levels, precision, scale=scale)
    st = _CorrState(pyr, fmap1.detach().float().contiguous(), fmap2.detach().float().contiguous(), precision)
    token = _CorrPyramidFn.apply(fmap1, fmap2, st)
    return pyr, st, token


def corr_lookup_autograd(token, state, coords, radius, mask_costs=()):
    return _CorrLookupFn.apply(token, coords, state, radius, tuple(mask_costs))


# ---- DICL cost volumes and DAP ------------------------------------------------------------------

def _stream(t):
    return _lib.stream_ptr(t.device)


def dicl_stack(fmap1, fmap2, coords, radius, level=0, norm_hw=None, extra_delta=False):
    """(B,C,h,w), (B,C,hl,wl), (B,2,h,w) -> (B, 2r+1, 2r+1, 2C[+2], h, w) MatchingNet input
    (torch.ops.rmd.dicl_stack; corr/dicl.py:26-54)."""
    _same_device(fmap1, fmap2, coords)
    nh, nw = norm_hw if norm_hw is not None else fmap1.shape[-2:]
    return torch.ops.rmd.dicl_stack(fmap1, fmap2, coords, radius, level, int(nh), int(nw), bool(extra_delta))


def dicl_stack_int(fmap1, fmap2, ru, rv):
    """Integer-displacement matching volume with occlusion mask (torch.ops.rmd.dicl_stack_int;
    impls/dicl.py:212-238)."""
    _same_device(fmap1, fmap2)
    return torch.ops.rmd.dicl_stack_int(fmap1, fmap2, ru, rv)


def dicl_stack_int_warped(fmap1, fmap2, flow, ru, rv):
    """Masked integer volume of (fmap1, warp_backwards(fmap2, flow)) in one fused pass pair
    (torch.ops.rmd.dicl_stack_int_warped; impls/dicl.py:178-181 + 212-238)."""
    _same_device(fmap1, fmap2, flow)
    return torch.ops.rmd.dicl_stack_int_warped(fmap1, fmap2, flow, ru, rv)


def dap(x, weight):
    """x (B, D, ...) -> W x over the displacement dim; weight (D, D[, 1, 1]) (torch.ops.rmd.dap;
    blocks/dicl.py:143-150)."""
    _same_device(x, weight)
    return torch.ops.rmd.dap(x, weight)


def up8(mask, flow, temperature=4.0):
    """mask (B, 576, h, w) logits, flow (B, 2, h, w) -> convex-upsampled flow (B, 2, 8h, 8w)
    (torch.ops.rmd.up8; raft.py:319-331)."""
    _same_device(mask, flow)
    return torch.ops.rmd.up8(mask, flow, float(temperature))


def softargmax(cost, levels, radius, temperature=1.0):
    """cost (B, >= L*(2r+1)^2, h, w) -> list of L flows (B, 2, h, w), level l scaled by 2^l
    (torch.ops.rmd.softargmax; raft.py:112-135, corr/dot.py:83-90)."""
    _same_device(cost)
    return list(torch.ops.rmd.softargmax(cost, levels, radius, float(temperature)).unbind(0))
