"""torch.library registration of the rmd operators: `torch.ops.rmd.*` over the C ABI of librmd.so.

Every operator has a CUDA (HIP) kernel — the ctypes call into include/rmd.h on torch's current
stream —, a fake (meta) implementation that only computes output shapes (torch.compile /
torch.export / FakeTensor tracing), a CPU kernel for CPU tensors (rmd/cpu.py: the reference's ATen
algorithm, registered for CPU and AutogradCPU — a dispatch by device, never a fallback for a GPU
tensor), and, where the reference's module is trained through it, an autograd formula whose backward
is again an rmd operator.  Schemas follow SURVEY.md §8(b):

  corr_pyramid(fmap1, fmap2, levels, compute, storage, scale) -> pyramid     raft.py:18-47
  corr_lookup(pyramid, coords, levels, radius, level_mask) -> corr           raft.py:49-95
  corr_otf_prepare / corr_otf_lookup                                        raft_fs.py:13-87, corr/dot.py:25-57
  dicl_stack(fmap1, fmap2, coords, radius, level, norm_h, norm_w, extra) ->  corr/dicl.py:26-54,
        (B, 2r+1, 2r+1, 2C[+2], h, w)                                        dicl_emb.py:51-89, raft_dicl_ml.py:294-315
  dicl_stack_int(fmap1, fmap2, ru, rv), dicl_stack_int_warped(.., flow, ..) impls/dicl.py:178-238
  dap(x, weight)                                                             blocks/dicl.py:143-150
  up8(mask, flow, temperature), softargmax(cost, levels, radius, T)          raft.py:98-190, 319-331
  warp_backwards(img2, flow, eps) -> (est, mask)                             common/warp.py:5-33

The RAFT correlation's training path keeps rmd.ops' token-linked autograd functions: all lookups of
one CorrBlock accumulate into ONE dense pyramid gradient (query-minor, fp32) whose layout differs from
the pyramid tensor's own (chunked, fp16 in the perf mode), which a per-op autograd formula (gradient
shaped and typed like its input) cannot express.  corr_pyramid / corr_lookup here are the inference
operators.
"""

import ctypes

import torch

from . import _lib

_ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

LIB = torch.library.Library("rmd", "DEF")

_SCHEMAS = {
    "corr_pyramid": "corr_pyramid(Tensor fmap1, Tensor fmap2, int levels, int compute, int storage, float scale) -> Tensor",
    "corr_lookup": "corr_lookup(Tensor pyramid, Tensor coords, int levels, int radius, int level_mask) -> Tensor",
    "corr_otf_prepare": "corr_otf_prepare(Tensor fmap1, Tensor fmap2, int levels, int compute, float scale) -> Tensor",
    "corr_otf_lookup": ("corr_otf_lookup(Tensor workspace, Tensor coords, int channels, int levels, int compute, "
                        "int radius, int level_mask) -> Tensor"),
    "dicl_stack": ("dicl_stack(Tensor fmap1, Tensor fmap2, Tensor coords, int radius, int level, int norm_h, "
                   "int norm_w, bool extra_delta) -> Tensor"),
    "dicl_stack_backward": ("dicl_stack_backward(Tensor grad, Tensor coords, int channels, int level_h, int level_w, "
                            "int radius, int level, int norm_h, int norm_w, bool extra_delta) -> (Tensor, Tensor)"),
    "dicl_stack_int": "dicl_stack_int(Tensor fmap1, Tensor fmap2, int ru, int rv) -> Tensor",
    "dicl_stack_int_backward": "dicl_stack_int_backward(Tensor grad, Tensor fmap2, int ru, int rv) -> (Tensor, Tensor)",
    "dicl_stack_int_warped": "dicl_stack_int_warped(Tensor fmap1, Tensor fmap2, Tensor flow, int ru, int rv) -> Tensor",
    "dicl_stack_int_warped_backward": ("dicl_stack_int_warped_backward(Tensor grad, Tensor fmap2, Tensor flow, int ru, "
                                       "int rv) -> (Tensor, Tensor)"),
    "dap": "dap(Tensor x, Tensor weight) -> Tensor",
    "dap_transpose": "dap_transpose(Tensor grad, Tensor weight) -> Tensor",
    "dap_weight_grad": "dap_weight_grad(Tensor grad, Tensor x, int disp) -> Tensor",
    "up8": "up8(Tensor mask, Tensor flow, float temperature) -> Tensor",
    "up8_backward": "up8_backward(Tensor grad, Tensor mask, Tensor flow, float temperature) -> (Tensor, Tensor)",
    "softargmax": "softargmax(Tensor cost, int levels, int radius, float temperature) -> Tensor",
    "softargmax_backward": ("softargmax_backward(Tensor grad, Tensor cost, int levels, int radius, float temperature) "
                            "-> Tensor"),
    "warp_backwards": "warp_backwards(Tensor img2, Tensor flow, float eps) -> (Tensor, Tensor)",
    "warp_backwards_backward": "warp_backwards_backward(Tensor grad, Tensor flow, float eps) -> Tensor",
}
for _s in _SCHEMAS.values():
    LIB.define(_s)


def _cuda(name):
    """The HIP kernel of an operator (CUDA dispatch key); its CPU kernel lives in rmd/cpu.py.  Every
    tensor argument must be a GPU tensor (the dispatcher picks this kernel when any one is)."""
    def deco(fn):
        def kernel(*args):
            for a in args:
                if isinstance(a, torch.Tensor) and a.device.type != "cuda":
                    raise ValueError(f"rmd::{name}: all tensors must be on the GPU, got one on {a.device}")
            return fn(*args)
        LIB.impl(name, kernel, "CUDA")
        return fn
    return deco


def _fake(name):
    return torch.library.register_fake(f"rmd::{name}")


class _Dev:
    """Run a launch with the tensor's device current (only switches when it differs)."""

    def __init__(self, t):
        self.dev = t.device
        self.ctx = None

    def __enter__(self):
        if self.dev.index is not None and self.dev.index != torch.cuda.current_device():
            self.ctx = torch.cuda.device(self.dev)
            self.ctx.__enter__()
        return _lib.stream_ptr(self.dev)

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)


def _f32(t):
    """fp32, contiguous, detached (no aten.to call for fp32 inputs: an operator below autograd must
    not hand back its own input)."""
    t = t.detach()
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    return t.contiguous()


_DESC = {}


def describe(batch, height, width, levels, storage, layout=_lib.RMD_LAYOUT_ROWS):
    """rmd_pyramid_describe_layout, cached per geometry (host-only)."""
    key = (batch, height, width, levels, storage, layout)
    d = _DESC.get(key)
    if d is None:
        d = _DESC[key] = _lib.describe(batch, height, width, levels, storage, layout)
    return d


def describe_for(batch, height, width, levels, storage, channels, compute):
    """rmd_pyramid_describe_for: the layout the GEMM of (channels, compute) writes, cached."""
    key = ("for", batch, height, width, levels, storage, channels, compute)
    d = _DESC.get(key)
    if d is None:
        d = _DESC[key] = _lib.describe_for(batch, height, width, levels, storage, channels, compute)
    return d


_STORAGE = {_lib.RMD_F32: torch.float32, _lib.RMD_F16: torch.float16, _lib.RMD_S24: torch.uint8}
_STORAGE_CODE = {torch.float32: _lib.RMD_F32, torch.float16: _lib.RMD_F16, torch.uint8: _lib.RMD_S24}

# The pyramid tensor carries its layout and storage in its shape and dtype, so corr_lookup never
# trusts a caller's word for them: RMD_LAYOUT_ROWS pyramids are 1-D (total_elements,) float32/float16,
# RMD_LAYOUT_TILES pyramids 2-D (total_elements / 8, 8) float16 — one row per 2 x 4 chunk (every tiles
# level holds a multiple of 64 elements) — and RMD_S24 pyramids (row layout) uint8 (total_elements, 3).
TILES_ROW = 8
S24_BYTES = 3


def pyramid_view(data, layout):
    """The flat pyramid allocation shaped for its layout (see TILES_ROW)."""
    return data.view(-1, TILES_ROW) if layout == _lib.RMD_LAYOUT_TILES else data


def pyramid_layout(pyramid):
    """Layout of a pyramid tensor from its shape; ValueError for any other shape."""
    if pyramid.dtype == torch.uint8:
        if pyramid.dim() == 2 and pyramid.shape[1] == S24_BYTES:
            return _lib.RMD_LAYOUT_ROWS
    elif pyramid.dim() == 1:
        return _lib.RMD_LAYOUT_ROWS
    elif pyramid.dim() == 2 and pyramid.shape[1] == TILES_ROW:
        return _lib.RMD_LAYOUT_TILES
    raise ValueError(f"corr_lookup: a pyramid is 1-D (row layout), (n, {TILES_ROW}) (tiles layout) or uint8 "
                     f"(n, {S24_BYTES}) (S24 storage), got {pyramid.dtype} {tuple(pyramid.shape)}")


def pyramid_storage(pyramid):
    """RMD_F32 / RMD_F16 / RMD_S24 of a pyramid tensor (its dtype)."""
    if pyramid.dtype not in _STORAGE_CODE:
        raise ValueError(f"corr_lookup: pyramid dtype must be float32, float16 or uint8 (S24), got {pyramid.dtype}")
    return _STORAGE_CODE[pyramid.dtype]


def pyramid_elements(pyramid):
    """Pyramid elements held by a pyramid tensor (S24: 3 bytes each)."""
    return pyramid.shape[0] if pyramid.dtype == torch.uint8 else pyramid.numel()


def new_pyramid(like, d):
    """Uninitialised pyramid tensor for desc d on like's device (like.new_empty: fake tensors too)."""
    if d.storage == _lib.RMD_S24:
        return like.new_empty((d.total_elements, S24_BYTES), dtype=torch.uint8)
    return pyramid_view(like.new_empty((d.total_elements,), dtype=_STORAGE[d.storage]), d.layout)


def s24_encode(x):
    """float tensor -> RMD_S24 bytes (n, 3): the top 24 bits of each fp32 word, rounded half away from
    zero on the magnitude; NaN stays a quiet NaN (include/rmd.h RMD_S24, the x3 GEMM's epilogue)."""
    u = x.detach().float().contiguous().reshape(-1).view(torch.int32)
    nan = (u & 0x7fffffff) > 0x7f800000
    r = torch.where(nan, u | 0x00400000, u + 0x80)
    return r.view(torch.uint8).view(-1, 4)[:, 1:4].contiguous()


def s24_decode(b):
    """RMD_S24 bytes (n, 3) -> float32 (n,) (low mantissa byte zero)."""
    w = torch.zeros((b.shape[0], 4), dtype=torch.uint8, device=b.device)
    w[:, 1:4] = b
    return w.view(torch.float32).reshape(-1)


# ---- RAFT correlation pyramid + lookup (inference operators) -----------------------------------

def _check_fmaps(f1, f2):
    if f1.shape != f2.shape or f1.dim() != 4:
        raise ValueError(f"fmap1/fmap2 must be equal (B,C,H,W) shapes, got {tuple(f1.shape)} / {tuple(f2.shape)}")


@_cuda("corr_pyramid")
def _corr_pyramid(fmap1, fmap2, levels, compute, storage, scale):
    _check_fmaps(fmap1, fmap2)
    f1, f2 = _f32(fmap1), _f32(fmap2)
    b, c, h, w = f1.shape
    d = describe_for(b, h, w, levels, storage, c, compute)
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_corr_pyramid_workspace_bytes(ctypes.byref(d), c, compute), dtype=torch.uint8,
                     device=f1.device)
    data = new_pyramid(f1, d)                         # d.storage: S24 falls back to F32 off the x3 GEMM
    with _Dev(f1) as st:
        _lib.check(lib.rmd_corr_pyramid(_ptr(f1), _ptr(f2), c, float(scale), ctypes.byref(d), compute, _ptr(data),
                                        _ptr(ws), st), "rmd_corr_pyramid")
    return data


@_fake("corr_pyramid")
def _(fmap1, fmap2, levels, compute, storage, scale):
    _check_fmaps(fmap1, fmap2)
    b, c, h, w = fmap1.shape
    if fmap1.device.type == "cpu":                  # rmd/cpu.py writes the row layout, S24 as F32
        d = describe(b, h, w, levels, _lib.RMD_F32 if storage == _lib.RMD_S24 else storage)
    else:
        d = describe_for(b, h, w, levels, storage, c, compute)
    return new_pyramid(fmap1, d)


def _lookup_out(pyramid, coords, levels, radius):
    b, _, h, w = coords.shape
    return coords.new_empty((b, levels * (2 * radius + 1) ** 2, h, w), dtype=torch.float32)


def _check_device(name, *ts):
    dev = ts[0].device
    for t in ts[1:]:
        if t.device != dev:
            raise ValueError(f"{name}: tensors on different devices ({dev} / {t.device})")


@_cuda("corr_lookup")
def _corr_lookup(pyramid, coords, levels, radius, level_mask):
    b, two, h, w = coords.shape
    if pyramid.dtype not in _STORAGE_CODE or not pyramid.is_contiguous():
        raise ValueError(f"corr_lookup: pyramid must be a contiguous float32/float16/uint8 (S24) tensor, got "
                         f"{pyramid.dtype} {tuple(pyramid.shape)}")
    layout = pyramid_layout(pyramid)
    _check_device("corr_lookup", pyramid, coords)
    d = describe(b, h, w, levels, pyramid_storage(pyramid), layout)
    if two != 2 or pyramid_elements(pyramid) != d.total_elements:
        raise ValueError(f"corr_lookup: coords {tuple(coords.shape)} do not match the pyramid ({pyramid.numel()} elements)")
    co = _f32(coords)
    out = _lookup_out(pyramid, co, levels, radius)
    with _Dev(co) as st:
        _lib.check(_lib.lib().rmd_corr_lookup(_ptr(pyramid), ctypes.byref(d), _ptr(co), radius, level_mask, _ptr(out),
                                              st), "rmd_corr_lookup")
    return out


@_fake("corr_lookup")
def _(pyramid, coords, levels, radius, level_mask):
    pyramid_layout(pyramid)
    return _lookup_out(pyramid, coords, levels, radius)


@_cuda("corr_otf_prepare")
def _corr_otf_prepare(fmap1, fmap2, levels, compute, scale):
    _check_fmaps(fmap1, fmap2)
    f1, f2 = _f32(fmap1), _f32(fmap2)
    b, c, h, w = f1.shape
    lib = _lib.lib()
    nbytes = lib.rmd_corr_otf_workspace_bytes(b, c, h, w, levels, compute)
    if nbytes == 0:
        raise ValueError(f"otf: unsupported sizes {tuple(f1.shape)} with {levels} levels")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=f1.device)
    with _Dev(f1) as st:
        _lib.check(lib.rmd_corr_otf_prepare(_ptr(f1), _ptr(f2), b, c, h, w, levels, float(scale), compute, _ptr(ws), st),
                   "rmd_corr_otf_prepare")
    return ws


@_fake("corr_otf_prepare")
def _(fmap1, fmap2, levels, compute, scale):
    b, c, h, w = fmap1.shape
    if fmap1.device.type == "cpu":                  # rmd/cpu.py: fmap1 * scale + pooled levels, float32
        n = b * c * (h * w + sum((h >> i) * (w >> i) for i in range(levels)))
        return fmap1.new_empty((n,), dtype=torch.float32)
    return fmap1.new_empty((_lib.lib().rmd_corr_otf_workspace_bytes(b, c, h, w, levels, compute),), dtype=torch.uint8)


@_cuda("corr_otf_lookup")
def _corr_otf_lookup(workspace, coords, channels, levels, compute, radius, level_mask):
    b, two, h, w = coords.shape
    # the workspace must be the one corr_otf_prepare built for these sizes and this compute mode: its
    # segment layout depends on all of them, and the kernel trusts it
    want = _lib.lib().rmd_corr_otf_workspace_bytes(b, channels, h, w, levels, compute)
    if (two != 2 or workspace.dtype != torch.uint8 or workspace.dim() != 1 or not workspace.is_contiguous()
            or want == 0 or workspace.numel() != want):
        raise ValueError(f"corr_otf_lookup: workspace ({workspace.dtype}, {workspace.numel()} B) does not match "
                         f"coords {tuple(coords.shape)}, channels={channels}, levels={levels}, compute={compute} "
                         f"({want} B expected)")
    _check_device("corr_otf_lookup", workspace, coords)
    co = _f32(coords)
    out = _lookup_out(workspace, co, levels, radius)
    with _Dev(co) as st:
        _lib.check(_lib.lib().rmd_corr_otf_lookup(_ptr(workspace), b, channels, h, w, levels, compute, _ptr(co), radius,
                                                  level_mask, _ptr(out), st), "rmd_corr_otf_lookup")
    return out


@_fake("corr_otf_lookup")
def _(workspace, coords, channels, levels, compute, radius, level_mask):
    return _lookup_out(workspace, coords, levels, radius)


# ---- DICL displacement stacks -------------------------------------------------------------------

def _stack_shape(f1, radius, extra):
    b, c, h, w = f1.shape
    d = 2 * radius + 1
    return (b, d, d, 2 * c + (2 if extra else 0), h, w)


@_cuda("dicl_stack")
def _dicl_stack(fmap1, fmap2, coords, radius, level, norm_h, norm_w, extra_delta):
    f1, f2, co = _f32(fmap1), _f32(fmap2), _f32(coords)
    b, c, h, w = f1.shape
    hl, wl = f2.shape[-2:]
    if f2.shape[:2] != (b, c) or tuple(co.shape) != (b, 2, h, w):
        raise ValueError("dicl_stack: fmap2 must be (B,C,hl,wl) and coords (B,2,h,w) matching fmap1")
    out = torch.empty(_stack_shape(f1, radius, extra_delta), dtype=torch.float32, device=f1.device)
    with _Dev(f1) as st:
        _lib.check(_lib.lib().rmd_dicl_stack(_ptr(f1), _ptr(f2), _ptr(co), b, c, h, w, hl, wl, radius, level, norm_h,
                                             norm_w, int(extra_delta), _ptr(out), st), "rmd_dicl_stack")
    return out


@_fake("dicl_stack")
def _(fmap1, fmap2, coords, radius, level, norm_h, norm_w, extra_delta):
    return fmap1.new_empty(_stack_shape(fmap1, radius, extra_delta), dtype=torch.float32)


@_cuda("dicl_stack_backward")
def _dicl_stack_backward(grad, coords, channels, level_h, level_w, radius, level, norm_h, norm_w, extra_delta):
    g, co = _f32(grad), _f32(coords)
    b, _, h, w = co.shape
    g1 = torch.empty((b, channels, h, w), dtype=torch.float32, device=g.device)
    g2 = torch.empty((b, channels, level_h, level_w), dtype=torch.float32, device=g.device)
    with _Dev(g) as st:
        _lib.check(_lib.lib().rmd_dicl_stack_backward(_ptr(g), _ptr(co), b, channels, h, w, level_h, level_w, radius,
                                                      level, norm_h, norm_w, int(extra_delta), _ptr(g1), _ptr(g2), st),
                   "rmd_dicl_stack_backward")
    return g1, g2


@_fake("dicl_stack_backward")
def _(grad, coords, channels, level_h, level_w, radius, level, norm_h, norm_w, extra_delta):
    b, _, h, w = coords.shape
    return (coords.new_empty((b, channels, h, w), dtype=torch.float32),
            coords.new_empty((b, channels, level_h, level_w), dtype=torch.float32))


def _dicl_stack_setup(ctx, inputs, output):
    fmap1, fmap2, coords, radius, level, norm_h, norm_w, extra = inputs
    ctx.save_for_backward(coords)
    ctx.meta = (fmap1.shape[1], fmap2.shape[-2], fmap2.shape[-1], radius, level, norm_h, norm_w, extra)


def _dicl_stack_bwd(ctx, grad):
    (coords,) = ctx.saved_tensors
    c, hl, wl, radius, level, nh, nw, extra = ctx.meta
    g1, g2 = torch.ops.rmd.dicl_stack_backward(grad, coords, c, hl, wl, radius, level, nh, nw, extra)
    return g1, g2, None, None, None, None, None, None


torch.library.register_autograd("rmd::dicl_stack", _dicl_stack_bwd, setup_context=_dicl_stack_setup)


def _int_shape(f1, ru, rv):
    b, c, h, w = f1.shape
    return (b, 2 * ru + 1, 2 * rv + 1, 2 * c, h, w)


@_cuda("dicl_stack_int")
def _dicl_stack_int(fmap1, fmap2, ru, rv):
    f1, f2 = _f32(fmap1), _f32(fmap2)
    b, c, h, w = f1.shape
    if tuple(f2.shape) != (b, c, h, w):
        raise ValueError("dicl_stack_int: fmap1 and fmap2 must have equal (B,C,h,w) shapes")
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_dicl_stack_int_workspace_bytes(b, h, w), dtype=torch.uint8, device=f1.device)
    out = torch.empty(_int_shape(f1, ru, rv), dtype=torch.float32, device=f1.device)
    with _Dev(f1) as st:
        _lib.check(lib.rmd_dicl_stack_int(_ptr(f1), _ptr(f2), b, c, h, w, ru, rv, _ptr(out), _ptr(ws), st),
                   "rmd_dicl_stack_int")
    return out


@_fake("dicl_stack_int")
def _(fmap1, fmap2, ru, rv):
    return fmap1.new_empty(_int_shape(fmap1, ru, rv), dtype=torch.float32)


@_cuda("dicl_stack_int_backward")
def _dicl_stack_int_backward(grad, fmap2, ru, rv):
    g, f2 = _f32(grad), _f32(fmap2)
    b, c, h, w = f2.shape
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_dicl_stack_int_workspace_bytes(b, h, w), dtype=torch.uint8, device=g.device)
    g1 = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
    g2 = torch.empty_like(g1)
    with _Dev(g) as st:
        _lib.check(lib.rmd_dicl_stack_int_backward(_ptr(g), _ptr(f2), b, c, h, w, ru, rv, _ptr(g1), _ptr(g2), _ptr(ws),
                                                   st), "rmd_dicl_stack_int_backward")
    return g1, g2


@_fake("dicl_stack_int_backward")
def _(grad, fmap2, ru, rv):
    return fmap2.new_empty(fmap2.shape, dtype=torch.float32), fmap2.new_empty(fmap2.shape, dtype=torch.float32)


def _int_setup(ctx, inputs, output):
    _, fmap2, ru, rv = inputs
    ctx.save_for_backward(_f32(fmap2))
    ctx.meta = (ru, rv)


def _int_bwd(ctx, grad):
    (f2,) = ctx.saved_tensors
    g1, g2 = torch.ops.rmd.dicl_stack_int_backward(grad, f2, *ctx.meta)
    return g1, g2, None, None


torch.library.register_autograd("rmd::dicl_stack_int", _int_bwd, setup_context=_int_setup)


@_cuda("dicl_stack_int_warped")
def _dicl_stack_int_warped(fmap1, fmap2, flow, ru, rv):
    f1, f2, fl = _f32(fmap1), _f32(fmap2), _f32(flow)
    b, c, h, w = f1.shape
    if tuple(f2.shape) != (b, c, h, w) or tuple(fl.shape) != (b, 2, h, w):
        raise ValueError("dicl_stack_int_warped: need fmap1, fmap2 (B,C,h,w) and flow (B,2,h,w)")
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_dicl_stack_int_warped_workspace_bytes(b, c, h, w), dtype=torch.uint8, device=f1.device)
    out = torch.empty(_int_shape(f1, ru, rv), dtype=torch.float32, device=f1.device)
    with _Dev(f1) as st:
        _lib.check(lib.rmd_dicl_stack_int_warped(_ptr(f1), _ptr(f2), _ptr(fl), b, c, h, w, ru, rv, _ptr(out), _ptr(ws),
                                                 st), "rmd_dicl_stack_int_warped")
    return out


@_fake("dicl_stack_int_warped")
def _(fmap1, fmap2, flow, ru, rv):
    return fmap1.new_empty(_int_shape(fmap1, ru, rv), dtype=torch.float32)


@_cuda("dicl_stack_int_warped_backward")
def _dicl_stack_int_warped_backward(grad, fmap2, flow, ru, rv):
    g, f2, fl = _f32(grad), _f32(fmap2), _f32(flow)
    b, c, h, w = f2.shape
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_dicl_stack_int_warped_workspace_bytes(b, c, h, w), dtype=torch.uint8, device=g.device)
    g1 = torch.empty((b, c, h, w), dtype=torch.float32, device=g.device)
    g2 = torch.empty_like(g1)
    with _Dev(g) as st:
        _lib.check(lib.rmd_dicl_stack_int_warped_backward(_ptr(g), _ptr(f2), _ptr(fl), b, c, h, w, ru, rv, _ptr(g1),
                                                          _ptr(g2), _ptr(ws), st), "rmd_dicl_stack_int_warped_backward")
    return g1, g2


@_fake("dicl_stack_int_warped_backward")
def _(grad, fmap2, flow, ru, rv):
    return fmap2.new_empty(fmap2.shape, dtype=torch.float32), fmap2.new_empty(fmap2.shape, dtype=torch.float32)


def _warped_setup(ctx, inputs, output):
    _, fmap2, flow, ru, rv = inputs
    ctx.save_for_backward(_f32(fmap2), _f32(flow))
    ctx.meta = (ru, rv)


def _warped_bwd(ctx, grad):
    f2, fl = ctx.saved_tensors
    g1, g2 = torch.ops.rmd.dicl_stack_int_warped_backward(grad, f2, fl, *ctx.meta)
    return g1, g2, None, None, None


torch.library.register_autograd("rmd::dicl_stack_int_warped", _warped_bwd, setup_context=_warped_setup)


# ---- displacement-aware projection ---------------------------------------------------------------

def _dap_launch(x, weight, transpose, name):
    b, dd = x.shape[0], weight.shape[0]
    if x.numel() % (b * dd) or weight.numel() != dd * dd:
        raise ValueError(f"dap: x {tuple(x.shape)} does not hold {dd} displacement channels per batch")
    xc = _f32(x)
    wc = _f32(weight).reshape(dd, dd)
    out = torch.empty_like(xc)
    with _Dev(xc) as st:
        _lib.check(_lib.lib().rmd_dap(_ptr(xc), _ptr(wc), b, dd, xc.numel() // (b * dd), transpose, _ptr(out), st), name)
    return out


@_cuda("dap")
def _dap(x, weight):
    return _dap_launch(x, weight, 0, "rmd_dap")


@_fake("dap")
def _(x, weight):
    return x.new_empty(x.shape, dtype=torch.float32)


@_cuda("dap_transpose")
def _dap_transpose(grad, weight):
    return _dap_launch(grad, weight, 1, "rmd_dap^T")


@_fake("dap_transpose")
def _(grad, weight):
    return grad.new_empty(grad.shape, dtype=torch.float32)


@_cuda("dap_weight_grad")
def _dap_weight_grad(grad, x, disp):
    """dW = sum_b g_b x_b^T (rmd_dap_weight_grad: split-bf16 MFMA, deterministic split-K)."""
    b = x.shape[0]
    if grad.shape != x.shape or x.numel() % (b * disp):
        raise ValueError(f"dap_weight_grad: grad {tuple(grad.shape)} / x {tuple(x.shape)} with {disp} displacements")
    gc, xc = _f32(grad), _f32(x)
    n = xc.numel() // (b * disp)
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_dap_weight_grad_workspace_bytes(b, disp, n), dtype=torch.uint8, device=xc.device)
    out = torch.empty((disp, disp), dtype=torch.float32, device=xc.device)
    with _Dev(xc) as st:
        _lib.check(lib.rmd_dap_weight_grad(_ptr(gc), _ptr(xc), b, disp, n, _ptr(out), _ptr(ws), st),
                   "rmd_dap_weight_grad")
    return out


@_fake("dap_weight_grad")
def _(grad, x, disp):
    return x.new_empty((disp, disp), dtype=torch.float32)


def _dap_setup(ctx, inputs, output):
    x, weight = inputs
    ctx.save_for_backward(x, weight)


def _dap_bwd(ctx, grad):
    x, weight = ctx.saved_tensors
    b, dd = x.shape[0], weight.shape[0]
    gx = torch.ops.rmd.dap_transpose(grad, weight) if ctx.needs_input_grad[0] else None
    gw = None
    if ctx.needs_input_grad[1]:
        gw = torch.ops.rmd.dap_weight_grad(grad, x, dd).reshape(weight.shape).to(weight.dtype)
    return gx, gw


torch.library.register_autograd("rmd::dap", _dap_bwd, setup_context=_dap_setup)


# ---- flow heads ----------------------------------------------------------------------------------

@_cuda("up8")
def _up8(mask, flow, temperature):
    b, c, h, w = flow.shape
    if c != 2 or tuple(mask.shape) != (b, 576, h, w):
        raise ValueError(f"up8: need flow (B,2,h,w) and mask (B,576,h,w), got {tuple(flow.shape)}, {tuple(mask.shape)}")
    mc, fc = _f32(mask), _f32(flow)
    out = torch.empty((b, 2, 8 * h, 8 * w), dtype=torch.float32, device=fc.device)
    with _Dev(fc) as st:
        _lib.check(_lib.lib().rmd_up8(_ptr(mc), _ptr(fc), b, h, w, float(temperature), _ptr(out), st), "rmd_up8")
    return out


@_fake("up8")
def _(mask, flow, temperature):
    b, _, h, w = flow.shape
    return flow.new_empty((b, 2, 8 * h, 8 * w), dtype=torch.float32)


@_cuda("up8_backward")
def _up8_backward(grad, mask, flow, temperature):
    g, mc, fc = _f32(grad), _f32(mask), _f32(flow)
    b, _, h, w = fc.shape
    lib = _lib.lib()
    ws = torch.empty(lib.rmd_up8_workspace_bytes(b, h, w), dtype=torch.uint8, device=g.device)
    gm = torch.empty_like(mc)
    gf = torch.empty_like(fc)
    with _Dev(g) as st:
        _lib.check(lib.rmd_up8_backward(_ptr(mc), _ptr(fc), _ptr(g), b, h, w, float(temperature), _ptr(gm), _ptr(gf),
                                        _ptr(ws), st), "rmd_up8_backward")
    return gm, gf


@_fake("up8_backward")
def _(grad, mask, flow, temperature):
    return mask.new_empty(mask.shape, dtype=torch.float32), flow.new_empty(flow.shape, dtype=torch.float32)


def _up8_setup(ctx, inputs, output):
    mask, flow, temperature = inputs
    ctx.save_for_backward(mask, flow)
    ctx.temperature = temperature


def _up8_bwd(ctx, grad):
    mask, flow = ctx.saved_tensors
    gm, gf = torch.ops.rmd.up8_backward(grad, mask, flow, ctx.temperature)
    return gm.to(mask.dtype), gf.to(flow.dtype), None


torch.library.register_autograd("rmd::up8", _up8_bwd, setup_context=_up8_setup)


def _sam_shape(cost, levels):
    b = cost.shape[0]
    return (levels, b, 2) + tuple(cost.shape[2:])


@_cuda("softargmax")
def _softargmax(cost, levels, radius, temperature):
    b, ctot = cost.shape[:2]
    n = cost[0, 0].numel()
    if ctot < levels * (2 * radius + 1) ** 2:
        raise ValueError(f"softargmax: {ctot} channels < {levels} levels x {(2 * radius + 1) ** 2} displacements")
    cc = _f32(cost)
    flows = torch.empty(_sam_shape(cc, levels), dtype=torch.float32, device=cc.device)
    with _Dev(cc) as st:
        _lib.check(_lib.lib().rmd_softargmax(_ptr(cc), b, ctot, n, levels, radius, float(temperature), _ptr(flows), st),
                   "rmd_softargmax")
    return flows


@_fake("softargmax")
def _(cost, levels, radius, temperature):
    return cost.new_empty(_sam_shape(cost, levels), dtype=torch.float32)


@_cuda("softargmax_backward")
def _softargmax_backward(grad, cost, levels, radius, temperature):
    cc, g = _f32(cost), _f32(grad)
    b, ctot = cc.shape[:2]
    n = cc[0, 0].numel()
    gc = torch.zeros_like(cc) if ctot > levels * (2 * radius + 1) ** 2 else torch.empty_like(cc)
    with _Dev(g) as st:
        _lib.check(_lib.lib().rmd_softargmax_backward(_ptr(cc), _ptr(g), b, ctot, n, levels, radius, float(temperature),
                                                      _ptr(gc), st), "rmd_softargmax_backward")
    return gc


@_fake("softargmax_backward")
def _(grad, cost, levels, radius, temperature):
    return cost.new_empty(cost.shape, dtype=torch.float32)


def _sam_setup(ctx, inputs, output):
    cost, levels, radius, temperature = inputs
    ctx.save_for_backward(cost)
    ctx.meta = (levels, radius, temperature)


def _sam_bwd(ctx, grad):
    (cost,) = ctx.saved_tensors
    gc = torch.ops.rmd.softargmax_backward(grad, cost, *ctx.meta)
    return gc.to(cost.dtype), None, None, None


torch.library.register_autograd("rmd::softargmax", _sam_bwd, setup_context=_sam_setup)


# ---- backward warp -------------------------------------------------------------------------------

@_cuda("warp_backwards")
def _warp_backwards(img2, flow, eps):
    b, c, h, w = img2.shape
    if tuple(flow.shape) != (b, 2, h, w):
        raise ValueError(f"warp_backwards: flow {tuple(flow.shape)} must be (B, 2, h, w) for img2 {tuple(img2.shape)}")
    ic, fc = _f32(img2), _f32(flow)
    out = torch.empty_like(ic)
    mask = torch.empty((b, 1, h, w), dtype=torch.uint8, device=ic.device)
    with _Dev(ic) as st:
        _lib.check(_lib.lib().rmd_warp_backwards(_ptr(ic), _ptr(fc), b, c, h, w, float(eps), _ptr(out), _ptr(mask), st),
                   "rmd_warp_backwards")
    return out, mask.bool()


@_fake("warp_backwards")
def _(img2, flow, eps):
    b, c, h, w = img2.shape
    return img2.new_empty(img2.shape, dtype=torch.float32), img2.new_empty((b, 1, h, w), dtype=torch.bool)


@_cuda("warp_backwards_backward")
def _warp_backwards_backward(grad, flow, eps):
    g, fc = _f32(grad), _f32(flow)
    b, c, h, w = g.shape
    gi = torch.empty_like(g)
    with _Dev(g) as st:
        _lib.check(_lib.lib().rmd_warp_backwards_backward(_ptr(g), _ptr(fc), b, c, h, w, float(eps), _ptr(gi), st),
                   "rmd_warp_backwards_backward")
    return gi


@_fake("warp_backwards_backward")
def _(grad, flow, eps):
    return grad.new_empty(grad.shape, dtype=torch.float32)


def _warp_setup(ctx, inputs, output):
    img2, flow, eps = inputs
    ctx.save_for_backward(flow)
    ctx.eps = eps
    ctx.dtype = img2.dtype
    ctx.mark_non_differentiable(output[1])


def _warp_bwd(ctx, grad, _gmask):
    (flow,) = ctx.saved_tensors
    return torch.ops.rmd.warp_backwards_backward(grad, flow, ctx.eps).to(ctx.dtype), None, None


torch.library.register_autograd("rmd::warp_backwards", _warp_bwd, setup_context=_warp_setup)


def operators():
    """Names of the registered torch.ops.rmd operators."""
    return sorted(_SCHEMAS)
