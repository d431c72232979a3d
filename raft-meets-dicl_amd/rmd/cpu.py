"""CPU kernels of the torch.ops.rmd operators: ATen composites of the reference's own algorithms.

The reference's modules run on any device (src/models/impls/raft.py:15-95 is plain torch), so a user
who evaluates on the CPU keeps the drop-ins: every rmd operator has a kernel here, registered for the
CPU and AutogradCPU dispatch keys (SURVEY.md §7 "CPU dispatch").

Dispatch, not fallback: a CUDA tensor always reaches the HIP kernel of rmd/library.py (which raises if
librmd.so is missing); only CPU tensors come here.  Each kernel restates the reference lines it names
with the same ATen calls (matmul, avg_pool2d, grid_sample, ...), in fp32 whatever the compute mode
(the storage dtype of a pyramid is honoured), so CPU results follow the reference op for op.
Registered at AutogradCPU, the kernels record their ATen graph: the modules train on CPU through
ordinary autograd (the alias-key formulas of rmd/library.py serve the CUDA kernels).

CPU-side formats:
  * corr_pyramid returns the row layout (1-D, include/rmd.h RMD_LAYOUT_ROWS) for every precision;
  * corr_otf_prepare returns a float32 "workspace" holding fmap1 * scale and the pooled fmap2 levels
    (the HIP workspace is an opaque byte buffer in the kernel's operand order).
"""

import torch
import torch.nn.functional as F

from . import _lib
from .library import LIB, _SCHEMAS, _STORAGE, pyramid_elements, pyramid_layout, pyramid_storage, s24_decode


def _delta(r, device):
    """(2r+1, 2r+1, 2) displacement grid, meshgrid(dx, dy, indexing='ij') (raft.py:55-59)."""
    d = torch.linspace(-r, r, 2 * r + 1, device=device)
    return torch.stack(torch.meshgrid(d, d, indexing="ij"), dim=-1)


def _normalise(cen, w_den, h_den):
    """grid_sample coordinates as the reference computes them in place (raft.py:69-70)."""
    x = 2 * cen[..., 0] / w_den - 1
    y = 2 * cen[..., 1] / h_den - 1
    return torch.stack((x, y), dim=-1)


# ---- RAFT correlation pyramid + lookup (raft.py:18-95) ------------------------------------------

def _corr_levels(f1, f2, levels, scale):
    """raft.py:26-47: corr = fmap1^T fmap2 (B, H, W, 1, H, W) normalised, then 2x2 average pools."""
    b, c, h, w = f1.shape
    corr = torch.matmul(f1.reshape(b, c, h * w).transpose(1, 2), f2.reshape(b, c, h * w))
    if abs(scale * (c ** 0.5) - 1.0) < 1e-6:
        corr = corr / torch.tensor(c).float().sqrt()        # raft.CorrBlock's normalisation, op for op
    elif scale != 1.0:
        corr = corr * scale
    lv = [corr.reshape(b * h * w, 1, h, w)]
    for _ in range(1, levels):
        lv.append(F.avg_pool2d(lv[-1], kernel_size=2, stride=2))
    return lv


def _pack_rows(lv, desc, dtype):
    """Levels (B*N, 1, H_l, W_l) -> the row-layout pyramid (include/rmd.h element formula)."""
    b, n = desc.batch, desc.height * desc.width
    parts, at = [], 0
    for i, x in enumerate(lv):
        hl, wl, cw, tx = desc.level_h[i], desc.level_w[i], desc.tile_w[i], desc.tiles_x[i]
        if desc.level_offset[i] != at:
            parts.append(x.new_zeros(desc.level_offset[i] - at))
        x = F.pad(x.reshape(b, n, hl, wl), (0, tx * cw - wl))
        parts.append(x.reshape(b, n, hl, tx, cw).permute(0, 2, 3, 1, 4).reshape(-1))
        at = desc.level_offset[i] + parts[-1].numel()
    if desc.total_elements != at:
        parts.append(lv[0].new_zeros(desc.total_elements - at))
    return torch.cat(parts).to(dtype)


def _unpack(pyramid, desc, i):
    """Level i of a pyramid tensor (either layout) as (B*N, 1, H_i, W_i) float32."""
    b, h, w = desc.batch, desc.height, desc.width
    th, tw, ty, tx = desc.tile_h[i], desc.tile_w[i], desc.tiles_y[i], desc.tiles_x[i]
    s, off = desc.query_slots, desc.level_offset[i]
    x = pyramid.reshape(-1)[off: off + b * ty * tx * s * th * tw].view(b, ty, tx, s, th, tw)
    x = x.permute(0, 3, 1, 4, 2, 5).reshape(b, s, ty * th, tx * tw)[..., :desc.level_h[i], :desc.level_w[i]]
    if desc.layout == _lib.RMD_LAYOUT_TILES:
        from .ops import tiles_slots
        x = x.index_select(1, tiles_slots(h, w).to(x.device))
    return x.float().reshape(b * h * w, 1, desc.level_h[i], desc.level_w[i])


def corr_pyramid(fmap1, fmap2, levels, compute, storage, scale):
    f1, f2 = fmap1.float(), fmap2.float()
    b, c, h, w = f1.shape
    if storage == _lib.RMD_S24:
        # S24 is the x3 GEMM's output format; every other GEMM (this one too) stores F32, as
        # rmd_pyramid_describe_for resolves it — which also keeps the ATen graph differentiable
        storage = _lib.RMD_F32
    desc = _lib.describe(b, h, w, levels, storage, _lib.RMD_LAYOUT_ROWS)
    return _pack_rows(_corr_levels(f1, f2, levels, float(scale)), desc, _STORAGE[storage])


def corr_lookup(pyramid, coords, levels, radius, level_mask):
    """raft.py:49-95 over the levels stored in `pyramid`."""
    b, _, h, w = coords.shape
    desc = _lib.describe(b, h, w, levels, pyramid_storage(pyramid), pyramid_layout(pyramid))
    if pyramid_elements(pyramid) != desc.total_elements:
        raise ValueError(f"corr_lookup: coords {tuple(coords.shape)} do not match the pyramid "
                         f"({pyramid_elements(pyramid)} elements)")
    if desc.storage == _lib.RMD_S24:
        pyramid = s24_decode(pyramid)
    r = radius
    co = coords.float().permute(0, 2, 3, 1)
    delta = _delta(r, coords.device)
    out = []
    for i in range(levels):
        corr = _unpack(pyramid, desc, i)
        h2, w2 = corr.shape[-2:]
        cen = co.reshape(b, h, w, 1, 1, 2) / 2 ** i + delta
        cen = _normalise(cen, w2 - 1, h2 - 1).reshape(b * h * w, 2 * r + 1, 2 * r + 1, 2)
        corr = F.grid_sample(corr, cen, align_corners=True).view(b, h, w, -1)
        if (level_mask >> i) & 1:
            corr = torch.zeros_like(corr)
        out.append(corr)
    return torch.cat(out, dim=-1).permute(0, 3, 1, 2).contiguous().float()


# ---- on-the-fly lookup (raft_fs.py:13-87) -------------------------------------------------------

def _otf_split(workspace, b, c, h, w, levels):
    sizes = [(h >> i, w >> i) for i in range(levels)]
    n1 = b * c * h * w
    f1 = workspace[:n1].view(b, c, h, w)
    pyr, at = [], n1
    for hl, wl in sizes:
        k = b * c * hl * wl
        pyr.append(workspace[at: at + k].view(b, c, hl, wl))
        at += k
    if at != workspace.numel():
        raise ValueError(f"corr_otf_lookup: workspace of {workspace.numel()} floats does not match "
                         f"({b}, {c}, {h}, {w}) with {levels} levels")
    return f1, pyr


def corr_otf_prepare(fmap1, fmap2, levels, compute, scale):
    """raft_fs.py:16-31: fmap2 and its avg-pooled levels, kept with fmap1 * scale."""
    f2 = fmap2.float()
    parts = [(fmap1.float() * float(scale)).reshape(-1), f2.reshape(-1)]
    for _ in range(1, levels):
        f2 = F.avg_pool2d(f2, kernel_size=2, stride=2)
        parts.append(f2.reshape(-1))
    return torch.cat(parts)


def corr_otf_lookup(workspace, coords, channels, levels, compute, radius, level_mask):
    """raft_fs.py:33-87: grid-sample each pooled level at the window and dot it with fmap1."""
    b, _, h, w = coords.shape
    if workspace.dtype != torch.float32:
        raise ValueError("corr_otf_lookup: a CPU workspace comes from the CPU corr_otf_prepare (float32)")
    f1, pyr = _otf_split(workspace, b, channels, h, w, levels)
    c, r = channels, radius
    f1 = f1.permute(0, 2, 3, 1).reshape(b, h, w, c, 1)
    delta = _delta(r, coords.device).view(1, 2 * r + 1, 1, 2 * r + 1, 1, 2)
    co = coords.float().permute(0, 2, 3, 1).reshape(b, 1, h, 1, w, 2)
    out = []
    for i, f2 in enumerate(pyr):
        h2, w2 = f2.shape[-2:]
        cen = _normalise(co / 2 ** i + delta, w2 - 1, h2 - 1).reshape(b, (2 * r + 1) * h, (2 * r + 1) * w, 2)
        s = F.grid_sample(f2, cen, align_corners=True).view(b, c, 2 * r + 1, h, 2 * r + 1, w)
        s = s.permute(0, 3, 5, 2, 4, 1).reshape(b, h, w, (2 * r + 1) ** 2, c)
        corr = torch.matmul(s, f1).view(b, h, w, (2 * r + 1) ** 2)
        if (level_mask >> i) & 1:
            corr = torch.zeros_like(corr)
        out.append(corr)
    return torch.cat(out, dim=-1).permute(0, 3, 1, 2).contiguous().float()


# ---- DICL displacement stacks (corr/dicl.py:26-54, dicl_emb.py:51-89, raft_dicl_ml.py:294-315) ----

def _stack_f2(f2, coords, h, w, radius, level, norm_h, norm_w):
    b, c = f2.shape[:2]
    r = radius
    delta = _delta(r, coords.device).view(1, 2 * r + 1, 1, 2 * r + 1, 1, 2)
    co = coords.float().permute(0, 2, 3, 1).reshape(b, 1, h, 1, w, 2)
    cen = (co / 2 ** level if level else co) + delta
    cen = _normalise(cen, norm_w - 1, norm_h - 1).reshape(b, (2 * r + 1) * h, (2 * r + 1) * w, 2)
    s = F.grid_sample(f2, cen, align_corners=True).view(b, c, 2 * r + 1, h, 2 * r + 1, w)
    return s.permute(0, 2, 4, 1, 3, 5)                      # (B, 2r+1, 2r+1, C, h, w)


def dicl_stack(fmap1, fmap2, coords, radius, level, norm_h, norm_w, extra_delta):
    f1, f2 = fmap1.float(), fmap2.float()
    b, c, h, w = f1.shape
    d = 2 * radius + 1
    parts = [f1.view(b, 1, 1, c, h, w).expand(-1, d, d, -1, -1, -1),
             _stack_f2(f2, coords, h, w, radius, level, norm_h, norm_w)]
    if extra_delta:                                          # dicl_emb.py:82-86: delta as positional encoding
        parts.append(_delta(radius, f1.device).view(1, d, d, 2, 1, 1).expand(b, -1, -1, -1, h, w))
    return torch.cat(parts, dim=-3)


def dicl_stack_backward(grad, coords, channels, level_h, level_w, radius, level, norm_h, norm_w, extra_delta):
    b, _, h, w = coords.shape
    g = grad.float()
    g1 = g[:, :, :, :channels].sum(dim=(1, 2))
    with torch.enable_grad():
        f2 = torch.zeros(b, channels, level_h, level_w, device=grad.device, requires_grad=True)
        s = _stack_f2(f2, coords.detach(), h, w, radius, level, norm_h, norm_w)
        (g2,) = torch.autograd.grad(s, f2, g[:, :, :, channels:2 * channels])
    return g1, g2


def dicl_stack_int(fmap1, fmap2, ru, rv):
    """impls/dicl.py:212-238: integer-displacement volume, zeroed where the f2 half sums to 0."""
    f1, f2 = fmap1.float(), fmap2.float()
    b, c, h, w = f1.shape
    du, dv = 2 * ru + 1, 2 * rv + 1
    rows = []
    for i in range(du):
        cols = []
        for j in range(dv):
            di, dj = i - ru, j - rv
            w0, w1, h0, h1 = max(0, -di), min(w, w - di), max(0, -dj), min(h, h - dj)
            dw0, dw1, dh0, dh1 = max(0, di), min(w, w + di), max(0, dj), min(h, h + dj)
            a = F.pad(f1[:, :, h0:h1, w0:w1], (w0, w - w1, h0, h - h1))
            z = F.pad(f2[:, :, dh0:dh1, dw0:dw1], (w0, w - w1, h0, h - h1))
            cols.append(torch.cat((a, z), dim=1))
        rows.append(torch.stack(cols, dim=1))
    mvol = torch.stack(rows, dim=1)                          # (B, du, dv, 2C, h, w)
    valid = mvol[:, :, :, c:].detach().sum(dim=-3) != 0
    return mvol * valid.unsqueeze(3)


def _int_grads(grad, fmap1_like, fmap2, fn):
    with torch.enable_grad():
        f1 = torch.zeros_like(fmap1_like, dtype=torch.float32, requires_grad=True)
        f2 = fmap2.detach().float().requires_grad_(True)
        out = fn(f1, f2)
        return torch.autograd.grad(out, (f1, f2), grad.float())


def dicl_stack_int_backward(grad, fmap2, ru, rv):
    return _int_grads(grad, fmap2, fmap2, lambda a, z: dicl_stack_int(a, z, ru, rv))


# ---- backward warp (common/warp.py:5-33) --------------------------------------------------------

def _warp_grid(flow, h, w):
    cx = torch.arange(0, w, device=flow.device).view(1, w).expand(h, -1)
    cy = torch.arange(0, h, device=flow.device).view(h, 1).expand(-1, w)
    fpos = (torch.stack((cx, cy), dim=0).float() + flow.float()).permute(0, 2, 3, 1)
    return _normalise(fpos, max(w - 1, 0), max(h - 1, 0))


def warp_backwards(img2, flow, eps):
    b, c, h, w = img2.shape
    fpos = _warp_grid(flow, h, w)
    est = F.grid_sample(img2.float(), fpos, align_corners=True)
    mask = F.grid_sample(torch.ones(b, 1, h, w, device=img2.device), fpos, align_corners=True) > (1.0 - eps)
    return est * mask, mask


def warp_backwards_backward(grad, flow, eps):
    with torch.enable_grad():
        img = torch.zeros(grad.shape, device=grad.device, requires_grad=True)
        est, _ = warp_backwards(img, flow.detach(), eps)
        return torch.autograd.grad(est, img, grad.float())[0]


def dicl_stack_int_warped(fmap1, fmap2, flow, ru, rv):
    """impls/dicl.py:178-181 (warp_backwards of feat2 by the coarse flow, eps 1e-5) + :212-238."""
    warped, _ = warp_backwards(fmap2, flow.detach(), 1e-5)
    return dicl_stack_int(fmap1, warped, ru, rv)


def dicl_stack_int_warped_backward(grad, fmap2, flow, ru, rv):
    return _int_grads(grad, fmap2, fmap2, lambda a, z: dicl_stack_int_warped(a, z, flow, ru, rv))


# ---- displacement-aware projection (blocks/dicl.py:143-150) -------------------------------------

def _dap_view(x, weight):
    b, dd = x.shape[0], weight.shape[0]
    if x.numel() % (b * dd) or weight.numel() != dd * dd:
        raise ValueError(f"dap: x {tuple(x.shape)} does not hold {dd} displacement channels per batch")
    return x.float().reshape(b, dd, -1, 1), weight.float().reshape(dd, dd, 1, 1)


def dap(x, weight):
    xv, wv = _dap_view(x, weight)
    return F.conv2d(xv, wv).reshape(x.shape)                 # the reference's 1x1 nn.Conv2d, no bias


def dap_transpose(grad, weight):
    gv, wv = _dap_view(grad, weight)
    return F.conv2d(gv, wv.reshape(wv.shape[0], -1).t().reshape(wv.shape)).reshape(grad.shape)


def dap_weight_grad(grad, x, disp):
    b = x.shape[0]
    g, xx = grad.float().reshape(b, disp, -1), x.float().reshape(b, disp, -1)
    return torch.einsum("bop,bip->oi", g, xx)


# ---- flow heads (raft.py:98-190, 319-331) -------------------------------------------------------

def up8(mask, flow, temperature):
    b, c, h, w = flow.shape
    m = torch.softmax(mask.float().view(b, 1, 9, 8, 8, h, w) / temperature, dim=2)
    up = F.unfold(8 * flow.float(), (3, 3), padding=1).view(b, c, 9, 1, 1, h, w)
    up = torch.sum(m * up, dim=2).permute(0, 1, 4, 2, 5, 3)
    return up.reshape(b, 2, h * 8, w * 8)


def up8_backward(grad, mask, flow, temperature):
    with torch.enable_grad():
        m = mask.detach().float().requires_grad_(True)
        f = flow.detach().float().requires_grad_(True)
        return torch.autograd.grad(up8(m, f, temperature), (m, f), grad.float())


def softargmax(cost, levels, radius, temperature):
    b = cost.shape[0]
    dd = (2 * radius + 1) ** 2
    if cost.shape[1] < levels * dd:
        raise ValueError(f"softargmax: {cost.shape[1]} channels < {levels} levels x {dd} displacements")
    rest = tuple(cost.shape[2:])
    c = cost.float().reshape(b, cost.shape[1], 1, -1)
    delta = _delta(radius, cost.device).view(1, dd, 2, 1)
    flows = []
    for lvl in range(levels):
        score = F.softmax(c[:, lvl * dd:(lvl + 1) * dd] / temperature, dim=1)
        flows.append(torch.sum(delta * 2 ** lvl * score, dim=1).reshape((b, 2) + rest))
    return torch.stack(flows)


def softargmax_backward(grad, cost, levels, radius, temperature):
    with torch.enable_grad():
        c = cost.detach().float().requires_grad_(True)
        return torch.autograd.grad(softargmax(c, levels, radius, temperature), c, grad.float())[0]


_KERNELS = {
    "corr_pyramid": corr_pyramid, "corr_lookup": corr_lookup,
    "corr_otf_prepare": corr_otf_prepare, "corr_otf_lookup": corr_otf_lookup,
    "dicl_stack": dicl_stack, "dicl_stack_backward": dicl_stack_backward,
    "dicl_stack_int": dicl_stack_int, "dicl_stack_int_backward": dicl_stack_int_backward,
    "dicl_stack_int_warped": dicl_stack_int_warped, "dicl_stack_int_warped_backward": dicl_stack_int_warped_backward,
    "dap": dap, "dap_transpose": dap_transpose, "dap_weight_grad": dap_weight_grad,
    "up8": up8, "up8_backward": up8_backward, "softargmax": softargmax, "softargmax_backward": softargmax_backward,
    "warp_backwards": warp_backwards, "warp_backwards_backward": warp_backwards_backward,
}
assert sorted(_KERNELS) == sorted(_SCHEMAS), "every rmd operator needs a CPU kernel"

for _name, _fn in _KERNELS.items():
    LIB.impl(_name, _fn, "CPU")
    LIB.impl(_name, _fn, "AutogradCPU")
