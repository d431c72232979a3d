"""Oracle: DICL cost-volume construction and displacement-aware projection (numpy).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Reference semantics restated here (qzed/raft-meets-dicl v2):
  * dicl_stack — src/models/common/corr/dicl.py:26-54 (same body in dicl_1x1.py:51-79):
      stack[b,a,bb,0:C,y,x]  = f1[b,:,y,x]                              (expand, :51-52)
      stack[b,a,bb,C:2C,y,x] = bilinear(f2, x_c + a - r, y_c + bb - r)  (grid_sample, :36-48)
    zero padding per tap, align_corners=True, no validity mask.  The multi-level module
    src/models/impls/raft_dicl_ml.py:294-315 samples level i of the fmap2 pyramid at
    (x/2^i + a - r, y/2^i + bb - r) normalised with fmap1's (w-1),(h-1) and un-normalised with the
    level's (w_i-1),(h_i-1): sample position = (x/2^i + a - r) * (w_i-1)/(w-1).
  * dicl_stack_int — src/models/impls/dicl.py:212-238: integer displacements di = i - ru (x),
    dj = j - rv (y); both halves copied where (x+di, y+dj) is inside, zero elsewhere; then the
    whole 2C vector is zeroed where sum_c of the f2 half == 0 (detached mask, :236-238).
  * dap — src/models/common/blocks/dicl.py:121-150: 1x1 conv D->D without bias.
"""

import numpy as np

from .corr import _sample_features


def dicl_stack(f1, f2, coords, radius, level=0, norm_hw=None):
    """(B,C,h,w) f1, (B,C,h_i,w_i) f2, coords (B,2,h,w) -> stack (B, d, d, 2C, h, w)."""
    b, c, h, w = f1.shape
    hl, wl = f2.shape[-2:]
    nh, nw = norm_hw if norm_hw is not None else (h, w)
    d = 2 * radius + 1
    s = 2.0 ** level
    cx = coords[:, 0].reshape(b, h * w) / s
    cy = coords[:, 1].reshape(b, h * w) / s
    sx = (wl - 1) / (nw - 1)
    sy = (hl - 1) / (nh - 1)
    samp = _sample_features(f2, cx, cy, radius, sx, sy)                    # (B,C,P,a,b)
    samp = samp.reshape(b, c, h, w, d, d).transpose(0, 4, 5, 1, 2, 3)     # (B,a,b,C,h,w)
    f1e = np.broadcast_to(f1[:, None, None], (b, d, d, c, h, w))
    return np.ascontiguousarray(np.concatenate([f1e, samp], axis=3))


def dicl_stack_backward(f2_shape, coords, radius, grad_stack, level=0, norm_hw=None):
    """Gradients of dicl_stack w.r.t. f1 (sum over displacements) and f2 (bilinear scatter)."""
    b, d, _, c2, h, w = grad_stack.shape
    c = c2 // 2
    hl, wl = f2_shape[-2:]
    nh, nw = norm_hw if norm_hw is not None else (h, w)
    dt = grad_stack.dtype
    gf1 = grad_stack[:, :, :, :c].sum(axis=(1, 2))
    gf2 = np.zeros((b, c, hl, wl), dtype=dt)
    s = 2.0 ** level
    sx = (wl - 1) / (nw - 1)
    sy = (hl - 1) / (nh - 1)
    cx = coords[:, 0] / s
    cy = coords[:, 1] / s
    bi = np.arange(b)[:, None, None]
    one = np.asarray(1, dtype=dt)
    for a in range(d):
        for bb in range(d):
            px = (cx + (a - radius)) * sx
            py = (cy + (bb - radius)) * sy
            x0 = np.floor(px)
            y0 = np.floor(py)
            fx, fy = px - x0, py - y0
            x0 = x0.astype(np.int64)
            y0 = y0.astype(np.int64)
            g = grad_stack[:, a, bb, c:]                                     # (B,C,h,w)
            for ddy, wy in ((0, one - fy), (1, fy)):
                for ddx, wx in ((0, one - fx), (1, fx)):
                    xx, yy = x0 + ddx, y0 + ddy
                    v = (xx >= 0) & (xx < wl) & (yy >= 0) & (yy < hl)
                    contrib = g * (wx * wy * v)[:, None]                     # (B,C,h,w)
                    idx_y = np.clip(yy, 0, hl - 1)
                    idx_x = np.clip(xx, 0, wl - 1)
                    for ch in range(c):
                        np.add.at(gf2[:, ch], (bi, idx_y, idx_x), contrib[:, ch])
    return gf1, gf2


def dicl_stack_int(f1, f2, ru, rv):
    """(B,C,h,w) x2 -> mvol (B, 2ru+1, 2rv+1, 2C, h, w) with the occlusion validity mask."""
    b, c, h, w = f1.shape
    du, dv = 2 * ru + 1, 2 * rv + 1
    mvol = np.zeros((b, du, dv, 2 * c, h, w), dtype=f1.dtype)
    for i in range(du):
        for j in range(dv):
            di, dj = i - ru, j - rv
            w0, w1 = max(0, -di), min(w, w - di)
            h0, h1 = max(0, -dj), min(h, h - dj)
            if w1 <= w0 or h1 <= h0:
                continue
            mvol[:, i, j, :c, h0:h1, w0:w1] = f1[:, :, h0:h1, w0:w1]
            mvol[:, i, j, c:, h0:h1, w0:w1] = f2[:, :, h0 + dj:h1 + dj, w0 + di:w1 + di]
    valid = mvol[:, :, :, c:].sum(axis=3) != 0
    return mvol * valid[:, :, :, None]


def dicl_stack_int_at(f1, f2, ru, rv, idx):
    """dicl_stack_int evaluated only at sampled positions (full-size parity checks).

    idx = (b, i, j, y, x) integer arrays of equal length n -> (n, 2C): the same copy + occlusion
    mask as dicl_stack_int (src/models/impls/dicl.py:212-238), one displacement vector per sample.
    """
    b, i, j, y, x = (np.asarray(a, dtype=np.int64) for a in idx)
    c, h, w = f1.shape[1:]
    di, dj = i - ru, j - rv
    xx, yy = x + di, y + dj
    inside = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
    v1 = f1[b, :, y, x]                                                   # (n, C)
    v2 = f2[b, :, np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)] * inside[:, None]
    out = np.concatenate([v1 * inside[:, None], v2], axis=1)
    valid = v2.sum(axis=1) != 0
    return out * valid[:, None]


def dicl_stack_at(f1, f2, coords, radius, idx, level=0, norm_hw=None):
    """dicl_stack evaluated only at sampled positions: idx = (b, a, bb, y, x) -> (n, 2C).

    Same sample position as dicl_stack (src/models/common/corr/dicl.py:26-54; level scaling of
    src/models/impls/raft_dicl_ml.py:294-315): ((x_c/2^i + a - r) * sx, (y_c/2^i + bb - r) * sy),
    bilinear with zero padding per tap.
    """
    b, a, bb, y, x = (np.asarray(t, dtype=np.int64) for t in idx)
    _, c, h, w = f1.shape
    hl, wl = f2.shape[-2:]
    nh, nw = norm_hw if norm_hw is not None else (h, w)
    s = 2.0 ** level
    sx = (wl - 1) / (nw - 1)
    sy = (hl - 1) / (nh - 1)
    px = (coords[b, 0, y, x] / s + (a - radius)) * sx
    py = (coords[b, 1, y, x] / s + (bb - radius)) * sy
    x0, y0 = np.floor(px), np.floor(py)
    fx, fy = (px - x0)[:, None], (py - y0)[:, None]
    x0, y0 = x0.astype(np.int64), y0.astype(np.int64)

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < wl) & (yy >= 0) & (yy < hl)
        return f2[b, :, np.clip(yy, 0, hl - 1), np.clip(xx, 0, wl - 1)] * ok[:, None]

    samp = ((1 - fx) * (1 - fy) * tap(y0, x0) + fx * (1 - fy) * tap(y0, x0 + 1) +
            (1 - fx) * fy * tap(y0 + 1, x0) + fx * fy * tap(y0 + 1, x0 + 1))
    return np.concatenate([f1[b, :, y, x], samp], axis=1)


def dicl_stack_int_backward(f1, f2, ru, rv, grad_mvol):
    """Gradients of dicl_stack_int w.r.t. f1, f2 (mask is detached, dicl.py:236)."""
    b, c, h, w = f1.shape
    du, dv = 2 * ru + 1, 2 * rv + 1
    mvol = dicl_stack_int(f1, f2, ru, rv)
    valid = (mvol[:, :, :, c:].sum(axis=3) != 0)                            # (B,du,dv,h,w)
    g1 = np.zeros_like(f1)
    g2 = np.zeros_like(f2)
    for i in range(du):
        for j in range(dv):
            di, dj = i - ru, j - rv
            w0, w1 = max(0, -di), min(w, w - di)
            h0, h1 = max(0, -dj), min(h, h - dj)
            if w1 <= w0 or h1 <= h0:
                continue
            m = valid[:, i, j, None, h0:h1, w0:w1]
            g1[:, :, h0:h1, w0:w1] += grad_mvol[:, i, j, :c, h0:h1, w0:w1] * m
            g2[:, :, h0 + dj:h1 + dj, w0 + di:w1 + di] += grad_mvol[:, i, j, c:, h0:h1, w0:w1] * m
    return g1, g2


def dap(x, weight):
    """x (B, du, dv, h, w) or (B, D, h, w); weight (D, D[,1,1]) -> same shape as x."""
    wgt = weight.reshape(weight.shape[0], weight.shape[1])
    b = x.shape[0]
    h, w = x.shape[-2:]
    xf = x.reshape(b, -1, h * w)
    return np.matmul(wgt, xf).reshape(x.shape)


def dap_backward(x, weight, grad_out):
    wgt = weight.reshape(weight.shape[0], weight.shape[1])
    b = x.shape[0]
    h, w = x.shape[-2:]
    xf = x.reshape(b, -1, h * w)
    g = grad_out.reshape(b, -1, h * w)
    gx = np.matmul(wgt.T, g).reshape(x.shape)
    gw = np.einsum("bop,bip->oi", g, xf).reshape(weight.shape)
    return gx, gw


def _warp_taps(flow):
    """Bilinear taps of warp_backwards: positions (x + fx, y + fy) in float32 like the reference's grid + flow."""
    b, _, h, w = flow.shape
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    ix = (xs[None].astype(np.float32) + flow[:, 0].astype(np.float32)).astype(np.float64)
    iy = (ys[None].astype(np.float32) + flow[:, 1].astype(np.float32)).astype(np.float64)
    x0, y0 = np.floor(ix), np.floor(iy)
    fx, fy = ix - x0, iy - y0
    taps = []
    for dy, wy in ((0, 1.0 - fy), (1, fy)):
        for dx, wx in ((0, 1.0 - fx), (1, fx)):
            xx, yy = x0.astype(np.int64) + dx, y0.astype(np.int64) + dy
            inb = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
            taps.append((np.where(inb, yy * w + xx, 0), np.where(inb, wx * wy, 0.0)))
    return taps


def warp_backwards(img2, flow, eps=1e-5):
    """common/warp.py:5-33: bilinear sample of img2 at grid + flow (zero padding, align_corners), times
    the validity mask (in-bounds bilinear weight > 1 - eps).  -> (est * mask (B,C,h,w), mask (B,h,w) bool)."""
    b, c, h, w = img2.shape
    flat = img2.reshape(b, c, h * w)
    est = np.zeros((b, c, h * w))
    wsum = np.zeros((b, h * w))
    for idx, wt in _warp_taps(flow):
        idx, wt = idx.reshape(b, -1), wt.reshape(b, -1)
        est += np.take_along_axis(flat, np.broadcast_to(idx[:, None], (b, c, h * w)), axis=2) * wt[:, None]
        wsum += wt
    mask = wsum > np.float32(1.0 - eps)
    return (est * mask[:, None]).reshape(b, c, h, w), mask.reshape(b, h, w)


def warp_backwards_backward(flow, grad_out, eps=1e-5):
    """d img2 of warp_backwards (flow and mask carry no gradient, dicl.py:178 detaches the flow)."""
    b, c, h, w = grad_out.shape
    _, mask = warp_backwards(np.zeros((b, 1, h, w)), flow, eps)
    g = grad_out.reshape(b, c, h * w) * mask.reshape(b, 1, h * w)
    out = np.zeros((b, c, h * w))
    for idx, wt in _warp_taps(flow):
        idx, wt = idx.reshape(b, -1), wt.reshape(b, -1)
        for bi in range(b):
            for ci in range(c):
                np.add.at(out[bi, ci], idx[bi], g[bi, ci] * wt[bi])
    return out.reshape(b, c, h, w)
