"""Oracle: RAFT all-pairs correlation, pooled pyramid and windowed bilinear lookup (numpy).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Arithmetic is carried out in the dtype of the
inputs (float64 for checking, float32 for the timed CPU baseline).

Reference semantics restated here (qzed/raft-meets-dicl v2):
  * corr0[b,p,q] = sum_c f1[b,c,p] f2[b,c,q] / sqrt(C)           src/models/impls/raft.py:26-33
  * level l = avg_pool2d(level l-1, 2, 2) over the target dims, floor sizes   raft.py:38-47
  * lookup: level i is sampled at (x/2^i + dx, y/2^i + dy), dx,dy in {-r..r}, bilinear,
    align_corners=True, zero padding per tap                        raft.py:57-80
  * output channel = i*(2r+1)^2 + a*(2r+1) + b with x-offset a-r, y-offset b-r
    (meshgrid(dx, dy, indexing='ij'))                                raft.py:57-59,83,92-95
  * levels listed in mask_costs (as index i+3) are zeroed            raft.py:86-87
  * a level with height or width 1 divides by zero in the [-1,1] normalisation
    (raft.py:73-74) and yields NaN for every query                   (fixture corr_b1_c16_12x20_nan)
  * raft/fs: fmap2 is avg-pooled instead of the volume, no 1/sqrt(C)  src/models/impls/raft_fs.py:13-87

The bilinear lookup is restated in pixel coordinates (no [-1,1] round trip) with one weight set
per query and level: all (2r+1)^2 offsets are integers, so every tap shares frac(x/2^i),
frac(y/2^i).
"""

import numpy as np


def pyramid_level_shapes(h, w, levels):
    """Floor-sized level shapes of the avg-pool pyramid (raft.py:38-47)."""
    shapes = [(h, w)]
    for _ in range(1, levels):
        h, w = h // 2, w // 2
        shapes.append((h, w))
    return shapes


def corr_volume(fmap1, fmap2):
    """(B,C,H,W) x2 -> (B, H*W, H, W): raft.py:26-33.

    fmap1 may hold any subset of query pixels (B,C,h1,w1); targets always follow fmap2's grid.
    """
    b, c, h1, w1 = fmap1.shape
    h, w = fmap2.shape[-2:]
    f1 = fmap1.reshape(b, c, h1 * w1)
    f2 = fmap2.reshape(b, c, h * w)
    corr = np.matmul(f1.transpose(0, 2, 1), f2)
    corr = corr / np.sqrt(np.asarray(c, dtype=fmap1.dtype))
    return corr.reshape(b, h1 * w1, h, w)


def _avg_pool2(x):
    """2x2/2 average pool over the last two dims, floor sizes (F.avg_pool2d, raft.py:42)."""
    h2, w2 = x.shape[-2] // 2, x.shape[-1] // 2
    x = x[..., : 2 * h2, : 2 * w2]
    return 0.25 * (x[..., 0::2, 0::2] + x[..., 0::2, 1::2] + x[..., 1::2, 0::2] + x[..., 1::2, 1::2])


def corr_pyramid(fmap1, fmap2, levels):
    """List of levels, each (B, H*W, H_i, W_i): raft.py:18-47."""
    pyr = [corr_volume(fmap1, fmap2)]
    for _ in range(1, levels):
        pyr.append(_avg_pool2(pyr[-1]))
    return pyr


def _bilinear_window(maps, cx, cy, r):
    """Sample the (2r+1)^2 integer-offset window of each query's own map.

    maps: (B, P, Hl, Wl)   one target map per query
    cx, cy: (B, P)         centre in this level's pixel coordinates
    returns (B, P, 2r+1 [x-offset a], 2r+1 [y-offset b])
    """
    bsz, p, hl, wl = maps.shape
    x0 = np.floor(cx)
    y0 = np.floor(cy)
    fx = (cx - x0)[..., None, None]
    fy = (cy - y0)[..., None, None]
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    k = 2 * r + 2
    offs = np.arange(-r, r + 2)
    xs = x0[..., None] + offs                                  # (B,P,k) patch columns
    ys = y0[..., None] + offs                                  # (B,P,k) patch rows
    vx = (xs >= 0) & (xs < wl)
    vy = (ys >= 0) & (ys < hl)
    xs_c = np.clip(xs, 0, wl - 1)
    ys_c = np.clip(ys, 0, hl - 1)
    bi = np.arange(bsz)[:, None, None, None]
    pi = np.arange(p)[None, :, None, None]
    patch = maps[bi, pi, ys_c[..., :, None], xs_c[..., None, :]]          # (B,P,k rows,k cols)
    patch = patch * (vy[..., :, None] & vx[..., None, :])                 # zero padding per tap
    top = patch[..., :-1, :]                                              # rows y0-r .. y0+r
    bot = patch[..., 1:, :]
    # out[a, b] (a = x index, b = y index)
    v00 = top[..., :, :-1]
    v01 = top[..., :, 1:]
    v10 = bot[..., :, :-1]
    v11 = bot[..., :, 1:]
    one = np.asarray(1, dtype=maps.dtype)
    out_yx = ((one - fx) * (one - fy) * v00 + fx * (one - fy) * v01 +
              (one - fx) * fy * v10 + fx * fy * v11)                      # (B,P,b,a)
    del k
    return np.swapaxes(out_yx, -1, -2)                                    # (B,P,a,b)


def corr_lookup(pyramid, coords, radius, mask_costs=()):
    """Windowed bilinear lookup over the pyramid -> (B, L*(2r+1)^2, H, W): raft.py:49-95.

    pyramid: list of (B, H*W, H_i, W_i);  coords: (B,2,H,W), ch0 = x, ch1 = y (level-0 pixels).
    """
    b, _, h, w = coords.shape
    d = 2 * radius + 1
    cx = coords[:, 0].reshape(b, h * w)
    cy = coords[:, 1].reshape(b, h * w)
    out = []
    for i, lvl in enumerate(pyramid):
        hl, wl = lvl.shape[-2:]
        if i + 3 in mask_costs:
            o = np.zeros((b, h * w, d, d), dtype=lvl.dtype)
        elif hl < 2 or wl < 2:
            o = np.full((b, h * w, d, d), np.nan, dtype=lvl.dtype)
        else:
            s = np.asarray(2.0 ** i, dtype=lvl.dtype)
            o = _bilinear_window(lvl, cx / s, cy / s, radius)
        out.append(o.reshape(b, h * w, d * d))
    out = np.concatenate(out, axis=-1)                                    # (B, P, L*d*d)
    return np.ascontiguousarray(out.transpose(0, 2, 1).reshape(b, -1, h, w))


def _pool_fmap(f):
    return _avg_pool2(f)


def corr_lookup_fs(fmap1, fmap2, coords, levels, radius, mask_costs=(), scale=None):
    """On-the-fly lookup: dot(fmap1, bilinear(pooled fmap2)) — raft_fs.py:13-87.

    ``scale`` multiplies the result: None → 1 (raft_fs has no 1/sqrt(C)); corr/dot.py:55-57 uses
    1/sqrt(C), raft.CorrBlock equals this times 1/sqrt(C).
    """
    b, c, h, w = fmap1.shape
    d = 2 * radius + 1
    f2s = [fmap2]
    for _ in range(1, levels):
        f2s.append(_pool_fmap(f2s[-1]))
    cx = coords[:, 0].reshape(b, h * w)
    cy = coords[:, 1].reshape(b, h * w)
    f1 = fmap1.reshape(b, c, h * w)
    out = []
    for i, f2 in enumerate(f2s):
        hl, wl = f2.shape[-2:]
        if i + 3 in mask_costs:
            o = np.zeros((b, h * w, d * d), dtype=fmap1.dtype)
        elif hl < 2 or wl < 2:
            o = np.full((b, h * w, d * d), np.nan, dtype=fmap1.dtype)
        else:
            s = np.asarray(2.0 ** i, dtype=fmap1.dtype)
            samp = _sample_features(f2, cx / s, cy / s, radius)           # (B,C,P,a,b)
            o = np.einsum("bcp,bcpxy->bpxy", f1, samp).reshape(b, h * w, d * d)
        if scale is not None:
            o = o * np.asarray(scale, dtype=o.dtype)
        out.append(o)
    out = np.concatenate(out, axis=-1)
    return np.ascontiguousarray(out.transpose(0, 2, 1).reshape(b, -1, h, w))


def _sample_features(f, cx, cy, r, sx=1.0, sy=1.0):
    """Bilinear zero-padded samples of feature map f (B,C,Hl,Wl) at ((cx+a-r)*sx, (cy+b-r)*sy).

    returns (B, C, P, 2r+1 [a], 2r+1 [b]).  With sx = sy = 1 all taps share one weight set.
    """
    bsz, c, hl, wl = f.shape
    d = 2 * r + 1
    off = np.arange(-r, r + 1, dtype=f.dtype)
    px = (cx[..., :, None] + off) * np.asarray(sx, dtype=f.dtype)          # (B,P,a)
    py = (cy[..., :, None] + off) * np.asarray(sy, dtype=f.dtype)          # (B,P,b)
    px = np.broadcast_to(px[..., :, None], px.shape + (d,))                # (B,P,a,b)
    py = np.broadcast_to(py[..., None, :], py.shape[:-1] + (d, d))
    x0 = np.floor(px)
    y0 = np.floor(py)
    fx = px - x0
    fy = py - y0
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    bi = np.arange(bsz)[:, None, None, None]
    out = np.zeros((bsz, c) + px.shape[1:], dtype=f.dtype)
    one = np.asarray(1, dtype=f.dtype)
    for dy, wy in ((0, one - fy), (1, fy)):
        for dx, wx in ((0, one - fx), (1, fx)):
            xx = x0 + dx
            yy = y0 + dy
            v = (xx >= 0) & (xx < wl) & (yy >= 0) & (yy < hl)
            vals = f[bi, :, np.clip(yy, 0, hl - 1), np.clip(xx, 0, wl - 1)]   # (B,P,a,b,C)
            out += np.moveaxis(vals * (wx * wy * v)[..., None], -1, 1)
    return out


def corr_lookup_backward(fmap1, fmap2, coords, levels, radius, grad_out, mask_costs=()):
    """d(sum(out*grad_out))/d(fmap1, fmap2) for raft.CorrBlock (dense restatement, small sizes).

    Transposes the lookup (bilinear scatter), the pooling (equal spread over each 2x2 block of
    the floor-cropped region) and the GEMM.  Coordinates carry no gradient (raft.py:402).
    """
    b, c, h, w = fmap1.shape
    d = 2 * radius + 1
    n = h * w
    shapes = pyramid_level_shapes(h, w, levels)
    g = grad_out.reshape(b, levels, d, d, n)                               # (B,L,a,b,P)
    cx = coords[:, 0].reshape(b, n)
    cy = coords[:, 1].reshape(b, n)
    one = np.asarray(1, dtype=fmap1.dtype)
    gcorr0 = np.zeros((b, n, h, w), dtype=fmap1.dtype)
    bi = np.arange(b)[:, None]
    pi = np.arange(n)[None, :]
    for i, (hl, wl) in enumerate(shapes):
        if i + 3 in mask_costs:
            continue
        s = np.asarray(2.0 ** i, dtype=fmap1.dtype)
        gl = np.zeros((b, n, hl, wl), dtype=fmap1.dtype)
        lx, ly = cx / s, cy / s
        x0 = np.floor(lx)
        y0 = np.floor(ly)
        fx, fy = lx - x0, ly - y0
        x0 = x0.astype(np.int64)
        y0 = y0.astype(np.int64)
        for a in range(d):
            for bb in range(d):
                gv = g[:, i, a, bb, :]
                for ddy, wy in ((0, one - fy), (1, fy)):
                    for ddx, wx in ((0, one - fx), (1, fx)):
                        xx = x0 + a - radius + ddx
                        yy = y0 + bb - radius + ddy
                        v = (xx >= 0) & (xx < wl) & (yy >= 0) & (yy < hl)
                        np.add.at(gl, (bi, pi, np.clip(yy, 0, hl - 1), np.clip(xx, 0, wl - 1)),
                                  gv * wx * wy * v)
        # transpose of i successive 2x2 average pools: spread over 2^i x 2^i blocks
        k = 2 ** i
        up = np.repeat(np.repeat(gl, k, axis=-2), k, axis=-1) / np.asarray(k * k, dtype=gl.dtype)
        gcorr0[..., : hl * k, : wl * k] += up
    gcorr0 = gcorr0.reshape(b, n, n) / np.sqrt(np.asarray(c, dtype=fmap1.dtype))
    f1 = fmap1.reshape(b, c, n)
    f2 = fmap2.reshape(b, c, n)
    gf1 = np.matmul(f2, gcorr0.transpose(0, 2, 1)).reshape(b, c, h, w)
    gf2 = np.matmul(f1, gcorr0).reshape(b, c, h, w)
    return gf1, gf2


def corr_lookup_fs_backward(fmap1, fmap2, coords, levels, radius, grad_out, mask_costs=(), scale=None):
    """d(sum(out*grad_out))/d(fmap1, fmap2) for raft_fs.CorrBlock (raft_fs.py:13-87; autograd of its
    avg_pool2d chain, grid_sample and matmul), with corr_lookup_fs's ``scale`` (None -> 1).

    raft_fs's output equals raft.CorrBlock's times sqrt(C) (pooling fmap2
    commutes with the product), so its gradient is corr_lookup_backward's times sqrt(C) * scale.
    """
    c = fmap1.shape[1]
    k = np.sqrt(np.asarray(c, dtype=fmap1.dtype)) * np.asarray(1.0 if scale is None else scale, dtype=fmap1.dtype)
    g1, g2 = corr_lookup_backward(fmap1, fmap2, coords, levels, radius, grad_out, mask_costs)
    return g1 * k, g2 * k

