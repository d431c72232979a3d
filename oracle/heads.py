"""Per-iteration flow heads around the cost volume — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* Up8 convex upsampling, ``Up8Network.forward`` after its convolutions
  (reference src/models/impls/raft.py:313-331).
* Soft-argmax flow regression (raft.py:98-135; corr/dicl.py:64-85, corr/dot.py:69-90 and the identical
  classes of corr/dicl_1x1.py, corr/dicl_emb.py).

Forward and backward, float64 numpy.  The backward formulas are the chain rule of the reference's
softmax / unfold / weighted sum; tests pin them against the reference's autograd (golden vectors).
"""

import numpy as np


def _softmax(x, axis):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def _unfold3(f):
    """(B, C, h, w) -> (B, C, 9, h, w): F.unfold(f, (3, 3), padding=1), neighbour k = 3*ky + kx."""
    b, c, h, w = f.shape
    p = np.zeros((b, c, h + 2, w + 2), dtype=f.dtype)
    p[:, :, 1:-1, 1:-1] = f
    return np.stack([p[:, :, ky:ky + h, kx:kx + w] for ky in range(3) for kx in range(3)], axis=2)


def up8(mask, flow, temperature=4.0):
    """mask (B, 576, h, w) logits, flow (B, 2, h, w) -> (B, 2, 8h, 8w) — raft.py:319-331."""
    b, c, h, w = flow.shape
    p = _softmax(mask.reshape(b, 1, 9, 8, 8, h, w) / temperature, axis=2)   # (b,1,9,8i,8j,h,w)
    u = _unfold3(8 * flow).reshape(b, c, 9, 1, 1, h, w)
    up = (p * u).sum(axis=2)                                                # (b, c, 8, 8, h, w)
    return up.transpose(0, 1, 4, 2, 5, 3).reshape(b, c, 8 * h, 8 * w)


def up8_backward(mask, flow, grad_out, temperature=4.0):
    """-> (d mask (B, 576, h, w), d flow (B, 2, h, w))."""
    b, c, h, w = flow.shape
    p = _softmax(mask.reshape(b, 1, 9, 8, 8, h, w) / temperature, axis=2)   # (b,1,9,8,8,h,w)
    u = _unfold3(8 * flow).reshape(b, c, 9, 1, 1, h, w)
    g = grad_out.reshape(b, c, h, 8, w, 8).transpose(0, 1, 3, 5, 2, 4)      # (b, c, 8i, 8j, h, w)
    g = g[:, :, None]                                                       # (b, c, 1, 8, 8, h, w)
    gk = (g * u).sum(axis=1, keepdims=True)                                 # d up / d p_k summed over c
    dl = p * (gk - (p * gk).sum(axis=2, keepdims=True)) / temperature
    dmask = dl.reshape(b, 576, h, w)
    q = (p * g).sum(axis=(3, 4))                                            # (b, c, 9, h, w)
    dflow = np.zeros_like(flow)
    for ky in range(3):
        for kx in range(3):
            qk = 8 * q[:, :, 3 * ky + kx]                                   # contributes to (y+ky-1, x+kx-1)
            ys0, ys1 = max(0, 1 - ky), min(h, h + 1 - ky)
            xs0, xs1 = max(0, 1 - kx), min(w, w + 1 - kx)
            dflow[:, :, ys0 + ky - 1:ys1 + ky - 1, xs0 + kx - 1:xs1 + kx - 1] += qk[:, :, ys0:ys1, xs0:xs1]
    return dmask, dflow


def _deltas(radius):
    d = 2 * radius + 1
    a, bb = np.meshgrid(np.arange(d) - radius, np.arange(d) - radius, indexing="ij")
    return a.reshape(-1).astype(np.float64), bb.reshape(-1).astype(np.float64)   # k = a*d + b -> (dx, dy)


def softargmax(cost, levels, radius, temperature=1.0, first_level=0):
    """cost (B, L*(2r+1)^2, h, w) -> list of L flows (B, 2, h, w); level l scaled by 2^(first_level+l)."""
    b, _, h, w = cost.shape
    dd = (2 * radius + 1) ** 2
    dx, dy = _deltas(radius)
    out = []
    for lvl in range(levels):
        p = _softmax(cost[:, lvl * dd:(lvl + 1) * dd] / temperature, axis=1)
        s = 2.0 ** (first_level + lvl)
        out.append(np.stack([(p * (s * dx)[None, :, None, None]).sum(1),
                             (p * (s * dy)[None, :, None, None]).sum(1)], axis=1))
    return out


def softargmax_backward(cost, levels, radius, grad_flows, temperature=1.0, first_level=0):
    """grad_flows: list of L (B, 2, h, w) -> d cost (B, L*(2r+1)^2, h, w)."""
    dd = (2 * radius + 1) ** 2
    dx, dy = _deltas(radius)
    g = np.zeros_like(cost)
    for lvl in range(levels):
        p = _softmax(cost[:, lvl * dd:(lvl + 1) * dd] / temperature, axis=1)
        s = 2.0 ** (first_level + lvl)
        gv = s * (dx[None, :, None, None] * grad_flows[lvl][:, 0:1] + dy[None, :, None, None] * grad_flows[lvl][:, 1:2])
        g[:, lvl * dd:(lvl + 1) * dd] = p * (gv - (p * gv).sum(1, keepdims=True)) / temperature
    return g
