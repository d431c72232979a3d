"""Deterministic synthetic frame pair for the end-to-end test — test infrastructure only.

Shared by tests/golden/gen_e2e.py (reference run, build container) and tests/test_gpu_e2e.py (GPU
box) so the images are regenerated bit-identically instead of being committed.  A smooth random
texture (sum of seeded sinusoids, numpy float64 -> float32) in [-1, 1] (the post-InputSpec range,
input.py:220-221); img2 is img1 moved by an integer flow (u, v), so the ground-truth flow is
constant; both are zero-padded at the bottom/right to a multiple of 8 (ModuloPadding, input.py:79-138,
cfg/model/raft-baseline.yaml:21-28).
"""

import numpy as np


def frame_pair(h, w, flow=(3, 5), seed=1234, pad=8):
    rng = np.random.Generator(np.random.PCG64(seed))
    u, v = flow
    hh, ww = h + abs(v), w + abs(u)
    ys, xs = np.meshgrid(np.arange(hh, dtype=np.float64), np.arange(ww, dtype=np.float64), indexing="ij")
    tex = np.zeros((3, hh, ww))
    for c in range(3):
        for _ in range(12):
            fx, fy = rng.uniform(0.01, 0.15, 2)
            ph = rng.uniform(0, 2 * np.pi)
            tex[c] += rng.uniform(0.3, 1.0) * np.sin(fx * xs + fy * ys + ph)
    tex /= np.abs(tex).max()
    # img1(y, x) = tex(y + v, x + u) and img2(y, x) = tex(y, x): a point of img1 at (x, y) appears
    # in img2 at (x + u, y + v) -> ground-truth flow (u, v)
    img1 = tex[:, v:v + h, u:u + w]
    img2 = tex[:, :h, :w]
    hp, wp = (h + pad - 1) // pad * pad, (w + pad - 1) // pad * pad
    out = []
    for im in (img1, img2):
        p = np.zeros((3, hp, wp), dtype=np.float32)
        p[:, :h, :w] = im
        out.append(p[None])
    gt = np.zeros((1, 2, h, w), dtype=np.float32)
    gt[0, 0], gt[0, 1] = u, v
    return out[0], out[1], gt


def epe(flow, gt):
    """Mean end-point error over the unpadded region (src/metrics/epe.py:36)."""
    h, w = gt.shape[-2:]
    f = np.asarray(flow, dtype=np.float64)[..., :h, :w]
    return float(np.sqrt(((f - gt) ** 2).sum(1)).mean())
