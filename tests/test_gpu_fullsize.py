"""Full-size GPU parity: the BASELINE configurations' own shapes, batch 8, against the float64 oracle.

The volumes here are 0.1-1.3 GB each, so the oracle is evaluated at sampled positions only
(oracle.dicl_stack_int_at / dicl_stack_at: the same restatement, per displacement vector) — every
sampled vector is compared whole — plus size-independent properties checked over the whole
volume on the GPU (zero pattern = occlusion mask, the f1 half constant over displacements).

Tolerances are ELEMENTWISE (conftest.assert_close_elementwise: |got - ref| <= atol + rtol*|ref|):
  * integer DICL volume (cfg3, copy + mask): bit-exact
  * bilinear DICL stack (cfg4 levels): rtol 1e-5, atol 1e-6 — fp32 pixel-coordinate bilinear vs the
    float64 restatement
  * DAP (cfg3 D=49, cfg4 D=81): rtol 5e-5, atol 5e-5 * max|ref| — split-bf16 MFMA (hi.hi + hi.lo +
    lo.hi, fp32 accumulate): ~1.5e-5 * max|ref| absolute
SURVEY.md §8(d): cfg3 = DICL 384x512 b8, levels 2..6 (96x128 .. 6x8), C=32, D=49; cfg4 = KITTI
376x1242 padded to 384x1280, ctf-l3 levels 1/8, 1/16, 1/32 (48x160, 24x80, 12x40), C=32, D=81.
"""

import numpy as np
import pytest
import torch

import oracle
from conftest import assert_close_elementwise

pytestmark = pytest.mark.gpu
DEV = "cuda"
NS = 60000                       # sampled displacement vectors per volume


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _feat(rng, b, c, h, w, holes=True):
    f = rng.standard_normal((b, c, h, w)).astype(np.float32)
    if holes:                                   # zero feature vectors -> occlusion-masked displacements
        f[0, :, h // 4: h // 4 + max(1, h // 8), w // 3: w // 3 + max(1, w // 6)] = 0.0
        f[b - 1, :, h - 1, :] = 0.0
        f[1, : c // 2, 0, 0] = 0.0              # partially zero vector stays valid
    return f


def _sample(rng, shape, n):
    return tuple(rng.integers(0, s, n) for s in shape)


@pytest.mark.parametrize("h,w", [(96, 128), (48, 64), (24, 32), (12, 16), (6, 8)])
def test_cfg3_dicl_volume_b8_bit_exact(h, w):
    import rmd
    rng = np.random.default_rng(h * 1000 + w)
    b, c, ru, rv = 8, 32, 3, 3
    f1 = _feat(rng, b, c, h, w, holes=False)
    f2 = _feat(rng, b, c, h, w)
    mvol = rmd.ops.dicl_stack_int(_t(f1), _t(f2), ru, rv)          # (B, 7, 7, 2C, h, w)
    assert tuple(mvol.shape) == (b, 2 * ru + 1, 2 * rv + 1, 2 * c, h, w)
    n = min(NS, b * 49 * h * w)
    idx = _sample(rng, (b, 2 * ru + 1, 2 * rv + 1, h, w), n)
    ti = [torch.from_numpy(a).to(DEV) for a in idx]
    got = mvol[ti[0], ti[1], ti[2], :, ti[3], ti[4]].cpu().numpy()   # (n, 2C)
    ref = oracle.dicl_stack_int_at(f1, f2, ru, rv, idx)
    assert np.array_equal(got, ref)
    # whole-volume properties: a displacement vector is either all zero (outside / occluded) or its
    # f1 half is f1 itself; the number of zero vectors equals the oracle's mask count
    zero = (mvol == 0).all(dim=3)
    f1t = _t(f1)[:, None, None].expand(-1, 2 * ru + 1, 2 * rv + 1, -1, -1, -1)
    assert bool(((mvol[:, :, :, :c] == f1t).all(dim=3) | zero).all())
    m_ref = oracle.dicl_stack_int(f1[:1], f2[:1], ru, rv)             # image 0 in full
    assert np.array_equal(mvol[:1].cpu().numpy(), m_ref)


@pytest.mark.parametrize("level,h,w", [(0, 48, 160), (0, 24, 80), (0, 12, 40)])
def test_cfg4_dicl_stack_b8(level, h, w):
    import rmd
    rng = np.random.default_rng(7 * h + w)
    b, c, r = 8, 32, 4
    f1 = _feat(rng, b, c, h, w, holes=False)
    f2 = _feat(rng, b, c, h, w)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 3.0, (b, 2, h, w))).astype(np.float32)
    co[0, :, 0, 0] = (-40.0, -40.0)                                    # far outside
    co[1, :, 1, 1] = (w - 1.0, h - 1.0)                                # exact far corner
    st = rmd.ops.dicl_stack(_t(f1), _t(f2), _t(co), r)                 # (B, 9, 9, 2C, h, w)
    d = 2 * r + 1
    assert tuple(st.shape) == (b, d, d, 2 * c, h, w)
    n = min(NS, b * d * d * h * w)
    idx = _sample(rng, (b, d, d, h, w), n)
    ti = [torch.from_numpy(a).to(DEV) for a in idx]
    got = st[ti[0], ti[1], ti[2], :, ti[3], ti[4]].cpu().numpy()
    ref = oracle.dicl_stack_at(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64), r, idx)
    assert_close_elementwise(got, ref, rtol=1e-5, atol=1e-6)
    f1t = _t(f1)[:, None, None].expand(-1, d, d, -1, -1, -1)
    assert bool((st[:, :, :, :c] == f1t).all())                       # no mask on the bilinear stack


@pytest.mark.parametrize("d,h,w", [(49, 96, 128), (81, 48, 160), (324, 48, 160)])
def test_dap_b8_full_size(d, h, w):
    import rmd
    rng = np.random.default_rng(d)
    b = 8
    x = rng.standard_normal((b, d, h, w)).astype(np.float32)
    wt = (np.eye(d) + 0.05 * rng.standard_normal((d, d))).astype(np.float32)[:, :, None, None]
    y = rmd.ops.dap(_t(x), _t(wt))
    assert tuple(y.shape) == (b, d, h, w)
    n = 20000
    bi, yi, xi = _sample(rng, (b, h, w), n)
    got = y[torch.from_numpy(bi).to(DEV), :, torch.from_numpy(yi).to(DEV), torch.from_numpy(xi).to(DEV)]
    ref = x.astype(np.float64)[bi, :, yi, xi] @ wt[:, :, 0, 0].astype(np.float64).T    # (n, D)
    assert_close_elementwise(got.cpu().numpy(), ref, rtol=5e-5, atol=5e-5 * np.abs(ref).max())


def test_cfg2_whole_volume_across_gemm_kernels():
    """cfg2 (B=8, 55x128, C=256) whole volume, every level and a whole lookup output, across three
    independent GEMM kernels (each pinned to the oracle on samples in test_gpu_corr.py):
      * fp32 parity mode (corr_pyramid_x3s, split-bf16 MFMA, S24 row layout) and fp32-f32 (the same GEMM,
        F32 row layout) vs fp32-exact (corr_pyramid_tiled, exact f32 MFMA): max|d| / max|ref| <= 1e-4
        (north_star fp32 gate);
      * bf16 perf mode (corr_pyramid_w8, tiles layout, fp16 storage) vs fp32-exact: <= 1e-2.
    1.3e10 pyramid values per mode are compared on the GPU (no oracle can run at this size)."""
    import rmd
    g = torch.Generator(device="cpu").manual_seed(2024)
    b, c, h, w = 8, 256, 55, 128
    f1 = torch.randn(b, c, h, w, generator=g).to(DEV)
    f2 = torch.randn(b, c, h, w, generator=g).to(DEV)
    ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32), indexing="ij")
    flow = torch.nn.functional.interpolate(torch.randn(b, 2, 4, 8, generator=g) * 3.0, size=(h, w), mode="bilinear",
                                           align_corners=True)
    co = (torch.stack([xs, ys])[None] + flow + torch.randn(b, 2, 1, 1, generator=g) * 4.0).to(DEV)
    ref = rmd.ops.corr_pyramid(f1, f2, 4, "fp32-exact")
    out_ref = rmd.ops.corr_lookup(ref, co, 4)
    for precision, tol, layout in (("fp32", 1e-4, 0), ("fp32-f32", 1e-4, 0), ("bf16", 1e-2, 1)):
        pyr = rmd.ops.corr_pyramid(f1, f2, 4, precision)
        assert pyr.desc.layout == layout
        for i in range(4):
            a, r = pyr.unpack(i), ref.unpack(i)
            err = float((a - r).abs().max() / r.abs().max())
            assert err < tol, f"{precision} level {i}: {err:.3e}"
            del a, r
        out = rmd.ops.corr_lookup(pyr, co, 4)
        err = float((out - out_ref).abs().max() / out_ref.abs().max())
        assert err < tol, f"{precision} lookup: {err:.3e}"
        del pyr, out
        torch.cuda.empty_cache()
