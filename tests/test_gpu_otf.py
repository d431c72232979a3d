"""GPU parity of the on-the-fly lookup (rmd_corr_otf_prepare / rmd_corr_otf_lookup).

raft_fs.CorrBlock(method="otf") (reference src/models/impls/raft_fs.py:13-87) against the golden
vectors the reference produced, against oracle.corr_lookup_fs (float64) on seeded inputs covering
ragged sizes, channel counts that are not a multiple of the operand padding, masked levels, 1-pixel
levels (NaN) and flow spreads that overflow the per-block target box (per-query fallback), and at the
full cfg2 size against the volume path (same kernels' results must agree).

Tolerances (max|got-ref| / max|ref|): fp32 mode (split-bf16 MFMA, ~1e-5) and fp32-exact (f32 MFMA) 1e-4,
bf16 mode 1e-2.
"""

import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden, rel_max_err

pytestmark = pytest.mark.gpu

TOL = {"fp32": 1e-4, "fp32-exact": 1e-4, "bf16": 1e-2}
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _grid_coords(rng, b, h, w, spread):
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    base = np.stack([xs, ys])[None].astype(np.float64)
    return (base + spread * rng.standard_normal((b, 2, h, w))).astype(np.float32)


@pytest.mark.parametrize("precision", ["fp32", "fp32-exact", "bf16"])
@pytest.mark.parametrize("name", ["corr_fs_b2_c32_24x40", "corr_fs_b2_c16_16x24_nonfinite"])
def test_otf_matches_reference_golden(precision, name):
    import rmd
    g = load_golden(name)
    cb = rmd.raft_fs.CorrBlock(_t(g["fmap1"]), _t(g["fmap2"]), int(g["levels"]), int(g["radius"]),
                               precision=precision, method="otf")
    out = cb(_t(g["coords"]))
    torch.cuda.synchronize()
    assert out.dtype == torch.float32 and out.is_contiguous() and tuple(out.shape) == g["out"].shape
    assert rel_max_err(out.cpu().numpy(), g["out"]) < TOL[precision]


CASES = [
    # b, c, h, w, levels, radius, spread, mask
    (2, 32, 24, 40, 4, 4, 2.0, ()),
    (1, 40, 17, 23, 3, 3, 3.0, (4,)),          # C not a multiple of 32, ragged map, level 1 masked
    (2, 64, 12, 20, 4, 2, 1.0, ()),            # level 3 is 1x2 -> NaN
    (1, 16, 30, 50, 2, 7, 25.0, ()),           # huge spread: union boxes span many bands
    (1, 256, 46, 62, 4, 4, 4.0, (3, 6)),       # cfg1 feature shape, levels 0 and 3 masked
    (1, 8, 9, 70, 1, 1, 0.5, ()),              # one level, r=1, wide map
    (1, 320, 14, 20, 3, 3, 2.0, ()),           # C > 256: runtime-channel path (Cp 384: 12 bf16 / 24 f32 load steps)
]


@pytest.mark.parametrize("precision", ["fp32", "fp32-exact", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=[f"b{c[0]}c{c[1]}_{c[2]}x{c[3]}_l{c[4]}r{c[5]}" for c in CASES])
def test_otf_matches_oracle(case, precision):
    import rmd
    b, c, h, w, levels, r, spread, mask = case
    rng = np.random.default_rng(c * 1000 + h)
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    co = _grid_coords(rng, b, h, w, spread)
    ref = oracle.corr_lookup_fs(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64), levels, r, mask)
    cb = rmd.raft_fs.CorrBlock(_t(f1), _t(f2), levels, r, precision=precision, method="otf")
    got = cb(_t(co), list(mask)).cpu().numpy()
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    assert rel_max_err(got[fin], ref[fin]) < TOL[precision]


@pytest.mark.parametrize("precision", ["fp32", "fp32-exact", "bf16"])
def test_otf_wide_box_per_query_path(precision):
    """Flow scattered over a 600-pixel-wide map: union boxes wider than kMaxT take the per-query path."""
    import rmd
    rng = np.random.default_rng(9)
    b, c, h, w = 1, 24, 4, 600
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    co = np.stack([rng.uniform(-5, w + 5, (b, h, w)), rng.uniform(-2, h + 2, (b, h, w))], 1).astype(np.float32)
    ref = oracle.corr_lookup_fs(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64), 2, 3)
    got = rmd.raft_fs.CorrBlock(_t(f1), _t(f2), 2, 3, precision=precision, method="otf")(_t(co)).cpu().numpy()
    assert rel_max_err(got, ref) < TOL[precision]


def test_otf_dot_scale_one_level():
    """corr/dot.py:25-57 semantics: one level, products scaled by 1/sqrt(C) in the query operand."""
    from rmd import ops
    rng = np.random.default_rng(5)
    f1 = rng.standard_normal((2, 32, 12, 16)).astype(np.float32)
    f2 = rng.standard_normal((2, 32, 12, 16)).astype(np.float32)
    co = _grid_coords(rng, 2, 12, 16, 1.5)
    st = ops.otf_prepare(_t(f1), _t(f2), 1, "fp32", scale=32 ** -0.5)
    got = ops.otf_lookup(st, _t(co), 3).cpu().numpy()
    ref = oracle.corr_lookup_fs(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64), 1, 3,
                                scale=32 ** -0.5)
    assert rel_max_err(got, ref) < 1e-4


@pytest.mark.parametrize("precision", ["fp32", "fp32-exact", "bf16"])
def test_otf_full_size_agrees_with_volume_path(precision):
    """cfg2 size (B=8, C=256, 55x128, 4 levels, r=4): on-the-fly == pyramid + lookup, and deterministic."""
    import rmd
    g = torch.Generator(device="cpu").manual_seed(3)
    f1 = torch.randn(8, 256, 55, 128, generator=g).to(DEV)
    f2 = torch.randn(8, 256, 55, 128, generator=g).to(DEV)
    ys, xs = torch.meshgrid(torch.arange(55.0), torch.arange(128.0), indexing="ij")
    co = (torch.stack([xs, ys])[None] + 6 * torch.randn(8, 2, 55, 128, generator=g)).to(DEV)
    otf = rmd.raft_fs.CorrBlock(f1, f2, 4, 4, precision=precision, method="otf")
    vol = rmd.raft_fs.CorrBlock(f1, f2, 4, 4, precision="fp32")
    a = otf(co)
    b = otf(co)
    ref = vol(co)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert rel_max_err(a.cpu().numpy(), ref.cpu().numpy()) < TOL[precision]


def test_otf_is_inference_only():
    import rmd
    f1 = torch.randn(1, 8, 8, 8, device=DEV, requires_grad=True)
    with pytest.raises(RuntimeError, match="inference-only"):
        rmd.raft_fs.CorrBlock(f1, f1.detach(), 2, 2, method="otf")
    with torch.no_grad():
        rmd.raft_fs.CorrBlock(f1, f1.detach(), 2, 2, method="otf")
