"""GPU parity of the on-the-fly lookup (rmd_corr_otf_prepare / rmd_corr_otf_lookup).

raft_fs.CorrBlock(method="otf") (reference src/models/impls/raft_fs.py:13-87) against the golden
vectors the reference produced, against oracle.corr_lookup_fs (float64) on seeded inputs covering
ragged sizes, channel counts that are not a multiple of the operand padding, masked levels, 1-pixel
levels (NaN) and flow spreads that overflow the per-block target box (per-query fallback), and at the
full cfg2 size against the volume path (same kernels' results must agree).  The backward
(rmd_corr_otf_record + rmd_corr_otf_backward) against the reference's autograd gradients
(gen_golden_fs_backward.py), the float64 oracle over several lookups, and the volume path's backward.

Tolerances (max|got-ref| / max|ref|): fp32 mode (split-bf16 MFMA, ~1e-5) and fp32-exact (f32 MFMA) 1e-4,
bf16 mode 1e-2; the forward fp32 modes also per element, |err| <= 1e-4 |ref| + 1e-5 max|ref|
(conftest.assert_fp32_gate).
"""

import numpy as np
import pytest
import torch

import oracle
from conftest import assert_fp32_gate, load_golden, rel_max_err

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
    if precision.startswith("fp32"):
        assert_fp32_gate(out.cpu().numpy(), g["out"])


CASES = [
    # b, c, h, w, levels, radius, spread, mask
    (2, 32, 24, 40, 4, 4, 2.0, ()),
    (1, 40, 17, 23, 3, 3, 3.0, (4,)),          # C not a multiple of 32, ragged map, level 1 masked
    (2, 64, 12, 20, 4, 2, 1.0, ()),            # level 3 is 1x2 -> NaN
    (1, 16, 30, 50, 2, 7, 25.0, ()),           # huge spread: union boxes span many bands
    (1, 256, 46, 62, 4, 4, 4.0, (3, 6)),       # cfg1 feature shape, levels 0 and 3 masked
    (1, 8, 9, 70, 1, 1, 0.5, ()),              # one level, r=1, wide map
    (1, 320, 14, 20, 3, 3, 2.0, ()),           # C > 256: runtime-channel path (Cp 384: 12 bf16 / 24 f32 load steps)
    (1, 48, 20, 36, 2, 8, 3.0, ()),            # r=8: 17 x 17 window, three interpolation items per thread
    (2, 128, 18, 40, 3, 5, 2.0, (5,)),         # r=5, C=128, level 0 masked
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
    if precision.startswith("fp32"):
        assert_fp32_gate(got, ref)


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


@pytest.mark.parametrize("radius", [4, 7])
def test_otf_wide_map_agrees_with_volume_path(radius):
    """bf16 on a wide map (B=4, 128x256: 4,096 16x2 query blocks) takes the 16x4-block kernel
    (csrc/corr_otf.hip kWideBlocks); it must equal the pyramid + lookup within the bf16 tolerance, with
    large and small displacements, and be deterministic."""
    import rmd
    g = torch.Generator(device="cpu").manual_seed(11)
    f1 = torch.randn(4, 256, 128, 256, generator=g).to(DEV)
    f2 = torch.randn(4, 256, 128, 256, generator=g).to(DEV)
    ys, xs = torch.meshgrid(torch.arange(128.0), torch.arange(256.0), indexing="ij")
    co = torch.stack([xs, ys])[None] + 6 * torch.randn(4, 2, 128, 256, generator=g)
    co[1] += 40.0                                      # one image with a large shift (boxes off the map)
    co = co.to(DEV)
    otf = rmd.raft_fs.CorrBlock(f1, f2, 4, radius, precision="bf16", method="otf")
    a = otf(co)
    b = otf(co)
    vol = rmd.raft_fs.CorrBlock(f1, f2, 4, radius, precision="fp32")
    ref = vol(co)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert rel_max_err(a.cpu().numpy(), ref.cpu().numpy()) < TOL["bf16"]


def _grads(cb_factory, f1, f2, coords_list, gouts, mask=()):
    t1 = _t(f1).requires_grad_(True)
    t2 = _t(f2).requires_grad_(True)
    cb = cb_factory(t1, t2)
    loss = 0
    for co, go in zip(coords_list, gouts):
        loss = loss + (cb(_t(co), list(mask)) * _t(go)).sum()
    g1, g2 = torch.autograd.grad(loss, (t1, t2))
    torch.cuda.synchronize()
    return cb, g1.cpu().numpy(), g2.cpu().numpy()


@pytest.mark.parametrize("precision", ["fp32", "fp32-exact", "bf16"])
@pytest.mark.parametrize("name", ["corr_fs_bwd_b2_c32_24x40", "corr_fs_bwd_b1_c48_21x35_l3r3"])
def test_otf_backward_matches_reference_golden(precision, name):
    """raft_fs.CorrBlock(method='otf') gradients against the reference's own autograd gradients
    (tests/golden/gen_golden_fs_backward.py: avg_pool2d chain + grid_sample + matmul backward)."""
    import rmd
    g = load_golden(name)
    levels, r = int(g["levels"]), int(g["radius"])
    mask = tuple(g["mask_costs"].tolist())
    cb, g1, g2 = _grads(lambda a, b: rmd.raft_fs.CorrBlock(a, b, levels, r, precision=precision, method="otf"),
                        g["fmap1"], g["fmap2"], [g["coords"]], [g["grad_out"]], mask)
    assert cb.method == "otf"
    assert rel_max_err(g1, g["grad_fmap1"]) < TOL[precision]
    assert rel_max_err(g2, g["grad_fmap2"]) < TOL[precision]


BWD_CASES = [
    # b, c, h, w, levels, radius, spread, mask, lookups
    (2, 32, 24, 40, 4, 4, 2.0, (), 3),            # several lookups accumulate into one backward
    (1, 40, 17, 23, 3, 3, 3.0, (4,), 2),          # C not a multiple of 32, ragged map, level 1 masked
    (1, 256, 46, 62, 4, 4, 4.0, (), 2),           # cfg1 feature shape
    (1, 16, 30, 50, 2, 7, 25.0, (), 2),           # huge spread: wide union boxes (several bands per row)
    (2, 8, 9, 70, 1, 1, 0.5, (), 35),             # 35 lookups: records split over two launches (32 max)
    (1, 32, 40, 96, 3, 4, "split", (), 3),        # divergent flow: two patch clusters far apart per query tile
]


def _case_coords(rng, b, h, w, spread):
    if spread != "split":
        return _grid_coords(rng, b, h, w, spread)
    # left/right halves of every query row pulled 30 columns apart (occlusion-edge-like divergence)
    co = _grid_coords(rng, b, h, w, 0.5)
    co[:, 0, :, ::2] += 30.0
    co[:, 0, :, 1::2] -= 30.0
    return co


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("case", BWD_CASES, ids=[f"b{c[0]}c{c[1]}_{c[2]}x{c[3]}_l{c[4]}r{c[5]}_n{c[8]}"
                                                for c in BWD_CASES])
def test_otf_backward_matches_oracle(case, precision):
    """Gradients of several on-the-fly lookups of one block (each with its own coords and upstream
    gradient) against the float64 oracle summed over the lookups."""
    import rmd
    b, c, h, w, levels, r, spread, mask, n = case
    rng = np.random.default_rng(c * 100 + w)
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    cos = [_case_coords(rng, b, h, w, spread) for _ in range(n)]
    d = (2 * r + 1) ** 2
    gos = [rng.standard_normal((b, levels * d, h, w)).astype(np.float32) for _ in range(n)]
    _, g1, g2 = _grads(lambda a, bb: rmd.raft_fs.CorrBlock(a, bb, levels, r, precision=precision, method="otf"),
                       f1, f2, cos, gos, mask)
    r1 = np.zeros(f1.shape)
    r2 = np.zeros(f2.shape)
    for co, go in zip(cos, gos):
        a1, a2 = oracle.corr_lookup_fs_backward(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64),
                                                levels, r, go.astype(np.float64), mask)
        r1 += a1
        r2 += a2
    assert rel_max_err(g1, r1) < TOL[precision]
    assert rel_max_err(g2, r2) < TOL[precision]


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_otf_backward_is_deterministic(precision):
    """Run-to-run identical gradients (G built in fixed record order, d P summed in fp64): 12 lookups at
    a cfg1-like map with a spread flow, so many query tiles add into the same pooled targets."""
    import rmd
    rng = np.random.default_rng(99)
    b, c, h, w = 2, 64, 46, 62
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    cos = [_grid_coords(rng, b, h, w, 3.0) for _ in range(12)]
    gos = [rng.standard_normal((b, 324, h, w)).astype(np.float32) for _ in range(12)]
    runs = [_grads(lambda a, bb: rmd.raft_fs.CorrBlock(a, bb, 4, 4, precision=precision, method="otf"),
                   f1, f2, cos, gos)[1:] for _ in range(3)]
    for g1, g2 in runs[1:]:
        assert np.array_equal(g1, runs[0][0]) and np.array_equal(g2, runs[0][1])


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_otf_backward_deterministic_across_wide_dynamic_range(precision):
    """d P contributions whose magnitudes span far more than 2^29 (upstream gradients
    scaled per query by 2^-40 .. 2^+8, so a pooled target sums terms ~2^48 apart) stay run-to-run bitwise
    equal (64-bit fixed-point accumulation is associative) and match the float64 oracle."""
    import rmd
    rng = np.random.default_rng(5)
    b, c, h, w, levels, r = 1, 32, 24, 40, 3, 3
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    cos = [_grid_coords(rng, b, h, w, 1.5) for _ in range(4)]
    d = (2 * r + 1) ** 2
    mag = np.exp2(rng.integers(-40, 9, size=(b, 1, h, w))).astype(np.float32)
    gos = [(rng.standard_normal((b, levels * d, h, w)) * mag).astype(np.float32) for _ in range(4)]
    runs = [_grads(lambda a, bb: rmd.raft_fs.CorrBlock(a, bb, levels, r, precision=precision, method="otf"),
                   f1, f2, cos, gos)[1:] for _ in range(3)]
    for g1, g2 in runs[1:]:
        assert np.array_equal(g1, runs[0][0]) and np.array_equal(g2, runs[0][1])
    r1 = np.zeros(f1.shape)
    r2 = np.zeros(f2.shape)
    for co, go in zip(cos, gos):
        a1, a2 = oracle.corr_lookup_fs_backward(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64),
                                                levels, r, go.astype(np.float64), ())
        r1 += a1
        r2 += a2
    assert rel_max_err(runs[0][0], r1) < TOL[precision]
    assert rel_max_err(runs[0][1], r2) < TOL[precision]


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_otf_backward_bound_beyond_float_range(precision):
    """the fixed-point exponent's bound records x N x max|w| x max|q~| exceeds FLT_MAX
    (upstream gradients ~1e31, features ~1e3 at a 48 x 80 map: ~1e39) while every gradient stays finite.
    The bound is formed in double, so s is chosen for it (a float bound overflowed to inf and took s = 60,
    overflowing every int64 sum); gradients finite, run-to-run equal, and at the float64 oracle."""
    import rmd
    rng = np.random.default_rng(31)
    b, c, h, w, levels, r = 1, 32, 48, 80, 2, 3
    f1 = (rng.standard_normal((b, c, h, w)) * 1e3).astype(np.float32)
    f2 = (rng.standard_normal((b, c, h, w)) * 1e3).astype(np.float32)
    cos = [_grid_coords(rng, b, h, w, 1.5) for _ in range(2)]
    d = (2 * r + 1) ** 2
    gos = [(rng.standard_normal((b, levels * d, h, w)) * 1e31).astype(np.float32) for _ in range(2)]
    qmax = float(np.abs(f1).max())                       # raft_fs: q~ = fmap1 (scale 1)
    assert 2 * h * w * float(np.abs(gos[0]).max()) * qmax > np.finfo(np.float32).max
    runs = [_grads(lambda a, bb: rmd.raft_fs.CorrBlock(a, bb, levels, r, precision=precision, method="otf"),
                   f1, f2, cos, gos)[1:] for _ in range(2)]
    assert np.isfinite(runs[0][0]).all() and np.isfinite(runs[0][1]).all()
    assert np.array_equal(runs[0][0], runs[1][0]) and np.array_equal(runs[0][1], runs[1][1])
    r1 = np.zeros(f1.shape)
    r2 = np.zeros(f2.shape)
    for co, go in zip(cos, gos):
        a1, a2 = oracle.corr_lookup_fs_backward(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64),
                                                levels, r, go.astype(np.float64), ())
        r1 += a1
        r2 += a2
    assert rel_max_err(runs[0][0], r1) < TOL[precision]
    assert rel_max_err(runs[0][1], r2) < TOL[precision]


def test_otf_backward_propagates_non_finite_gradients():
    """A NaN in the upstream gradient reaches the pooled-target gradient (through the float side buffer
    of the fixed-point accumulation) as it does through the reference's autograd; finite inputs stay
    finite."""
    import rmd
    rng = np.random.default_rng(8)
    b, c, h, w = 1, 16, 12, 20
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    co = _grid_coords(rng, b, h, w, 0.5)
    go = rng.standard_normal((b, 2 * 25, h, w)).astype(np.float32)
    _, g1, g2 = _grads(lambda a, bb: rmd.raft_fs.CorrBlock(a, bb, 2, 2, precision="fp32", method="otf"), f1, f2, [co],
                       [go])
    assert np.isfinite(g1).all() and np.isfinite(g2).all()
    go[0, 12, 5, 7] = np.nan
    _, g1, g2 = _grads(lambda a, bb: rmd.raft_fs.CorrBlock(a, bb, 2, 2, precision="fp32", method="otf"), f1, f2, [co],
                       [go])
    assert np.isnan(g2).any() and np.isnan(g1).any()


def test_otf_backward_equals_volume_backward_raft_scale():
    """rmd.raft.CorrBlock (scale 1/sqrt(C)) trained through the on-the-fly path gives the volume path's
    gradients (fp32 mode, 12 lookups with a flow that moves every iteration, B=2 at the cfg2 map size)."""
    import rmd
    gen = torch.Generator(device="cpu").manual_seed(11)
    b, c, h, w = 2, 256, 55, 128
    f1 = torch.randn(b, c, h, w, generator=gen).numpy()
    f2 = torch.randn(b, c, h, w, generator=gen).numpy()
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    base = np.stack([xs, ys])[None].astype(np.float32)
    drift = torch.randn(b, 2, 1, 1, generator=gen).numpy() * 4
    cos = [(base + (k + 1) / 12 * drift + 0.5 * torch.randn(b, 2, h, w, generator=gen).numpy()).astype(np.float32)
           for k in range(12)]
    gos = [torch.randn(b, 324, h, w, generator=gen).numpy() for _ in range(12)]
    cb_o, o1, o2 = _grads(lambda a, bb: rmd.raft.CorrBlock(a, bb, 4, 4, precision="fp32", method="otf"), f1, f2, cos, gos)
    cb_v, v1, v2 = _grads(lambda a, bb: rmd.raft.CorrBlock(a, bb, 4, 4, precision="fp32", method="volume"), f1, f2, cos,
                          gos)
    assert cb_o.method == "otf" and cb_v.method == "volume"
    assert rel_max_err(o1, v1) < 1e-4
    assert rel_max_err(o2, v2) < 1e-4


def test_auto_method_follows_memory_budget():
    """method='auto' (the default) takes the volume while it fits the budget (rmd.config), else otf; the
    two paths give the same lookup."""
    import rmd
    rng = np.random.default_rng(3)
    f1 = _t(rng.standard_normal((1, 32, 24, 40)).astype(np.float32))
    f2 = _t(rng.standard_normal((1, 32, 24, 40)).astype(np.float32))
    co = _t(_grid_coords(rng, 1, 24, 40, 2.0))
    big = rmd.raft_fs.CorrBlock(f1, f2, 4, 4)
    small = rmd.raft_fs.CorrBlock(f1, f2, 4, 4, memory_budget=1 << 16)
    assert big.method == "volume" and small.method == "otf"
    prev = rmd.config.configure({"corr-method": "auto", "corr-memory-budget": "64KiB"})
    try:
        assert rmd.raft_fs.CorrBlock(f1, f2, 4, 4).method == "otf"
    finally:
        rmd.config.restore(prev)
    assert rel_max_err(small(co).cpu().numpy(), big(co).cpu().numpy()) < 1e-4


def test_otf_workspace_mismatch_raises():
    """The operator checks the workspace against its sizes / compute mode (a bf16 workspace read as
    fp32 would index past it)."""
    from rmd import ops
    f = torch.randn(1, 32, 12, 16, device=DEV)
    st = ops.otf_prepare(f, f, 2, "bf16")
    co = torch.zeros(1, 2, 12, 16, device=DEV)
    with pytest.raises(ValueError, match="workspace"):
        torch.ops.rmd.corr_otf_lookup(st.ws, co, 32, 2, ops.PRECISIONS["fp32"][0], 3, 0)
    with pytest.raises(ValueError, match="workspace"):
        torch.ops.rmd.corr_otf_lookup(st.ws, co, 64, 2, st.compute, 3, 0)
