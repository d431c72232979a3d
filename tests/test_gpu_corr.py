"""GPU parity of the RAFT correlation pyramid + lookup (rmd_corr_pyramid / rmd_corr_lookup).

Checked against (1) golden vectors produced by the reference itself (tests/golden), (2) the
float64 CPU oracle at the same seeded inputs, and (3) at the full cfg2 size (B=8, 55x128, C=256)
against the oracle on a random sample of queries plus determinism.

Tolerances (max|got-ref| / max|ref|, conftest.rel_max_err):
  * fp32 modes (split-bf16 MFMA hi.hi + hi.lo + lo.hi; fp32-exact: exact f32 MFMA): 1e-4 — north_star's
    cost-volume gate — and, per element, |err| <= 1e-4 |ref| + 1e-5 max|ref| (conftest.assert_fp32_gate)
  * bf16 mode (bf16 operands, f32 accumulation, fp16 pyramid): 1e-2 — operand rounding 2^-9
"""

import numpy as np
import pytest
import torch

import oracle
from conftest import assert_close_elementwise, assert_fp32_gate, load_golden, rel_max_err

pytestmark = pytest.mark.gpu

TOL = {"fp32": 1e-4, "fp32-f32": 1e-4, "fp32-exact": 1e-4, "bf16": 1e-2, "bf16-f32": 1e-2, "fp32-f16": 2e-3}
CORR_CASES = ["corr_b2_c32_24x40", "corr_b2_c32_24x40_mask", "corr_b1_c256_16x24_pyr",
              "corr_b1_c16_12x20_nan", "corr_b1_c32_20x28_r7_l2", "corr_b2_c64_17x23_l1",
              "corr_b2_c16_16x24_nonfinite"]      # NaN / +-inf coordinates -> NaN windows (grid_sample)
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("precision", ["fp32", "fp32-f32", "fp32-exact", "bf16", "bf16-f32", "fp32-f16"])
@pytest.mark.parametrize("name", CORR_CASES)
def test_corr_block_matches_reference_golden(name, precision):
    import rmd
    g = load_golden(name)
    cb = rmd.raft.CorrBlock(_t(g["fmap1"]), _t(g["fmap2"]), num_levels=int(g["levels"]),
                            radius=int(g["radius"]), precision=precision)
    out = cb(_t(g["coords"]), g["mask_costs"].tolist())
    torch.cuda.synchronize()
    assert out.dtype == torch.float32 and out.is_contiguous()
    assert tuple(out.shape) == g["out"].shape
    assert rel_max_err(out.cpu().numpy(), g["out"]) < TOL[precision]
    if precision.startswith("fp32") and precision != "fp32-f16":
        assert_fp32_gate(out.cpu().numpy(), g["out"])


@pytest.mark.parametrize("precision,tol", [("fp32-exact", 1e-5), ("fp32", 1e-4), ("fp32-f32", 1e-4)])
def test_pyramid_levels_match_reference_golden(precision, tol):
    import rmd
    g = load_golden("corr_b1_c256_16x24_pyr")
    cb = rmd.raft.CorrBlock(_t(g["fmap1"]), _t(g["fmap2"]), 4, 4, precision=precision)
    for i, lvl in enumerate(cb.corr_pyramid):
        assert tuple(lvl.shape) == g[f"pyr{i}"].shape
        assert rel_max_err(lvl.cpu().numpy(), g[f"pyr{i}"]) < tol
        assert_fp32_gate(lvl.cpu().numpy(), g[f"pyr{i}"])


@pytest.mark.parametrize("precision", ["fp32", "fp32-f32", "fp32-exact", "bf16"])
def test_cfg1_shape_matches_oracle(precision):
    """cfg1 feature shape (368x496 -> 46x62), C=256, B=1, full oracle comparison."""
    import rmd
    rng = np.random.default_rng(11)
    f1 = rng.standard_normal((1, 256, 46, 62)).astype(np.float32)
    f2 = rng.standard_normal((1, 256, 46, 62)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(46), np.arange(62), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 4, (1, 2, 46, 62))).astype(np.float32)
    cb = rmd.raft.CorrBlock(_t(f1), _t(f2), 4, 4, precision=precision)
    out = cb(_t(co)).cpu().numpy()
    ref = oracle.corr_lookup(oracle.corr_pyramid(f1.astype(np.float64), f2.astype(np.float64), 4),
                             co.astype(np.float64), 4)
    assert rel_max_err(out, ref) < TOL[precision]
    if precision.startswith("fp32"):
        assert_fp32_gate(out, ref)


@pytest.mark.parametrize("radius", [1, 2, 3, 5, 6, 8])
def test_lookup_every_radius_row_split_vs_oracle(radius):
    """The lookup splits each window's 2r+1 output rows over 3 lanes (PR = ceil((2r+1)/3); for
    r = 2, 3, 5, 6, 8 the last part overlaps the previous one and stores only its own rows).  Checks
    every radius the kernel is built for against the oracle, with a masked level (zeros), a 1-pixel
    level (NaN, raft.py:73-74) and coordinates far outside the map."""
    import rmd
    rng = np.random.default_rng(100 + radius)
    f1 = rng.standard_normal((2, 32, 12, 20)).astype(np.float32)
    f2 = rng.standard_normal((2, 32, 12, 20)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(12), np.arange(20), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 3, (2, 2, 12, 20))).astype(np.float32)
    co[1, :, 3:5, 7:11] += 40.0
    for precision in ("fp32", "bf16"):
        cb = rmd.raft.CorrBlock(_t(f1), _t(f2), 4, radius, precision=precision)
        out = cb(_t(co), [4]).cpu().numpy()
        ref = oracle.corr_lookup(oracle.corr_pyramid(f1.astype(np.float64), f2.astype(np.float64), 4),
                                 co.astype(np.float64), radius, [4])
        assert out.shape == ref.shape
        assert np.array_equal(np.isnan(out), np.isnan(ref))
        fin = ~np.isnan(ref)
        d = (2 * radius + 1) ** 2
        assert np.all(out[:, d:2 * d] == 0)                                # masked level 1
        assert rel_max_err(out[fin], ref[fin]) < TOL[precision]


def _cfg2_inputs(seed=5, b=8):
    rng = np.random.default_rng(seed)
    f1 = rng.standard_normal((b, 256, 55, 128)).astype(np.float32)
    f2 = rng.standard_normal((b, 256, 55, 128)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(55), np.arange(128), indexing="ij")
    flow = rng.normal(0, 6, (b, 2, 1, 1)) + rng.normal(0, 2, (b, 2, 55, 128))
    co = (np.stack([xs, ys])[None] + flow).astype(np.float32)
    return f1, f2, co


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_cfg2_full_size_sampled_queries(precision):
    """BASELINE cfg2 size (Sintel 440x1024 -> 55x128, C=256, B=8): oracle on 384 sampled queries/batch."""
    import rmd
    f1, f2, co = _cfg2_inputs()
    b, c, h, w = f1.shape
    cb = rmd.raft.CorrBlock(_t(f1), _t(f2), 4, 4, precision=precision)
    out = cb(_t(co)).cpu().numpy().reshape(b, 324, h * w)
    rng = np.random.default_rng(3)
    sel = np.sort(rng.choice(h * w, 384, replace=False))
    sel[:4] = [0, w - 1, (h - 1) * w, h * w - 1]                      # image corners
    f1s = f1.reshape(b, c, h * w)[:, :, sel][:, :, None, :].astype(np.float64)
    cos = co.reshape(b, 2, h * w)[:, :, sel][:, :, None, :].astype(np.float64)
    ref = oracle.corr_lookup(oracle.corr_pyramid(f1s, f2.astype(np.float64), 4), cos, 4)
    assert rel_max_err(out[:, :, sel], ref.reshape(b, 324, -1)) < TOL[precision]
    if precision.startswith("fp32"):
        # the cost-volume gate elementwise: |err| <= 1e-4 |ref| + 1e-5 max|ref|
        ref = ref.reshape(b, 324, -1)
        assert_close_elementwise(out[:, :, sel], ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())


def test_stationary_path_4k_sampled_vs_oracle():
    """A 4K frame's 1/8-resolution map (2160x3840 -> 270x480, C=256, B=1): one wave's 16 level-0
    rows exceed 32-bit store offsets, so the bf16 GEMM routes to corr_pyramid_stationary (64-bit
    addressing, hand-placed vmcnt window audited in tests/test_asm_audit.py).  Pyramid 44.6 GB fp16;
    oracle on 256 sampled queries, flow up to +-40 px, image corners included."""
    import rmd
    from rmd import _lib
    h, w = 270, 480
    d = _lib.describe(1, h, w, 4, _lib.RMD_F16)
    assert _lib.lib().rmd_corr_gemm_kernel(d, 256, _lib.RMD_BF16) == b"stationary"
    rng = np.random.default_rng(17)
    f1 = rng.standard_normal((1, 256, h, w)).astype(np.float32)
    f2 = rng.standard_normal((1, 256, h, w)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    flow = rng.normal(0, 15, (1, 2, 1, 1)) + rng.normal(0, 8, (1, 2, h, w))
    co = (np.stack([xs, ys])[None] + flow).astype(np.float32)
    cb = rmd.raft.CorrBlock(_t(f1), _t(f2), 4, 4, precision="bf16")
    out = cb(_t(co))
    sel = np.sort(rng.choice(h * w, 256, replace=False))
    sel[:4] = [0, w - 1, (h - 1) * w, h * w - 1]
    got = out.reshape(1, 324, h * w)[:, :, torch.from_numpy(sel).to(DEV)].cpu().numpy()
    del out, cb
    torch.cuda.empty_cache()
    f1s = f1.reshape(1, 256, h * w)[:, :, sel][:, :, None, :].astype(np.float64)
    cos = co.reshape(1, 2, h * w)[:, :, sel][:, :, None, :].astype(np.float64)
    ref = oracle.corr_lookup(oracle.corr_pyramid(f1s, f2.astype(np.float64), 4), cos, 4)
    assert rel_max_err(got, ref.reshape(1, 324, -1)) < TOL["bf16"]


def test_gemm_kernel_routing():
    """cfg2 bf16 -> w8, fp32 -> x3 (split bf16), fp32-exact -> tiled (exact f32 MFMA), 4K bf16 -> stationary."""
    from rmd import _lib
    lib = _lib.lib()
    assert lib.rmd_corr_gemm_kernel(_lib.describe(8, 55, 128, 4, _lib.RMD_F32), 256, _lib.RMD_BF16X3) == b"x3"
    assert lib.rmd_corr_gemm_kernel(_lib.describe(8, 55, 128, 4, _lib.RMD_F32), 320, _lib.RMD_BF16X3) == b"tiled"
    assert lib.rmd_corr_gemm_kernel(_lib.describe(8, 55, 128, 4, _lib.RMD_F16), 256, _lib.RMD_BF16X3) == b"tiled"
    assert lib.rmd_corr_gemm_kernel(_lib.describe(8, 55, 128, 4, _lib.RMD_F16), 256, _lib.RMD_BF16) == b"w8"
    assert lib.rmd_corr_gemm_kernel(_lib.describe(8, 55, 128, 4, _lib.RMD_F32), 256, _lib.RMD_F32) == b"tiled"
    assert lib.rmd_corr_gemm_kernel(_lib.describe(8, 55, 128, 4, _lib.RMD_F16), 128, _lib.RMD_BF16) == b"tiled"
    assert lib.rmd_corr_gemm_kernel(_lib.describe(1, 270, 480, 4, _lib.RMD_F16), 256, _lib.RMD_BF16) == b"stationary"


def test_lookup_deterministic_and_pyramid_reusable():
    import rmd
    f1, f2, co = _cfg2_inputs(seed=9, b=2)
    cb = rmd.raft.CorrBlock(_t(f1), _t(f2), 4, 4, precision="bf16")
    a = cb(_t(co))
    b_ = cb(_t(co))
    c2 = cb(_t(co + 0.5))
    torch.cuda.synchronize()
    assert torch.equal(a, b_)
    assert not torch.equal(a, c2)


@pytest.mark.parametrize("precision", ["fp32", "fp32-exact", "bf16"])
def test_corr_block_backward_matches_reference_golden(precision):
    """a11: d(sum(out * grad_out)) / d(fmap1, fmap2) vs the reference's autograd (golden), radius 4,
    4 levels.  The gradient does not depend on the stored pyramid values: the fp32 modes (split-bf16
    backward GEMMs) meet the fp32 gate (1e-4); the bf16 mode runs its backward GEMMs on bf16 products
    (fp32 accumulation) and meets its own 1e-2."""
    import rmd
    g = load_golden("corr_b2_c32_24x40")
    f1 = _t(g["fmap1"]).requires_grad_(True)
    f2 = _t(g["fmap2"]).requires_grad_(True)
    cb = rmd.raft.CorrBlock(f1, f2, 4, 4, precision=precision)
    out = cb(_t(g["coords"]))
    (out * _t(g["grad_out"])).sum().backward()
    tol = 1e-4 if precision.startswith("fp32") else TOL[precision]
    assert rel_max_err(f1.grad.cpu().numpy(), g["grad_fmap1"]) < tol
    assert rel_max_err(f2.grad.cpu().numpy(), g["grad_fmap2"]) < tol


def test_corr_block_backward_accumulates_over_iterations_and_masks():
    """Several lookups of one block (the GRU iterations) sum their gradients into one pyramid
    gradient; masked levels contribute nothing; coords receive none.  Oracle: float64 restatement."""
    import rmd
    rng = np.random.default_rng(4)
    b, c, h, w = 2, 48, 19, 26
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    grid = np.stack([xs, ys])[None].astype(np.float64)
    t1, t2 = _t(f1).requires_grad_(True), _t(f2).requires_grad_(True)
    cb = rmd.raft.CorrBlock(t1, t2, 4, 3, precision="fp32")
    loss = 0.0
    ref1 = np.zeros((b, c, h, w))
    ref2 = np.zeros((b, c, h, w))
    cots = []
    for mask in ([], [4], [3, 6]):
        co = (grid + rng.normal(0, 3, (b, 2, h, w))).astype(np.float32)
        go = rng.standard_normal((b, 4 * 49, h, w)).astype(np.float32)
        cot = _t(co).requires_grad_(True)
        cots.append(cot)
        loss = loss + (cb(cot, mask) * _t(go)).sum()
        r1, r2 = oracle.corr_lookup_backward(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64),
                                             4, 3, go.astype(np.float64), mask)
        ref1 += r1
        ref2 += r2
    loss.backward()
    assert rel_max_err(t1.grad.cpu().numpy(), ref1) < 1e-4
    assert rel_max_err(t2.grad.cpu().numpy(), ref2) < 1e-4
    assert all(c.grad is None for c in cots)


def test_corr_block_no_grad_builds_no_autograd_state():
    import rmd
    f1, f2, co = _cfg2_inputs(seed=1, b=1)
    t1 = _t(f1).requires_grad_(True)
    with torch.no_grad():
        cb = rmd.raft.CorrBlock(t1, _t(f2), 4, 4, precision="bf16")
        out = cb(_t(co))
    assert cb._token is None and not out.requires_grad


def test_zero_flow_centre_channel_is_self_correlation():
    """Property: at integer coords = grid, level-0 centre tap (a=b=r) is f1_p . f2_p / sqrt(C)."""
    import rmd
    rng = np.random.default_rng(2)
    f1 = rng.standard_normal((2, 64, 21, 37)).astype(np.float32)
    f2 = rng.standard_normal((2, 64, 21, 37)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(21), np.arange(37), indexing="ij")
    co = np.broadcast_to(np.stack([xs, ys])[None], (2, 2, 21, 37)).astype(np.float32)
    out = rmd.raft.CorrBlock(_t(f1), _t(f2), 2, 3, precision="fp32")(_t(co)).cpu().numpy()
    centre = out[:, 3 * 7 + 3]
    ref = (f1.astype(np.float64) * f2).sum(1) / 8.0
    assert rel_max_err(centre, ref) < 1e-5


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_raft_fs_corr_block_matches_reference_golden(precision):
    """a4: raft_fs.CorrBlock (pooled-feature window dot, no 1/sqrt(C)) vs the reference's output."""
    import rmd
    g = load_golden("corr_fs_b2_c32_24x40")
    cb = rmd.raft_fs.CorrBlock(_t(g["fmap1"]), _t(g["fmap2"]), int(g["levels"]), int(g["radius"]),
                               precision=precision)
    out = cb(_t(g["coords"]))
    assert out.dtype == torch.float32 and out.is_contiguous() and tuple(out.shape) == g["out"].shape
    assert rel_max_err(out.cpu().numpy(), g["out"]) < TOL[precision]
    if precision.startswith("fp32") and precision != "fp32-f16":
        assert_fp32_gate(out.cpu().numpy(), g["out"])


def test_dot_correlation_module_matches_reference_golden():
    """a5: corr.dot.CorrelationModule forward (with and without DAP) and gradients vs the reference."""
    import rmd
    from detinit import det_init
    g = load_golden("dot_b2_c32_12x16")
    mod = rmd.corr.make_cmod("dot", 32, int(g["radius"]), dap_init="standard")
    assert sorted(mod.state_dict().keys()) == sorted(g["sd.keys"].tolist())
    det_init(mod)
    mod = mod.to(DEV)
    f1 = _t(g["fmap1"]).requires_grad_(True)
    f2 = _t(g["fmap2"]).requires_grad_(True)
    out = mod(f1, f2, _t(g["coords"]), dap=True)
    assert rel_max_err(out.detach().cpu().numpy(), g["out"]) < 1e-4
    d1, d2, dw = torch.autograd.grad(out, (f1, f2, mod.dap.conv1.weight), _t(g["grad_out"]))
    assert rel_max_err(d1.cpu().numpy(), g["grad_fmap1"]) < 1e-4
    assert rel_max_err(d2.cpu().numpy(), g["grad_fmap2"]) < 1e-4
    assert rel_max_err(dw.cpu().numpy(), g["grad_dap"]) < 1e-4
    with torch.no_grad():
        nodap = mod(_t(g["fmap1"]), _t(g["fmap2"]), _t(g["coords"]), dap=False)
    assert rel_max_err(nodap.cpu().numpy(), g["out_nodap"]) < 1e-4


def _gemm_operand(bl, layout):
    """Storage of the logical B operand bl (b, k, nc) in rmd_corr_grad_gemm layout 0-3 (include/rmd.h)
    and its ldb."""
    b, k, nc = bl.shape
    if layout == 0:
        return bl.contiguous(), nc
    if layout == 1:
        return bl.transpose(1, 2).contiguous(), k
    if layout == 2:                                  # ((n/8) ldb + k) 8 + n%8, ldb = k
        npad = (nc + 7) // 8 * 8
        t = torch.zeros(b, k, npad)
        t[:, :, :nc] = bl
        return t.view(b, k, npad // 8, 8).permute(0, 2, 1, 3).contiguous(), k
    kpad = (k + 7) // 8 * 8                          # layout 3: ((k/8) ldb + n) 8 + k%8, ldb = nc
    t = torch.zeros(b, kpad, nc)
    t[:, :k] = bl
    return t.view(b, kpad // 8, 8, nc).permute(0, 1, 3, 2).contiguous(), nc


@pytest.mark.parametrize("compute", ["x3", "bf16"])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
@pytest.mark.parametrize("b,m,k,nc", [(6, 256, 3790, 2852), (2, 100, 37, 45), (1, 300, 129, 130), (3, 32, 1000, 7),
                                     (1, 33, 4096, 35)])
def test_corr_grad_gemm_vs_fp64(layout, b, m, k, nc, compute):
    """rmd_corr_grad_gemm (split-bf16 x3 MFMA) against a float64 GEMM, elementwise, in all four B
    layouts (2 / 3: the 8-target blocked order of the pyramid gradient).  Shapes: the cfg5 backward
    (B6, C256, T = 3790 pooled targets, N = 2852 queries; lda = 3790 is not 16-B aligned), ragged
    tiles and 8-blocks, M over two 256-row tiles, a K split into several workgroups; (1, 33, 4096, 35)
    splits K and has batch*m*nc % 4 != 0 (the split-K reduction's scalar tail)."""
    import ctypes
    from rmd import _lib
    g = torch.Generator(device="cpu").manual_seed(m + k)
    a = torch.randn(b, m, k, generator=g)
    bl = torch.randn(b, k, nc, generator=g)
    ref = torch.bmm(a.double(), bl.double())
    bm, ldb = _gemm_operand(bl, layout)
    lib = _lib.lib()
    ad, bd = a.to(DEV), bm.to(DEV)
    out = torch.full((b, m, nc), float("nan"), device=DEV)
    ws = torch.empty(max(lib.rmd_corr_grad_gemm_workspace_bytes(b, m, k, nc), 1), dtype=torch.uint8, device=DEV)
    cmp = _lib.RMD_BF16X3 if compute == "x3" else _lib.RMD_BF16
    rc = lib.rmd_corr_grad_gemm(ctypes.c_void_p(ad.data_ptr()), k, ctypes.c_void_p(bd.data_ptr()), ldb, b, m, k, nc,
                                layout, cmp, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()), None)
    assert rc == 0
    torch.cuda.synchronize()
    got = out.cpu().double()
    if compute == "x3":
        # fp32-accurate: |err| <= 2e-5 * sqrt(k) * rms(|a||b|) — the dropped lo.lo term and fp32 accumulation
        tol = 2e-5 * np.sqrt(k) + 1e-6
        assert_close_elementwise(got.numpy(), ref.numpy(), rtol=1e-4, atol=tol)
    else:
        # bf16 products (the bf16 mode's backward): each operand rounded to 8 significant bits; gated like
        # the bf16 mode's other outputs, max-normalised (TOL["bf16"] = 1e-2; measured ~2e-3)
        assert rel_max_err(got.numpy(), ref.numpy()) < 5e-3


@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_corr_grad_gemm_misaligned_base_pointers(layout):
    """The C ABI takes plain strided pointers: operands that start 4 B past a 16-B boundary (an offset
    view) must take the scalar load path, not misaligned float4 loads."""
    import ctypes
    from rmd import _lib
    b, m, k, nc = 2, 70, 136, 72
    g = torch.Generator(device="cpu").manual_seed(7)
    a = torch.randn(b, m, k, generator=g)
    bl = torch.randn(b, k, nc, generator=g)
    ref = torch.bmm(a.double(), bl.double())
    bm, ldb = _gemm_operand(bl, layout)
    lib = _lib.lib()
    abuf = torch.zeros(a.numel() + 4, device=DEV)
    bbuf = torch.zeros(bm.numel() + 4, device=DEV)
    abuf[1:1 + a.numel()] = a.reshape(-1).to(DEV)
    bbuf[1:1 + bm.numel()] = bm.reshape(-1).to(DEV)
    out = torch.full((b, m, nc), float("nan"), device=DEV)
    ws = torch.empty(max(lib.rmd_corr_grad_gemm_workspace_bytes(b, m, k, nc), 1), dtype=torch.uint8, device=DEV)
    rc = lib.rmd_corr_grad_gemm(ctypes.c_void_p(abuf.data_ptr() + 4), k, ctypes.c_void_p(bbuf.data_ptr() + 4), ldb,
                                b, m, k, nc, layout, _lib.RMD_BF16X3, ctypes.c_void_p(out.data_ptr()),
                                ctypes.c_void_p(ws.data_ptr()), None)
    assert rc == 0
    torch.cuda.synchronize()
    assert_close_elementwise(out.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=2e-5 * np.sqrt(k) + 1e-6)


@pytest.mark.parametrize("b,h,w", [(1, 55, 128), (2, 40, 64), (1, 23, 96), (3, 55, 128), (1, 46, 62)])
def test_w8_balanced_schedule_levels_vs_oracle(b, h, w):
    """The bf16 GEMM's balanced schedule (corr_pyramid.hip w8_balance): a last block row of <= 8 target
    rows is paired two blocks per workgroup (55 = 3*16 + 7; 40 = 2*16 + 8 also stores a level-3 row
    from the pair's second half), and helper workgroups run the query tiles past qfull.  Every level
    of sampled queries (including the last query tiles, which the helpers write) against the oracle;
    (1, 23, 96) has an odd number of column blocks, (1, 46, 62) neither pairs nor splits."""
    import rmd
    rng = np.random.default_rng(h * w + b)
    c = 256
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    pyr = rmd.ops.corr_pyramid(_t(f1), _t(f2), 4, "bf16")
    n = h * w
    sel = np.unique(np.concatenate([rng.choice(n, 96, replace=False), np.arange(max(0, n - 40), n),
                                    np.arange(0, 8)]))
    ref = oracle.corr_pyramid(f1.reshape(b, c, n)[:, :, sel][:, :, None, :].astype(np.float64),
                              f2.astype(np.float64), 4)
    torch.cuda.synchronize()
    for i in range(4):
        got = pyr.unpack(i).cpu().numpy().reshape(b, n, *ref[i].shape[-2:])[:, sel]
        r = ref[i].reshape(b, len(sel), *ref[i].shape[-2:])
        assert rel_max_err(got, r) < 1e-2, f"level {i}"


@pytest.mark.parametrize("b,h,w,c", [(8, 48, 96, 256), (8, 55, 128, 256), (16, 55, 128, 256), (8, 9, 70, 256),
                                     (8, 39, 121, 256), (8, 39, 121, 96)])
def test_x3_balanced_schedule_whole_pyramid_vs_exact(b, h, w, c):
    """The fp32-mode GEMM's balanced schedule (corr_pyramid_x3.hip X3Sched): when one workgroup per
    (image, block) leaves a partial last round, each XCD's remaining blocks run as query-tile parts
    (8x48x96: 36 blocks per XCD -> 32 whole + 4 x 8 parts; cfg2 b8: 32 + 24 x 4; b16: 96 + 16 x 2;
    8x9x70: 2 x 5 blocks per image, 80 units, one round, no split; 8x39x121: 40 blocks per XCD -> 32 + 8 x 4
    parts with a partial last query tile (N = 4719) and ragged columns, also at C = 96).  Every element of
    every level (a missed or doubled query tile would show) against the exact-f32 GEMM's pyramid:
    max-normalised 1e-4 and north_star's elementwise gate (S24 storage, <= 2^-16 relative rounding)."""
    import rmd
    rng = np.random.default_rng(b * 1000 + h * w + c)
    f1 = _t(rng.standard_normal((b, c, h, w)).astype(np.float32))
    f2 = _t(rng.standard_normal((b, c, h, w)).astype(np.float32))
    p24 = rmd.ops.corr_pyramid(f1, f2, 4, "fp32")
    p32 = rmd.ops.corr_pyramid(f1, f2, 4, "fp32-exact")
    for i in range(4):
        got = p24.unpack(i).reshape(-1).double()         # compared on the GPU (b16: 0.9 G elements)
        ref = p32.unpack(i).reshape(-1).double()
        assert torch.isfinite(ref).all() and torch.equal(torch.isnan(got), torch.isnan(ref))
        scale = ref.abs().max()
        err = (got - ref).abs()
        assert float(err.max() / scale) < 1e-4, f"level {i}"
        assert bool((err <= 1e-4 * ref.abs() + 1e-5 * scale).all()), f"level {i} elementwise"
        del got, ref, err
    del p24, p32
    torch.cuda.empty_cache()


@pytest.mark.parametrize("precision,c,b,h,w", [("bf16", 200, 2, 23, 40), ("bf16", 193, 1, 17, 33),
                                               ("fp32", 200, 2, 23, 40), ("fp32", 96, 3, 9, 70),
                                               ("fp32", 256, 1, 8, 8)])
def test_gemm_paths_odd_shapes_vs_oracle(precision, c, b, h, w):
    """Channel counts that zero-pad to the w8 kernel's 256 (bf16: C = 193, 200) or run the x3 kernel
    below 256 (fp32: C = 96, 200), ragged maps (23x40, 17x33, 9x70 -> level 3 of 1 row) and a map of one
    8x8 block: full pyramid of every query against the oracle."""
    import rmd
    from rmd import _lib
    lib = _lib.lib()
    compute = _lib.RMD_BF16 if precision == "bf16" else _lib.RMD_BF16X3
    storage = _lib.RMD_F16 if precision == "bf16" else _lib.RMD_F32
    kern = lib.rmd_corr_gemm_kernel(_lib.describe(b, h, w, 4, storage), c, compute)
    assert kern == (b"w8" if precision == "bf16" else b"x3")
    rng = np.random.default_rng(c * h + w)
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    pyr = rmd.ops.corr_pyramid(_t(f1), _t(f2), 4, precision)
    ref = oracle.corr_pyramid(f1.astype(np.float64), f2.astype(np.float64), 4)
    torch.cuda.synchronize()
    for i in range(4):
        got = pyr.unpack(i).cpu().numpy().reshape(ref[i].shape)
        assert rel_max_err(got, ref[i]) < TOL[precision], f"level {i}"


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_large_batch_offsets_vs_oracle(precision):
    """B = 40 at the cfg2 map (pyramid 5.2 GB fp16 / 10.4 GB fp32, lookup output 365 MB): the last images' level
    offsets run far past 2^32 bytes, so any 32-bit batch arithmetic in the GEMM epilogue or the lookup
    would land in the wrong image.  Sampled queries of the first and the last image vs the oracle."""
    import rmd
    b, c, h, w = 40, 256, 55, 128
    g = torch.Generator(device="cpu").manual_seed(5)
    f1 = torch.randn(b, c, h, w, generator=g)
    f2 = torch.randn(b, c, h, w, generator=g)
    ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32), indexing="ij")
    co = torch.stack([xs, ys])[None] + 3.0 * torch.randn(b, 2, h, w, generator=g)
    cb = rmd.raft.CorrBlock(f1.to(DEV), f2.to(DEV), 4, 4, precision=precision)
    out = cb(co.to(DEV))
    rng = np.random.default_rng(9)
    n = h * w
    sel = np.sort(rng.choice(n, 64, replace=False))
    for bi in (0, b - 1):
        got = out[bi].reshape(324, n)[:, torch.from_numpy(sel).to(DEV)].cpu().numpy()
        f1s = f1[bi:bi + 1].reshape(1, c, n)[:, :, sel][:, :, None, :].double().numpy()
        cos = co[bi:bi + 1].reshape(1, 2, n)[:, :, sel][:, :, None, :].double().numpy()
        ref = oracle.corr_lookup(oracle.corr_pyramid(f1s, f2[bi:bi + 1].double().numpy(), 4), cos, 4)
        assert rel_max_err(got, ref.reshape(324, -1)) < TOL[precision], f"image {bi}"


def test_pyramid_tensor_carries_its_layout_48x64():
    """at an even shape (48x64, C=256, bf16) the row and tiles descs of the pyramid have the
    same element count, so a layout flag the caller passes could silently scramble the lookup.  The
    pyramid tensor carries its layout in its shape instead: the w8 GEMM's tiles pyramid is (n, 8), the
    lookup reads it correctly, and any other 2-D view is rejected."""
    import rmd
    from rmd import _lib
    rng = np.random.default_rng(48)
    f1 = rng.standard_normal((1, 256, 48, 64)).astype(np.float32)
    f2 = rng.standard_normal((1, 256, 48, 64)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(48), np.arange(64), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 2, (1, 2, 48, 64))).astype(np.float32)
    rows = _lib.describe(1, 48, 64, 4, _lib.RMD_F16, _lib.RMD_LAYOUT_ROWS)
    tiles = _lib.describe(1, 48, 64, 4, _lib.RMD_F16, _lib.RMD_LAYOUT_TILES)
    assert rows.total_elements == tiles.total_elements            # the ambiguous case
    pyr = torch.ops.rmd.corr_pyramid(_t(f1), _t(f2), 4, _lib.RMD_BF16, _lib.RMD_F16, 1 / 16)
    assert pyr.shape == (tiles.total_elements // 8, 8)
    out = torch.ops.rmd.corr_lookup(pyr, _t(co), 4, 4, 0).cpu().numpy()
    ref = oracle.corr_lookup(oracle.corr_pyramid(f1.astype(np.float64), f2.astype(np.float64), 4), co.astype(np.float64), 4)
    assert rel_max_err(out, ref) < TOL["bf16"]
    with pytest.raises(ValueError, match="tiles layout"):
        torch.ops.rmd.corr_lookup(pyr.view(-1, 16), _t(co), 4, 4, 0)


@pytest.mark.parametrize("c,b,h,w", [(256, 8, 55, 128), (96, 3, 9, 70), (200, 2, 23, 40), (256, 1, 8, 8),
                                     (64, 1, 17, 33), (256, 2, 46, 62)])
def test_s24_pyramid_is_rounded_f32_pyramid(c, b, h, w):
    """The x3 GEMM's S24 epilogue (fp32 mode) against its F32 epilogue (fp32-f32) on the same inputs:
    every stored element equals the F32 value rounded by the RMD_S24 rule (rmd.library.s24_encode),
    bit for bit — all four levels, odd / even query parity of the 6-byte level-3 chunks, ragged maps and
    C < 256 — and the lookup of the S24 pyramid equals the lookup of the rounded values in an F32 pyramid."""
    import rmd
    from rmd import _lib, library
    rng = np.random.default_rng(c * 7 + h * w + b)
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f1[0, :, 0, 0] = np.nan                                         # a NaN query row stays NaN
    p24 = rmd.ops.corr_pyramid(_t(f1), _t(f2), 4, "fp32-s24")
    p32 = rmd.ops.corr_pyramid(_t(f1), _t(f2), 4, "fp32-f32")
    assert p24.desc.storage == _lib.RMD_S24 and p24.data.dtype == torch.uint8
    assert p24.data.shape == (p24.desc.total_elements, 3)
    assert p24.desc.tile_w[3] == 4                                  # S24 level 3: 1 x 4 chunks
    for i in range(4):
        got = p24.unpack(i).reshape(-1)
        ref = library.s24_decode(library.s24_encode(p32.unpack(i)))
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), f"level {i}"
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    co = _t((np.stack([xs, ys])[None] + rng.normal(0, 3, (b, 2, h, w))).astype(np.float32))
    a = torch.ops.rmd.corr_lookup(p24.data, co, 4, 4, 0)
    # the F32 pyramid rounded in place (F32 layout, the S24 values): the same lookup arithmetic
    r = torch.ops.rmd.corr_lookup(library.s24_decode(library.s24_encode(p32.data)), co, 4, 4, 0)
    assert torch.equal(torch.nan_to_num(a, nan=7.0), torch.nan_to_num(r, nan=7.0))


def test_s24_storage_falls_back_to_f32_off_the_x3_gemm():
    """S24 is the x3 GEMM's output format: describe_for resolves it to F32 for any other GEMM (C > 256,
    exact f32, bf16) and rmd_corr_pyramid refuses an S24 desc there."""
    import rmd
    from rmd import _lib
    d = _lib.describe_for(1, 16, 24, 4, _lib.RMD_S24, 320, _lib.RMD_BF16X3)        # C > 256: tiled f32
    assert d.storage == _lib.RMD_F32
    d = _lib.describe_for(1, 16, 24, 4, _lib.RMD_S24, 256, _lib.RMD_BF16X3)
    assert d.storage == _lib.RMD_S24
    f = torch.randn(1, 320, 16, 24, device=DEV)
    pyr = torch.ops.rmd.corr_pyramid(f, f, 4, _lib.RMD_BF16X3, _lib.RMD_S24, 1.0)
    assert pyr.dtype == torch.float32 and pyr.dim() == 1
    with pytest.raises(RuntimeError, match="S24"):
        d = _lib.describe(1, 16, 24, 4, _lib.RMD_S24)
        lib = _lib.lib()
        import ctypes
        ws = torch.empty(lib.rmd_corr_pyramid_workspace_bytes(ctypes.byref(d), 320, _lib.RMD_F32), dtype=torch.uint8,
                         device=DEV)
        out = torch.empty(d.total_elements * 3, dtype=torch.uint8, device=DEV)
        _lib.check(lib.rmd_corr_pyramid(ctypes.c_void_p(f.data_ptr()), ctypes.c_void_p(f.data_ptr()), 320, 1.0,
                                        ctypes.byref(d), _lib.RMD_F32, ctypes.c_void_p(out.data_ptr()),
                                        ctypes.c_void_p(ws.data_ptr()), None), "rmd_corr_pyramid")
