"""GPU parity of the DICL cost volumes and DAP (rmd_dicl_stack*, rmd_dap) against reference
golden vectors (tests/golden) and the float64 oracle.

Tolerances (max-normalised, conftest.rel_max_err): stacks 1e-5 (bilinear in pixel coordinates vs
the reference's [-1,1] round trip), integer volume bit-exact (pure copy + mask), DAP 1e-4 (north_star's
fp32 tolerance; rmd_dap is a split-bf16 MFMA GEMM, hi.hi + hi.lo + lo.hi, measured ~1.5e-5 — the
reference's own GPU conv runs in TF32 by default, ~5e-4), DAP weight gradient (torch GEMM) 1e-5,
full modules through MatchingNet (MIOpen convolutions) 1e-4.
"""

import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden, rel_max_err

DAP_TOL = 1e-4
from detinit import det_init

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a, grad=False):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV).requires_grad_(grad)


def test_dicl_stack_forward_backward_golden():
    import rmd
    g = load_golden("dicl_b1_c16_8x12")
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    st = rmd.ops.dicl_stack(f1, f2, _t(g["coords"]), int(g["radius"]))
    assert tuple(st.shape) == g["stack"].shape and st.is_contiguous()
    assert rel_max_err(st.detach().cpu().numpy(), g["stack"]) < 1e-5
    g1, g2 = torch.autograd.grad(st, (f1, f2), _t(g["grad_stack"]))
    assert rel_max_err(g1.cpu().numpy(), g["grad_fmap1"]) < 1e-5
    assert rel_max_err(g2.cpu().numpy(), g["grad_fmap2"]) < 1e-5


def test_dicl_correlation_module_golden():
    """Whole drop-in module (gather -> MatchingNet -> DAP) with the reference's weights/state keys."""
    import rmd
    g = load_golden("dicl_b1_c16_8x12")
    mod = rmd.corr.make_cmod("dicl", 16, int(g["radius"]), dap_init="standard")
    assert sorted(mod.state_dict().keys()) == sorted(g["sd.keys"].tolist())
    det_init(mod)
    mod = mod.to(DEV).eval()
    cap = {}
    mod.mnet.register_forward_hook(lambda m, i, o: cap.update(cost=o))
    with torch.no_grad():
        out = mod(_t(g["fmap1"]), _t(g["fmap2"]), _t(g["coords"]), dap=True)
    assert rel_max_err(cap["cost"].cpu().numpy(), g["cost"]) < 1e-4
    assert rel_max_err(out.cpu().numpy(), g["out"]) < 1e-4


@pytest.mark.parametrize("dap_type", ["separate", "full"])
def test_dicl_ml_level_stacks_golden(dap_type):
    import rmd
    g = load_golden(f"ml_{dap_type}_b1_c8_8x12")
    co = _t(g["coords"])
    h, w = g["coords"].shape[-2:]
    for i in range(int(g["levels"])):
        f2 = g[f"fmap2_{i}"]
        st = rmd.ops.dicl_stack(_t(g[f"fmap1_{i}"]), _t(f2), co, int(g["radius"]), level=i, norm_hw=(h, w))
        assert rel_max_err(st.cpu().numpy(), g[f"stack_{i}"]) < 1e-5


@pytest.mark.parametrize("kind,fixture", [("dicl-1x1", "dicl1x1_b2_c16_8x12"), ("dicl-emb", "diclemb_b2_c16_8x12")])
def test_dicl_variant_module_golden_forward_and_gradients(kind, fixture):
    """Whole 'dicl-1x1' / 'dicl-emb' modules (corr/dicl_1x1.py:33-86, corr/dicl_emb.py:32-104) in train
    mode against the reference's outputs: MatchingNet output (hook), module output and the gradients of
    a seeded upstream gradient w.r.t. both feature maps, with and without DAP, and w.r.t. every
    parameter (dap=True).  Our stack kernel feeds MIOpen convolutions here, so the gradient tolerances
    cover MIOpen's fp32 algorithms (forward 1e-4, feature gradients 2e-4, parameter gradients 1e-3)."""
    import rmd
    g = load_golden(fixture)
    mod = rmd.corr.make_cmod(kind, 16, int(g["radius"]), dap_init="standard")
    assert sorted(mod.state_dict().keys()) == sorted(g["sd.keys"].tolist())
    det_init(mod)
    mod = mod.to(DEV).train()
    for dap in (True, False):
        tag = "dap" if dap else "nodap"
        cap = {}
        hook = mod.mnet.register_forward_hook(lambda m, i, o: cap.update(cost=o))
        f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
        out = mod(f1, f2, _t(g["coords"]), dap=dap)
        hook.remove()
        assert tuple(out.shape) == g[f"{tag}.out"].shape
        assert rel_max_err(cap["cost"].detach().cpu().numpy(), g[f"{tag}.cost"]) < 1e-4
        assert rel_max_err(out.detach().cpu().numpy(), g[f"{tag}.out"]) < 1e-4
        params = [(k, p) for k, p in mod.named_parameters()] if dap else []
        grads = torch.autograd.grad(out, [f1, f2] + [p for _, p in params], _t(g[f"{tag}.grad_out"]))
        assert rel_max_err(grads[0].cpu().numpy(), g[f"{tag}.grad_fmap1"]) < 2e-4
        assert rel_max_err(grads[1].cpu().numpy(), g[f"{tag}.grad_fmap2"]) < 2e-4
        for (k, _), gp in zip(params, grads[2:]):
            assert rel_max_err(gp.cpu().numpy(), g[f"{tag}.pg.{k}"]) < 1e-3, k


def test_dicl_emb_stack_has_delta_channels():
    import rmd
    g = load_golden("dicl_b1_c16_8x12")
    st = rmd.ops.dicl_stack(_t(g["fmap1"]), _t(g["fmap2"]), _t(g["coords"]), 4, extra_delta=True).cpu().numpy()
    assert st.shape[3] == 2 * 16 + 2
    assert rel_max_err(st[:, :, :, :32], g["stack"]) < 1e-5
    a = np.arange(9)[:, None] - 4
    assert np.array_equal(st[0, :, :, 32, 0, 0], np.broadcast_to(a, (9, 9)).astype(np.float32))
    assert np.array_equal(st[0, :, :, 33, 0, 0], np.broadcast_to(a.T, (9, 9)).astype(np.float32))


def test_dicl_stack_cfg4_shape_vs_oracle():
    """KITTI ctf-l3 1/16 level (24x80), C=32, r=4, B=2, fractional smooth flow."""
    import rmd
    rng = np.random.default_rng(4)
    b, c, h, w = 2, 32, 24, 80
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 3, (b, 2, h, w))).astype(np.float32)
    st = rmd.ops.dicl_stack(_t(f1), _t(f2), _t(co), 4).cpu().numpy()
    ref = oracle.dicl_stack(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64), 4)
    assert rel_max_err(st, ref) < 1e-5


@pytest.mark.parametrize("level,radius,extra", [(1, 4, False), (2, 4, False), (1, 3, True), (3, 4, False)])
def test_dicl_stack_scaled_grid_vs_oracle(level, radius, extra):
    """raft_dicl_ml levels > 0 (grid scaled by (w_l-1)/(w-1)): the separable patch kernel (r = 3, 4;
    K = 4, 6 at levels 1, 2) and, at level 3 (K = 4), large flows whose samples leave the map."""
    import rmd
    rng = np.random.default_rng(40 + level)
    b, c, h, w = 2, 16, 24, 80
    hl, wl = h >> level, w >> level
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, hl, wl)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 3 if level < 3 else 30, (b, 2, h, w))).astype(np.float32)
    st = rmd.ops.dicl_stack(_t(f1), _t(f2), _t(co), radius, level=level, norm_hw=(h, w), extra_delta=extra)
    st = st.cpu().numpy()
    ref = oracle.dicl_stack(f1.astype(np.float64), f2.astype(np.float64), co.astype(np.float64), radius,
                            level=level, norm_hw=(h, w))
    assert rel_max_err(st[:, :, :, :2 * c], ref) < 1e-5
    if extra:
        a = (np.arange(2 * radius + 1) - radius).astype(np.float32)
        assert np.array_equal(st[0, :, :, 2 * c, 3, 5], np.broadcast_to(a[:, None], st.shape[1:3]))
        assert np.array_equal(st[0, :, :, 2 * c + 1, 3, 5], np.broadcast_to(a[None, :], st.shape[1:3]))


def test_dicl_stack_int_golden_bit_exact():
    import rmd
    g = load_golden("dicl_cost_b2_c16_10x12")
    ru, rv = g["maxdisp"].tolist()
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    mvol = rmd.ops.dicl_stack_int(f1, f2, ru, rv)
    assert np.array_equal(mvol.detach().cpu().numpy(), g["mvol"])
    g1, g2 = torch.autograd.grad(mvol, (f1, f2), _t(g["grad_mvol"]))
    assert rel_max_err(g1.cpu().numpy(), g["grad_fmap1"]) < 1e-6
    assert rel_max_err(g2.cpu().numpy(), g["grad_fmap2"]) < 1e-6


def test_dicl_compute_cost_golden():
    import rmd
    g = load_golden("dicl_cost_b2_c16_10x12")
    mnet = rmd.blocks.dicl.MatchingNet(32)
    assert sorted(mnet.state_dict().keys()) == sorted(g["sd.keys"].tolist())
    holder = torch.nn.Module()
    holder.mnet = mnet                      # det_init keys as inside FlowLevel: 'mnet.0.0.weight', ...
    det_init(holder)
    mnet = mnet.to(DEV).eval()
    with torch.no_grad():
        cost = rmd.dicl.compute_cost(mnet, _t(g["fmap1"]), _t(g["fmap2"]), g["maxdisp"].tolist())
    assert rel_max_err(cost.cpu().numpy(), g["cost"]) < 1e-4


def test_dicl_stack_int_cfg3_level2_vs_oracle():
    """DICL baseline level-2 shape of cfg3 (96x128), C=32, 7x7, with zero holes."""
    import rmd
    rng = np.random.default_rng(8)
    b, c, h, w = 1, 32, 96, 128
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2[:, :, 10:20, 30:50] = 0
    mvol = rmd.ops.dicl_stack_int(_t(f1), _t(f2), 3, 3).cpu().numpy()
    assert np.array_equal(mvol, oracle.dicl_stack_int(f1, f2, 3, 3))


def test_dap_golden():
    import rmd
    g = load_golden("dap_b2_r4_6x8")
    x = _t(g["x"], True)
    wt = _t(g["weight"], True)
    y = rmd.ops.dap(x, wt)
    assert rel_max_err(y.detach().cpu().numpy(), g["out"]) < DAP_TOL
    gx, gw = torch.autograd.grad(y, (x, wt), _t(g["grad_out"]))
    assert rel_max_err(gx.cpu().numpy(), g["grad_x"]) < DAP_TOL
    assert rel_max_err(gw.cpu().numpy(), g["grad_weight"]) < DAP_TOL


@pytest.mark.parametrize("b,d,h,w", [(8, 81, 48, 160), (3, 25, 7, 9), (2, 324, 12, 16), (1, 49, 96, 128),
                                     (2, 130, 5, 13), (1, 1, 4, 4), (8, 324, 48, 160)])
def test_dap_weight_grad_vs_oracle(b, d, h, w):
    """rmd_dap_weight_grad (split-bf16 MFMA, deterministic split-K over batch x pixels) against float64:
    cfg4 1/8 level at b8 (D = 81, K = 61440), ragged D / pixel counts, D = 1, the 324 'full' DAP at b8;
    and bitwise determinism."""
    import rmd  # noqa: F401
    rng = np.random.default_rng(d + h)
    x = rng.standard_normal((b, d, h, w)).astype(np.float32)
    gr = rng.standard_normal((b, d, h, w)).astype(np.float32)
    tx, tg = _t(x), _t(gr)
    gw = torch.ops.rmd.dap_weight_grad(tg, tx, d)
    gw2 = torch.ops.rmd.dap_weight_grad(tg, tx, d)
    torch.cuda.synchronize()
    assert torch.equal(gw, gw2)
    ref = np.einsum("bop,bip->oi", gr.reshape(b, d, -1).astype(np.float64), x.reshape(b, d, -1).astype(np.float64))
    assert rel_max_err(gw.cpu().numpy(), ref) < DAP_TOL


def test_dap_full_324_vs_oracle():
    """'full' DAP of raft_dicl_ml (324x324, weight streamed, not LDS-resident)."""
    import rmd
    rng = np.random.default_rng(6)
    x = rng.standard_normal((2, 324, 12, 16)).astype(np.float32)
    wt = (rng.standard_normal((324, 324, 1, 1)) * 0.05).astype(np.float32)
    y = rmd.ops.dap(_t(x), _t(wt)).cpu().numpy()
    assert rel_max_err(y, oracle.dap(x.astype(np.float64), wt.astype(np.float64))) < DAP_TOL


@pytest.mark.parametrize("transpose", [False, True])
@pytest.mark.parametrize("b,d,h,w", [(3, 25, 7, 9), (2, 130, 5, 13), (1, 200, 33, 1), (2, 1, 4, 4),
                                     (1, 1000, 3, 5), (2, 324, 12, 16), (3, 258, 17, 29), (2, 336, 6, 7),
                                     (1, 352, 9, 40), (3, 260, 6, 10), (1, 1000, 4, 9), (2, 132, 20, 20),
                                     (1, 144, 16, 17)])
def test_dap_ragged_vs_oracle(b, d, h, w, transpose):
    """rmd_dap's split-bf16 MFMA GEMM at ragged shapes: D not a multiple of 16 or 32, several M-blocks
    (D = 130, 132, 144, 200, 258, 260: 2-3 blocks; 324, 336, 352: 4 with a short or full last block;
    1000: 32 one-tile blocks, 8-wave workgroups), pixel counts that are not a multiple of the 32-pixel
    tile, D = 1; forward and transposed (the input gradient W^T g)."""
    import rmd  # noqa: F401
    rng = np.random.default_rng(d * 7 + h)
    x = rng.standard_normal((b, d, h, w)).astype(np.float32)
    wt = (np.eye(d) + rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)
    op = torch.ops.rmd.dap_transpose if transpose else torch.ops.rmd.dap
    y = op(_t(x), _t(wt[:, :, None, None])).cpu().numpy()
    w64 = wt.astype(np.float64)
    ref = oracle.dap(x.astype(np.float64), (w64.T if transpose else w64)[:, :, None, None])
    assert rel_max_err(y, ref) < DAP_TOL


@pytest.mark.parametrize("dap_type", ["separate", "full"])
def test_dicl_ml_correlation_module_golden(dap_type):
    """a7: raft_dicl_ml.CorrelationModule end to end (gather -> MatchingNet -> mask -> DAP) vs the
    reference module's output with the same name-keyed weights."""
    import rmd
    g = load_golden(f"ml_{dap_type}_b1_c8_8x12")
    L, r = int(g["levels"]), int(g["radius"])
    mod = rmd.raft_dicl_ml.CorrelationModule(feature_dim=8, levels=L, radius=r, dap_init="standard",
                                             dap_type=dap_type)
    assert sorted(mod.state_dict().keys()) == sorted(g["sd.keys"].tolist())
    det_init(mod)
    mod = mod.to(DEV).eval()
    with torch.no_grad():
        out = mod([_t(g[f"fmap1_{i}"]) for i in range(L)], [_t(g[f"fmap2_{i}"]) for i in range(L)],
                  _t(g["coords"]), dap=True, mask_costs=g["mask_costs"].tolist())
    assert tuple(out.shape) == g["out"].shape
    assert rel_max_err(out.cpu().numpy(), g["out"]) < 1e-4


@pytest.mark.parametrize("level,radius", [(0, 4), (0, 6), (1, 4), (2, 3)])
def test_dicl_stack_backward_vs_oracle(level, radius):
    """a6/a7 backward at a cfg4-like size: unit-step patch kernel (level 0, r <= 4), general kernel
    (r > 4, and raft_dicl_ml levels > 0 whose grid is scaled by (w_l-1)/(w-1)), both with the LDS
    window.  Oracle: float64 restatement (bilinear scatter)."""
    import rmd
    rng = np.random.default_rng(5 + level)
    b, c, h, w = 2, 16, 24, 80
    hl, wl = h >> level, w >> level
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, hl, wl)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 2, (b, 2, h, w))).astype(np.float32)
    t1, t2 = _t(f1, True), _t(f2, True)
    st = rmd.ops.dicl_stack(t1, t2, _t(co), radius, level=level, norm_hw=(h, w))
    gst = rng.standard_normal(tuple(st.shape)).astype(np.float32)
    g1, g2 = torch.autograd.grad(st, (t1, t2), _t(gst))
    r1, r2 = oracle.dicl_stack_backward(f2.shape, co.astype(np.float64), radius, gst.astype(np.float64),
                                        level=level, norm_hw=(h, w))
    assert rel_max_err(g1.cpu().numpy(), r1) < 1e-5
    assert rel_max_err(g2.cpu().numpy(), r2) < 1e-4


@pytest.mark.parametrize("radius", [4, 2])
def test_dicl_stack_backward_smooth_flow_vs_oracle(radius):
    """Unit-step backward with a smooth flow (the case the cross-lane run merge of the patch
    backward takes: neighbouring pixels' patches start at consecutive columns), plus rows with
    jumps, out-of-map flows and map edges that break the chains."""
    import rmd
    rng = np.random.default_rng(77 + radius)
    b, c, h, w = 2, 8, 24, 160
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    flow = np.stack([np.full((h, w), 2.3), np.full((h, w), -1.6)])[None].repeat(b, 0)
    flow[1] += 0.01 * xs[None]                                  # slowly varying: chains break now and then
    flow[0, :, 5, 40:60] += 7.5                                 # a jump inside a row
    flow[1, :, 20:, :] -= 30.0                                  # patches partly / fully above the map
    co = (np.stack([xs, ys])[None] + flow).astype(np.float32)
    t1, t2 = _t(f1, True), _t(f2, True)
    st = rmd.ops.dicl_stack(t1, t2, _t(co), radius)
    gst = rng.standard_normal(tuple(st.shape)).astype(np.float32)
    g1, g2 = torch.autograd.grad(st, (t1, t2), _t(gst))
    r1, r2 = oracle.dicl_stack_backward(f2.shape, co.astype(np.float64), radius, gst.astype(np.float64))
    assert rel_max_err(g1.cpu().numpy(), r1) < 1e-5
    assert rel_max_err(g2.cpu().numpy(), r2) < 1e-4


@pytest.mark.parametrize("level,radius,amp", [(0, 4, 3.0), (0, 4, 8.0), (0, 3, 3.0), (0, 1, 8.0), (1, 4, 3.0),
                                              (1, 4, 8.0), (1, 3, 3.0)])
def test_dicl_stack_backward_graded_flow_vs_oracle(level, radius, amp):
    """Stack backward under flow fields with gradients (low-resolution noise upsampled x8, as the
    component bench): neighbouring pixels' window origins step by 0, 1 or 2 columns and change rows
    along x, so the two-pixel merges (unit step: joint (2r+3) x (2r+4) box; level 1: K x K separable
    patches) mix with chained, unchained and per-pixel lanes inside one wave."""
    import rmd
    rng = np.random.default_rng(int(100 * amp) + 10 * level + radius)
    b, c, h, w = 2, 8, 24, 96
    hl, wl = h >> level, w >> level
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, hl, wl)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    low = torch.from_numpy(rng.standard_normal((b, 2, h // 8, w // 8)) * amp)
    flow = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=True).numpy()
    co = (np.stack([xs, ys])[None] + flow).astype(np.float32)
    t1, t2 = _t(f1, True), _t(f2, True)
    st = rmd.ops.dicl_stack(t1, t2, _t(co), radius, level=level, norm_hw=(h, w))
    gst = rng.standard_normal(tuple(st.shape)).astype(np.float32)
    g1, g2 = torch.autograd.grad(st, (t1, t2), _t(gst))
    r1, r2 = oracle.dicl_stack_backward(f2.shape, co.astype(np.float64), radius, gst.astype(np.float64),
                                        level=level, norm_hw=(h, w))
    assert rel_max_err(g1.cpu().numpy(), r1) < 1e-5
    assert rel_max_err(g2.cpu().numpy(), r2) < 1e-4
