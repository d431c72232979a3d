"""CPU dispatch of the torch.ops.rmd operators (rmd/cpu.py) against the reference's golden vectors.

The drop-in modules run on device='cpu' as the reference's do (raft.py:15-95 is plain torch): CPU
tensors reach the operators' ATen kernels, GPU tensors the HIP kernels (tests/test_gpu_*.py hold the
GPU parity tests).  The CPU kernels restate the reference op for op, so in fp32 they reproduce the
fixtures bitwise where the reference's CPU ran the same ATen calls (corr, raft_fs forward) and to
1e-5 elsewhere (summation order of a conv / einsum); the bf16 modes keep their 1e-2 tolerance (fp16
pyramid storage).  Gradients flow through the kernels' own ATen graph (AutogradCPU registration).
"""

import numpy as np
import pytest
import torch

from conftest import load_golden, rel_max_err
from detinit import det_init, det_init_fanin

CORR_CASES = ["corr_b2_c32_24x40", "corr_b2_c32_24x40_mask", "corr_b1_c256_16x24_pyr",
              "corr_b1_c16_12x20_nan", "corr_b1_c32_20x28_r7_l2", "corr_b2_c64_17x23_l1",
              "corr_b2_c16_16x24_nonfinite"]


def _t(a, grad=False):
    return torch.from_numpy(np.ascontiguousarray(a)).requires_grad_(grad)


# the CPU GEMM stores F32 for fp32 (S24 is the x3 GEMM's format): the fp32 modes reproduce the
# reference bit for bit
@pytest.mark.parametrize("precision,tol", [("fp32", 0.0), ("fp32-f32", 0.0), ("fp32-exact", 0.0), ("bf16", 1e-2)])
@pytest.mark.parametrize("name", CORR_CASES)
def test_corr_block_cpu_matches_reference_golden(name, precision, tol):
    import rmd
    g = load_golden(name)
    cb = rmd.raft.CorrBlock(_t(g["fmap1"]), _t(g["fmap2"]), num_levels=int(g["levels"]), radius=int(g["radius"]),
                            precision=precision, method="volume")
    out = cb(_t(g["coords"]), g["mask_costs"].tolist())
    assert out.device.type == "cpu" and out.dtype == torch.float32 and out.is_contiguous()
    assert tuple(out.shape) == g["out"].shape
    assert rel_max_err(out.numpy(), g["out"]) <= tol
    assert rmd.library.pyramid_layout(cb.pyramid.data) == rmd._lib.RMD_LAYOUT_ROWS   # CPU pyramids: row layout


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-6), ("fp32-f32", 1e-6)])
def test_corr_pyramid_levels_cpu(precision, tol):
    import rmd
    g = load_golden("corr_b1_c256_16x24_pyr")
    cb = rmd.raft.CorrBlock(_t(g["fmap1"]), _t(g["fmap2"]), 4, 4, precision=precision)
    for i, lvl in enumerate(cb.corr_pyramid):
        assert rel_max_err(lvl.numpy(), g[f"pyr{i}"]) < tol


def test_s24_encoding_rounds_half_away_and_keeps_specials():
    """RMD_S24 (include/rmd.h): top 24 bits of the fp32 word, round half away from zero on the
    magnitude; inf stays inf, NaN stays NaN, the largest finite values round to inf."""
    import rmd
    lib = rmd.library
    x = torch.tensor([0.0, -0.0, 1.0, -1.0, 1.0 + 2.0 ** -17, 1.0 + 2.0 ** -16, 1.0 + 3 * 2.0 ** -17,
                      float("inf"), float("-inf"), float("nan"), 3.4028235e38, -3.4028235e38, 1e-40],
                     dtype=torch.float32)
    y = lib.s24_decode(lib.s24_encode(x))
    # 15 stored mantissa bits: ulp(1) = 2^-15, ties (1 + 2^-16) round away from zero
    exp = torch.tensor([0.0, -0.0, 1.0, -1.0, 1.0, 1.0 + 2.0 ** -15, 1.0 + 2.0 ** -15,
                        float("inf"), float("-inf"), float("nan"), float("inf"), float("-inf"), 0.0])
    exp[-1] = lib.s24_decode(lib.s24_encode(torch.tensor([1e-40])))[0]    # subnormal: 8 low bits dropped
    assert torch.equal(torch.signbit(y), torch.signbit(exp))
    assert torch.equal(torch.isnan(y), torch.isnan(exp))
    m = ~torch.isnan(exp)
    assert torch.equal(y[m], exp[m])
    r = torch.randn(100000) * torch.exp(torch.randn(100000) * 10)
    assert ((lib.s24_decode(lib.s24_encode(r)) - r).abs() <= r.abs() * 2.0 ** -16).all()


def test_cpu_lookup_reads_s24_pyramids():
    """An S24 pyramid (uint8 (n, 3), the x3 GEMM's output format: 1 x (8, 8, 4, 4) chunks) looked up on
    the CPU: its shape and dtype carry the storage, and the result is the reference's within the
    2^-16 relative rounding of the stored values."""
    import rmd
    from rmd import _lib, cpu, library
    g = load_golden("corr_b2_c32_24x40")
    f1, f2, co = _t(g["fmap1"]), _t(g["fmap2"]), _t(g["coords"])
    lv, r = int(g["levels"]), int(g["radius"])
    b, c, h, w = f1.shape
    p32 = torch.ops.rmd.corr_pyramid(f1, f2, lv, _lib.RMD_BF16X3, _lib.RMD_S24, 1.0 / c ** 0.5)
    assert p32.dtype == torch.float32 and p32.dim() == 1          # the CPU GEMM stores F32
    d24 = _lib.describe(b, h, w, lv, _lib.RMD_S24)
    assert d24.tile_w[lv - 1] == (4 if lv == 4 else d24.tile_w[lv - 1])
    p24 = library.s24_encode(cpu._pack_rows(cpu._corr_levels(f1, f2, lv, 1.0 / c ** 0.5), d24, torch.float32))
    assert p24.dtype == torch.uint8 and p24.shape == (d24.total_elements, 3)
    assert library.pyramid_storage(p24) == _lib.RMD_S24
    a = torch.ops.rmd.corr_lookup(p24, co, lv, r, 0)
    ref = torch.ops.rmd.corr_lookup(p32, co, lv, r, 0)
    assert rel_max_err(a.numpy(), ref.numpy()) < 2e-5
    assert rel_max_err(a.numpy(), g["out"]) < 2e-5


@pytest.mark.parametrize("name", ["corr_fs_b2_c32_24x40", "corr_fs_b2_c16_16x24_nonfinite"])
@pytest.mark.parametrize("method", ["otf", "volume"])
def test_raft_fs_cpu_matches_reference_golden(name, method):
    import rmd
    g = load_golden(name)
    cb = rmd.raft_fs.CorrBlock(_t(g["fmap1"]), _t(g["fmap2"]), int(g["levels"]), int(g["radius"]),
                               precision="fp32", method=method)
    assert cb.method == method
    out = cb(_t(g["coords"]))
    assert rel_max_err(out.numpy(), g["out"]) < 1e-5


@pytest.mark.parametrize("method", ["otf", "volume"])
@pytest.mark.parametrize("name", ["corr_fs_bwd_b2_c32_24x40", "corr_fs_bwd_b1_c48_21x35_l3r3"])
def test_raft_fs_cpu_backward_matches_reference_golden(name, method):
    """Training on the CPU: gradients through the operators' ATen graph vs the reference's autograd."""
    import rmd
    g = load_golden(name)
    t1, t2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    cb = rmd.raft_fs.CorrBlock(t1, t2, int(g["levels"]), int(g["radius"]), precision="fp32", method=method)
    loss = (cb(_t(g["coords"]), g["mask_costs"].tolist()) * _t(g["grad_out"])).sum()
    g1, g2 = torch.autograd.grad(loss, (t1, t2))
    assert rel_max_err(g1.numpy(), g["grad_fmap1"]) < 1e-5
    assert rel_max_err(g2.numpy(), g["grad_fmap2"]) < 1e-5


def test_dot_module_cpu_golden():
    import rmd
    g = load_golden("dot_b2_c32_12x16")
    mod = rmd.corr.make_cmod("dot", 32, int(g["radius"]), dap_init="standard")
    det_init(mod)
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    out = mod(f1, f2, _t(g["coords"]), dap=True)
    assert rel_max_err(out.detach().numpy(), g["out"]) < 1e-5


def test_dicl_stack_cpu_forward_backward_golden():
    import rmd
    g = load_golden("dicl_b1_c16_8x12")
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    st = rmd.ops.dicl_stack(f1, f2, _t(g["coords"]), int(g["radius"]))
    assert rel_max_err(st.detach().numpy(), g["stack"]) == 0.0
    g1, g2 = torch.autograd.grad(st, (f1, f2), _t(g["grad_stack"]))
    assert rel_max_err(g1.numpy(), g["grad_fmap1"]) < 1e-6
    assert rel_max_err(g2.numpy(), g["grad_fmap2"]) < 1e-6
    # the backward operator itself (what the HIP autograd formula calls) agrees with the ATen graph
    b1, b2 = torch.ops.rmd.dicl_stack_backward(_t(g["grad_stack"]), _t(g["coords"]), 16, 8, 12, int(g["radius"]), 0,
                                               8, 12, False)
    assert rel_max_err(b1.numpy(), g["grad_fmap1"]) < 1e-6
    assert rel_max_err(b2.numpy(), g["grad_fmap2"]) < 1e-6


@pytest.mark.parametrize("dap_type", ["separate", "full"])
def test_dicl_ml_cpu_golden(dap_type):
    import rmd
    g = load_golden(f"ml_{dap_type}_b1_c8_8x12")
    L, r = int(g["levels"]), int(g["radius"])
    h, w = g["coords"].shape[-2:]
    for i in range(L):
        st = rmd.ops.dicl_stack(_t(g[f"fmap1_{i}"]), _t(g[f"fmap2_{i}"]), _t(g["coords"]), r, level=i, norm_hw=(h, w))
        assert rel_max_err(st.numpy(), g[f"stack_{i}"]) < 1e-6
    mod = rmd.raft_dicl_ml.CorrelationModule(feature_dim=8, levels=L, radius=r, dap_init="standard", dap_type=dap_type)
    det_init(mod)
    mod.eval()
    with torch.no_grad():
        out = mod([_t(g[f"fmap1_{i}"]) for i in range(L)], [_t(g[f"fmap2_{i}"]) for i in range(L)], _t(g["coords"]),
                  dap=True, mask_costs=g["mask_costs"].tolist())
    assert rel_max_err(out.numpy(), g["out"]) < 1e-5


@pytest.mark.parametrize("kind,fixture", [("dicl-1x1", "dicl1x1_b2_c16_8x12"), ("dicl-emb", "diclemb_b2_c16_8x12")])
def test_dicl_variant_modules_cpu_golden(kind, fixture):
    import rmd
    g = load_golden(fixture)
    mod = rmd.corr.make_cmod(kind, 16, int(g["radius"]), dap_init="standard")
    det_init(mod)
    mod = mod.train()
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    out = mod(f1, f2, _t(g["coords"]), dap=True)
    assert rel_max_err(out.detach().numpy(), g["dap.out"]) < 1e-5
    g1, g2 = torch.autograd.grad(out, (f1, f2), _t(g["dap.grad_out"]))
    assert rel_max_err(g1.numpy(), g["dap.grad_fmap1"]) < 1e-5
    assert rel_max_err(g2.numpy(), g["dap.grad_fmap2"]) < 1e-5


def test_dicl_stack_int_cpu_golden_bit_exact():
    import rmd
    g = load_golden("dicl_cost_b2_c16_10x12")
    ru, rv = g["maxdisp"].tolist()
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    mvol = rmd.ops.dicl_stack_int(f1, f2, ru, rv)
    assert np.array_equal(mvol.detach().numpy(), g["mvol"])
    g1, g2 = torch.autograd.grad(mvol, (f1, f2), _t(g["grad_mvol"]))
    assert rel_max_err(g1.numpy(), g["grad_fmap1"]) == 0.0
    assert rel_max_err(g2.numpy(), g["grad_fmap2"]) == 0.0
    b1, b2 = torch.ops.rmd.dicl_stack_int_backward(_t(g["grad_mvol"]), _t(g["fmap2"]), ru, rv)
    assert rel_max_err(b1.numpy(), g["grad_fmap1"]) == 0.0 and rel_max_err(b2.numpy(), g["grad_fmap2"]) == 0.0


def test_warp_and_warped_volume_cpu_golden():
    import rmd
    g = load_golden("warp_b2_c8_10x12")
    img = _t(g["img2"], True)
    est, mask = rmd.warp.warp_backwards(img, _t(g["flow"]))
    assert np.array_equal(mask.numpy(), g["mask"])
    assert rel_max_err(est.detach().numpy(), g["est"]) == 0.0
    (gi,) = torch.autograd.grad(est, img, _t(g["grad_out"]))
    assert rel_max_err(gi.numpy(), g["grad_img2"]) < 1e-6
    g = load_golden("warp_dicl_cost_b2_c16_10x12")
    ru, rv = g["maxdisp"].tolist()
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    mvol = rmd.ops.dicl_stack_int_warped(f1, f2, _t(g["flow_up"]), ru, rv)
    assert rel_max_err(mvol.detach().numpy(), g["mvol"]) < 1e-6
    d1, d2 = torch.autograd.grad(mvol, (f1, f2), _t(g["grad_mvol"]))
    assert rel_max_err(d1.numpy(), g["grad_fmap1"]) < 1e-6
    assert rel_max_err(d2.numpy(), g["grad_fmap2"]) < 1e-6


def test_dap_cpu_golden():
    import rmd
    g = load_golden("dap_b2_r4_6x8")
    dap = rmd.blocks.dicl.DisplacementAwareProjection((4, 4), init="standard")
    with torch.no_grad():
        dap.conv1.weight.copy_(_t(g["weight"]))
    x = _t(g["x"], True)
    y = dap(x)
    assert rel_max_err(y.detach().numpy(), g["out"]) < 1e-6
    gx, gw = torch.autograd.grad(y, (x, dap.conv1.weight), _t(g["grad_out"]))
    assert rel_max_err(gx.numpy(), g["grad_x"]) < 1e-6
    assert rel_max_err(gw.numpy(), g["grad_weight"]) < 1e-5
    d = int(np.prod(g["x"].shape[1:3]))
    gw_op = torch.ops.rmd.dap_weight_grad(_t(g["grad_out"]), _t(g["x"]), d)
    assert rel_max_err(gw_op.numpy(), g["grad_weight"].reshape(d, d)) < 1e-5


def test_up8_network_cpu_golden():
    import rmd
    g = load_golden("heads_up8_b2_h32_6x9")
    mod = det_init_fanin(rmd.raft.Up8Network(hidden_dim=g["hidden"].shape[1]))
    hid, flow = _t(g["hidden"], True), _t(g["flow"], True)
    out = mod(hid, flow)
    assert rel_max_err(out.detach().numpy(), g["out"]) < 1e-5
    dh, dfl = torch.autograd.grad(out, (hid, flow), _t(g["grad_out"]))
    assert rel_max_err(dh.numpy(), g["grad_hidden"]) < 1e-5
    assert rel_max_err(dfl.numpy(), g["grad_flow"]) < 1e-5


@pytest.mark.parametrize("kind", ["plain", "dap"])
def test_softargmax_cpu_golden(kind):
    import rmd
    g = load_golden(f"heads_softargmax_raft_{kind}_b2_5x7")
    L, r, t = int(g["levels"]), int(g["radius"]), float(g["temperature"])
    mod = rmd.raft.make_flow_regression("softargmax" if kind == "plain" else "softargmax+dap", L, r, temperature=t)
    det_init_fanin(mod)
    cost = _t(g["cost"], True)
    flows = mod(cost)
    for i, f in enumerate(flows):
        assert rel_max_err(f.detach().numpy(), g[f"flow{i}"]) < 1e-6
    loss = sum((f * _t(g[f"grad_flow{i}"])).sum() for i, f in enumerate(flows))
    (dc,) = torch.autograd.grad(loss, cost)
    assert rel_max_err(dc.numpy(), g["grad_cost"]) < 1e-5


def test_cpu_ops_opcheck():
    """torch.library.opcheck on CPU tensors: schema, fake kernel and dispatch consistency."""
    import rmd  # noqa: F401
    rng = np.random.default_rng(0)
    f = _t(rng.standard_normal((2, 16, 6, 8)).astype(np.float32))
    co = _t((np.stack(np.meshgrid(np.arange(8.0), np.arange(6.0))[::1])[None].repeat(2, 0)
             + rng.normal(0, 1, (2, 2, 6, 8))).astype(np.float32))
    torch.library.opcheck(torch.ops.rmd.dicl_stack, (f, f, co, 2, 0, 6, 8, False),
                          test_utils=("test_schema", "test_faketensor"))
    torch.library.opcheck(torch.ops.rmd.up8, (_t(rng.standard_normal((2, 576, 6, 8)).astype(np.float32)), co, 4.0),
                          test_utils=("test_schema", "test_faketensor"))
    pyr = torch.ops.rmd.corr_pyramid(f, f, 2, 0, 0, 0.25)
    torch.library.opcheck(torch.ops.rmd.corr_lookup, (pyr, co, 2, 2, 0), test_utils=("test_schema", "test_faketensor"))
    ws = torch.ops.rmd.corr_otf_prepare(f, f, 2, 0, 1.0)
    torch.library.opcheck(torch.ops.rmd.corr_otf_lookup, (ws, co, 16, 2, 0, 2, 0),
                          test_utils=("test_schema", "test_faketensor"))
