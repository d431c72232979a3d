"""GPU parity of the per-iteration flow heads (rmd_up8, rmd_softargmax and their backward passes)
against reference golden vectors (tests/golden/heads_*.npz, made by tests/golden/gen_golden_heads.py)
and the float64 oracle (oracle/heads.py).

Tolerances (max-normalised, conftest.rel_max_err): kernels vs oracle 1e-5 (fp32 softmax/expf vs
float64); whole modules with MIOpen convolutions vs the reference's fp32 CPU autograd 1e-4; modules
with a DAP layer 1e-4 (north_star's fp32 tolerance: rmd_dap computes in split-bf16 MFMA, ~1.5e-5).
Edge cases: 1-pixel and 1-row maps (every neighbour tap out of bounds), large logits (softmax
overflow safety), non-multiple-of-wave pixel counts, extra trailing channels (dicl_emb).
"""

import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden, rel_max_err
from detinit import det_init_fanin

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a, grad=False):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV).requires_grad_(grad)


def test_up8_network_matches_reference_golden():
    import rmd
    g = load_golden("heads_up8_b2_h32_6x9")
    mod = rmd.raft.Up8Network(hidden_dim=g["hidden"].shape[1])
    assert sorted(mod.state_dict().keys()) == sorted(g["keys"].tolist())
    mod = det_init_fanin(mod).to(DEV)
    assert mod.temperature == float(g["temperature"])
    cap = {}
    mod.conv2.register_forward_hook(lambda m, i, o: cap.update(mask=o))
    hid, flow = _t(g["hidden"], True), _t(g["flow"], True)
    out = mod(hid, flow)
    assert tuple(out.shape) == g["out"].shape and out.is_contiguous()
    assert rel_max_err(cap["mask"].detach().cpu().numpy(), g["mask"]) < 1e-4
    assert rel_max_err(out.detach().cpu().numpy(), g["out"]) < 1e-4
    dh, dfl, dw = torch.autograd.grad(out, (hid, flow, mod.conv2.weight), _t(g["grad_out"]))
    assert rel_max_err(dh.cpu().numpy(), g["grad_hidden"]) < 1e-4
    assert rel_max_err(dfl.cpu().numpy(), g["grad_flow"]) < 1e-4
    assert rel_max_err(dw.cpu().numpy(), g["grad_conv2"]) < 1e-4


@pytest.mark.parametrize("b,h,w,t", [(2, 6, 9, 4.0), (1, 1, 1, 4.0), (3, 1, 37, 0.5), (2, 55, 128, 4.0),
                                     (1, 17, 70, 1.0)])
def test_up8_kernel_vs_oracle(b, h, w, t):
    import rmd
    rng = np.random.default_rng(b * 1000 + h * 10 + w)
    mask = (3.0 * rng.standard_normal((b, 576, h, w))).astype(np.float32)
    flow = (4.0 * rng.standard_normal((b, 2, h, w))).astype(np.float32)
    go = rng.standard_normal((b, 2, 8 * h, 8 * w)).astype(np.float32)
    tm, tf = _t(mask, True), _t(flow, True)
    out = rmd.ops.up8(tm, tf, t)
    m64, f64 = mask.astype(np.float64), flow.astype(np.float64)
    assert rel_max_err(out.detach().cpu().numpy(), oracle.up8(m64, f64, t)) < 1e-5
    dm, df = torch.autograd.grad(out, (tm, tf), _t(go))
    rm, rf = oracle.up8_backward(m64, f64, go.astype(np.float64), t)
    assert rel_max_err(dm.cpu().numpy(), rm) < 1e-5
    assert rel_max_err(df.cpu().numpy(), rf) < 1e-5


def test_up8_large_logits_no_overflow():
    import rmd
    rng = np.random.default_rng(5)
    mask = (400.0 * rng.standard_normal((1, 576, 4, 5))).astype(np.float32)
    flow = rng.standard_normal((1, 2, 4, 5)).astype(np.float32)
    tm, tf = _t(mask, True), _t(flow, True)
    out = rmd.ops.up8(tm, tf, 4.0)
    assert torch.isfinite(out).all()
    m64, f64 = mask.astype(np.float64), flow.astype(np.float64)
    assert rel_max_err(out.detach().cpu().numpy(), oracle.up8(m64, f64, 4.0)) < 1e-5
    # peaked softmax: the mask gradient must not lose accuracy to cancellation
    go = rng.standard_normal(out.shape).astype(np.float32)
    dm, df = torch.autograd.grad(out, (tm, tf), _t(go))
    rm, rf = oracle.up8_backward(m64, f64, go.astype(np.float64), 4.0)
    assert rel_max_err(dm.cpu().numpy(), rm) < 1e-5
    assert rel_max_err(df.cpu().numpy(), rf) < 1e-5


def _dap_sd(mod):
    return det_init_fanin(mod).to(DEV)


@pytest.mark.parametrize("kind", ["plain", "dap"])
def test_softargmax_raft_matches_reference_golden(kind):
    import rmd
    g = load_golden(f"heads_softargmax_raft_{kind}_b2_5x7")
    L, r, t = int(g["levels"]), int(g["radius"]), float(g["temperature"])
    mod = rmd.raft.make_flow_regression("softargmax" if kind == "plain" else "softargmax+dap", L, r, temperature=t)
    assert sorted(mod.state_dict().keys()) == sorted(g["keys"].tolist())
    mod = _dap_sd(mod)
    cost = _t(g["cost"], True)
    flows = mod(cost)
    tol = 1e-4 if kind == "dap" else 1e-5
    assert len(flows) == L
    for i, f in enumerate(flows):
        assert rel_max_err(f.detach().cpu().numpy(), g[f"flow{i}"]) < tol
    loss = sum((f * _t(g[f"grad_flow{i}"])).sum() for i, f in enumerate(flows))
    (dc,) = torch.autograd.grad(loss, cost)
    assert rel_max_err(dc.cpu().numpy(), g["grad_cost"]) < tol


@pytest.mark.parametrize("cmod", ["dot", "dicl", "dicl-1x1", "dicl-emb"])
@pytest.mark.parametrize("kind", ["plain", "dap"])
def test_softargmax_corr_module_matches_reference_golden(cmod, kind):
    import rmd
    g = load_golden(f"heads_softargmax_dot_{kind}_b2_5x7")
    r, t = int(g["radius"]), float(g["temperature"])
    mod = rmd.corr.make_flow_regression(cmod, "softargmax" if kind == "plain" else "softargmax+dap", r, temperature=t)
    assert sorted(mod.state_dict().keys()) == sorted(g["keys"].tolist())
    mod = _dap_sd(mod)
    cost_np = g["cost"]
    if cmod == "dicl-emb":          # embedding input: cost channels followed by 5 embedding channels
        extra = np.random.default_rng(1).standard_normal((cost_np.shape[0], 5) + cost_np.shape[2:]).astype(np.float32)
        cost_np = np.concatenate([cost_np, extra], axis=1)
    cost = _t(cost_np, True)
    f = mod(cost)
    tol = 1e-4 if kind == "dap" else 1e-5
    assert rel_max_err(f.detach().cpu().numpy(), g["flow"]) < tol
    (dc,) = torch.autograd.grad(f, cost, _t(g["grad_flow"]))
    dd = (2 * r + 1) ** 2
    assert rel_max_err(dc[:, :dd].cpu().numpy(), g["grad_cost"]) < tol
    assert not dc[:, dd:].any()


@pytest.mark.parametrize("b,L,r,h,w", [(8, 4, 4, 55, 128), (1, 1, 1, 1, 1), (2, 2, 3, 13, 21), (3, 1, 2, 7, 9)])
def test_softargmax_kernel_vs_oracle(b, L, r, h, w):
    import rmd
    rng = np.random.default_rng(L * 100 + r * 10 + h)
    cost = (5.0 * rng.standard_normal((b, L * (2 * r + 1) ** 2, h, w))).astype(np.float32)
    tc = _t(cost, True)
    flows = rmd.ops.softargmax(tc, L, r, 0.8)
    ref = oracle.softargmax(cost.astype(np.float64), L, r, 0.8)
    for f, rf in zip(flows, ref):
        assert rel_max_err(f.detach().cpu().numpy(), rf) < 1e-5
    gfl = [rng.standard_normal(f.shape).astype(np.float32) for f in flows]
    (dc,) = torch.autograd.grad(flows, tc, [_t(x) for x in gfl])
    rdc = oracle.softargmax_backward(cost.astype(np.float64), L, r, [x.astype(np.float64) for x in gfl], 0.8)
    assert rel_max_err(dc.cpu().numpy(), rdc) < 1e-5


def test_heads_reject_bad_shapes():
    import rmd
    with pytest.raises(ValueError):
        rmd.ops.up8(torch.zeros(1, 575, 2, 2, device=DEV), torch.zeros(1, 2, 2, 2, device=DEV))
    with pytest.raises(ValueError):
        rmd.ops.softargmax(torch.zeros(1, 80, 2, 2, device=DEV), 1, 4)
    with pytest.raises(RuntimeError):
        rmd.ops.softargmax(torch.zeros(1, 17 * 17, 2, 2, device=DEV), 1, 8)      # radius > 4: C-ABI error
