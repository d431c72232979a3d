#!/usr/bin/env python3
"""Golden vectors for the per-iteration flow heads, produced by RUNNING the reference.

Test infrastructure only; same import recipe as gen_golden.py (inert stubs for the reference's
absent non-hot-path imports).  Functions exercised (reference file:line):
  * raft.Up8Network                              src/models/impls/raft.py:299-331
  * raft.SoftArgMaxFlowRegression(+WithDap)      src/models/impls/raft.py:98-181
  * corr.dot.SoftArgMaxFlowRegression(+WithDap)  src/models/common/corr/dot.py:69-120

Weights are never stored: both sides fill them with detinit (name-keyed, seeded).
Usage:  python tests/golden/gen_golden_heads.py        (writes tests/golden/heads_*.npz)
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from detinit import det_init_fanin  # noqa: E402
from gen_golden import OUT, _import_reference  # noqa: E402


def main():
    import torch
    ref = _import_reference()
    from src.models.common.corr import dot as corr_dot
    torch.manual_seed(0)
    rng = np.random.default_rng(4321)
    t = torch.from_numpy

    def save(name, **arrays):
        path = os.path.join(OUT, name + ".npz")
        np.savez_compressed(path, **arrays)
        print(f"{name}.npz  {os.path.getsize(path) / 1e6:.2f} MB  keys={sorted(arrays)}")

    # ---- Up8Network: module forward + gradients (hidden, flow, conv2 weight) ---------------------
    b, hdim, h, w = 2, 32, 6, 9
    up = det_init_fanin(ref["raft"].Up8Network(hidden_dim=hdim))
    hid = rng.standard_normal((b, hdim, h, w), dtype=np.float32)
    flow = (3.0 * rng.standard_normal((b, 2, h, w))).astype(np.float32)
    th, tf = t(hid).requires_grad_(True), t(flow).requires_grad_(True)
    cap = {}
    up.conv2.register_forward_hook(lambda m, i, o: cap.update(mask=o))
    out = up(th, tf)
    g = rng.standard_normal(out.shape, dtype=np.float32)
    dh, dfl, dw = torch.autograd.grad(out, (th, tf, up.conv2.weight), t(g))
    save("heads_up8_b2_h32_6x9", hidden=hid, flow=flow, mask=cap["mask"].detach().numpy(),
         out=out.detach().numpy(), grad_out=g, grad_hidden=dh.numpy(), grad_flow=dfl.numpy(),
         grad_conv2=dw.numpy(), temperature=np.float32(up.temperature),
         keys=np.asarray(sorted(up.state_dict().keys())))

    # ---- raft soft-argmax regression, 4 levels r=4 (plain and with per-level DAP) ----------------
    b, h, w, L, r = 2, 5, 7, 4, 4
    cost = (4.0 * rng.standard_normal((b, L * (2 * r + 1) ** 2, h, w))).astype(np.float32)
    for name, mod in (("plain", ref["raft"].SoftArgMaxFlowRegression(L, r, temperature=0.7)),
                      ("dap", det_init_fanin(ref["raft"].SoftArgMaxFlowRegressionWithDap(L, r, temperature=1.3)))):
        tc = t(cost).requires_grad_(True)
        flows = mod(tc)
        gs = [rng.standard_normal(f.shape, dtype=np.float32) for f in flows]
        loss = sum((f * t(gg)).sum() for f, gg in zip(flows, gs))
        dc = torch.autograd.grad(loss, tc)[0]
        arrays = dict(cost=cost, levels=np.int32(L), radius=np.int32(r), temperature=np.float32(mod.temperature),
                      grad_cost=dc.numpy(), keys=np.asarray(sorted(mod.state_dict().keys())))
        for i, (f, gg) in enumerate(zip(flows, gs)):
            arrays[f"flow{i}"], arrays[f"grad_flow{i}"] = f.detach().numpy(), gg
        save(f"heads_softargmax_raft_{name}_b2_5x7", **arrays)

    # ---- corr-module soft-argmax (one level, no level scaling), dot flavour, r=3 -----------------
    r = 3
    cost = (3.0 * rng.standard_normal((b, (2 * r + 1) ** 2, h, w))).astype(np.float32)
    for name, mod in (("plain", corr_dot.SoftArgMaxFlowRegression(r)),
                      ("dap", det_init_fanin(corr_dot.SoftArgMaxFlowRegressionWithDap(r)))):
        tc = t(cost).requires_grad_(True)
        f = mod(tc)
        gg = rng.standard_normal(f.shape, dtype=np.float32)
        dc = torch.autograd.grad(f, tc, t(gg))[0]
        save(f"heads_softargmax_dot_{name}_b2_5x7", cost=cost, radius=np.int32(r),
             temperature=np.float32(mod.temperature), flow=f.detach().numpy(), grad_flow=gg,
             grad_cost=dc.numpy(), keys=np.asarray(sorted(mod.state_dict().keys())))


if __name__ == "__main__":
    main()
