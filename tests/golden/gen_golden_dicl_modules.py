#!/usr/bin/env python3
"""Golden vectors for the whole 'dicl-1x1' and 'dicl-emb' correlation modules (test infrastructure).

Runs the reference's own modules from /root/reference (qzed/raft-meets-dicl v2) in the build
container, on seeded inputs, with the name-keyed weights of detinit.det_init, and stores inputs,
the MatchingNet output (forward hook), the module output and the gradients of a seeded upstream
gradient w.r.t. both feature maps (and, with dap=True, every parameter):

  * corr.dicl_1x1.CorrelationModule   src/models/common/corr/dicl_1x1.py:33-86
  * corr.dicl_emb.CorrelationModule   src/models/common/corr/dicl_emb.py:32-104

The modules run in train mode (batch statistics, as in the reference's training step) with
dap=True and dap=False.  Weights are never stored: the test rebuilds them with det_init.

Usage:  python tests/golden/gen_golden_dicl_modules.py   (writes tests/golden/dicl1x1_*.npz, diclemb_*.npz)
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from detinit import det_init  # noqa: E402
from gen_golden import _coords, _import_reference, _state_keys  # noqa: E402

OUT = HERE


def main():
    import torch
    ref = _import_reference()
    from src.models.common.corr import dicl_1x1, dicl_emb
    del ref
    t = torch.from_numpy
    rng = np.random.default_rng(4321)
    b, c, h, w, r = 2, 16, 8, 12, 3
    for name, cls in (("dicl1x1", dicl_1x1.CorrelationModule), ("diclemb", dicl_emb.CorrelationModule)):
        torch.manual_seed(0)
        mod = det_init(cls(feature_dim=c, radius=r, dap_init="standard")).train()
        f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
        f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
        co = _coords(rng, b, h, w, 1.5)
        arrays = dict(fmap1=f1, fmap2=f2, coords=co, radius=np.int32(r), **_state_keys(mod, "sd."))
        for dap in (True, False):
            cap = {}
            hook = mod.mnet.register_forward_hook(lambda m, i, o: cap.update(stack=i[0], cost=o))
            tf1, tf2 = t(f1).requires_grad_(True), t(f2).requires_grad_(True)
            out = mod(tf1, tf2, t(co), dap=dap)
            hook.remove()
            g = rng.standard_normal(out.shape, dtype=np.float32)
            # parameter gradients for the dap=True pass only (keeps the fixture small)
            params = [(k, p) for k, p in mod.named_parameters()] if dap else []
            grads = torch.autograd.grad(out, [tf1, tf2] + [p for _, p in params], t(g))
            tag = "dap" if dap else "nodap"
            arrays[f"{tag}.out"] = out.detach().numpy()
            arrays[f"{tag}.cost"] = cap["cost"].detach().numpy()
            arrays[f"{tag}.grad_out"] = g
            arrays[f"{tag}.grad_fmap1"] = grads[0].numpy()
            arrays[f"{tag}.grad_fmap2"] = grads[1].numpy()
            for (k, _), gp in zip(params, grads[2:]):
                arrays[f"{tag}.pg.{k}"] = gp.numpy()
        path = os.path.join(OUT, f"{name}_b{b}_c{c}_{h}x{w}.npz")
        np.savez_compressed(path, **arrays)
        print(f"{os.path.basename(path)}  {os.path.getsize(path) / 1e6:.2f} MB  {len(arrays)} arrays")


if __name__ == "__main__":
    main()
