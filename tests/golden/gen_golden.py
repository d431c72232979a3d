#!/usr/bin/env python3
"""Generate golden vectors for the cost-volume hot path by RUNNING the reference.

Test infrastructure only.  This script imports the read-only reference checkout at
/root/reference (qzed/raft-meets-dicl v2) in the build container, feeds it seeded synthetic
inputs and writes inputs + reference outputs as small compressed ``.npz`` fixtures next to
this file.  The reference itself never travels: only the numeric vectors are committed.

The reference's non-hot-path imports (cv2, parse, git, tensorboard, torchvision) are absent in
this image and are replaced by inert ``sys.modules`` stubs; none of them is touched by the
functions exercised here.

Functions exercised (reference file:line):
  * raft.CorrBlock                      src/models/impls/raft.py:15-95
  * raft_fs.CorrBlock                   src/models/impls/raft_fs.py:13-87
  * corr.dot.CorrelationModule          src/models/common/corr/dot.py:8-66
  * corr.dicl.CorrelationModule         src/models/common/corr/dicl.py:8-61
  * impls.dicl.FlowLevel.compute_cost   src/models/impls/dicl.py:212-241
  * blocks.dicl.DisplacementAwareProjection  src/models/common/blocks/dicl.py:121-150
  * raft_dicl_ml.CorrelationModule      src/models/impls/raft_dicl_ml.py:235-343

Usage:  python tests/golden/gen_golden.py        (writes tests/golden/*.npz)
"""

import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from detinit import det_init  # noqa: E402

REF = os.environ.get("RMD_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True

    class _Stub(types.ModuleType):
        def __getattr__(self, name):
            if name.startswith("__"):
                raise AttributeError(name)
            return object

    for n in ["cv2", "parse", "git", "tensorboard", "tensorboard.compat", "tensorboard.compat.proto",
              "tensorboard.backend", "tensorboard.backend.event_processing",
              "tensorboard.backend.event_processing.event_file_loader", "torch.utils.tensorboard",
              "torchvision", "torchvision.transforms", "torchvision.transforms.functional"]:
        sys.modules.setdefault(n, _Stub(n))
    sys.path.insert(0, REF)

    import src.models  # noqa: F401  (loads every model + hot-path module)
    from src.models.impls import raft, raft_fs, dicl, raft_dicl_ml
    from src.models.common.corr import dot as corr_dot, dicl as corr_dicl
    from src.models.common.blocks import dicl as blocks_dicl
    return dict(raft=raft, raft_fs=raft_fs, dicl=dicl, ml=raft_dicl_ml, dot=corr_dot,
                cdicl=corr_dicl, blocks=blocks_dicl)


def _grid(b, h, w):
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32), indexing="ij")
    g = np.stack([xs, ys], 0)[None].repeat(b, 0)           # ch0 = x, ch1 = y (grid.py:4-12)
    return g


def _coords(rng, b, h, w, sigma, oob=True):
    c = _grid(b, h, w) + rng.normal(0.0, sigma, size=(b, 2, h, w)).astype(np.float32)
    if oob:
        # a few far out-of-bounds queries, exact-integer queries and border queries
        c[0, :, 0, 0] = (-50.0, -50.0)
        c[0, :, 0, 1] = (w + 40.0, 3.0)
        c[0, :, 1, 0] = (2.0, 5.0)                           # exact integer
        c[0, :, 1, 1] = (w - 1.0, h - 1.0)                   # exact far border
        c[-1, :, h - 1, w - 1] = (0.0, 0.0)
        c[-1, :, h - 1, w - 2] = (-4.5, h + 3.25)
    return c.astype(np.float32)


def _state_keys(module, prefix):
    # weights are NOT stored: both sides fill them with detinit.det_init (name-keyed, seeded)
    return {f"{prefix}keys": np.asarray(sorted(module.state_dict().keys()))}


def main():
    import torch
    ref = _import_reference()
    torch.manual_seed(0)
    torch.set_grad_enabled(True)
    rng = np.random.default_rng(1234)
    t = torch.from_numpy

    def save(name, **arrays):
        path = os.path.join(OUT, name + ".npz")
        np.savez_compressed(path, **arrays)
        print(f"{name}.npz  {os.path.getsize(path) / 1e6:.2f} MB  keys={sorted(arrays)}")

    # ---- (1) RAFT all-pairs correlation + pyramid + lookup (a1-a3) -------------------------
    def corr_case(name, b, c, h, w, levels, radius, sigma, mask_costs=(), pyramid=False, grad=False):
        f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
        f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
        co = _coords(rng, b, h, w, sigma)
        tf1, tf2 = t(f1).requires_grad_(grad), t(f2).requires_grad_(grad)
        cb = ref["raft"].CorrBlock(tf1, tf2, num_levels=levels, radius=radius)
        out = cb(t(co), list(mask_costs))
        arrays = dict(fmap1=f1, fmap2=f2, coords=co, out=out.detach().numpy(),
                      levels=np.int32(levels), radius=np.int32(radius),
                      mask_costs=np.asarray(mask_costs, dtype=np.int32))
        if pyramid:
            for i, lvl in enumerate(cb.corr_pyramid):       # reference layout (B,H,W,1,H2,W2)
                arrays[f"pyr{i}"] = lvl.detach().numpy()
        if grad:
            g = rng.standard_normal(out.shape, dtype=np.float32)
            d1, d2 = torch.autograd.grad(out, (tf1, tf2), t(g))
            arrays.update(grad_out=g, grad_fmap1=d1.numpy(), grad_fmap2=d2.numpy())
        save(name, **arrays)
        return f1, f2, co

    f1, f2, co = corr_case("corr_b2_c32_24x40", 2, 32, 24, 40, 4, 4, 3.0, grad=True)
    corr_case("corr_b2_c32_24x40_mask", 2, 32, 24, 40, 4, 4, 3.0, mask_costs=(4, 6))
    corr_case("corr_b1_c256_16x24_pyr", 1, 256, 16, 24, 4, 4, 4.0, pyramid=True)
    corr_case("corr_b1_c16_12x20_nan", 1, 16, 12, 20, 4, 4, 2.0)         # level 3 is 1x2 -> NaN
    corr_case("corr_b1_c32_20x28_r7_l2", 1, 32, 20, 28, 2, 7, 5.0)
    corr_case("corr_b2_c64_17x23_l1", 2, 64, 17, 23, 1, 4, 3.0)           # odd sizes, 1 level

    # ---- (2) on-the-fly lookup, raft/fs semantics (a4): no 1/sqrt(C) ------------------------
    cbfs = ref["raft_fs"].CorrBlock(t(f1), t(f2), num_levels=4, radius=4)
    out_fs = cbfs(t(co), [])
    save("corr_fs_b2_c32_24x40", fmap1=f1, fmap2=f2, coords=co, out=out_fs.detach().numpy(),
         levels=np.int32(4), radius=np.int32(4))

    # ---- (3) windowed dot-product correlation + DAP (a5) -----------------------------------
    b, c, h, w, r = 2, 32, 12, 16, 4
    mod = det_init(ref["dot"].CorrelationModule(radius=r, dap_init="standard"))
    f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    co = _coords(rng, b, h, w, 2.5)
    tf1, tf2 = t(f1).requires_grad_(True), t(f2).requires_grad_(True)
    out = mod(tf1, tf2, t(co), dap=True)
    out_nodap = mod(t(f1), t(f2), t(co), dap=False)
    g = rng.standard_normal(out.shape, dtype=np.float32)
    d1, d2, dw = torch.autograd.grad(out, (tf1, tf2, mod.dap.conv1.weight), t(g))
    save("dot_b2_c32_12x16", fmap1=f1, fmap2=f2, coords=co, out=out.detach().numpy(),
         out_nodap=out_nodap.detach().numpy(), radius=np.int32(r), grad_out=g,
         grad_fmap1=d1.numpy(), grad_fmap2=d2.numpy(), grad_dap=dw.numpy(),
         **_state_keys(mod, "sd."))

    # ---- (4) DICL displacement gather -> MatchingNet -> DAP (a6) ---------------------------
    b, c, h, w, r = 1, 16, 8, 12, 4
    mod = det_init(ref["cdicl"].CorrelationModule(feature_dim=c, radius=r, dap_init="standard")).eval()
    cap = {}
    mod.mnet.register_forward_hook(lambda m, i, o: cap.update(stack=i[0], cost=o))
    f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    co = _coords(rng, b, h, w, 1.7)
    tf1, tf2 = t(f1).requires_grad_(True), t(f2).requires_grad_(True)
    out = mod(tf1, tf2, t(co), dap=True)
    gs = rng.standard_normal(cap["stack"].shape, dtype=np.float32)
    d1, d2 = torch.autograd.grad(cap["stack"], (tf1, tf2), t(gs))
    save("dicl_b1_c16_8x12", fmap1=f1, fmap2=f2, coords=co, stack=cap["stack"].detach().numpy(),
         cost=cap["cost"].detach().numpy(), out=out.detach().numpy(), radius=np.int32(r),
         grad_stack=gs, grad_fmap1=d1.numpy(), grad_fmap2=d2.numpy(), **_state_keys(mod, "sd."))

    # ---- (5) DICL baseline integer cost volume with validity mask (a8) ---------------------
    b, c, h, w = 2, 16, 10, 12
    lvl = det_init(ref["dicl"].FlowLevel(c, 3, (3, 3))).eval()
    cap = {}
    lvl.mnet.register_forward_hook(lambda m, i, o: cap.update(mvol=i[0], cost=o))
    f1 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    f2 = rng.standard_normal((b, c, h, w), dtype=np.float32)
    f2[0, :, 2:4, 3:7] = 0.0                        # zero feature vectors (occlusion holes, dicl.py:236)
    f2[1, :, 9, :] = 0.0
    f2[1, :5, 0, 0] = 0.0                            # partially zero vector stays valid
    tf1, tf2 = t(f1).requires_grad_(True), t(f2).requires_grad_(True)
    cost = lvl.compute_cost(tf1, tf2)
    gm = rng.standard_normal(cap["mvol"].shape, dtype=np.float32)
    d1, d2 = torch.autograd.grad(cap["mvol"], (tf1, tf2), t(gm))
    save("dicl_cost_b2_c16_10x12", fmap1=f1, fmap2=f2, maxdisp=np.int32([3, 3]),
         mvol=cap["mvol"].detach().numpy(), cost=cost.detach().numpy(), grad_mvol=gm,
         grad_fmap1=d1.numpy(), grad_fmap2=d2.numpy(), **_state_keys(lvl.mnet, "sd."))

    # ---- (6) displacement-aware projection (a9) ---------------------------------------------
    dap = det_init(ref["blocks"].DisplacementAwareProjection((4, 4), init="standard"))
    x = rng.standard_normal((2, 9, 9, 6, 8), dtype=np.float32)
    tx = t(x).requires_grad_(True)
    y = dap(tx)
    g = rng.standard_normal(y.shape, dtype=np.float32)
    dx, dw = torch.autograd.grad(y, (tx, dap.conv1.weight), t(g))
    save("dap_b2_r4_6x8", x=x, weight=dap.conv1.weight.detach().numpy(), out=y.detach().numpy(),
         grad_out=g, grad_x=dx.numpy(), grad_weight=dw.numpy())

    # ---- (7) multi-level DICL with RAFT lookup (a7), 'full' and 'separate' DAP -------------
    for dap_type in ("separate", "full"):
        b, c, h, w, r, L = 1, 8, 8, 12, 4, 2
        mod = det_init(ref["ml"].CorrelationModule(feature_dim=c, levels=L, radius=r, dap_init="standard",
                                                   dap_type=dap_type)).eval()
        stacks = []
        for m in mod.mnet:
            m.register_forward_hook(lambda m, i, o: stacks.append(i[0].detach().numpy()))
        # fmap1 is a stack kept at full resolution, fmap2 a pyramid (raft_dicl_ml.py:181-200);
        # the reference normalises the level-i sample positions with fmap1's (w-1),(h-1) (:300-305)
        f1s = [rng.standard_normal((b, c, h, w), dtype=np.float32) for i in range(L)]
        f2s = [rng.standard_normal((b, c, h >> i, w >> i), dtype=np.float32) for i in range(L)]
        co = _coords(rng, b, h, w, 2.0)
        out = mod([t(a) for a in f1s], [t(a) for a in f2s], t(co), dap=True, mask_costs=[4])
        arrays = dict(coords=co, out=out.detach().numpy(), radius=np.int32(r), levels=np.int32(L),
                      mask_costs=np.int32([4]), **_state_keys(mod, "sd."))
        for i in range(L):
            arrays[f"fmap1_{i}"], arrays[f"fmap2_{i}"], arrays[f"stack_{i}"] = f1s[i], f2s[i], stacks[i]
        save(f"ml_{dap_type}_b1_c8_8x12", **arrays)


if __name__ == "__main__":
    main()
