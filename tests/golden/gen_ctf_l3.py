#!/usr/bin/env python3
"""Generate the RAFT+DICL ctf-l3 fixtures by RUNNING the reference model (build container only).

Test infrastructure (SURVEY.md §8(c) fixtures 6b and 7).  Builds the reference
`raft+dicl/ctf-l3` RaftPlusDiclModule (src/models/impls/raft_dicl_ctf_l3.py:19-260, defaults of
cfg/model/raft+dicl-ctf3l.yaml), fills it with detinit.det_init_fanin (name-keyed, seeded, flow head gain 0.02: the GPU
test regenerates the same weights on tests/e2e/ctf_l3_net.CtfL3Net) and stores only numbers:

  ctf_l3_fwd_384x512.npz  (6b) inference, eval mode, iterations (4, 3, 3), one synthetic 384x512
      pair (frame_pair(368, 496) padded to 64, cfg4/cfg5 padding): the 1/32 and 1/16 flows of every
      iteration in full, the mean EPE of the three full-resolution outputs and their flow at 4096
      fixed pixels.
  ctf_l3_train_384x512.npz  (7) one training step at cfg5 shape, batch 2: train mode with frozen
      BatchNorm (on-stage freeze_batchnorm, norm.py:17-24), loss raft+dicl/mlseq (ord 1, gamma
      0.85, alpha (0.38, 0.6, 1.0); loss/mlseq.py:34-57), backward, clip_grad_norm_(1.0), AdamW
      (lr 4e-4, weight decay 1e-4, eps 1e-8: the train/chairs2-1 stage); stores the loss, the total
      gradient norm, every parameter's gradient norm, and the loss of a second forward after the step.

  ctf_l3_fwd_376x1242.npz  (6b at the cfg4 size) the same inference fixture for a KITTI-shape
      376x1242 pair padded to 384x1280 (cfg/model/raft+dicl-ctf3l.yaml:26-33), BASELINE configs[3].
  ctf_l3_train_b6_384x512.npz  (7 at the benched batch) the training step with the cfg5 per-GPU
      batch 6 (pairs: the two of the batch-2 fixture plus four more seeded textures and flows).

Before writing, the restatement tests/e2e/ctf_l3_net.py (given the reference's own make_cmod) is
checked against the reference forward and loss: they must agree bitwise on the CPU.

usage: python tests/golden/gen_ctf_l3.py [fwd512] [train] [fwd1242] [train6]   (default: all)
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
from detinit import det_init_fanin  # noqa: E402
from gen_golden import _import_reference  # noqa: E402
from synth import epe, frame_pair  # noqa: E402

H, W = 368, 496                    # FlyingChairs frame, padded to 384x512 (modulo 64)
PAD = 64
ITERS = (4, 3, 3)
SAMPLES = 4096
# the update block's flow head is scaled down so the coarse level's random-weight updates (x2 per
# level up to 1/8, x8 to full resolution) stay at a few pixels, like real flows of this size
HEAD_GAIN = 0.02
OPT = dict(lr=4e-4, weight_decay=1e-4, eps=1e-8)


def sample_pixels(h, w, n, seed=7):
    rng = np.random.Generator(np.random.PCG64(seed))
    return np.sort(rng.choice(h * w, n, replace=False))


# (texture seed, integer flow) of the training pairs; batch n takes the first n
TRAIN_PAIRS = ((1234, (3, 5)), (99, (6, 2)), (7, (2, 4)), (21, (5, 1)), (314, (1, 6)), (2718, (4, 3)))


def train_batch(n=2):
    """n synthetic pairs (different textures and flows) + padded targets and validity masks."""
    import torch
    imgs1, imgs2, flows, valids = [], [], [], []
    for seed, flow in TRAIN_PAIRS[:n]:
        i1, i2, gt = frame_pair(H, W, flow=flow, seed=seed, pad=PAD)
        hp, wp = i1.shape[-2:]
        f = np.zeros((1, 2, hp, wp), np.float32)
        f[:, :, :H, :W] = gt
        v = np.zeros((1, hp, wp), bool)
        v[:, :H, :W] = True
        imgs1.append(i1), imgs2.append(i2), flows.append(f), valids.append(v)
    cat = lambda xs: torch.from_numpy(np.concatenate(xs))  # noqa: E731
    return cat(imgs1), cat(imgs2), cat(flows), cat(valids)


def train_step(model, loss_fn, freeze, img1, img2, flow, valid):
    import torch
    model.train()
    freeze(model)
    opt = torch.optim.AdamW(model.parameters(), **OPT)
    opt.zero_grad()
    loss = loss_fn(model(img1, img2, iterations=ITERS), flow, valid)
    loss.backward()
    names = [n for n, p in model.named_parameters() if p.grad is not None]
    gnorm = {n: float(p.grad.norm()) for n, p in model.named_parameters() if p.grad is not None}
    total = float(torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0, norm_type=2.0))
    opt.step()
    with torch.no_grad():
        loss1 = loss_fn(model(img1, img2, iterations=ITERS), flow, valid)
    return float(loss), total, names, gnorm, float(loss1)


def _models():
    import torch
    mods = _import_reference()  # noqa: F841
    from src.models.impls import raft_dicl_ctf_l3 as ctf
    from src.models.common import corr as rcorr
    from e2e.ctf_l3_net import CtfL3Net
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count() or 8)
    ref = det_init_fanin(ctf.RaftPlusDiclModule(), head_gain=HEAD_GAIN)
    mine = det_init_fanin(CtfL3Net(rcorr.make_cmod, rcorr.make_flow_regression), head_gain=HEAD_GAIN)
    assert sorted(ref.state_dict().keys()) == sorted(mine.state_dict().keys())
    return ref, mine


def gen_forward(ref, mine, h, w, name):
    """(6b) inference at h x w padded to PAD, eval mode, iterations ITERS."""
    import torch
    img1, img2, gt = frame_pair(h, w, pad=PAD)
    i1, i2 = torch.from_numpy(img1), torch.from_numpy(img2)
    ref.eval(), mine.eval()
    with torch.no_grad():
        out_r = ref(i1, i2, iterations=ITERS)
        out_m = mine(i1, i2, iterations=ITERS)
    for lr_, lm in zip(out_r, out_m):
        for a, b in zip(lr_, lm):
            assert torch.equal(a, b), float((a - b).abs().max())
    print("restatement == reference (forward, bitwise)")
    sel = sample_pixels(h, w, SAMPLES)
    arrays = dict(height=np.int32(h), width=np.int32(w), pad=np.int32(PAD), iterations=np.asarray(ITERS, np.int32),
                  pixels=sel, keys=np.asarray(sorted(ref.state_dict().keys())),
                  epe3=np.asarray([epe(f.numpy(), gt) for f in out_r[2]]))
    for lvl, nm in ((0, "flow5"), (1, "flow4")):
        arrays[nm] = np.stack([f.numpy() for f in out_r[lvl]]).astype(np.float32)
    for k, f in enumerate(out_r[2]):
        f = f.numpy()[0, :, :h, :w].reshape(2, -1)
        assert np.isfinite(f).all()
        arrays[f"flow3_it{k}"] = f[:, sel].astype(np.float32)
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(path, os.path.getsize(path), "bytes; EPE (1/8 level):", np.round(arrays["epe3"], 4).tolist(),
          "flow5 range", float(np.abs(arrays["flow5"]).max()))


def gen_train(ref, mine, n, name):
    """(7) one training step at cfg5 shape with batch n."""
    from src.models.common import norm as rnorm
    from src.models.common.loss import mlseq
    from e2e.ctf_l3_net import freeze_batchnorm, mlseq_loss
    ref_loss = mlseq.MultiLevelSequenceLoss({"ord": 1, "gamma": 0.85, "alpha": (0.38, 0.6, 1.0)})
    b1, b2, fl, va = train_batch(n)
    res_r = train_step(ref, lambda r, f, v: ref_loss(None, r, f, v), lambda m: rnorm.freeze_batchnorm(m, True),
                       b1, b2, fl, va)
    res_m = train_step(mine, mlseq_loss, freeze_batchnorm, b1, b2, fl, va)
    assert res_r[0] == res_m[0] and res_r[1] == res_m[1] and res_r[4] == res_m[4], (res_r[0], res_m[0])
    assert res_r[2] == res_m[2] and all(res_r[3][k] == res_m[3][k] for k in res_r[2])
    print("restatement == reference (training step: loss, gradient norms, loss after AdamW, bitwise)")
    loss0, total, names, gnorm, loss1 = res_r
    path = os.path.join(HERE, name)
    np.savez_compressed(path, height=np.int32(H), width=np.int32(W), pad=np.int32(PAD), batch=np.int32(n),
                        iterations=np.asarray(ITERS, np.int32), loss=np.float64(loss0), grad_norm=np.float64(total),
                        names=np.asarray(names), grad_norms=np.asarray([gnorm[k] for k in names]),
                        loss_after_step=np.float64(loss1), lr=np.float64(OPT["lr"]),
                        weight_decay=np.float64(OPT["weight_decay"]), eps=np.float64(OPT["eps"]),
                        pair_seeds=np.asarray([p[0] for p in TRAIN_PAIRS[:n]], np.int64),
                        pair_flows=np.asarray([p[1] for p in TRAIN_PAIRS[:n]], np.int64))
    print(path, os.path.getsize(path), "bytes; loss", loss0, "grad norm", total, "loss after step", loss1,
          "params with grads", len(names))


def main():
    which = set(sys.argv[1:]) or {"fwd512", "train", "fwd1242", "train6"}
    # every fixture starts from freshly initialised weights (a training step changes them)
    if "fwd512" in which:
        gen_forward(*_models(), H, W, "ctf_l3_fwd_384x512.npz")
    if "train" in which:
        gen_train(*_models(), 2, "ctf_l3_train_384x512.npz")
    if "fwd1242" in which:
        gen_forward(*_models(), 376, 1242, "ctf_l3_fwd_376x1242.npz")
    if "train6" in which:
        gen_train(*_models(), 6, "ctf_l3_train_b6_384x512.npz")


if __name__ == "__main__":
    main()
