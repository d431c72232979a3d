"""Hybrid-model parity: RAFT+DICL ctf-l3 (src/models/impls/raft_dicl_ctf_l3.py:19-260) through the HIP
DICL path, against fixtures the reference itself produced (tests/golden/gen_ctf_l3.py, SURVEY.md
§8(c) fixtures 6b and 7).

tests/e2e/ctf_l3_net.py restates the network with the reference's module names (checked bitwise
against the reference on the CPU by the generator); here its three correlation modules are
rmd.corr.make_cmod('dicl') (rmd_dicl_stack + MatchingNet + rmd_dap, forward and backward on the
GPU) and its convex upsampling rmd.raft.Up8Network.  Weights: detinit.det_init_fanin (name-keyed,
flow head gain 0.02), regenerated here.

Tolerances:
  * inference (384x512 and 376x1242 -> 384x1280, b1, iterations (4, 3, 3)): |EPE - EPE_ref| <= 1e-3 px for every 1/8-level
    output (north_star's EPE gate); 1/32 and 1/16 flows of every iteration and sampled full-resolution
    flows within 1e-2 px (MIOpen vs CPU ATen convolutions: summation order only).
  * training step (cfg5 shape 384x512, batch 2 and 6, mlseq loss, clip 1.0, AdamW): loss and total gradient
    norm within 1e-4 relative; every parameter's gradient norm within 1e-3 relative, except gradients
    that are zero in exact arithmetic and rounding noise in both runs (biases of convolutions followed
    by InstanceNorm, e.g. fnet.conv1.bias: ~1e-6 against a total norm of ~2.6e3), which must stay below
    1e-8 x the total norm; the loss after the AdamW step within 1e-3 relative (the first Adam step
    moves each weight by ~lr * sign(g), so near-zero gradients whose sign depends on summation order
    perturb it slightly).
"""

import json
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden
from detinit import det_init_fanin
from e2e.ctf_l3_net import CtfL3Net, freeze_batchnorm, mlseq_loss
from synth import epe, frame_pair

pytestmark = pytest.mark.gpu

HEAD_GAIN = 0.02


def _net():
    import rmd
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    net = CtfL3Net(rmd.corr.make_cmod, rmd.corr.make_flow_regression, upnet_cls=rmd.raft.Up8Network)
    return det_init_fanin(net, head_gain=HEAD_GAIN).cuda()


def _report(name, rep):
    print(json.dumps(rep))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, f"{name}.json"), "w") as fh:
            json.dump(rep, fh)


@pytest.mark.parametrize("fixture", ["ctf_l3_fwd_384x512", "ctf_l3_fwd_376x1242"])
def test_ctf_l3_forward_matches_reference(fixture):
    """384x512 (cfg5 frame) and the cfg4 KITTI shape 376x1242 padded to 384x1280 (BASELINE configs[3])."""
    g = load_golden(fixture)
    h, w, pad = int(g["height"]), int(g["width"]), int(g["pad"])
    iters = tuple(int(i) for i in g["iterations"])
    net = _net().eval()
    assert sorted(net.state_dict().keys()) == sorted(g["keys"].tolist())
    img1, img2, gt = frame_pair(h, w, pad=pad)
    with torch.no_grad():
        out5, out4, out3 = net(torch.from_numpy(img1).cuda(), torch.from_numpy(img2).cuda(), iters)
    d5 = float(np.abs(np.stack([f.cpu().numpy() for f in out5]) - g["flow5"]).max())
    d4 = float(np.abs(np.stack([f.cpu().numpy() for f in out4]) - g["flow4"]).max())
    flows = [f.cpu().numpy() for f in out3]
    d_epe = [abs(epe(f, gt) - float(r)) for f, r in zip(flows, g["epe3"])]
    d3 = max(float(np.abs(f[0, :, :h, :w].reshape(2, -1)[:, g["pixels"]] - g[f"flow3_it{k}"]).max())
             for k, f in enumerate(flows))
    rep = {"epe_ref": g["epe3"].tolist(), "epe": [epe(f, gt) for f in flows], "max_abs_epe_diff": max(d_epe),
           "max_flow_diff_px": {"1/32": d5, "1/16": d4, "full": d3}}
    _report(fixture, rep)
    assert max(d_epe) <= 1e-3, rep
    assert max(d5, d4, d3) <= 1e-2, rep


def _train_batch(h, w, pad, pairs):
    imgs1, imgs2, flows, valids = [], [], [], []
    for seed, flow in pairs:
        i1, i2, gt = frame_pair(h, w, flow=flow, seed=seed, pad=pad)
        hp, wp = i1.shape[-2:]
        f = np.zeros((1, 2, hp, wp), np.float32)
        f[:, :, :h, :w] = gt
        v = np.zeros((1, hp, wp), bool)
        v[:, :h, :w] = True
        imgs1.append(i1), imgs2.append(i2), flows.append(f), valids.append(v)
    return [torch.from_numpy(np.concatenate(x)).cuda() for x in (imgs1, imgs2, flows, valids)]


@pytest.mark.parametrize("fixture", ["ctf_l3_train_384x512", "ctf_l3_train_b6_384x512"])
def test_ctf_l3_training_step_matches_reference(fixture):
    """cfg5 shape at batch 2 and at the benched per-GPU batch 6."""
    g = load_golden(fixture)
    h, w, pad = int(g["height"]), int(g["width"]), int(g["pad"])
    iters = tuple(int(i) for i in g["iterations"])
    if "pair_seeds" in g:
        pairs = [(int(s), tuple(int(v) for v in f)) for s, f in zip(g["pair_seeds"], g["pair_flows"])]
    else:
        pairs = [(1234, (3, 5)), (99, (6, 2))]
    assert len(pairs) == int(g["batch"])
    img1, img2, flow, valid = _train_batch(h, w, pad, pairs)
    net = _net()
    net.train()
    freeze_batchnorm(net)
    opt = torch.optim.AdamW(net.parameters(), lr=float(g["lr"]), weight_decay=float(g["weight_decay"]),
                            eps=float(g["eps"]))
    opt.zero_grad()
    loss = mlseq_loss(net(img1, img2, iters), flow, valid)
    loss.backward()
    params = dict(net.named_parameters())
    names = [str(n) for n in g["names"]]
    assert sorted(names) == sorted(n for n, p in params.items() if p.grad is not None)
    gn = np.asarray([float(params[n].grad.norm()) for n in names])
    total = float(torch.nn.utils.clip_grad_norm_(net.parameters(), 1.0, norm_type=2.0))
    opt.step()
    with torch.no_grad():
        loss1 = float(mlseq_loss(net(img1, img2, iters), flow, valid))
    ref_gn = g["grad_norms"]
    noise = 1e-8 * float(g["grad_norm"])                 # rounding-noise level of exactly-zero gradients
    zero = (ref_gn <= noise) & (gn <= noise)
    rel_gn = np.abs(gn - ref_gn) / np.maximum(np.abs(ref_gn), 1e-30)
    ok_gn = (rel_gn <= 1e-3) | zero
    worst = int(np.argmax(np.where(zero, 0, rel_gn)))
    loss = float(loss.detach())
    rep = {"loss": loss, "loss_ref": float(g["loss"]),
           "loss_rel_diff": abs(loss - float(g["loss"])) / abs(float(g["loss"])),
           "grad_norm": total, "grad_norm_ref": float(g["grad_norm"]),
           "grad_norm_rel_diff": abs(total - float(g["grad_norm"])) / float(g["grad_norm"]),
           "param_grad_norm_max_rel_diff": float(rel_gn[worst]), "worst_param": names[worst],
           "zero_gradient_params": [names[i] for i in np.nonzero(zero)[0]],
           "loss_after_step": loss1, "loss_after_step_ref": float(g["loss_after_step"]),
           "loss_after_step_rel_diff": abs(loss1 - float(g["loss_after_step"])) / abs(float(g["loss_after_step"]))}
    _report(fixture, rep)
    assert rep["loss_rel_diff"] <= 1e-4, rep
    assert rep["grad_norm_rel_diff"] <= 1e-4, rep
    assert ok_gn.all(), [(names[i], gn[i], ref_gn[i]) for i in np.nonzero(~ok_gn)[0][:10]]
    assert rep["loss_after_step_rel_diff"] <= 1e-3, rep
