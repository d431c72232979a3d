"""End-to-end gate of the north star: RAFT 12-iteration inference at 436x1024 with the HIP correlation
path matches the reference's EPE within 1e-3 px.

The fixture (tests/golden/e2e_raft_436x1024.npz, made by tests/golden/gen_e2e.py) holds the
reference model's mean EPE after every iteration and its flow at 4096 fixed pixels after
iterations 1, 4 and 12, for name-keyed deterministic weights (detinit.det_init_fanin) and the
synthetic pair of synth.frame_pair (known constant flow).  tests/e2e/raft_net.py restates the
network with the reference's module names (verified bitwise against the reference on CPU when given
the reference's CorrBlock); here its correlation is rmd.raft.CorrBlock and its convex upsampling
rmd.raft.Up8Network (rmd_up8), both on the GPU.

Tolerances: |EPE - EPE_ref| <= 1e-3 px after every iteration (north_star) in both precision modes;
sampled flow max |d| <= 1e-2 px (fp32 mode: MIOpen convolutions vs CPU ATen differ in summation
order only) and <= 5e-2 px (bf16 mode: bf16 GEMM operands, fp16 pyramid).
"""

import json
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden
from detinit import det_init_fanin
from e2e.raft_net import RaftNet
from synth import epe, frame_pair

pytestmark = pytest.mark.gpu

FLOW_TOL = {"fp32": 1e-2, "bf16": 5e-2}


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_raft_12_iterations_epe_matches_reference(precision):
    import rmd
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    g = load_golden("e2e_raft_436x1024")
    h, w, iters = int(g["height"]), int(g["width"]), int(g["iterations"])
    net = det_init_fanin(RaftNet(rmd.raft.CorrBlock, precision=precision,
                                 upnet_cls=rmd.raft.Up8Network)).eval().cuda()
    assert sorted(net.state_dict().keys()) == sorted(g["keys"].tolist())
    img1, img2, gt = frame_pair(h, w)
    with torch.no_grad():
        flows = [f.cpu().numpy() for f in net(torch.from_numpy(img1).cuda(), torch.from_numpy(img2).cuda(), iters)]
    d_epe = [abs(epe(f, gt) - float(r)) for f, r in zip(flows, g["epe"])]
    d_flow = {}
    for k in (1, 4, 12):
        f = flows[k - 1][0, :, :h, :w].reshape(2, -1)[:, g["pixels"]]
        d_flow[k] = float(np.abs(f - g[f"flow_it{k}"]).max())
    report = {"precision": precision, "epe_ref_it12": float(g["epe"][-1]), "epe_it12": epe(flows[-1], gt),
              "max_abs_epe_diff": max(d_epe), "epe_diff_it12": d_epe[-1], "max_flow_diff_px": d_flow}
    print(json.dumps(report))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, f"e2e_{precision}.json"), "w") as fh:
            json.dump(report, fh)
    assert max(d_epe) <= 1e-3, report
    assert max(d_flow.values()) <= FLOW_TOL[precision], report
