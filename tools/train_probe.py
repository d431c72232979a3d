#!/usr/bin/env python3
"""bench.py's train_step leg (cfg5: RAFT+DICL ctf-l3, b6, 384x512, (4,3,3) iterations, mlseq loss,
backward, clip, AdamW) for a rocprofv3 --kernel-trace run: `warmup` steps (MIOpen algorithm search
happens here), then a 1.5 s idle gap, then `steps` timed steps — tools/train_profile_summary.py sums
the kernels after the last gap.  usage: python3 tools/train_probe.py [warmup] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch
    # the same network, data and step as bench.train_leg (which times its own loop)
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
        sys.path.insert(0, p)
    import numpy as np
    import rmd
    from detinit import det_init_fanin
    from e2e.ctf_l3_net import CtfL3Net, freeze_batchnorm, mlseq_loss
    from synth import frame_pair
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda", 0)
    h, w, pad, bsz = 368, 496, 64, 6
    net = det_init_fanin(CtfL3Net(rmd.corr.make_cmod, rmd.corr.make_flow_regression, upnet_cls=rmd.raft.Up8Network),
                         head_gain=0.02).to(dev)
    net.train()
    freeze_batchnorm(net)
    opt = torch.optim.AdamW(net.parameters(), lr=4e-4, weight_decay=1e-4, eps=1e-8)
    ims = []
    for k in range(bsz):
        rng = np.random.default_rng(k)
        i1, i2, gt = frame_pair(h, w, flow=tuple(int(v) for v in rng.integers(0, 8, 2)), seed=k, pad=pad)
        hp, wp = i1.shape[-2:]
        f = np.zeros((1, 2, hp, wp), np.float32)
        f[:, :, :h, :w] = gt
        v = np.zeros((1, hp, wp), bool)
        v[:, :h, :w] = True
        ims.append((i1, i2, f, v))
    img1, img2, flow, valid = (torch.from_numpy(np.concatenate([x[i] for x in ims])).to(dev) for i in range(4))

    def step():
        opt.zero_grad(set_to_none=True)
        loss = mlseq_loss(net(img1, img2, (4, 3, 3)), flow, valid)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 1.0, norm_type=2.0)
        opt.step()

    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    time.sleep(1.5)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"train_probe: {(time.perf_counter() - t0) / steps * 1e3:.1f} ms per step ({steps} steps after {warm} warm-up)")


if __name__ == "__main__":
    main()
