#!/usr/bin/env python3
"""Generate the end-to-end RAFT fixture by RUNNING the reference model (build container only).

Test infrastructure.  Builds the reference raft/baseline RaftModule (src/models/impls/raft.py:334,
defaults of cfg/model/raft-baseline.yaml), fills it with detinit.det_init_fanin (name-keyed, seeded — the
GPU test regenerates the same weights on its own copy of the architecture), runs 12 GRU iterations in
eval mode on the synthetic Sintel-shape pair of synth.frame_pair (436x1024 -> padded 440x1024) and
stores only numbers: mean EPE vs the known flow after every iteration and the flow at 4096 fixed
pixels after iterations 1, 4 and 12.  The reference itself never travels.

usage: python tests/golden/gen_e2e.py   (writes tests/golden/e2e_raft_436x1024.npz)
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from detinit import det_init_fanin  # noqa: E402
from gen_golden import _import_reference  # noqa: E402
from synth import epe, frame_pair  # noqa: E402

H, W, ITERS, SAMPLES = 436, 1024, 12, 4096
KEEP = (1, 4, 12)


def sample_pixels(h, w, n, seed=7):
    rng = np.random.Generator(np.random.PCG64(seed))
    return np.sort(rng.choice(h * w, n, replace=False))


def main():
    import torch
    _import_reference()
    from src.models.impls import raft
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count() or 8)
    model = det_init_fanin(raft.RaftModule()).eval()
    img1, img2, gt = frame_pair(H, W)
    with torch.no_grad():
        flows = model(torch.from_numpy(img1), torch.from_numpy(img2), iterations=ITERS)
    sel = sample_pixels(H, W, SAMPLES)
    arrays = dict(height=np.int32(H), width=np.int32(W), iterations=np.int32(ITERS), pixels=sel,
                  epe=np.asarray([epe(f.numpy(), gt) for f in flows]),
                  keys=np.asarray(sorted(model.state_dict().keys())))
    for k in KEEP:
        f = flows[k - 1].numpy()[0, :, :H, :W].reshape(2, -1)
        assert np.isfinite(f).all()
        arrays[f"flow_it{k}"] = f[:, sel].astype(np.float32)
    path = os.path.join(HERE, "e2e_raft_436x1024.npz")
    np.savez_compressed(path, **arrays)
    print(path, os.path.getsize(path), "bytes; EPE per iteration:", np.round(arrays["epe"], 4).tolist())


if __name__ == "__main__":
    main()
