#!/usr/bin/env python3
"""Model-level context for the headline: RAFT 12-iteration inference at 436x1024 (padded 440x1024),
batch 8, on one MI355X — the whole network (encoders, GRU, heads) with
  * ref      : the reference's eager-torch correlation (raft.py:15-95 restated: matmul / sqrt(C),
               avg_pool2d pyramid, grid_sample lookup) and eager convex upsampling (raft.py:319-331)
  * rmd_fp32 : rmd.raft.CorrBlock (exact-fp32 MFMA, fp32 pyramid) + rmd.raft.Up8Network
  * rmd_bf16 : rmd.raft.CorrBlock (bf16 MFMA, fp16 pyramid) + rmd.raft.Up8Network
Convolutions are MIOpen fp32 in all three (TF32 off).  Synthetic smooth frame pair, name-keyed random
weights (tests/golden/detinit), no dataset.  Not the bench.py metric (that times the §8 hot path
alone); this shows what the hot path is worth inside the model.
usage: python tools/bench_e2e.py [reps] [batch]  -> one JSON document on stdout
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "raft-meets-dicl_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    import rmd
    from detinit import det_init_fanin
    from e2e.raft_net import RaftNet
    from e2e.eager_corr import EagerCorrBlock
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    h, w = 440, 1024
    g = torch.Generator().manual_seed(1234)
    low = torch.rand(b, 3, h // 8, w // 8, generator=g) * 2 - 1
    img1 = F.interpolate(low, size=(h, w), mode="bilinear", align_corners=True)
    img2 = torch.roll(img1, shifts=(3, 5), dims=(2, 3))
    img1, img2 = img1.cuda(), img2.cuda()
    variants = {"ref": (EagerCorrBlock, None, "fp32"),
                "rmd_fp32": (rmd.raft.CorrBlock, rmd.raft.Up8Network, "fp32"),
                "rmd_bf16": (rmd.raft.CorrBlock, rmd.raft.Up8Network, "bf16")}
    res = {"config": {"image": "436x1024 padded 440x1024", "batch": b, "iterations": 12, "convs": "MIOpen fp32",
                      "data": "synthetic smooth pair, random name-keyed weights"}}
    flows = {}
    for name, (cb, up, prec) in variants.items():
        net = det_init_fanin(RaftNet(cb, precision=prec, upnet_cls=up)).eval().cuda()
        with torch.no_grad():
            for _ in range(2):
                out = net(img1, img2, 12)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                out = net(img1, img2, 12)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / reps
        flows[name] = out[-1]
        res[name] = {"ms_per_batch": ms, "frame_pairs_per_s": b * 1e3 / ms}
        del net, out
        torch.cuda.empty_cache()
    for name in ("rmd_fp32", "rmd_bf16"):
        res[name]["speedup_vs_ref"] = res["ref"]["ms_per_batch"] / res[name]["ms_per_batch"]
        res[name]["max_abs_flow_diff_vs_ref_px"] = float((flows[name] - flows["ref"]).abs().max())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
