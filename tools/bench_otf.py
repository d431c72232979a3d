#!/usr/bin/env python3
"""On-the-fly (raft/fs) path vs the all-pairs volume: forward (12 lookups) and training (forward +
backward of 12 lookups) at cfg2 (B=8, 55x128, C=256) and inference at a 4K 1/8 map (270x480, C=256, B=2),
HIP-event timed.  Prints one JSON object.  bench.py's 'highres_fs' key runs the 4K leg.

usage: python3 tools/bench_otf.py [--reps 5] [--skip-4k] [--precision bf16]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        z = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        z.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(z))
    return float(np.median(ms))


def inputs(b, c, h, w, iters, seed=1234):
    import bench
    return bench.synthetic(b, c, h, w, iters, seed, "cuda")


def infer(method, precision, f1, f2, coords, levels=4, radius=4):
    import rmd
    with torch.no_grad():
        cb = rmd.raft_fs.CorrBlock(f1, f2, levels, radius, precision=precision, method=method)
        out = None
        for co in coords:
            out = cb(co)
    return out


def train(method, precision, f1, f2, coords, gouts, levels=4, radius=4):
    import rmd
    t1 = f1.detach().requires_grad_(True)
    t2 = f2.detach().requires_grad_(True)
    cb = rmd.raft_fs.CorrBlock(t1, t2, levels, radius, precision=precision, method=method)
    loss = 0
    for co, go in zip(coords, gouts):
        loss = loss + (cb(co) * go).sum()
    return torch.autograd.grad(loss, (t1, t2))


def highres(precision, reps, b=2, h=270, w=480, c=256, iters=12):
    """4K frame (2160x3840 -> 1/8 map 270x480): on-the-fly vs volume inference, 12 lookups."""
    import rmd
    f1, f2, coords = inputs(b, c, h, w, iters)
    res = {"map": f"{h}x{w}", "batch": b, "channels": c, "iterations": iters, "precision": precision,
           "volume_bytes": rmd.config.volume_bytes(b, h, w, 4, precision, False)}
    res["otf_ms"] = timed(lambda: infer("otf", precision, f1, f2, coords), reps)
    try:
        res["volume_ms"] = timed(lambda: infer("volume", precision, f1, f2, coords), max(2, reps // 2), warm=1)
        res["otf_speedup"] = res["volume_ms"] / res["otf_ms"]
    except (RuntimeError, torch.cuda.OutOfMemoryError) as e:      # noqa: BLE001
        res["volume_error"] = f"{type(e).__name__}: {e}"[:300]
    torch.cuda.empty_cache()
    res["otf_frame_pairs_per_s"] = b * 1e3 / res["otf_ms"]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--skip-4k", action="store_true")
    ap.add_argument("--cfg2-off", action="store_true", help="only the 4K leg")
    a = ap.parse_args()
    out = {}
    if a.cfg2_off:
        out["highres_4k"] = highres(a.precision, a.reps)
        print(json.dumps(out, indent=1))
        return
    b, c, h, w, iters = 8, 256, 55, 128, 12
    f1, f2, coords = inputs(b, c, h, w, iters)
    g = torch.Generator(device="cpu").manual_seed(5)
    gouts = [torch.randn(b, 324, h, w, generator=g).cuda() for _ in range(iters)]
    for p in (a.precision, "fp32"):
        r = {}
        r["otf_forward_ms"] = timed(lambda: infer("otf", p, f1, f2, coords), a.reps)
        r["volume_forward_ms"] = timed(lambda: infer("volume", p, f1, f2, coords), a.reps)
        r["otf_train_ms"] = timed(lambda: train("otf", p, f1, f2, coords, gouts), a.reps)
        r["volume_train_ms"] = timed(lambda: train("volume", p, f1, f2, coords, gouts), a.reps)
        r["otf_backward_ms"] = r["otf_train_ms"] - r["otf_forward_ms"]
        r["volume_backward_ms"] = r["volume_train_ms"] - r["volume_forward_ms"]
        out[f"cfg2_b8_{p}"] = r
        torch.cuda.empty_cache()
    if not a.skip_4k:
        del f1, f2, coords, gouts
        torch.cuda.empty_cache()
        out["highres_4k"] = highres(a.precision, a.reps)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
