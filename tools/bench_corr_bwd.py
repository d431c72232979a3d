#!/usr/bin/env python3
"""RAFT correlation forward + backward timing (training path, diagnostic; MI355X only).

rmd.raft.CorrBlock with feature maps that require gradients: the pyramid (GEMM + pooled epilogue),
12 lookups, then autograd: G of the 12 lookups written in one pass (rmd_corr_grad_build; with
RMD_GRAD_BUILD=0 the round-4 path: 12 rmd_corr_lookup_backward into a zeroed G), the pooled target
features, two GEMMs and the unpool kernel.  Shape: FlyingChairs 368x496 -> 46x62 (RAFT pads
modulo 8), C = 256, batch 6 (SURVEY.md §8(d) cfg5 batch), smooth moving coordinates.
usage: bench_corr_bwd.py [reps] [precision] [cfg5|cfg2]   -> one JSON document on stdout
(cfg2: bench.py's headline shape, 55x128, batch 8)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    import rmd
    from rmd import ops
    ops.GRAD_BUILD = os.environ.get("RMD_GRAD_BUILD", "1") != "0"
    ops.GRAD_BF16 = os.environ.get("RMD_GRAD_BF16", "1") != "0"
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    shape = sys.argv[3] if len(sys.argv) > 3 else "cfg5"
    dev = torch.device("cuda", 0)
    b, c, h, w = (8, 256, 55, 128) if shape == "cfg2" else (6, 256, 46, 62)
    f1, f2, coords = bench.synthetic(b, c, h, w, 12, 1234, dev)
    f1.requires_grad_(True)
    f2.requires_grad_(True)
    g = torch.Generator(device="cpu").manual_seed(3)
    gos = [torch.randn(b, 324, h, w, generator=g).to(dev) for _ in range(12)]

    def fwd():
        cb = rmd.raft.CorrBlock(f1, f2, 4, 4, precision=prec)
        return sum((cb(coords[i]) * gos[i]).sum() for i in range(12))

    def run(fn, n):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / n

    def fwd_only():
        cb = rmd.raft.CorrBlock(f1.detach(), f2.detach(), 4, 4, precision=prec)
        return [cb(coords[i]) for i in range(12)]

    def fwd_outs():
        cb = rmd.raft.CorrBlock(f1, f2, 4, 4, precision=prec)
        return [cb(coords[i]) for i in range(12)]

    with torch.no_grad():
        t_f = run(fwd_only, reps)
    t_fb = run(lambda: torch.autograd.grad(fwd(), (f1, f2)), reps)
    # the same backward driven by the 12 upstream gradients directly (no torch loss multiply / sum /
    # their backward): the correlation block's own backward kernels
    t_fb2 = run(lambda: torch.autograd.grad(fwd_outs(), (f1, f2), gos), reps)
    print(json.dumps({"shape": f"B{b} C{c} {h}x{w}, 12 lookups", "precision": prec,
                      "grad_build": ops.GRAD_BUILD, "grad_bf16": ops.GRAD_BF16,
                      "forward_ms": t_f,
                      "forward_backward_ms": t_fb, "backward_ms": t_fb - t_f,
                      "backward_ms_from_grad_out": t_fb2 - t_f,
                      "note": "backward_ms: forward_backward includes the loss multiply-adds (torch); "
                              "backward_ms_from_grad_out: autograd.grad(outputs, inputs, grad_outputs)"}))


if __name__ == "__main__":
    main()
