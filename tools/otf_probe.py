#!/usr/bin/env python3
"""Runs the on-the-fly lookup at cfg2 (B=8, C=256, 55x128, 4 levels, r=4) `reps` times, for
rocprofv3 kernel traces / counter passes.  usage: python tools/otf_probe.py [reps] [precision]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import torch  # noqa: E402


def main():
    from rmd import ops
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    b, c, h, w = 8, 256, 55, 128
    f1 = torch.randn(b, c, h, w, generator=g).to(dev)
    f2 = torch.randn(b, c, h, w, generator=g).to(dev)
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    low = torch.randn(b, 2, h // 8, w // 8, generator=g) * 3.0
    flow = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=True)
    co = (torch.stack([xs, ys]).float()[None] + flow).to(dev)
    st = ops.otf_prepare(f1, f2, 4, prec)
    for _ in range(reps):
        ops.otf_lookup(st, co, 4)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
