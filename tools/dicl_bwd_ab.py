#!/usr/bin/env python3
"""A/B of the unit-step DICL stack backward kernels (diagnostic build; RMD_DICL_BWD_GM=2: backward4, the
one-column merge + cross-lane chain; 1: the general two-pixel merge without a chain; 0 / default: the
product, general merge + cross-lane chain) at cfg4 1/8 (B8 C32 48x160 r4) with smooth coordinates
(bench_components.smooth_coords) and with a steeper flow field.  Gradients of each variant are
compared with the first's; times are medians of HIP-event-timed forward+backward minus forward.
usage: python tools/dicl_bwd_ab.py [reps] -> JSON"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import torch  # noqa: E402


def med(fn, reps):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        z.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(z))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from rmd import ops
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    b, c, h, w, r = 8, 32, 48, 160, 4
    f1 = torch.randn(b, c, h, w, generator=g).to(dev).requires_grad_(True)
    f2 = torch.randn(b, c, h, w, generator=g).to(dev).requires_grad_(True)
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    res = {}
    for name, amp in (("smooth_amp3", 3.0), ("steep_amp8", 8.0)):
        low = torch.randn(b, 2, h // 8, w // 8, generator=g) * amp
        flow = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=True)
        co = (torch.stack([xs, ys]).float()[None] + flow).to(dev)
        gst = torch.randn(b, 9, 9, 2 * c, h, w, generator=g).to(dev)
        out = {}
        ref = None
        for v in ("2", "1", "0"):
            os.environ["RMD_DICL_BWD_GM"] = v

            def fb():
                return torch.autograd.grad(ops.dicl_stack(f1, f2, co, r), (f1, f2), gst)
            got = fb()
            if ref is None:
                ref = [t.clone() for t in got]
            err = max(float((x - y).abs().max() / y.abs().max()) for x, y in zip(got, ref))
            fwd = med(lambda: ops.dicl_stack(f1.detach(), f2.detach(), co, r), reps)
            out[v] = {"fwd_bwd_ms": med(fb, reps), "fwd_ms": fwd, "max_rel_err_vs_first": err}
            out[v]["bwd_ms"] = out[v]["fwd_bwd_ms"] - fwd
        os.environ.pop("RMD_DICL_BWD_GM", None)
        res[name] = out
        # raft_dicl_ml level 1 (fmap2 at 24x80, separable kernels): RMD_DICL_BWD_SEP2=2 one pixel per
        # lane, 0 / default two pixels per lane with merged + chained adds
        f2l = torch.randn(b, c, h // 2, w // 2, generator=g).to(dev).requires_grad_(True)
        outl, refl = {}, None
        for v in ("2", "0"):
            os.environ["RMD_DICL_BWD_SEP2"] = v

            def fbl():
                return torch.autograd.grad(ops.dicl_stack(f1, f2l, co, r, level=1, norm_hw=(h, w)), (f1, f2l), gst)
            got = fbl()
            if refl is None:
                refl = [t.clone() for t in got]
            err = max(float((x - y).abs().max() / y.abs().max()) for x, y in zip(got, refl))
            fwd = med(lambda: ops.dicl_stack(f1.detach(), f2l.detach(), co, r, level=1, norm_hw=(h, w)), reps)
            outl[v] = {"fwd_bwd_ms": med(fbl, reps), "fwd_ms": fwd, "max_rel_err_vs_first": err}
            outl[v]["bwd_ms"] = outl[v]["fwd_bwd_ms"] - fwd
        os.environ.pop("RMD_DICL_BWD_SEP2", None)
        res[name + "_ml_level1"] = outl
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
