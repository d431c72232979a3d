#!/usr/bin/env python3
"""A/B of the DICL volume kernel variants (RMD_DICL_PATCH / RMD_DICL_GENERAL / RMD_DICL_INT, read per launch) at the
BASELINE shapes: a6 rmd_dicl_stack at cfg4 1/8 (B8 C32 48x160 r4), a7 its raft_dicl_ml level-1 form (f2 at 24x80), a8 rmd_dicl_stack_int at cfg3
level 2 (B8 C32 96x128 ru=rv=3).  Each variant's output is compared bitwise with variant 1's (the
previous formulation); times are medians of HIP-event-timed launches, interleaved over rounds.
usage: python tools/dicl_ab.py [reps] [name filter] -> one JSON document on stdout"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import torch  # noqa: E402


def med_ms(fn, reps):
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def main():
    from rmd import ops
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {}
    cases = []
    b, c, h, w, r = 8, 32, 48, 160, 4
    f1 = torch.randn(b, c, h, w, generator=g).to(dev)
    f2 = torch.randn(b, c, h, w, generator=g).to(dev)
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    low = torch.randn(b, 2, h // 8, w // 8, generator=g) * 3.0
    flow = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=True)
    co = (torch.stack([xs, ys]).float()[None] + flow).to(dev)
    nb = b * 81 * 2 * c * h * w * 4 + 2 * f1.numel() * 4 + co.numel() * 4
    out = torch.empty(b, 9, 9, 2 * c, h, w, device=dev)
    cases.append(("a6_stack_cfg4", "RMD_DICL_PATCH", ["1", "0", "2", "3", "4", "5"], lambda: ops.dicl_stack(f1, f2, co, r), nb))
    f2l = torch.randn(b, c, h // 2, w // 2, generator=g).to(dev)
    cases.append(("a7_ml_level1_cfg4", "RMD_DICL_GENERAL", ["1", "3", "0"],
                  lambda: ops.dicl_stack(f1, f2l, co, r, level=1, norm_hw=(h, w)), nb - f2.numel() * 3))
    b3, c3, h3, w3 = 8, 32, 96, 128
    g1 = torch.randn(b3, c3, h3, w3, generator=g).to(dev)
    g2 = torch.randn(b3, c3, h3, w3, generator=g).to(dev)
    g2[:, :, 10:20, 30:40] = 0
    nb3 = b3 * 49 * 2 * c3 * h3 * w3 * 4 + 2 * g1.numel() * 4
    cases.append(("a8_int_cfg3", "RMD_DICL_INT", ["1", "0", "2", "3", "4"], lambda: ops.dicl_stack_int(g1, g2, 3, 3), nb3))
    del out
    # backward (training): forward+backward minus forward; window variants (atomics: compare allclose)
    f1g, f2g, f2lg = (t.clone().requires_grad_(True) for t in (f1, f2, f2l))
    gst = torch.randn(b, 9, 9, 2 * c, h, w, generator=g).to(dev)

    def bwd6():
        return torch.autograd.grad(ops.dicl_stack(f1g, f2g, co, r), (f1g, f2g), gst)

    def bwd7():
        return torch.autograd.grad(ops.dicl_stack(f1g, f2lg, co, r, level=1, norm_hw=(h, w)), (f1g, f2lg), gst)
    only = sys.argv[2] if len(sys.argv) > 2 else ""
    cases = [cs for cs in cases if only in cs[0]]
    for name, fn in (("a6_backward_cfg4", bwd6), ("a7_backward_cfg4", bwd7)):
        if only not in name:
            continue
        out = {}
        os.environ["RMD_DICL_BWD_WIN"] = "1"
        ref = [t.clone() for t in fn()]
        tt = {"1": [], "0": []}
        for _ in range(3):
            for v in ("1", "0"):
                os.environ["RMD_DICL_BWD_WIN"] = v
                fn()
                tt[v].append(med_ms(fn, reps))
        for v in ("1", "0"):
            os.environ["RMD_DICL_BWD_WIN"] = v
            got = fn()
            err = max(float((a - b_).abs().max() / b_.abs().max()) for a, b_ in zip(got, ref))
            out[v] = dict(fwd_bwd_ms=min(tt[v]), all_ms=tt[v], max_rel_err_vs_v1=err)
        os.environ.pop("RMD_DICL_BWD_WIN", None)
        res[name] = out
        del ref
    del gst, f1g, f2g, f2lg
    torch.cuda.empty_cache()
    for name, env, variants, fn, nbytes in cases:
        os.environ[env] = "1"
        ref = fn().clone()
        times = {v: [] for v in variants}
        same = {}
        for v in variants:
            os.environ[env] = v
            o = fn()
            torch.cuda.synchronize()
            same[v] = bool(torch.equal(o, ref)) or float((o - ref).abs().max() / ref.abs().max())
            del o
        for _ in range(3):
            for v in variants:
                os.environ[env] = v
                for _ in range(2):
                    fn()
                times[v].append(med_ms(fn, reps))
        os.environ.pop(env, None)
        res[name] = {v: dict(ms=min(times[v]), all_ms=times[v], GBps=nbytes / (min(times[v]) * 1e-3) / 1e9,
                             frac_of_8TBps=nbytes / (min(times[v]) * 1e-3) / 8e12, bitwise_equal_v1_or_max_rel_err=same[v])
                     for v in variants}
        del ref
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
