#!/usr/bin/env python3
"""Ablation of the unit-step DICL stack backward at cfg4 (B8 C32 48x160 r4): RMD_DICL_BWD_ABL =
0 full (default 2-pixel merged-row kernel with the cross-lane chain), nochain without the chain, px1 the 1-pixel kernel, px4 the 4-pixel merged kernel; on the 1-pixel kernel: 1 no window flush (global atomics), 2 no LDS atomics, 3 no gradient loads.  Times the
backward launch alone (rmd_dicl_stack_backward through the ctypes binding), HIP events, median.
Diagnostic only (ablated results are wrong).  usage: python tools/dicl_bwd_ablate.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import torch  # noqa: E402


def main():
    from rmd import _lib
    from rmd.ops import _ptr, _stream
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    b, c, h, w, r = 8, 32, 48, 160, 4
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    low = torch.randn(b, 2, h // 8, w // 8, generator=g) * 3.0
    flow = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=True)
    co = (torch.stack([xs, ys]).float()[None] + flow).to(dev).contiguous()
    gst = torch.randn(b, 9, 9, 2 * c, h, w, generator=g).to(dev)
    g1 = torch.empty(b, c, h, w, device=dev)
    g2 = torch.empty(b, c, h, w, device=dev)

    def fn():
        _lib.check(_lib.lib().rmd_dicl_stack_backward(_ptr(gst), _ptr(co), b, c, h, w, h, w, r, 0, h, w, 0,
                                                      _ptr(g1), _ptr(g2), _stream(gst)), "rmd_dicl_stack_backward")
    res = {}
    for v in ("px1", "nochain", "0", "px4", "1", "2", "3", "4", "0"):
        os.environ["RMD_DICL_BWD_PX"] = {"0": "0", "nochain": "0", "px4": "4"}.get(v, "1")     # ablations: 1-pixel kernel
        os.environ["RMD_DICL_BWD_CHAIN"] = "1" if v == "nochain" else "0"
        os.environ["RMD_DICL_BWD_ABL"] = v if v in ("1", "2", "3", "4") else "0"
        for _ in range(3):
            fn()
        ev = []
        for _ in range(reps):
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            z.record()
            ev.append((a, z))
        torch.cuda.synchronize()
        t = sorted(x.elapsed_time(y) for x, y in ev)
        res.setdefault(v, []).append(t[len(t) // 2])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
