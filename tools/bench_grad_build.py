#!/usr/bin/env python3
"""rmd_corr_grad_build alone at cfg2 b8 (55x128, 4 levels, r = 4): 12 lookups (bench.synthetic's
smooth moving coordinates), 0 lookups (the kernel's store stream alone), and the round-4 path (zero
fill + 12 rmd_corr_lookup_backward).  Diagnostic; MI355X only.  -> JSON lines on stdout"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from rmd import _lib as L
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = L.lib()
    b, h, w, levels, r, n = 8, 55, 128, 4, 4, 12
    dev = torch.device("cuda", 0)
    _, _, coords = bench.synthetic(b, 8, h, w, n, 1234, dev)
    g = torch.Generator(device="cpu").manual_seed(3)
    gos = [torch.randn(b, levels * 81, h, w, generator=g).to(dev) for _ in range(n)]
    d = L.PyramidDesc()
    L.check(lib.rmd_pyramid_describe(b, h, w, levels, L.RMD_F32, ctypes.byref(d)), "describe")
    t = lib.rmd_corr_grad_targets(h, w, levels)
    G = torch.empty(b * h * w * t, dtype=torch.float32, device=dev)
    cos = [coords[i].contiguous() for i in range(n)]

    def build(k):
        gp = (ctypes.c_void_p * max(k, 1))(*[x.data_ptr() for x in gos[:k]])
        cp = (ctypes.c_void_p * max(k, 1))(*[x.data_ptr() for x in cos[:k]])
        L.check(lib.rmd_corr_grad_build(gp, cp, None, k, ctypes.byref(d), r, 0, ctypes.c_void_p(G.data_ptr()),
                                        None), "build")

    def seq():
        G.zero_()
        for i in range(n):
            L.check(lib.rmd_corr_lookup_backward(ctypes.c_void_p(gos[i].data_ptr()), ctypes.byref(d),
                                                 ctypes.c_void_p(cos[i].data_ptr()), r, 0,
                                                 ctypes.c_void_p(G.data_ptr()), None), "seq")

    def timed(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    gb = G.numel() * 4
    for name, fn in (("build12", lambda: build(n)), ("build0", lambda: build(0)), ("sequential", seq)):
        us = timed(fn)
        print(json.dumps({"case": name, "us": round(us, 1), "G_GB": round(gb / 1e9, 3),
                          "G_write_TBps": round(gb / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
