#!/usr/bin/env python3
"""Diagnostic: compare the x3 GEMM's S24 pyramid with its F32 pyramid rounded on the host, level by level,
and print where they differ (positions decoded as (image, query, level row, level col)).  Also probes
v_permlane16_swap / v_permlane32_swap lane semantics through a tiny HIP kernel if tools/_ab/perm_probe exists.
usage: python3 tools/s24_debug.py [b c h w]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import rmd
    from rmd import library
    b, c, h, w = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (2, 32, 24, 40)
    rng = np.random.default_rng(0)
    f1 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    f2 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    p24 = rmd.ops.corr_pyramid(f1, f2, 4, "fp32-s24")
    p32 = rmd.ops.corr_pyramid(f1, f2, 4, "fp32-f32")
    for i in range(4):
        got = p24.unpack(i)
        ref = library.s24_decode(library.s24_encode(p32.unpack(i)))
        shp = tuple(got.shape)
        g = got.view(torch.int32).cpu().numpy().reshape(b, h * w, -1)
        r = ref.view(torch.int32).cpu().numpy().reshape(b, h * w, -1)
        bad = np.argwhere(g != r)
        print(f"level {i} shape {shp}: {len(bad)} of {g.size} differ")
        lh, lw = p24.desc.level_h[i], p24.desc.level_w[i]
        for bi, q, t in bad[:12]:
            gv = np.frombuffer(np.int32(g[bi, q, t]).tobytes(), np.float32)[0]
            rv = np.frombuffer(np.int32(r[bi, q, t]).tobytes(), np.float32)[0]
            print(f"   img {bi} query {q} (y{q // w} x{q % w}) target ({t // lw},{t % lw}) got {gv:.6g} ref {rv:.6g}")
        if len(bad):
            ys, xs = bad[:, 2] // lw, bad[:, 2] % lw
            print("   bad target rows", np.unique(ys)[:20], "cols", np.unique(xs)[:40])
            print("   bad queries mod 32", np.unique(bad[:, 1] % 32)[:40])


if __name__ == "__main__":
    main()
