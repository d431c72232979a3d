#!/usr/bin/env python3
"""MFMA work the on-the-fly lookup (csrc/corr_otf.hip) issues at cfg2 for bench.py's synthetic coordinates
(CPU only): per query block of QSX x QSY 16-query segments and level, the box of its queries' windows
clipped to the map and widened to 16-target segments; every (box target segment, query segment) pair is
one 16x16 MFMA tile of C = 256 channels.  Compared with the algorithmic work (each query's in-map
(2r+2)^2 window).  usage: python tools/otf_work_model.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

B, C, H, W, R = 8, 256, 55, 128, 4
K = 2 * R + 2


def work(coords, qsx, qsy, levels=4):
    tiles, need = 0, 0
    bx, by = 16 * qsx, qsy
    for L in range(levels):
        lh, lw = H >> L, W >> L
        x = np.floor(coords[:, 0] / 2 ** L).astype(np.int64) - R
        y = np.floor(coords[:, 1] / 2 ** L).astype(np.int64) - R
        for b in range(B):
            for qy0 in range(0, H, by):
                for qx0 in range(0, W, bx):
                    xs, ys = x[b, qy0:qy0 + by, qx0:qx0 + bx], y[b, qy0:qy0 + by, qx0:qx0 + bx]
                    x0, x1 = max(xs.min(), 0), min(xs.max() + K - 1, lw - 1)
                    y0, y1 = max(ys.min(), 0), min(ys.max() + K - 1, lh - 1)
                    if x1 < x0 or y1 < y0:
                        continue
                    nseg = (x1 >> 4) - (x0 >> 4) + 1
                    tiles += (y1 - y0 + 1) * nseg * qsx * qsy
                    inx = np.clip(np.minimum(xs + K, lw) - np.maximum(xs, 0), 0, None)
                    iny = np.clip(np.minimum(ys + K, lh) - np.maximum(ys, 0), 0, None)
                    need += int((inx * iny).sum())
    return tiles * 16 * 16 * C * 2, need * C * 2


def main():
    _, _, co = bench.synthetic(B, 4, H, W, 12, 1234, "cpu")
    c = co[5].numpy()
    for qsx, qsy in ((1, 1), (1, 2), (2, 1), (1, 4), (2, 2)):
        issued, algo = work(c, qsx, qsy)
        print(f"block {16 * qsx}x{qsy}: issued {issued / 1e9:.1f} GFLOP (bf16 MFMA), algorithmic {algo / 1e9:.2f} GFLOP, "
              f"x{issued / algo:.1f}; at 2.5 PF: {issued / 2.5e15 * 1e6:.1f} us (bf16) / {3 * issued / 2.5e15 * 1e6:.1f} us (x3)")


if __name__ == "__main__":
    main()
