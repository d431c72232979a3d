#!/usr/bin/env python3
"""Cache-line model of the lookup's pyramid reads (CPU only): for bench.py's cfg2 synthetic coords
(iteration 0), count the distinct 128-B lines of the query-minor row-chunk layout (rmd.h) that the
in-map part of every radius-4 window touches, per level, for chunk widths CW and an optional per-query
column skew s(l) = (l >> L) (l = query index within a line's query group, L = level) — the layout
alternative DESIGN.md §4 weighs.  The unskewed (8, 8, 4, 2) row reproduces the measured read bytes
(65.9 MB modelled vs 67.9 MB FETCH_SIZE, profiles/pmc_r01.json).
usage: python tools/lookup_line_model.py -> one line per variant"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

H, W, B, R = 55, 128, 8, 4
N = H * W
LEVELS = [(55, 128), (27, 64), (13, 32), (6, 16)]


def model(coords, cws, skew, line=128, esz=2):
    lines, need = [], []
    for lvl, (lh, lw) in enumerate(LEVELS):
        cw = cws[lvl]
        qpl = line // (cw * esz)                       # queries sharing one line of a chunk
        x = coords[:, 0].reshape(B, N) / 2 ** lvl
        y = coords[:, 1].reshape(B, N) / 2 ** lvl
        x0 = np.floor(x).astype(np.int64) - R
        y0 = np.floor(y).astype(np.int64) - R
        q = np.arange(N)
        s = (q % qpl >> lvl) * skew[lvl]
        bb = np.broadcast_to(np.arange(B)[:, None], (B, N))
        keys, nd = [], 0
        for j in range(2 * R + 2):
            yy = y0 + j
            for k in range(2 * R + 2):
                tx = x0 + k
                ok = (yy >= 0) & (yy < lh) & (tx >= 0) & (tx < lw)
                nd += int(ok.sum()) * esz
                ch = (tx - s[None, :] + 64) // cw
                keys.append((((bb * 64 + yy) * 400 + ch) * N * 2 + (q // qpl)[None, :])[ok])
        lines.append(len(np.unique(np.concatenate(keys))) * line / 1e6)
        need.append(nd / 1e6)
    return lines, need


def main():
    _, _, coords = bench.synthetic(B, 4, H, W, 12, 1234, "cpu")
    c = coords[0].numpy()
    for cws in [(8, 8, 4, 2), (4, 4, 4, 2)]:
        for skew in [(0, 0, 0, 0), (1, 0, 0, 0), (1, 1, 1, 0)]:
            lines, need = model(c, cws, skew)
            print(f"chunks {cws} skew {skew}: lines {sum(lines):.1f} MB {[round(v, 1) for v in lines]}, "
                  f"in-map bytes {sum(need):.1f} MB")


if __name__ == "__main__":
    main()
