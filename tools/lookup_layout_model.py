#!/usr/bin/env python3
"""Cache-line model of the lookup's pyramid reads for candidate query-minor layouts (CPU only).

For bench.py's cfg2 synthetic coords (iteration 0, B=8, 55x128, r=4), counts the distinct 128-B lines
that the in-map part of every query's radius-4 window touches, per level, for a layout given by
  * the query slot order (raster, or the tiles order of include/rmd.h), and
  * per level a target chunk shape th x tw (fp16): a line holds 128 / (2 th tw) consecutive slots'
    chunks of one chunk position.
The tiles layout row reproduces the measured FETCH traffic within a few % (58.3 MB measured,
profiles/lookup_layout_ab_r03.json).  usage: python tools/lookup_layout_model.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import bench  # noqa: E402

H, W, B, R = 55, 128, 8, 4
N = H * W
LEVELS = [(55, 128), (27, 64), (13, 32), (6, 16)]


def tiles_slots():
    y1, x1 = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    qx, hp = (W + 15) // 16, H // 2
    s = ((y1 // 2) * qx + x1 // 16) * 32 + ((x1 % 16) // 4) * 8 + (y1 % 2) * 4 + x1 % 4
    s = np.where(y1 < 2 * hp, s, hp * qx * 32 + x1)
    return s.reshape(-1)


def model(coords, slot, chunks, line=128, esz=2):
    lines, need = [], []
    bb = np.arange(B)[:, None]
    for lvl, (lh, lw) in enumerate(LEVELS):
        th, tw = chunks[lvl]
        spl = line // (th * tw * esz)                  # slots per line
        x = coords[:, 0].reshape(B, N) / 2 ** lvl
        y = coords[:, 1].reshape(B, N) / 2 ** lvl
        x0 = np.floor(x).astype(np.int64) - R
        y0 = np.floor(y).astype(np.int64) - R
        grp = (slot // spl)[None, :]
        keys, nd = [], 0
        for j in range(2 * R + 2):
            yy = y0 + j
            for k in range(2 * R + 2):
                tx = x0 + k
                ok = (yy >= 0) & (yy < lh) & (tx >= 0) & (tx < lw)
                nd += int(ok.sum()) * esz
                pos = ((bb * 64 + yy // th) * 256 + tx // tw)
                keys.append((pos * (N + 64) + grp)[ok])
        lines.append(len(np.unique(np.concatenate(keys))) * line / 1e6)
        need.append(nd / 1e6)
    return lines, need


def main():
    _, _, coords = bench.synthetic(B, 4, H, W, 12, 1234, "cpu")
    c = coords[0].numpy()
    raster, tiles = np.arange(N), tiles_slots()
    variants = [
        ("rows (round 2)", raster, [(1, 8), (1, 8), (1, 4), (1, 2)]),
        ("tiles (product)", tiles, [(2, 4), (2, 4), (1, 4), (1, 2)]),
        ("tiles, 2x4 on level 2", tiles, [(2, 4), (2, 4), (2, 4), (1, 2)]),
        ("tiles, 2x4 on levels 2-3", tiles, [(2, 4), (2, 4), (2, 4), (2, 4)]),
        ("tiles, 2x2 on level 2, 2x2 level 3", tiles, [(2, 4), (2, 4), (2, 2), (2, 2)]),
        ("tiles, 4x4 levels 0-1", tiles, [(4, 4), (4, 4), (1, 4), (1, 2)]),
        ("tiles, 2x8 levels 0-1", tiles, [(2, 8), (2, 8), (1, 4), (1, 2)]),
        ("tiles, 4x2 levels 0-1", tiles, [(4, 2), (4, 2), (1, 4), (1, 2)]),
        ("tiles, 4x2 levels 0-2, 2x2 level 3", tiles, [(4, 2), (4, 2), (4, 2), (2, 2)]),
    ]
    for name, slot, chunks in variants:
        lines, need = model(c, slot, chunks)
        print(f"{name:38s} chunks {chunks}: lines {sum(lines):5.1f} MB {[round(v, 1) for v in lines]}, "
              f"in-map {sum(need):.1f} MB {[round(v, 1) for v in need]}")


if __name__ == "__main__":
    main()
