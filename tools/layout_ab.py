#!/usr/bin/env python3
"""Same-box A/B of the lookup over the two fp16 pyramid layouts (include/rmd.h): the w8 GEMM's tiles
layout vs the row layout holding the SAME fp16 values (repacked on the device from the tiles pyramid),
12 cfg2 lookups per round on bench.py's synthetic coordinates, layouts interleaved, HIP events around
each launch; outputs must be bitwise equal.  Under rocprofv3 --kernel-trace the two kernels are told
apart by their LAY template argument (corr_lookup_kernel<__half, 4, 3, 0|1>).
usage: python tools/lookup_layout_ab.py [rounds] -> JSON on stdout"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import _lib, library, ops  # noqa: E402


def pack_rows(pyr_tiles):
    """The tiles pyramid's values in the row layout (rmd_pyramid_describe, fp16)."""
    d = pyr_tiles.desc
    dr = library.describe(d.batch, d.height, d.width, d.levels, _lib.RMD_F16)
    data = torch.zeros(dr.total_elements, dtype=torch.float16, device=pyr_tiles.data.device)
    b, n = d.batch, d.height * d.width
    for i in range(d.levels):
        lv = pyr_tiles.unpack(i).reshape(b, n, dr.level_h[i], dr.level_w[i]).half()
        cw, nc, hl, wl = dr.tile_w[i], dr.tiles_x[i], dr.level_h[i], dr.level_w[i]
        full = torch.zeros(b, n, hl, nc * cw, dtype=torch.float16, device=data.device)
        full[..., :wl] = lv
        off = dr.level_offset[i]
        data[off: off + b * hl * nc * n * cw] = full.view(b, n, hl, nc, cw).permute(0, 2, 3, 1, 4).reshape(-1)
    return ops.Pyramid(data, dr, pyr_tiles.channels, pyr_tiles.scale)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, dev)
    pt = ops.corr_pyramid(f1, f2, 4, "bf16")
    assert pt.desc.layout == _lib.RMD_LAYOUT_TILES
    pr = pack_rows(pt)
    pyrs = {"tiles": pt, "rows": pr}
    ref = [ops.corr_lookup(pt, coords[i], 4) for i in range(12)]
    res = {}
    for k, p in pyrs.items():
        outs = [ops.corr_lookup(p, coords[i], 4) for i in range(12)]
        res[k] = {"bitwise_equal_tiles": all(torch.equal(o, r) for o, r in zip(outs, ref))}
    del ref, outs
    times = {k: [] for k in pyrs}
    for _ in range(rounds):
        for k, p in pyrs.items():
            ev = []
            for i in range(12):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ops.corr_lookup(p, coords[i], 4)
                b.record()
                ev.append((a, b))
            torch.cuda.synchronize()
            times[k] += [a.elapsed_time(b) for a, b in ev]
    nbytes = 118497280
    for k in pyrs:
        t = sorted(times[k])
        med = t[len(t) // 2]
        res[k].update(median_us=med * 1e3, min_us=t[0] * 1e3, frac_of_8TBps=nbytes / (med * 1e-3) / 8e12)
    print(json.dumps({"cfg": "cfg2 b8 bf16 pyramid values, r=4, 12 lookups per round", "rounds": rounds,
                      "layouts": res}, indent=1))


if __name__ == "__main__":
    main()
