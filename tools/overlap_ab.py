#!/usr/bin/env python3
"""Diagnostic: does running the bench step's batch as two half-batches on two HIP streams (each half's
GEMM + 12 lookups; the GEMM of one half can overlap the other half's lookups) beat the sequential
step?  cfg2 (B=8, 55x128, C=256), bench.py's synthetic inputs; median ms per step over reps, both
precisions.  usage: python3 tools/overlap_ab.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, "cuda")
    halves = [(f1[4 * s:4 * s + 4].contiguous(), f2[4 * s:4 * s + 4].contiguous(),
               coords[:, 4 * s:4 * s + 4].contiguous()) for s in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    res = {}
    for prec in ("bf16", "fp32"):
        def seq():
            pyr = ops.corr_pyramid(f1, f2, 4, prec)
            for it in range(12):
                ops.corr_lookup(pyr, coords[it], 4)

        def two():
            cur = torch.cuda.current_stream()
            for s, (a, b, co) in zip(streams, halves):
                s.wait_stream(cur)
            for s, (a, b, co) in zip(streams, halves):
                with torch.cuda.stream(s):
                    pyr = ops.corr_pyramid(a, b, 4, prec)
                    for it in range(12):
                        ops.corr_lookup(pyr, co[it], 4)
            for s in streams:
                cur.wait_stream(s)

        def half_seq():          # the two halves one after the other on one stream
            for a, b, co in halves:
                pyr = ops.corr_pyramid(a, b, 4, prec)
                for it in range(12):
                    ops.corr_lookup(pyr, co[it], 4)

        out = {}
        for name, fn in (("seq", seq), ("two_streams", two), ("halves_one_stream", half_seq)) * 2:
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                z.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(z))
            ts.sort()
            out.setdefault(name, []).append(round(ts[len(ts) // 2], 4))
        res[prec] = out
    print(json.dumps(res))


if __name__ == "__main__":
    main()
