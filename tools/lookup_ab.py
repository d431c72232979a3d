#!/usr/bin/env python3
"""A/B of the cfg2 lookup variants (RMD_LOOKUP_NT, read per launch: 0 plain, 1 non-temporal output
stores, 2 non-temporal pyramid loads, 3 both) on bench.py's synthetic inputs: 12 lookups per
round, HIP events around each lookup launch, variants interleaved; outputs compared bitwise with
variant 0.  A variant name "NT:PR" also sets RMD_LOOKUP_SPLIT=PR (output rows per lane).  usage: python tools/lookup_ab.py [rounds] -> JSON on stdout"""
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, dev)
    names = os.environ.get("RMD_AB", "0,1,2,3").split(",")
    pyr = ops.corr_pyramid(f1, f2, 4, "bf16")
    def select(n):
        nt, _, pr = n.partition(":")
        os.environ["RMD_LOOKUP_NT"] = nt
        os.environ["RMD_LOOKUP_SPLIT"] = pr or "9"

    select("0")
    ref = [ops.corr_lookup(pyr, coords[i], 4) for i in range(12)]
    res = {}
    for n in names:
        select(n)
        res[n] = {"bitwise_equal_v0": all(torch.equal(ops.corr_lookup(pyr, coords[i], 4), ref[i]) for i in range(12))}
    del ref
    times = {n: [] for n in names}
    for _ in range(rounds):
        for n in names:
            select(n)
            ev = []
            for i in range(12):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ops.corr_lookup(pyr, coords[i], 4)
                b.record()
                ev.append((a, b))
            torch.cuda.synchronize()
            times[n] += [a.elapsed_time(b) for a, b in ev]
    nbytes = 8 * 7040 * (4 * 100 * 2 + 4 * 81 * 4 + 8)
    for n in names:
        t = sorted(times[n])
        med = t[len(t) // 2]
        res[n].update(median_us=med * 1e3, min_us=t[0] * 1e3, frac_of_8TBps=nbytes / (med * 1e-3) / 8e12)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
