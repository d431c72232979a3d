#!/usr/bin/env python3
"""A/B of cfg2 lookup variants on bench.py's synthetic inputs (diagnostic build: run with
RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so).  RMD_AB is a comma-separated list of variants,
each a '+'-joined list of NAME=VALUE settings of RMD_LOOKUP_<NAME> (e.g. "XCH=1,XCH=0",
"XCH=0+SPLIT=9"); unset knobs take the product default.  12 lookups per round with HIP events
around each launch, variants interleaved; outputs compared bitwise with the first variant.
usage: python tools/lookup_ab.py [rounds] [precision] -> JSON on stdout"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402

KNOBS = ("XCH", "NT", "SPLIT", "V")      # RMD_LOOKUP_<KNOB>; a name starting with RMD_ is set verbatim (RMD_ABLATE)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    precision = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, dev)
    names = os.environ.get("RMD_AB", "XCH=1,XCH=0").split(",")
    pyr = ops.corr_pyramid(f1, f2, 4, precision)
    if os.environ.get("LOOKUP_AB_SAME"):        # every lookup at iteration 6's coordinates (cache reuse bound)
        coords = coords[6:7].expand(12, -1, -1, -1, -1).contiguous()

    def select(n):
        for k in KNOBS:
            os.environ.pop("RMD_LOOKUP_" + k, None)
        os.environ.pop("RMD_ABLATE", None)
        for kv in filter(None, n.split("+")):
            k, v = kv.split("=")
            os.environ[k if k.startswith("RMD_") else "RMD_LOOKUP_" + k] = v

    select(names[0])
    ref = [ops.corr_lookup(pyr, coords[i], 4) for i in range(12)]
    res = {}
    for n in names:
        select(n)
        outs = [ops.corr_lookup(pyr, coords[i], 4) for i in range(12)]
        res[n] = {"bitwise_equal_first": all(torch.equal(o, r) for o, r in zip(outs, ref)),
                  "max_abs_diff_first": max(float((o - r).abs().max()) for o, r in zip(outs, ref))}
        del outs
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
    esz = pyr.data.element_size()
    nbytes = 8 * 7040 * (4 * 100 * esz + 4 * 81 * 4 + 8)
    for n in names:
        t = sorted(times[n])
        med = t[len(t) // 2]
        res[n].update(median_us=med * 1e3, min_us=t[0] * 1e3, frac_of_8TBps=nbytes / (med * 1e-3) / 8e12)
    print(json.dumps({"precision": precision, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
