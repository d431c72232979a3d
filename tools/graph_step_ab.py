#!/usr/bin/env python3
"""A/B of the bench step (prep + GEMM/pyramid + 12 lookups, cfg2 b8 bf16) launched eagerly vs
replayed from a HIP graph captured with torch.cuda.graph (the rmd ops launch on torch's current
stream, so they are captured).  Same inputs, outputs compared bitwise.  Measures how much of the
step is launch overhead.  usage: python tools/graph_step_ab.py [rounds] -> JSON"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = 50
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, dev)

    def step():
        pyr = ops.corr_pyramid(f1, f2, 4, "bf16")
        out = None
        for i in range(12):
            out = ops.corr_lookup(pyr, coords[i], 4)
        return out

    for _ in range(3):
        ref = step()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gout = step()
    g.replay()
    torch.cuda.synchronize()
    res = {"bitwise_equal": bool(torch.equal(gout, ref)), "eager_ms": [], "graph_ms": []}
    for _ in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        res["eager_ms"].append((time.perf_counter() - t0) / steps * 1e3)
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        res["graph_ms"].append((time.perf_counter() - t0) / steps * 1e3)
    for k in ("eager_ms", "graph_ms"):
        v = sorted(res[k])
        res[k + "_median"] = v[len(v) // 2]
    res["pairs_per_s_eager"] = 8 / res["eager_ms_median"] * 1e3
    res["pairs_per_s_graph"] = 8 / res["graph_ms_median"] * 1e3
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
