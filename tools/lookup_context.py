#!/usr/bin/env python3
"""Lookup time by position in the bench step, under different contexts (diagnostic, MI355X only; run
under rocprofv3 --kernel-trace, then tools/lookup_context.py --summary <kernel_trace.csv>).

bench.py times steps of (prep + GEMM + 12 lookups); in that sequence the lookups slow down with their
position after the GEMM, while back-to-back lookups on one pyramid (tools/lookup_time.py) run at the
speed of the second.  Modes, each `steps` steps separated by a 50 ms idle gap marker:
  bench    : bench.py's step (a new output per lookup; the previous one still alive: two alternating blocks)
  nogemm   : the same 12 lookups per step on one pyramid built once (no GEMM between steps)
  oneout   : bench step with every lookup writing one preallocated output (C ABI call)
  samecoord: bench step with coords[0] for all 12 lookups
  rev      : bench step with the coords in reverse order (coords[11] first)
  shift    : bench step with coords[0] + 0.02 px * position (new tensors, nearly the same lines)
  const11  : bench step with coords[11] for all 12 lookups
usage: python3 tools/lookup_context.py [steps]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)

MODES = os.environ.get("LOOKUP_CONTEXT_MODES", "bench,nogemm,oneout,samecoord").split(",")


def run(steps):
    import torch
    import bench
    from rmd import _lib, ops
    f1, f2, coords = bench.synthetic(8, 256, 55, 128, 12, 1234, "cuda")
    lib = _lib.lib()
    for mode in MODES:
        pyr = ops.corr_pyramid(f1, f2, 4, "bf16")
        fixed = torch.empty(8, 324, 55, 128, device="cuda")
        out = None
        for s in range(steps + 2):
            if mode != "nogemm":
                pyr = ops.corr_pyramid(f1, f2, 4, "bf16")
            for it in range(12):
                if mode == "samecoord":
                    co = coords[0]
                elif mode == "rev":
                    co = coords[11 - it]
                elif mode == "shift":
                    co = coords[0] + 0.02 * it
                elif mode == "const11":
                    co = coords[11]
                else:
                    co = coords[it]
                if mode == "oneout":
                    _lib.check(lib.rmd_corr_lookup(ctypes.c_void_p(pyr.data.data_ptr()), ctypes.byref(pyr.desc),
                                                   ctypes.c_void_p(co.data_ptr()), 4, 0,
                                                   ctypes.c_void_p(fixed.data_ptr()),
                                                   _lib.stream_ptr(fixed.device)), "lookup")
                else:
                    out = ops.corr_lookup(pyr, co, 4)
        torch.cuda.synchronize()
        time.sleep(0.05)
    del out


def summary(path):
    import csv
    import statistics as st
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    # split into modes at the idle gaps (> 20 ms)
    groups, cur, last = [], [], None
    for s, e, n in rows:
        if last is not None and s - last > 20_000_000:
            groups.append(cur)
            cur = []
        cur.append((s, e, n))
        last = e
    groups.append(cur)
    groups = [g for g in groups if any("corr_lookup" in n for _, _, n in g)][-len(MODES):]
    res = {}
    for mode, g in zip(MODES, groups):
        pos, k, gemm = {}, None, []
        for s, e, n in g:
            if "corr_pyramid" in n:
                gemm.append((e - s) / 1e3)
                k = 0
            elif "corr_lookup" in n:
                k = 0 if k is None else k
                pos.setdefault(k % 12, []).append((e - s) / 1e3)
                k += 1
        res[mode] = {p: round(st.median(v[2:] if len(v) > 4 else v), 2) for p, v in sorted(pos.items())}
        allv = [x for v in pos.values() for x in (v[2:] if len(v) > 4 else v)]
        res[mode]["mean"] = round(sum(allv) / len(allv), 2)
        if len(gemm) > 4:
            res[mode]["gemm"] = round(st.median(gemm[2:]), 2)
            res[mode]["gemm_plus_12"] = round(res[mode]["gemm"] + 12 * res[mode]["mean"], 1)
    print(json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
