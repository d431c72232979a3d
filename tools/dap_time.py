#!/usr/bin/env python3
"""Time rmd_dap (DAP 1x1 projection, blocks/dicl.py:121-150) with HIP events on its launch stream.

usage: dap_time.py [reps] [lib ...]  -> one JSON line per (lib, case): median / min µs and a checksum.
Cases: D = 324 'full' (raft_dicl_ml.py:268-273) forward and transposed (the input-gradient form), and
D = 81 forward, all at b8 over the cfg4 1/8 level (48 x 160).  Extra libraries (e.g. -D build variants
under tools/_bin) are loaded side by side through rmd._lib's loader so the A/B runs on one box."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raft-meets-dicl_amd"))
from rmd import _lib  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
libs = sys.argv[2:] or [None]
dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
g = torch.Generator().manual_seed(0)
cases = [("d324_fwd", 324, 0), ("d324_bwd", 324, 1), ("d81_fwd", 81, 0)]
b, h, w = 8, 48, 160
for path in libs:
    lib = _lib.lib() if path is None else ctypes.CDLL(os.path.abspath(path))
    lib.rmd_dap.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 4 + [ctypes.c_void_p] * 2
    lib.rmd_dap.restype = ctypes.c_int
    for name, d, tr in cases:
        x = torch.randn(b, d, h * w, generator=g).to(dev)
        wt = (torch.randn(d, d, generator=g) * 0.05).to(dev)
        out = torch.empty_like(x)

        def run():
            rc = lib.rmd_dap(x.data_ptr(), wt.data_ptr(), b, d, h * w, tr, out.data_ptr(),
                             ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, rc

        for _ in range(3):
            run()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run()
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        ref = (wt.t() if tr else wt) @ x
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"lib": path or "librmd.so", "case": name, "median_us": ts[len(ts) // 2], "min_us": ts[0],
                          "checksum": float(out.double().sum()), "max_rel_err_vs_torch": err}), flush=True)
