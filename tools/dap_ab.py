#!/usr/bin/env python3
"""A/B of the DAP kernels (diagnostic build: RMD_LIBRARY=raft-meets-dicl_amd/rmd/librmd_diag.so).
Variants (RMD_AB, comma-separated, '+'-joined NAME=VALUE env settings): "RMD_DAP_VALU=0" (product:
split-bf16 x3 MFMA), "RMD_DAP_VALU=1" (round-1 exact-f32 MFMA), "RMD_DAP_VALU=2" (VALU),
"RMD_DAP_VALU=3" (blocked exact-f32 MFMA, RMD_DAP_TPW tiles per wave).  Shapes: D=49 at cfg3 level 2 (96x128),
D=81 at cfg4 1/8 (48x160), D=324 'full' (48x160), batch 8; forward and transposed (input gradient).
Outputs compared with the first variant; median of `reps` HIP-event timings.
usage: python tools/dap_ab.py [reps] -> JSON"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import torch  # noqa: E402


def main():
    from rmd import ops
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    names = os.environ.get("RMD_AB", "RMD_DAP_VALU=0,RMD_DAP_VALU=1").split(",")
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {}

    def select(n):
        for k in ("RMD_DAP_VALU", "RMD_DAP_TPW", "RMD_DAP_STREAM", "RMD_DAP_MT", "RMD_DAP_NW", "RMD_DAP_NT", "RMD_DAP_RING"):
            os.environ.pop(k, None)
        for kv in filter(None, n.split("+")):
            k, v = kv.split("=")
            os.environ[k] = v

    for d, (h, w) in ((49, (96, 128)), (81, (48, 160)), (324, (48, 160))):
        x = torch.randn(8, d, h, w, generator=g).to(dev)
        wt = (torch.eye(d) + 0.05 * torch.randn(d, d, generator=g)).to(dev)[:, :, None, None]
        nbytes = 2 * x.numel() * 4 + wt.numel() * 4
        for tr in (False, True):
            key = f"D{d}_{h}x{w}_b8" + ("_transpose" if tr else "")
            fn = (lambda: torch.ops.rmd.dap_transpose(x, wt)) if tr else (lambda: ops.dap(x, wt))
            w64 = wt[:, :, 0, 0].double()
            ref = torch.einsum("oi,bihw->bohw", w64.t() if tr else w64, x.double())
            outs, times = {}, {}
            for n in names:
                select(n)
                outs[n] = fn().clone()
                ts = []
                for _ in range(3):
                    fn()
                for _ in range(reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    fn()
                    b.record()
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b))
                ts.sort()
                times[n] = ts[len(ts) // 2] * 1e3
            res[key] = {n: {"median_us": times[n], "GBps": nbytes / (times[n] * 1e-6) / 1e9,
                            "max_abs_diff_first": float((outs[n] - outs[names[0]]).abs().max()),
                            "max_norm_err_fp64": float((outs[n].double() - ref).abs().max() / ref.abs().max()),
                            "max_elem_rel_err_fp64": float(((outs[n].double() - ref).abs()
                                                            / (ref.abs() + 1e-3 * ref.abs().max())).max())} for n in names}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
