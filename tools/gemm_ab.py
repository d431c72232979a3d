#!/usr/bin/env python3
"""A/B timing of the cfg2 correlation-GEMM kernels (diagnostic; MI355X only, not product code).

For each kernel named in RMD_GEMM_KERNEL values (pipe = default path, stationary = previous one)
times rmd_corr_pyramid_prepared alone with HIP events on the launch stream and checks that every
variant's pyramid is bitwise identical to the first one's (same MFMA and pooling order).
usage: gemm_ab.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the A/B knobs exist only in the diagnostic build (make -C raft-meets-dicl_amd/csrc diag)
os.environ.setdefault("RMD_LIBRARY", os.path.join(ROOT, "raft-meets-dicl_amd", "rmd", "librmd_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from rmd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    f1, f2, _ = bench.synthetic(8, 256, 55, 128, 1, 1234, dev)
    names = os.environ.get("RMD_AB", "w8,stationary").split(",")
    rounds = int(os.environ.get("RMD_AB_ROUNDS", "5"))
    times = {n: [] for n in names}
    res, ref = {}, None

    def configure(name):
        kern, _, abl = name.partition(":")          # e.g. "pipe:1" = RMD_ABLATE=1 (stores dropped)
        kern, _, aux = kern.partition("@")          # e.g. "w8@2" = RMD_STORE_AUX=2
        kern, _, knobs = kern.partition("+")        # e.g. "w8+roll+stag4" = RMD_W8_ROLL=1, RMD_W8_STAGGER=4
        os.environ["RMD_W8_ROLL"] = "1" if "roll" in knobs else "0"
        os.environ["RMD_W8_PAD"] = "0" if "nopad" in knobs else "1"      # "w8+nopad" = XOR-swizzled LDS
        # "w8+ring" = B ring + double-buffered A; "w8+pp" = the same with ping-pong phases (barriers)
        # (default w8 = the product kernel: padded LDS + ring + ping-pong; "w8+plain" = neither)
        os.environ["RMD_W8_RING"] = "1" if "ring" in knobs else ("0" if "plain" in knobs or "nopad" in knobs else "2")
        stag = int(knobs.split("stag")[1].split("+")[0]) if "stag" in knobs else 0
        os.environ["RMD_W8_STAGGER"] = str(stag + (1000 if "prio" in knobs else 0))     # "w8+prio" = s_setprio 1 on waves 4-7
        # "w8+bal0" / "w8+bal2" = balanced schedule off / pairing + helpers (default 1: pairing only)
        os.environ["RMD_W8_BAL"] = "0" if "bal0" in knobs else ("2" if "bal2" in knobs else "1")
        os.environ["RMD_GEMM_KERNEL"] = kern
        os.environ["RMD_ABLATE"] = abl or "0"
        os.environ["RMD_STORE_AUX"] = aux or "2"
        return abl

    for _ in range(5):                              # chip warm-up (clocks) before any timed variant
        ops.corr_pyramid(f1, f2, 4, "bf16")
    for rnd in range(rounds):                       # variants interleaved round by round
        for name in names:
            abl = configure(name)
            ev = []
            for _ in range(2):
                pyr = ops.corr_pyramid(f1, f2, 4, "bf16")
            for _ in range(reps):
                pyr = ops.corr_pyramid(f1, f2, 4, "bf16", events=ev)
            torch.cuda.synchronize()
            times[name] += [a.elapsed_time(b) for a, b in ev]
            if rnd == 0 and not abl:
                if ref is None:
                    ref = pyr.data.clone()
                else:
                    res.setdefault(name, {})["bitwise_mismatch_vs_first"] = int(
                        (pyr.data.view(torch.int16) != ref.view(torch.int16)).sum().item())
    for name in names:
        ms = sorted(times[name])
        res.setdefault(name, {}).update(median_ms=ms[len(ms) // 2], min_ms=ms[0],
                                        write_TBps=pyr.data.numel() * 2 / (ms[len(ms) // 2] * 1e-3) / 1e12)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
