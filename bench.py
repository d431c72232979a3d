#!/usr/bin/env python3
"""Benchmark of the RAFT cost-volume hot path on MI355X — BASELINE.json configs[1].

Workload ("step"): one pass of the hot path over one batch of synthetic Sintel-shape frame pairs:
436x1024 padded to 440x1024 (modulo 8, cfg/model/raft-baseline.yaml:21-28) -> 1/8-resolution
feature maps 55x128, C=256, batch 8 per GPU; build the all-pairs correlation volume + 4-level
pooled pyramid (rmd_corr_pyramid, replaces raft.py:18-47) and run the 12 per-GRU-iteration
radius-4 lookups (rmd_corr_lookup, replaces raft.py:49-95) with the flow estimate moving every
iteration.  Inputs (feature maps, coordinates) are resident in HBM before the timed region.
The encoders / GRU update block (MIOpen convolutions) are outside the hot path and not timed.

Metric: frame-pairs/s over the whole job (all ranks).  One process per GPU (torchrun); frame
pairs are independent, so each rank runs its own batch of 8 ("weak" scaling, no data-path
collective; timing is max over ranks via one all_reduce after the timed region).

Also reported: roofline of the dominant kernel per step (GEMM: one launch; lookup: 12 launches),
measured live with HIP events on the launch stream (the GEMM launch alone, the 12 lookups as one
bracket), both kernels' rooflines and the GEMM's MFMA fraction, and the CPU oracle
(test infrastructure, numpy/BLAS float32 restatement of the reference path) timed on a bounded
sample on this host, rank 0 only.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
MFMA_PEAK = {"bf16": 2500.0, "fp32": 157.3}   # dense TFLOP/s (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="frame pairs per GPU")
    ap.add_argument("--height", type=int, default=436)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--channels", type=int, default=256)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--radius", type=int, default=4)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "bf16-f32", "fp32-f16"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=10.0)
    ap.add_argument("--event-every", type=int, default=5,
                    help="record the per-kernel HIP events (roofline) on every E-th timed step")
    return ap.parse_args()


def padded(h, w, mod=8):
    return (h + mod - 1) // mod * mod, (w + mod - 1) // mod * mod


def synthetic(b, c, h8, w8, iters, seed, device):
    """Feature maps in the encoder's output range and a smooth flow that moves every iteration."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    f1 = torch.randn(b, c, h8, w8, generator=g)
    f2 = torch.randn(b, c, h8, w8, generator=g)
    ys, xs = torch.meshgrid(torch.arange(h8, dtype=torch.float32), torch.arange(w8, dtype=torch.float32),
                            indexing="ij")
    grid = torch.stack([xs, ys])[None].expand(b, -1, -1, -1)
    base = torch.randn(b, 2, 1, 1, generator=g) * 4.0
    smooth = torch.nn.functional.interpolate(torch.randn(b, 2, 4, 8, generator=g) * 2.0, size=(h8, w8),
                                             mode="bilinear", align_corners=True)
    coords = []
    for it in range(iters):
        frac = (it + 1) / iters
        coords.append((grid + frac * (base + smooth)).contiguous())
    return f1.to(device), f2.to(device), torch.stack(coords).to(device)


def cpu_baseline(args, h8, w8):
    """Oracle (numpy float32 restatement of raft.py:18-95) on one frame pair, this host's cores."""
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0))))
    rng = np.random.default_rng(0)
    f1 = rng.standard_normal((1, args.channels, h8, w8)).astype(np.float32)
    f2 = rng.standard_normal((1, args.channels, h8, w8)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h8, dtype=np.float32), np.arange(w8, dtype=np.float32), indexing="ij")
    co = (np.stack([xs, ys])[None] + rng.normal(0, 4, (1, 2, h8, w8))).astype(np.float32)
    pairs = 0
    t0 = time.perf_counter()
    while True:
        pyr = oracle.corr_pyramid(f1, f2, args.levels)
        for _ in range(args.iters):
            oracle.corr_lookup(pyr, co, args.radius)
        pairs += 1
        el = time.perf_counter() - t0
        if el > args.cpu_budget_s:
            break
    return {"value": pairs / el, "unit": "frame-pairs/s", "cores": threads, "kind": "port",
            "sample": f"{pairs} frame pair(s) of the same workload (1x{args.channels}x{h8}x{w8}, "
                      f"pyramid + {args.iters} lookups), oracle/ numpy+BLAS float32, {el:.1f} s"}


def job_time(elapsed, world, device):
    """Whole-job time of the timed region: the MAX over ranks (one all_reduce after the region,
    nothing on the data path); identity for a single process."""
    if world <= 1:
        return elapsed
    import torch.distributed as dist
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    return float(t.item())


def rank_inputs(args, rank, h8, w8, device):
    """Each rank's own batch of frame pairs (weak scaling: per-rank work fixed, seeds differ)."""
    return synthetic(args.batch, args.channels, h8, w8, args.iters, 1234 + rank, device)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import rmd
    from rmd import ops

    H, W = padded(args.height, args.width)
    h8, w8 = H // 8, W // 8
    B = args.batch
    f1, f2, coords = rank_inputs(args, rank, h8, w8, device)

    stream = torch.cuda.current_stream(device)
    ev_gemm = []      # (start, end) around the GEMM launch alone (rmd_corr_pyramid_prepared)
    ev_look = []      # (start, end) around the 12 lookup launches of a step

    def step(record):
        pyr = ops.corr_pyramid(f1, f2, args.levels, args.precision, events=ev_gemm if record else None)
        if record:
            a = torch.cuda.Event(enable_timing=True)
            z = torch.cuda.Event(enable_timing=True)
            a.record(stream)
        out = None
        for it in range(args.iters):
            out = ops.corr_lookup(pyr, coords[it], args.radius)
        if record:
            z.record(stream)
            ev_look.append((a, z))
        return out

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i % max(1, args.event_every) == 0)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    elapsed = job_time(elapsed, world, device)

    gemm_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_gemm]))
    look_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_look])) / args.iters
    N = h8 * w8
    D = (2 * args.radius + 1) ** 2
    s = 2 if args.precision in ("bf16", "fp32-f16") else 4
    levels = [(h8 >> i, w8 >> i) for i in range(args.levels)]
    # algorithmic bytes
    look_bytes = B * N * (args.levels * (2 * args.radius + 2) ** 2 * s + args.levels * D * 4 + 8)
    op_bytes = 2 if args.precision.startswith("bf16") else 4
    gemm_bytes = B * N * sum(h * w for h, w in levels) * s + 2 * B * N * args.channels * op_bytes
    gemm_flop = 2.0 * B * N * N * args.channels
    compute_dt = "fp32" if args.precision.startswith("fp32") else "bf16"
    look_gbs = look_bytes / (look_ms * 1e-3) / 1e9
    gemm_gbs = gemm_bytes / (gemm_ms * 1e-3) / 1e9
    gemm_tfs = gemm_flop / (gemm_ms * 1e-3) / 1e12

    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", "pmc_r01.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as fh:
                pmc = json.load(fh).get(args.precision, {})
        except (OSError, ValueError):
            pmc = {}
    roof_gemm = {"kernel": "corr_pyramid_w8 (bf16 MFMA GEMM + fused pooled-pyramid epilogue)",
                 "bound": "hbm", "achieved": gemm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": gemm_gbs / HBM_PEAK_GBS, "traffic": pmc.get("gemm_hbm_bytes_per_launch"),
                 "algorithmic_bytes_per_launch": gemm_bytes, "avg_launch_ms": gemm_ms, "launches_per_step": 1,
                 "mfma_tflops": gemm_tfs, "mfma_peak_tflops": MFMA_PEAK[compute_dt],
                 "mfma_frac": gemm_tfs / MFMA_PEAK[compute_dt], "algorithmic_flop_per_launch": gemm_flop}
    roof_look = {"kernel": "corr_lookup_kernel", "bound": "hbm", "achieved": look_gbs, "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": look_gbs / HBM_PEAK_GBS,
                 "traffic": pmc.get("lookup_hbm_bytes_per_launch"),
                 "algorithmic_bytes_per_launch": look_bytes, "avg_launch_ms": look_ms,
                 "launches_per_step": args.iters}
    dominant_gemm = gemm_ms >= look_ms * args.iters

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    total_pairs = world * B * args.steps
    res = {
        "metric": "frame-pairs/s @436x1024 RAFT 12 iters (1-8 GPU); corr MFMA% + lookup HBM%",
        "value": total_pairs / elapsed,
        "unit": "frame-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": compute_dt,
        "data": "synthetic (seeded random 1/8-res feature maps + smooth moving flow; no dataset)",
        "config": {"workload": "RAFT all-pairs correlation + 4-level pyramid + 12 radius-4 lookups "
                               "(BASELINE configs[1])",
                   "image": f"{args.height}x{args.width} padded {H}x{W}", "feature_map": f"{h8}x{w8}",
                   "channels": args.channels, "batch_per_gpu": B, "global_batch": B * world,
                   "lookups_per_step": args.iters, "precision": args.precision,
                   "pyramid_storage": "fp16" if s == 2 else "fp32", "parallelism": f"batch-shard x{world}"},
        "roofline": roof_gemm if dominant_gemm else roof_look,
        "roofline_gemm": roof_gemm,
        "roofline_lookup": roof_look,
    }
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args, h8, w8)
    print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
