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
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8, help="frame pairs per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many frame pairs in total, split evenly over the ranks "
                         "(overrides --batch; must be a multiple of the rank count)")
    ap.add_argument("--height", type=int, default=436)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--channels", type=int, default=256)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--radius", type=int, default=4)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "fp32-f32", "fp32-s24", "fp32-exact", "bf16-f32", "fp32-f16"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=10.0)
    ap.add_argument("--event-every", type=int, default=5,
                    help="record the per-kernel HIP events (roofline) on every E-th timed step "
                         "(steps E-1, 2E-1, ...: never the first timed step)")
    ap.add_argument("--model-level", choices=["on", "off"], default="on",
                    help="also time the whole RAFT network (436x1024, 12 iterations) with the rmd path on every "
                         "rank, batch-sharded like the headline (extra key 'model_level')")
    ap.add_argument("--fp32-mode", choices=["on", "off"], default="on",
                    help="extra key 'fp32_mode': the headline step in the fp32 parity mode (x3 GEMM, fp32 "
                         "pyramid) on the same inputs, with its own rooflines")
    ap.add_argument("--fp32-steps", type=int, default=10)
    ap.add_argument("--live-pmc", choices=["on", "off"], default="on",
                    help="rank 0 (any N): roofline traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over "
                         "tools/pmc_probe.py run as child processes on rank 0's GPU after the timed region")
    ap.add_argument("--train", choices=["on", "off"], default="on",
                    help="also time the cfg5 training step (RAFT+DICL ctf-l3, DDP over RCCL when N > 1): "
                         "extra key 'train_step'")
    ap.add_argument("--train-steps", type=int, default=10)
    ap.add_argument("--train-warmup", type=int, default=3)
    ap.add_argument("--train-batch", type=int, default=6, help="frame pairs per GPU (train/chairs2-1 stage)")
    ap.add_argument("--hybrid", choices=["on", "off"], default="on",
                    help="extra leg: RAFT+DICL ctf-l3 inference at 376x1242 (BASELINE configs[3]) on every rank")
    ap.add_argument("--hybrid-steps", type=int, default=5)
    ap.add_argument("--hybrid-warmup", type=int, default=2)
    ap.add_argument("--hybrid-batch", type=int, default=8, help="frame pairs per GPU (weak; --global-batch splits)")
    ap.add_argument("--dicl", choices=["on", "off"], default="on",
                    help="extra leg: DICL cost volumes + MatchingNet coarse-to-fine at 384x512 (BASELINE configs[2])")
    ap.add_argument("--highres", choices=["on", "off"], default="on",
                    help="extra key 'highres_fs': raft/fs inference at a 4K 1/8 map (270x480, C=256, b2, 12 lookups), "
                         "on-the-fly lookup vs the all-pairs volume (rank 0 of single-GPU runs)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0 (pair with --backend gloo)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/collective plumbing only (no GPU work): for the CPU gloo tests")
    return ap.parse_args()


def maybe_launch(args):
    """`bench.py --gpus N` (N > 1) started as a plain process launches its own N ranks: one process
    per GPU through torch.distributed.run (127.0.0.1 rendezvous), as the driver does; returns only
    in a rank (or a single-GPU run).  Runs before anything touches the GPU; the child processes are
    started with subprocess (no exec from this process)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


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


def cpu_baseline(args):
    """BASELINE configs[0] on this host's cores: the whole RAFT network (raft/baseline, 12 GRU
    iterations, synthetic 368x496 pair, batch 1, fp32) with the reference's eager correlation
    (tests/e2e/eager_corr.EagerCorrBlock = raft.py:15-95 op for op) on torch-CPU; 1 warm-up, median of
    5.  Test infrastructure timed as the baseline, never the product path."""
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from detinit import det_init_fanin
    from e2e.eager_corr import EagerCorrBlock
    from e2e.raft_net import RaftNet
    from synth import frame_pair
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        net = det_init_fanin(RaftNet(EagerCorrBlock)).eval()
        img1, img2, _ = frame_pair(368, 496)
        i1, i2 = torch.from_numpy(img1), torch.from_numpy(img2)
        times = []
        with torch.no_grad():
            for k in range(6):
                t0 = time.perf_counter()
                net(i1, i2, 12)
                if k:
                    times.append(time.perf_counter() - t0)
                if k and sum(times) > args.cpu_budget_s * 3:
                    break
    finally:
        torch.set_num_threads(prev)
    med = float(np.median(times))
    comps = cpu_components(threads, args.cpu_budget_s)
    return {"value": 1.0 / med, "unit": "frame-pairs/s", "cores": threads, "kind": "port",
            "ms_per_pair": med * 1e3, "runs": len(times), "components_cfg2_b1": comps,
            "sample": f"BASELINE configs[0]: whole RAFT network (raft/baseline, 12 iterations) on one synthetic "
                      f"368x496 pair, batch 1, fp32 torch-CPU with the reference's eager correlation "
                      f"(tests/e2e/eager_corr.py); 1 warm-up + median of {len(times)}"}


def cpu_components(threads, budget_s):
    """BASELINE.md §3 / SURVEY.md §8(d) 'CPU beside GPU': the reference correlation's two components at
    cfg2 shape with batch 1 (55x128 feature maps, C=256) on torch-CPU — the all-pairs GEMM + pyramid
    build (raft.py:18-47) and one radius-4 lookup (raft.py:49-95) — through the op-for-op restatement
    tests/e2e/eager_corr.EagerCorrBlock (test infrastructure); 1 warm-up + median of up to 5."""
    from e2e.eager_corr import EagerCorrBlock
    f1, f2, coords = synthetic(1, 256, 55, 128, 12, 1234, "cpu")
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        tp, tl = [], []
        with torch.no_grad():
            for k in range(6):
                t0 = time.perf_counter()
                cb = EagerCorrBlock(f1, f2, 4, 4)
                t1 = time.perf_counter()
                cb(coords[k % 12])
                t2 = time.perf_counter()
                if k:
                    tp.append(t1 - t0)
                    tl.append(t2 - t1)
                if k and sum(tp) + sum(tl) > budget_s:
                    break
    finally:
        torch.set_num_threads(prev)
    return {"pyramid_ms": float(np.median(tp)) * 1e3, "lookup_ms": float(np.median(tl)) * 1e3, "cores": threads,
            "runs": len(tp), "kind": "port",
            "sample": "cfg2 shape, batch 1 (55x128, C=256, 4 levels, r=4): EagerCorrBlock constructor (GEMM + "
                      "avg-pool pyramid, raft.py:18-47) and one lookup (raft.py:49-95), fp32 torch-CPU"}


def model_level(rank_dev, precision, b=8, rank=0, dry_run=False):
    """The whole RAFT network at 436x1024 (padded 440x1024), batch b, MIOpen fp32 convolutions, with
    rmd.raft.CorrBlock + rmd.raft.Up8Network (tools/bench_e2e.py compares it with the eager reference
    correlation): network and a synthetic batch on the rank's device."""
    import torch.nn.functional as F
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import rmd
    from detinit import det_init_fanin
    from e2e.raft_net import RaftNet
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    h, w = (128, 128) if dry_run else (440, 1024)      # dry run: level 3 is 2x2 (a 1-pixel level is NaN)
    g = torch.Generator().manual_seed(1234 + rank)
    low = torch.rand(b, 3, h // 8, w // 8, generator=g) * 2 - 1
    img1 = F.interpolate(low, size=(h, w), mode="bilinear", align_corners=True).to(rank_dev)
    img2 = torch.roll(img1, shifts=(3, 5), dims=(2, 3))
    if dry_run:
        # --dry-run (CPU gloo tests): a small frame through the eager reference correlation on the CPU,
        # exercising the shard / seed / MAX-over-ranks plumbing of the leg, not the kernels
        from e2e.eager_corr import EagerCorrBlock
        net = det_init_fanin(RaftNet(EagerCorrBlock))
    else:
        net = det_init_fanin(RaftNet(rmd.raft.CorrBlock, precision=precision, upnet_cls=rmd.raft.Up8Network))
    net = net.eval().to(rank_dev)
    return net, img1, img2


def model_leg(args, world, rank, device):
    """BASELINE.md frame-pairs/s of the 'cfg2 model at 1/2/4/8 GPUs': the whole RAFT network at
    436x1024 (padded 440x1024), 12 iterations, on every rank with its own batch shard (per-GPU b8, or
    --global-batch split), no collective on the data path; job time = MAX over ranks."""
    b = args.global_batch // world if args.global_batch else args.batch
    net, img1, img2 = model_level(device, args.precision, b, rank, args.dry_run)
    reps = 1 if args.dry_run else 3
    iters = 2 if args.dry_run else 12

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    with torch.no_grad():
        for i in range(1 if args.dry_run else 2):
            net(img1, img2, iters)
            progress(rank, f"model_level warm-up {i + 1}")
        sync()
        if world > 1:
            torch.distributed.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = net(img1, img2, iters)
        sync()
        el = time.perf_counter() - t0
        shard_sum = float(out[-1].double().sum())
    if world > 1:
        torch.distributed.barrier()
    el = job_time(el, world, device)
    del net, img1, img2
    torch.cuda.empty_cache()
    return {"frame_pairs_per_s": world * b * reps / el, "ms_per_batch": el / reps * 1e3, "per_gpu_batch": b,
            "global_batch": world * b, "n_gpus": world, "iterations": iters, "precision": args.precision,
            "rank0_flow_checksum": shard_sum,
            "parallelism": f"batch-shard x{world} (no collective)",
            "scaling": "strong" if args.global_batch else "weak", "convs": "MIOpen fp32 (TF32 off)",
            "workload": "whole RAFT network 436x1024 (padded 440x1024): encoders + GRU + rmd correlation + rmd Up8"}


def train_leg(args, world, rank, device):
    """BASELINE configs[4] / SURVEY.md §8(d) cfg5: one RAFT+DICL ctf-l3 training step per timed step —
    synthetic FlyingChairs-shape pairs (368x496 padded to 384x512), per-GPU batch 6, iterations
    (4, 3, 3), loss raft+dicl/mlseq (ord 1, gamma 0.85, alpha (0.38, 0.6, 1.0)), backward through the
    HIP DICL stack / DAP / Up8 kernels, clip_grad_norm_(1.0), AdamW (lr one-cycle to 4e-4, weight decay
    1e-4) — src/strategy/training.py:232-289.  N > 1: DistributedDataParallel over RCCL (bucketed
    gradient all-reduce of the 12.68 M fp32 parameters, overlapped with backward), the replacement
    of the reference's nn.DataParallel (src/cmd/train.py:183-184).  Network: tests/e2e/ctf_l3_net.py
    (the reference's architecture and module names; encoders/GRU/MatchingNet are MIOpen convs)."""
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import rmd
    from detinit import det_init_fanin
    from e2e.ctf_l3_net import CtfL3Net, freeze_batchnorm, mlseq_loss
    from synth import frame_pair
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    h, w, pad, bsz = 368, 496, 64, args.train_batch
    net = det_init_fanin(CtfL3Net(rmd.corr.make_cmod, rmd.corr.make_flow_regression, upnet_cls=rmd.raft.Up8Network),
                         head_gain=0.02).to(device)
    n_params = sum(p.numel() for p in net.parameters())
    net.train()
    freeze_batchnorm(net)
    model = net
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(net, device_ids=[device.index])
    opt = torch.optim.AdamW(net.parameters(), lr=4e-4, weight_decay=1e-4, eps=1e-8)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=4e-4, total_steps=100000, pct_start=0.05,
                                                cycle_momentum=False, anneal_strategy="linear")
    i1s, i2s, fls, vas = [], [], [], []
    for k in range(bsz):
        seed = 1000 * rank + k
        rng = np.random.default_rng(seed)
        i1, i2, gt = frame_pair(h, w, flow=tuple(int(v) for v in rng.integers(0, 8, 2)), seed=seed, pad=pad)
        hp, wp = i1.shape[-2:]
        f = np.zeros((1, 2, hp, wp), np.float32)
        f[:, :, :h, :w] = gt
        v = np.zeros((1, hp, wp), bool)
        v[:, :h, :w] = True
        i1s.append(i1), i2s.append(i2), fls.append(f), vas.append(v)
    img1, img2, flow, valid = (torch.from_numpy(np.concatenate(x)).to(device) for x in (i1s, i2s, fls, vas))

    def step():
        opt.zero_grad(set_to_none=True)
        loss = mlseq_loss(model(img1, img2, (4, 3, 3)), flow, valid)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 1.0, norm_type=2.0)
        opt.step()
        sched.step()
        return loss

    for i in range(args.train_warmup):
        step()
        progress(rank, f"train_step warm-up {i + 1}/{args.train_warmup}")
    torch.cuda.synchronize(device)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.train_steps):
        loss = step()
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    el = job_time(el, world, device)
    last = float(loss.detach())
    del model, net, opt
    torch.cuda.empty_cache()
    return {"workload": "RAFT+DICL ctf-l3 training step (BASELINE configs[4], SURVEY cfg5): 368x496 padded "
                        "384x512, iterations (4,3,3), mlseq loss, backward, clip 1.0, AdamW",
            "frame_pairs_per_s": world * bsz * args.train_steps / el, "steps_per_s": args.train_steps / el,
            "ms_per_step": el / args.train_steps * 1e3, "per_gpu_batch": bsz, "global_batch": world * bsz,
            "n_gpus": world, "steps": args.train_steps, "warmup": args.train_warmup,
            "parallelism": (f"DDP x{world} ({'RCCL' if args.backend == 'nccl' else args.backend} bucketed gradient "
                            f"all-reduce)" if world > 1 else "single GPU"),
            "gradient_bytes_per_step": 4 * n_params, "parameters": n_params, "last_loss": last,
            "scaling": "weak", "dtype": "fp32", "data": "synthetic smooth pairs with known flow, name-keyed random weights"}


def hybrid_leg(args, world, rank, device):
    """BASELINE configs[3] / SURVEY.md §8(d) cfg4: RAFT+DICL ctf-l3 inference on KITTI-shape pairs
    (376x1242 padded to 384x1280, ModuloPadding 64), iterations (4, 3, 3), convex upsampling, batch
    sharded over the ranks with no collective on the data path (per-GPU b8 weak scaling, or
    --global-batch G split evenly: strong).  The correlation modules are rmd.corr.make_cmod('dicl')
    (the HIP DICL stack + MatchingNet on MIOpen + the split-bf16 DAP), the GRU update blocks stay
    PyTorch, the convex upsampling is rmd Up8 — the reference's raft_dicl_ctf_l3.py:79-260 through
    tests/e2e/ctf_l3_net.py.  The timed region (MAX over ranks) is whole forward passes."""
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import rmd
    from detinit import det_init_fanin
    from e2e.ctf_l3_net import CtfL3Net
    from synth import frame_pair
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    h, w, pad = 376, 1242, 64
    bsz = args.global_batch // world if args.global_batch else args.hybrid_batch
    net = det_init_fanin(CtfL3Net(rmd.corr.make_cmod, rmd.corr.make_flow_regression, upnet_cls=rmd.raft.Up8Network),
                         head_gain=0.02).to(device).eval()
    i1s, i2s = [], []
    for k in range(bsz):
        seed = 5000 + 1000 * rank + k
        rng = np.random.default_rng(seed)
        i1, i2, _ = frame_pair(h, w, flow=tuple(int(v) for v in rng.integers(0, 8, 2)), seed=seed, pad=pad)
        i1s.append(i1), i2s.append(i2)
    img1, img2 = (torch.from_numpy(np.concatenate(x)).to(device) for x in (i1s, i2s))
    with torch.no_grad():
        for i in range(args.hybrid_warmup):
            net(img1, img2, (4, 3, 3))
            progress(rank, f"hybrid_inference warm-up {i + 1}/{args.hybrid_warmup}")
        torch.cuda.synchronize(device)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(args.hybrid_steps):
            out = net(img1, img2, (4, 3, 3))
        torch.cuda.synchronize(device)
        el = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    el = job_time(el, world, device)
    fin = bool(torch.isfinite(out[-1][-1]).all())
    hp, wp = img1.shape[-2:]
    del net, out, img1, img2
    torch.cuda.empty_cache()
    return {"workload": "RAFT+DICL ctf-l3 inference (BASELINE configs[3], SURVEY cfg4): 376x1242 padded "
                        f"{hp}x{wp}, iterations (4,3,3), convex upsampling",
            "frame_pairs_per_s": world * bsz * args.hybrid_steps / el, "ms_per_batch": el / args.hybrid_steps * 1e3,
            "per_gpu_batch": bsz, "global_batch": world * bsz, "n_gpus": world, "steps": args.hybrid_steps,
            "warmup": args.hybrid_warmup, "parallelism": f"batch-shard x{world} (no collective)",
            "scaling": "strong" if args.global_batch else "weak", "dtype": "fp32", "finite": fin,
            "convs": "MIOpen fp32 (TF32 off)",
            "data": "synthetic smooth pairs (tests/golden/synth.py), name-keyed random weights"}


def _library_info():
    """The measured librmd.so: its path, version and source fingerprint, and whether that fingerprint
    matches the sources in this tree (csrc/Makefile; rmd/_lib.py build_info)."""
    from rmd import _lib
    info = _lib.build_info()
    info["path"] = os.path.relpath(_lib.LIB_PATH, ROOT)
    info["version"] = _lib.lib().rmd_version().decode()
    return info


def dicl_leg(args, world, rank, device):
    """BASELINE configs[2] / SURVEY.md §8(d) cfg3: the DICL baseline's matching stage coarse to fine at
    384x512, per-GPU b8, C = 32, displacement range (3, 3) (D = 49) on levels 6..2 (6x8 .. 96x128):
    per level the coarse flow upsampled x2 (impls/dicl.py:171-181), the warped masked integer volume
    (rmd_dicl_stack_int_warped: warp + a8 in one kernel pair, impls/dicl.py:178-238), MatchingNet
    (MIOpen, blocks/dicl.py:93-118), DAP (rmd_dap, split-bf16 MFMA) and the soft-argmin flow
    regression (impls/dicl.py:53-86, torch).  Feature maps are synthetic (the feature encoder and
    the context networks are outside §8); weights: torch default init, DAP identity, BN in eval."""
    import torch.nn.functional as F
    from rmd import ops
    from rmd.blocks.dicl import DisplacementAwareProjection, MatchingNet
    torch.backends.cudnn.allow_tf32 = False
    b = args.global_batch // world if args.global_batch else 8
    c, md, levels = 32, (3, 3), (6, 5, 4, 3, 2)
    g = torch.Generator().manual_seed(77 + rank)
    torch.manual_seed(77)
    mods = {}
    feats = {}
    for l in levels:
        h, w = 384 >> l, 512 >> l
        mods[l] = (MatchingNet(2 * c).to(device).eval(), DisplacementAwareProjection(md).to(device).eval())
        feats[l] = tuple(torch.randn(b, c, h, w, generator=g).to(device) for _ in range(2))
    du, dv = 2 * md[0] + 1, 2 * md[1] + 1
    disp = torch.stack(torch.meshgrid(torch.arange(-md[0], md[0] + 1.0), torch.arange(-md[1], md[1] + 1.0),
                                      indexing="ij")).view(1, 2, du, dv, 1, 1).to(device)
    vol_bytes = 0
    stack_args = {}

    def forward():
        nonlocal vol_bytes
        flow, vb = None, 0
        for l in levels:
            f1, f2 = feats[l]
            h, w = f1.shape[-2:]
            mnet, dap = mods[l]
            if flow is None:
                mvol = ops.dicl_stack_int(f1, f2, md[0], md[1])
                stack_args[l] = None
            else:
                up = 2.0 * F.interpolate(flow, (h, w), mode="bilinear", align_corners=True)
                mvol = ops.dicl_stack_int_warped(f1, f2, up, md[0], md[1])
                stack_args[l] = up
            vb += mvol.numel() * 4
            cost = dap(mnet(mvol))
            prob = F.softmax(cost.reshape(b, du * dv, h, w), dim=1).view(b, 1, du, dv, h, w)
            lf = (prob * disp).sum(dim=(2, 3))
            flow = lf if flow is None else lf + up
        vol_bytes = vb
        return flow

    with torch.no_grad():
        for _ in range(3):
            forward()
        torch.cuda.synchronize(device)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(device)
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            out = forward()
        torch.cuda.synchronize(device)
        el = time.perf_counter() - t0
        # the five volume launches alone, on the inputs of the last forward (HIP events on the stream
        # the C ABI launches on): algorithmic bytes = the fp32 volumes written + both feature maps (and
        # the upsampled flow) read once
        vreps = 20
        a = torch.cuda.Event(enable_timing=True)
        z = torch.cuda.Event(enable_timing=True)
        io_bytes = vol_bytes
        for l in levels:
            io_bytes += 2 * feats[l][0].numel() * 4 + (stack_args[l].numel() * 4 if stack_args[l] is not None else 0)
        a.record()
        for _ in range(vreps):
            for l in levels:
                f1, f2 = feats[l]
                if stack_args[l] is None:
                    ops.dicl_stack_int(f1, f2, md[0], md[1])
                else:
                    ops.dicl_stack_int_warped(f1, f2, stack_args[l], md[0], md[1])
        z.record()
        torch.cuda.synchronize(device)
        vol_ms = a.elapsed_time(z) / vreps
    if world > 1:
        torch.distributed.barrier()
    el = job_time(el, world, device)
    fin = bool(torch.isfinite(out).all())
    del mods, feats, out, stack_args
    torch.cuda.empty_cache()
    return {"workload": "DICL cost volumes + MatchingNet + DAP + soft-argmin, coarse to fine (levels 6..2) at "
                        "384x512 (BASELINE configs[2], SURVEY cfg3)",
            "frame_pairs_per_s": world * b * reps / el, "ms_per_batch": el / reps * 1e3, "per_gpu_batch": b,
            "global_batch": world * b, "n_gpus": world, "volume_bytes_per_batch": vol_bytes,
            "volume_ms_per_batch": vol_ms, "volume_io_bytes_per_batch": io_bytes,
            "volume_gbps": io_bytes / vol_ms / 1e6, "volume_frac_of_hbm_peak": io_bytes / vol_ms / 1e6 / 8000.0,
            "displacement_range": list(md), "channels": c, "finite": fin,
            "scaling": "strong" if args.global_batch else "weak", "dtype": "fp32",
            "data": "synthetic feature maps (encoder / context nets outside the hot path)"}


def highres_leg(args, precision):
    """SURVEY.md §8(f) rank 1 / raft_fs.py:13-87 at high resolution: a 4K frame pair (2160x3840 -> 1/8 map
    270x480, C=256, batch 2) through raft_fs.CorrBlock with 12 lookups, once with the on-the-fly lookup
    (no O(N^2) memory) and once with the all-pairs volume (an 89 GB fp16 pyramid at this size): the
    crossover the 'auto' method's memory budget stands for (tools/bench_otf.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_otf
    res = bench_otf.highres(precision, reps=3)
    import rmd
    res["auto_method_at_default_budget"] = rmd.config.choose_method("auto", 2, 270, 480, 4, precision, False,
                                                                    rmd.config.current().memory_budget)
    res["workload"] = ("raft/fs CorrBlock inference, 4K 1/8 map 270x480, C=256, b2, 4 levels, r=4, 12 lookups: "
                       "on-the-fly vs all-pairs volume")
    return res


def progress(rank, what):
    """One stderr line per leg and rank (the JSON line stays the only stdout output): shows where a
    long multi-rank run is."""
    print(f"[bench] rank {rank} {time.strftime('%H:%M:%S')} {what}", file=sys.stderr, flush=True)


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


def rank_inputs(args, rank, world, h8, w8, device):
    """Weak scaling: each rank's own batch of frame pairs (per-rank work fixed, seeds differ).
    Strong scaling (--global-batch G): rank r's contiguous G/world shard of one global batch."""
    if args.global_batch:
        b = args.global_batch // world
        f1, f2, co = synthetic(args.global_batch, args.channels, h8, w8, args.iters, 1234, "cpu")
        sl = slice(rank * b, (rank + 1) * b)
        return f1[sl].to(device), f2[sl].to(device), co[:, sl].contiguous().to(device)
    return synthetic(args.batch, args.channels, h8, w8, args.iters, 1234 + rank, device)


def init_distributed(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and world != args.gpus:
        raise SystemExit(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.dry_run:
        device = torch.device("cpu")
    else:
        device = torch.device("cuda", 0 if args.one_device else local)
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        import datetime
        tmo = datetime.timedelta(seconds=600)          # a stuck collective raises instead of hanging forever
        if device.type == "cuda" and args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=tmo)
        else:
            dist.init_process_group(args.backend, timeout=tmo)
        assert dist.get_world_size() == world
        global _HOST_GROUP
        # a gloo group for the closing barrier: ranks waiting there for rank 0's cpu_baseline block in a
        # socket read instead of spin-waiting on a RCCL stream (the CPU baseline is timed on an
        # otherwise idle host)
        _HOST_GROUP = dist.new_group(backend="gloo", timeout=tmo) if args.backend != "gloo" else None
    return world, rank, device


_HOST_GROUP = None


def host_barrier():
    """Barrier whose waiters sleep in a gloo socket read (not a spinning RCCL stream sync)."""
    import torch.distributed as dist
    dist.barrier(group=_HOST_GROUP) if _HOST_GROUP is not None else dist.barrier()


HBM_COPY_GBS = 6290.0          # measured float4 copy rate (MI355X_MICROARCH.md chip table)


def corr_leg(args, precision, inputs, world, device, steps, warmup):
    """Time `steps` hot-path steps (operand prep + correlation GEMM + `iters` lookups) after `warmup`
    untimed ones, bracketed by barrier + synchronize, job time = MAX over ranks; HIP events on the launch
    stream around the GEMM launch alone and around the lookups of every E-th timed step (never the first)."""
    ev_gemm, ev_look = [], []
    if args.dry_run:
        def step(record):
            return None
    else:
        from rmd import ops
        f1, f2, coords = inputs
        stream = torch.cuda.current_stream(device)

        def step(record):
            pyr = ops.corr_pyramid(f1, f2, args.levels, precision, events=ev_gemm if record else None)
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

    def sync():
        if not args.dry_run:
            torch.cuda.synchronize(device)

    for _ in range(warmup):
        step(False)
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    E = max(1, args.event_every)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i % E == E - 1)
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    return job_time(elapsed, world, device), ev_gemm, ev_look


def child_env(device):
    """Environment of a rank-0 child process that must run on this rank's GPU: HIP_VISIBLE_DEVICES
    narrowed to it (index into an inherited list, if any), and no torchrun rank variables."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "TORCHELASTIC_RUN_ID", "MASTER_ADDR", "MASTER_PORT")}
    if device is not None and device.type == "cuda":
        vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
        ids = vis.split(",") if vis else None
        idx = device.index or 0
        env["HIP_VISIBLE_DEVICES"] = ids[idx] if ids and idx < len(ids) else str(idx)
        env.pop("CUDA_VISIBLE_DEVICES", None)
    return env


def live_traffic(args, precision, batch, rank, device=None):
    """HBM bytes per launch of the GEMM and lookup kernels from rocprofv3 PMC counters collected in THIS
    run: separate FETCH_SIZE and WRITE_SIZE passes (one counter group each, MI355X_MICROARCH.md HBM /
    PMC sections) over tools/pmc_probe.py (the same step on the same synthetic inputs), each a child
    process under its own KILL timeout.  gfx950 corrections: both counters are KiB; FETCH_SIZE counts
    half the bytes of wide streaming reads, so it is doubled.  Returns ({kernel: bytes}, note)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not on PATH"
    d = tempfile.mkdtemp(prefix="rmd_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    per = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        out = os.path.join(d, counter.lower())
        cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "run",
               "--", sys.executable, os.path.join(ROOT, "tools", "pmc_probe.py"), "--precision", precision,
               "--batch", str(batch), "--height", str(args.height), "--width", str(args.width),
               "--channels", str(args.channels), "--iters", str(args.iters)]
        progress(rank, f"live PMC pass {counter} ({precision})")
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=d, env=child_env(device))
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            shutil.rmtree(d, ignore_errors=True)
            return None, f"rocprofv3 --pmc {counter} failed (rc {r.returncode}): {r.stderr.decode()[-200:]}"
        vals = {}
        for row in csv.DictReader(open(files[0])):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            key = "gemm" if "corr_pyramid_" in name else "lookup" if "corr_lookup_kernel" in name else None
            if key:
                vals.setdefault(key, []).append(float(row["Counter_Value"]) * 1024.0)
        for k, v in vals.items():
            per.setdefault(k, {})[counter] = (sum(v) / len(v), len(v))
    mfma = mfma_busy_pass(args, precision, batch, rank, device, d, exe)
    shutil.rmtree(d, ignore_errors=True)
    res = {}
    for k, c in per.items():
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            res[k] = {"read": 2.0 * c["FETCH_SIZE"][0], "write": c["WRITE_SIZE"][0],
                      "total": 2.0 * c["FETCH_SIZE"][0] + c["WRITE_SIZE"][0], "dispatches": c["FETCH_SIZE"][1]}
    if mfma:
        res.setdefault("gemm", {})["mfma_counters"] = mfma
    return res, ("live: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE (KiB -> B, gfx950 correction), this run, tools/pmc_probe.py "
                 f"on rank {rank}'s GPU")


def mfma_busy_pass(args, precision, batch, rank, device, d, exe):
    """Counter-evidenced MFMA utilisation of the GEMM (north_star: 'MFMA utilisation for the correlation
    GEMM'): one rocprofv3 pass of SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE with the kernel trace over
    tools/pmc_probe.py.  MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe cycles summed over
    every SIMD (32 per v_mfma_f32_32x32x16_bf16); GRBM_GUI_ACTIVE the busy cycles summed over the 8 XCDs.
      mfma_busy = MFMA cycles / (SIMDs x GRBM_GUI_ACTIVE / 8)   (fraction of the chip's matrix-pipe cycles)
      clock     = GRBM_GUI_ACTIVE / 8 / kernel duration          (the effective clock the launch ran at)
    The first dispatch (cold clocks) is dropped."""
    import csv
    import glob
    import subprocess
    out = os.path.join(d, "mfma")
    cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "--kernel-trace",
           "--output-format", "csv", "-d", out, "-o", "run",
           "--", sys.executable, os.path.join(ROOT, "tools", "pmc_probe.py"), "--precision", precision,
           "--batch", str(batch), "--height", str(args.height), "--width", str(args.width),
           "--channels", str(args.channels), "--iters", str(args.iters)]
    progress(rank, f"live PMC pass SQ_VALU_MFMA_BUSY_CYCLES ({precision})")
    r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=d, env=child_env(device))
    cfiles = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
    tfiles = glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True)
    if r.returncode != 0 or not cfiles:
        return {"error": f"rocprofv3 MFMA pass failed (rc {r.returncode}): {r.stderr.decode()[-200:]}"}
    vals, durs = {}, {}
    for row in csv.DictReader(open(cfiles[0])):
        if "corr_pyramid_" in row["Kernel_Name"]:
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals.setdefault(key, {}).setdefault(row["Counter_Name"], 0.0)
            vals[key][row["Counter_Name"]] += float(row["Counter_Value"])
    for f in tfiles:
        for row in csv.DictReader(open(f)):
            if "corr_pyramid_" in row["Kernel_Name"]:
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                durs[key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    keys = sorted((k for k in vals if "SQ_VALU_MFMA_BUSY_CYCLES" in vals[k] and "GRBM_GUI_ACTIVE" in vals[k]), key=int)
    if len(keys) > 1:
        keys = keys[1:]
    if not keys:
        return {"error": "no GEMM dispatch in the MFMA pass"}
    simds = 4 * torch.cuda.get_device_properties(device).multi_processor_count
    busy = sum(vals[k]["SQ_VALU_MFMA_BUSY_CYCLES"] for k in keys) / len(keys)
    grbm = sum(vals[k]["GRBM_GUI_ACTIVE"] for k in keys) / len(keys)
    res = {"mfma_busy": busy / (simds * grbm / 8), "SQ_VALU_MFMA_BUSY_CYCLES": busy, "GRBM_GUI_ACTIVE": grbm,
           "simds": simds, "dispatches": len(keys),
           "source": "live: rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace, this run, "
                     f"tools/pmc_probe.py on rank {rank}'s GPU"}
    dk = [durs[k] for k in keys if k in durs]
    if dk:
        res["profiled_duration_ms"] = sum(dk) / len(dk) * 1e3
        res["clock_ghz"] = grbm / 8 / (sum(dk) / len(dk)) / 1e9
    return res


def stored_traffic(precision):
    """Counter bytes of an earlier profiled run (profiles/pmc_r04.json, tiles layout; older files after it)
    — only where no live pass ran."""
    for name in ("pmc_r04.json", "pmc_r02.json", "pmc_r01.json"):
        path = os.path.join(ROOT, "profiles", name)
        if os.path.exists(path):
            try:
                with open(path) as fh:
                    e = json.load(fh).get(precision, {})
            except (OSError, ValueError):
                continue
            det = e.get("detail", {})
            res = {k: {"read": v.get("fetch_bytes"), "write": v.get("write_bytes"), "total": v.get("hbm_bytes_per_launch")}
                   for k, v in det.items() if k in ("gemm", "lookup")}
            if res:
                return res, f"stored: profiles/{name} (an earlier box and tree; no live pass in this run)"
    return {}, "none"


def storage_bytes(precision):
    """Bytes per stored pyramid element of a precision mode (fp32: RMD_S24, 3 bytes)."""
    from rmd import _lib, ops
    return {_lib.RMD_F32: 4, _lib.RMD_F16: 2, _lib.RMD_S24: 3}[ops.PRECISIONS[precision][1]]


STORAGE_NAME = {4: "fp32", 3: "s24 (fp32 rounded to 16 significant bits)", 2: "fp16"}


def rooflines(args, precision, B, h8, w8, gemm_ms, look_ms, traffic, traffic_note, n_gemm, n_look):
    """roofline dicts of the GEMM and of the lookup from their average launch times (algorithmic bytes /
    flops per launch) and the counter traffic."""
    from rmd import _lib, ops
    N = h8 * w8
    D = (2 * args.radius + 1) ** 2
    s = storage_bytes(precision)
    compute_dt = "fp32" if precision.startswith("fp32") else "bf16"
    levels = [(h8 >> i, w8 >> i) for i in range(args.levels)]
    look_bytes = B * N * (args.levels * (2 * args.radius + 2) ** 2 * s + args.levels * D * 4 + 8)
    op_bytes = 2 if precision.startswith("bf16") else 4
    gemm_bytes = B * N * sum(h * w for h, w in levels) * s + 2 * B * N * args.channels * op_bytes
    gemm_flop = 2.0 * B * N * N * args.channels
    # MFMA work actually issued: the fp32 mode runs three bf16 products per k-step (x3 kernel)
    mfma_dt, mfma_mult = ("bf16", 3.0) if precision in ("fp32", "fp32-f32", "fp32-s24") else (compute_dt, 1.0)
    look_gbs = look_bytes / (look_ms * 1e-3) / 1e9
    gemm_gbs = gemm_bytes / (gemm_ms * 1e-3) / 1e9
    gemm_tfs = gemm_flop / (gemm_ms * 1e-3) / 1e12
    traffic = traffic or {}
    kname = _lib.lib().rmd_corr_gemm_kernel(_lib.describe(B, h8, w8, args.levels, ops.PRECISIONS[precision][1]),
                                             args.channels, ops.PRECISIONS[precision][0]).decode()

    def tr(k, key):
        v = traffic.get(k, {}).get(key)
        return float(v) if v is not None else None

    gt, lt = tr("gemm", "total"), tr("lookup", "total")
    # MFMA fraction the HBM store stream allows: the algorithmic bytes moved at the measured copy rate
    # (and at the 8 TB/s spec) bound the launch time from below, so the flops over that time bound MFMA
    ceil = {r: gemm_flop * mfma_mult / (gemm_bytes / (gbs * 1e9)) / 1e12 / MFMA_PEAK[mfma_dt]
            for r, gbs in (("copy_rate", HBM_COPY_GBS), ("spec_peak", HBM_PEAK_GBS))}
    roof_gemm = {"kernel": f"corr_pyramid_{kname} (MFMA GEMM + fused pooled-pyramid epilogue)",
                 "bound": "hbm", "achieved": gemm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": gemm_gbs / HBM_PEAK_GBS, "traffic": gt,
                 "traffic_read": tr("gemm", "read"), "traffic_write": tr("gemm", "write"),
                 "traffic_over_algorithmic": gt / gemm_bytes if gt else None, "traffic_source": traffic_note,
                 "algorithmic_bytes_per_launch": gemm_bytes, "avg_launch_ms": gemm_ms, "launches_per_step": 1,
                 "event_samples": n_gemm,
                 "mfma_tflops": gemm_tfs, "mfma_peak_tflops": MFMA_PEAK[mfma_dt],
                 "mfma_frac": gemm_tfs * mfma_mult / MFMA_PEAK[mfma_dt], "mfma_products_per_flop": mfma_mult,
                 "mfma_ceiling_at_hbm": ceil["copy_rate"], "mfma_ceiling_at_hbm_spec": ceil["spec_peak"],
                 "mfma_ceiling_note": (f"algorithmic bytes at the {HBM_COPY_GBS / 1e3:.2f} TB/s measured copy rate "
                                       f"(spec {HBM_PEAK_GBS / 1e3:.0f} TB/s) cap the fused-pyramid GEMM's MFMA fraction"),
                 "algorithmic_flop_per_launch": gemm_flop}
    mc = traffic.get("gemm", {}).get("mfma_counters")
    if mc:
        roof_gemm["mfma_busy"] = mc.get("mfma_busy")
        roof_gemm["mfma_counters"] = mc
    roof_look = {"kernel": "corr_lookup_kernel", "bound": "hbm", "achieved": look_gbs, "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": look_gbs / HBM_PEAK_GBS, "traffic": lt,
                 "traffic_read": tr("lookup", "read"), "traffic_write": tr("lookup", "write"),
                 "traffic_over_algorithmic": lt / look_bytes if lt else None, "traffic_source": traffic_note,
                 "algorithmic_bytes_per_launch": look_bytes, "avg_launch_ms": look_ms,
                 "launches_per_step": args.iters, "event_samples": n_look}
    return roof_gemm, roof_look


def event_ms(evs):
    return float(np.mean([a.elapsed_time(b) for a, b in evs]))


def main():
    args = parse()
    maybe_launch(args)
    world, rank, device = init_distributed(args)
    H, W = padded(args.height, args.width)
    h8, w8 = H // 8, W // 8
    if args.global_batch:
        if args.global_batch % world:
            raise SystemExit(f"bench.py: --global-batch {args.global_batch} is not a multiple of {world} ranks")
        args.batch = args.global_batch // world
    B = args.batch

    inputs = None if args.dry_run else rank_inputs(args, rank, world, h8, w8, device)
    elapsed, ev_gemm, ev_look = corr_leg(args, args.precision, inputs, world, device, args.steps, args.warmup)

    s = storage_bytes(args.precision)
    compute_dt = "fp32" if args.precision.startswith("fp32") else "bf16"
    res = {
        "metric": "frame-pairs/s @436x1024 RAFT 12 iters (1-8 GPU); corr MFMA% + lookup HBM%",
        "value": world * B * args.steps / elapsed,
        "unit": "frame-pairs/s",
        "value_scope": ("the cost-volume hot path only (SURVEY §8): correlation GEMM + pooled pyramid + 12 "
                        "lookups per frame pair, not the whole RAFT network (that figure is "
                        "model_level.frame_pairs_per_s)"),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch else "weak",
        "vs_baseline": None,
        "dtype": compute_dt,
        "data": "synthetic (seeded random 1/8-res feature maps + smooth moving flow; no dataset)",
        "library": _library_info(),
        "config": {"workload": "RAFT all-pairs correlation + 4-level pyramid + 12 radius-4 lookups "
                               "(BASELINE configs[1]); the whole network is the 'model_level' key",
                   "image": f"{args.height}x{args.width} padded {H}x{W}", "feature_map": f"{h8}x{w8}",
                   "channels": args.channels, "batch_per_gpu": B, "global_batch": B * world,
                   "lookups_per_step": args.iters, "precision": args.precision,
                   "pyramid_storage": STORAGE_NAME[s], "parallelism": f"batch-shard x{world}"},
    }
    if args.dry_run:
        res["dry_run"] = "launcher / collective plumbing only: no GPU work, value meaningless"
        if args.model_level == "on":
            res["model_level"] = model_leg(args, world, rank, device)
    else:
        # rank 0 profiles its own GPU in child processes after the timed region (the other ranks go on
        # to the next leg and wait for rank 0 at its first barrier)
        live = rank == 0 and args.live_pmc == "on"
        # both timed legs run before any profiling child process: the counter passes leave the chip in
        # another power / thermal state for a while, and the power-bound x3 GEMM of the fp32 leg ran ~15 %
        # slower right after them (profiles/INDEX_r06.md)
        fp32_leg = args.fp32_mode == "on" and args.precision != "fp32"
        if fp32_leg:
            progress(rank, "fp32_mode leg")
            w32 = max(3, args.warmup)
            el32, eg32, el32l = corr_leg(args, "fp32", inputs, world, device, args.fp32_steps, w32)
        traffic, note = live_traffic(args, args.precision, B, rank, device) if live else (None, "")
        if traffic is None:
            fallback, fnote = stored_traffic(args.precision)
            traffic, note = fallback, (f"{note}; " if note else "") + fnote
        roof_gemm, roof_look = rooflines(args, args.precision, B, h8, w8, event_ms(ev_gemm),
                                         event_ms(ev_look) / args.iters, traffic, note, len(ev_gemm), len(ev_look))
        dominant_gemm = roof_gemm["avg_launch_ms"] >= roof_look["avg_launch_ms"] * args.iters
        res["roofline"] = roof_gemm if dominant_gemm else roof_look
        res["roofline_gemm"] = roof_gemm
        res["roofline_lookup"] = roof_look
        progress(rank, "headline leg done")
        if fp32_leg:
            # the parity mode (north_star's fp32 gate) on the same inputs: x3 GEMM + 24-bit pyramid
            tr32, n32 = live_traffic(args, "fp32", B, rank, device) if live else (None, "")
            if tr32 is None:
                fb, fn = stored_traffic("fp32")
                tr32, n32 = fb, (f"{n32}; " if n32 else "") + fn
            g32, l32 = rooflines(args, "fp32", B, h8, w8, event_ms(eg32), event_ms(el32l) / args.iters, tr32, n32,
                                 len(eg32), len(el32l))
            if rank == 0:
                res["fp32_mode"] = {"value": world * B * args.fp32_steps / el32, "unit": "frame-pairs/s",
                                    "ms_per_step": el32 / args.fp32_steps * 1e3, "steps": args.fp32_steps,
                                    "warmup": w32, "precision": "fp32", "dtype": "fp32",
                                    "pyramid_storage": STORAGE_NAME[storage_bytes("fp32")],
                                    "storage_note": ("'fp32' mode stores the pyramid as RMD_S24: each fp32 value "
                                                     "rounded to its top 24 bits (16 significant bits, <= 2^-16 "
                                                     "relative); 'fp32-f32' keeps 4-byte storage"),
                                    "gemm": "split-bf16 x3 MFMA (hi.hi + hi.lo + lo.hi), fp32 accumulate",
                                    "roofline_gemm": g32, "roofline_lookup": l32}
        del inputs
        torch.cuda.empty_cache()
        # extra legs run on every rank (batch shards / DDP collectives); a Python-level failure in one
        # (raised symmetrically on every rank, e.g. out of memory) is recorded instead of losing the
        # headline line
        for flag, key, leg in ((args.model_level, "model_level", model_leg), (args.dicl, "dicl_matching", dicl_leg),
                               (args.hybrid, "hybrid_inference", hybrid_leg), (args.train, "train_step", train_leg)):
            if flag != "on":
                continue
            progress(rank, f"{key} leg")
            try:
                out = leg(args, world, rank, device)
            except Exception as e:                      # noqa: BLE001 — reported in the JSON line
                out = {"error": f"{type(e).__name__}: {e}"[:500]}
                torch.cuda.empty_cache()
            if rank == 0:
                res[key] = out
    if rank == 0 and world == 1 and not args.dry_run and args.highres == "on":
        progress(rank, "highres_fs leg")
        try:
            res["highres_fs"] = highres_leg(args, args.precision)
        except Exception as e:                          # noqa: BLE001 — reported in the JSON line
            res["highres_fs"] = {"error": f"{type(e).__name__}: {e}"[:500]}
        torch.cuda.empty_cache()
    if rank == 0:
        if not args.no_cpu_baseline:
            # rank 0 only, after every GPU leg: the other ranks wait at the barrier below
            progress(rank, "cpu_baseline leg")
            res["cpu_baseline"] = cpu_baseline(args)
            if world > 1:
                res["cpu_baseline"]["note"] = (f"rank 0 of {world}, timed after every GPU leg while the other ranks "
                                               f"sleep in a gloo barrier (no spin-waiting HIP sync on the host)")
        print(json.dumps(res), flush=True)
    if world > 1:
        if not args.dry_run:
            torch.cuda.synchronize(device)
        host_barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
