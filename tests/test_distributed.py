"""Multi-process paths.

* Inference shards frame pairs across ranks with no data-path collective; the only exchange is the
  MAX of the timed region (bench.job_time).  Checked with world_size 2 on `gloo` (CPU).
* Training: DDP's bucketed gradient all-reduce over the custom autograd of rmd.raft.CorrBlock.
  Checked on the GPU box with two ranks sharing cuda:0 over `gloo` (the 8-GPU RCCL run is the
  driver's): DDP-averaged gradients equal the single-process gradient of the concatenated batch.
"""

import json
import os
import subprocess
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _job_time_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import argparse

    import bench
    _init(rank, world, port)
    try:
        t = bench.job_time(0.5 + rank, world, torch.device("cpu"))
        args = argparse.Namespace(batch=2, channels=8, iters=3, global_batch=0)
        f1, _, co = bench.rank_inputs(args, rank, world, 5, 6, torch.device("cpu"))
        # strong scaling: the ranks' shards are the consecutive slices of one global batch of 4
        sargs = argparse.Namespace(batch=0, channels=8, iters=3, global_batch=4)
        s1, _, sco = bench.rank_inputs(sargs, rank, world, 5, 6, torch.device("cpu"))
        g1, _, gco = bench.synthetic(4, 8, 5, 6, 3, 1234, "cpu")
        strong_ok = (tuple(s1.shape) == (2, 8, 5, 6) and torch.equal(s1, g1[2 * rank: 2 * rank + 2])
                     and torch.equal(sco, gco[:, 2 * rank: 2 * rank + 2]))
        q.put((rank, t, float(f1.sum()), tuple(co.shape), strong_ok))
    finally:
        dist.destroy_process_group()


def test_bench_job_time_is_max_over_ranks_and_shards_differ():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_job_time_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [1.5, 1.5]          # both ranks report the slowest rank's time
    assert res[0][2] != res[1][2]                     # each rank has its own frame pairs
    assert res[0][3] == (3, 2, 2, 5, 6)
    assert res[0][4] and res[1][4]                    # strong-scaling shards tile the global batch


class _TinyCorrNet(torch.nn.Module):
    """1x1-conv 'encoder' -> rmd.raft.CorrBlock -> 2 lookups: parameters get gradients only through
    the correlation autograd (rmd_corr_lookup_backward + pyramid backward)."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.enc = torch.nn.Conv2d(3, 32, 1)
        with torch.no_grad():
            self.enc.weight.copy_(torch.randn(self.enc.weight.shape, generator=g) * 0.3)
            self.enc.bias.zero_()

    def forward(self, img1, img2, coords):
        import rmd
        cb = rmd.raft.CorrBlock(self.enc(img1), self.enc(img2), 2, 2, precision="fp32")
        return sum(cb(coords + 0.5 * k).square().mean() for k in range(2))


def _inputs(b, seed):
    g = torch.Generator().manual_seed(seed)
    img1 = torch.randn(b, 3, 12, 16, generator=g)
    img2 = torch.randn(b, 3, 12, 16, generator=g)
    ys, xs = torch.meshgrid(torch.arange(12.0), torch.arange(16.0), indexing="ij")
    co = torch.stack([xs, ys])[None] + torch.randn(b, 2, 12, 16, generator=g)
    return img1, img2, co


def _ddp_worker(rank, world, port, q, device="cuda"):
    sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
    if device == "cpu":
        torch.set_num_threads(1)
    _init(rank, world, port)
    try:
        dev = torch.device("cuda", 0) if device == "cuda" else torch.device("cpu")
        net = torch.nn.parallel.DistributedDataParallel(_TinyCorrNet().to(dev))
        img1, img2, co = (t.to(dev) for t in _inputs(4, 10 + rank))
        net(img1, img2, co).backward()
        q.put((rank, net.module.enc.weight.grad.cpu().numpy(), net.module.enc.bias.grad.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def _ddp_check(world, device):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q, device)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
    dev = torch.device("cuda", 0) if device == "cuda" else torch.device("cpu")
    net = _TinyCorrNet().to(dev)
    loss = 0.0
    for r in range(world):             # mean over ranks of each rank's loss == DDP's averaged gradient
        img1, img2, co = (t.to(dev) for t in _inputs(4, 10 + r))
        loss = loss + net(img1, img2, co) / world
    loss.backward()
    ref_w = net.enc.weight.grad.cpu().numpy()
    ref_b = net.enc.bias.grad.cpu().numpy()
    for _, gw, gb in res:
        np.testing.assert_allclose(gw, ref_w, rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(gb, ref_b, rtol=1e-4, atol=1e-6)
    assert np.abs(ref_w).max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_ddp_gradient_allreduce_through_corr_autograd(world):
    """world ranks share cuda:0 over gloo: the HIP correlation forward/backward under DDP."""
    _ddp_check(world, "cuda")


@pytest.mark.parametrize("world", [4])
def test_ddp_gradient_allreduce_through_corr_autograd_cpu(world):
    """The same DDP gradient check on CPU tensors (the operators' CPU kernels, rmd/cpu.py) at world 4:
    the bucketed all-reduce over the correlation autograd, rehearsed without a GPU."""
    _ddp_check(world, "cpu")


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_launches_its_own_ranks(world):
    """`bench.py --gpus N` started as one plain process spawns N ranks through
    torch.distributed.run (the same launcher the driver uses) and reports n_gpus = the world size
    the process group reports.  --dry-run skips the GPU work (gloo on CPU here)."""
    import json
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dry-run",
                          "--backend", "gloo", "--no-cpu-baseline", "--steps", "2", "--warmup", "1",
                          "--model-level", "off"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout                      # rank 0 alone prints the JSON line
    res = json.loads(lines[0])
    assert res["n_gpus"] == world and res["config"]["global_batch"] == 8 * world
    assert res["steps"] == 2 and res["scaling"] == "weak"


def test_bench_strong_scaling_split():
    """--global-batch 8 over 2 ranks: 4 pairs per rank, scaling "strong", value counts 8 per step."""
    import json
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--backend", "gloo", "--no-cpu-baseline", "--steps", "2", "--warmup", "1",
                          "--global-batch", "8", "--model-level", "off"], capture_output=True, text=True, timeout=300,
                         env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert res["scaling"] == "strong" and res["config"]["global_batch"] == 8
    assert res["config"]["batch_per_gpu"] == 4
    assert abs(res["value"] - 8 * 2 / (res["ms_per_step"] * 2 / 1e3)) < 1e-6 * res["value"]


@pytest.mark.parametrize("gb", [0, 4])
def test_bench_model_level_leg_is_batch_sharded(gb):
    """The whole-network leg (BASELINE.md's frame-pairs/s of the cfg2 model at 1/2/4/8 GPUs) runs on
    EVERY rank with its own batch shard and reports the job time MAX over ranks: 2 gloo ranks, weak
    (8 pairs per rank) and strong (--global-batch 4 -> 2 per rank).  --dry-run runs a small frame through
    the eager correlation on the CPU: the plumbing, not the kernels."""
    import json
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--backend", "gloo",
           "--no-cpu-baseline", "--steps", "1", "--warmup", "0"] + (["--global-batch", str(gb)] if gb else [])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    ml = res["model_level"]
    per = gb // 2 if gb else 8
    assert ml["n_gpus"] == 2 and ml["per_gpu_batch"] == per and ml["global_batch"] == 2 * per
    assert ml["scaling"] == ("strong" if gb else "weak")
    assert abs(ml["frame_pairs_per_s"] - 2 * per / (ml["ms_per_batch"] / 1e3)) < 1e-6 * ml["frame_pairs_per_s"]
    assert np.isfinite(ml["rank0_flow_checksum"])
    # both ranks reached the leg (progress lines on stderr)
    assert "rank 0" in out.stderr and "rank 1" in out.stderr and "model_level" in out.stderr


def test_bench_rank0_cpu_baseline_at_two_ranks():
    """N > 1: rank 0 still times the CPU baseline (after every GPU leg, the other ranks waiting at a
    barrier) and the one JSON line carries it; gloo dry run on the CPU."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--backend",
                          "gloo", "--steps", "1", "--warmup", "0", "--model-level", "off", "--cpu-budget-s", "0.5"],
                         capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    cb = res["cpu_baseline"]
    assert res["n_gpus"] == 2 and cb["value"] > 0 and cb["cores"] >= 1 and "rank 0 of 2" in cb["note"]


def test_child_env_pins_rank_gpu():
    import importlib
    import torch
    bench = importlib.import_module("bench")
    os.environ["HIP_VISIBLE_DEVICES"] = "4,5,6,7"
    try:
        env = bench.child_env(torch.device("cuda", 2))
    finally:
        del os.environ["HIP_VISIBLE_DEVICES"]
    assert env["HIP_VISIBLE_DEVICES"] == "6" and "RANK" not in env and "WORLD_SIZE" not in env
    assert bench.child_env(torch.device("cuda", 1))["HIP_VISIBLE_DEVICES"] == "1"


def test_bench_rejects_world_size_mismatch():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run",
                          "--no-cpu-baseline"], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr


def _rccl_worker(port, q):
    """One rank on the RCCL ("nccl") backend: process-group init, an all_reduce and a DDP step through the
    correlation autograd on cuda:0 (RCCL cannot put two ranks on one GPU, so the 1-GPU box exercises
    the backend itself; the N-rank data path is the gloo test above and the driver's 8-GPU bench)."""
    sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        t = torch.full((4,), 2.0, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        net = torch.nn.parallel.DistributedDataParallel(_TinyCorrNet().to(dev), device_ids=[0])
        img1, img2, co = (x.to(dev) for x in _inputs(4, 10))
        net(img1, img2, co).backward()
        q.put((dist.get_backend(), float(t.sum()), net.module.enc.weight.grad.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_backend_ddp_step_one_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    backend, s, gw = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl" and s == 8.0
    sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
    dev = torch.device("cuda", 0)
    net = _TinyCorrNet().to(dev)
    img1, img2, co = (x.to(dev) for x in _inputs(4, 10))
    net(img1, img2, co).backward()
    np.testing.assert_allclose(gw, net.enc.weight.grad.cpu().numpy(), rtol=1e-5, atol=1e-7)
