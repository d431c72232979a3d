#!/usr/bin/env python3
"""Component benchmark of the non-headline §8 kernels at BASELINE.json's configs (MI355X only).

Times each op with HIP events on its launch stream (median of `reps` launches after warm-up) and
reports algorithmic HBM bytes per launch, GB/s and the fraction of the 8 TB/s HBM peak:
  * a6  rmd_dicl_stack        cfg4 (KITTI 384x1280 -> 1/8 level 48x160, C=32, r=4, B=8)
  * a6' rmd_dicl_stack_backward (same shape)
  * a8  rmd_dicl_stack_int    cfg3 (DICL 384x512 -> level 2 96x128, C=32, ru=rv=3, B=8)
  * a9  rmd_dap               cfg4 1/8 level, D=81, B=8 (and D=324 'full')
  * a11 rmd_corr_lookup_backward + pyramid backward (GEMMs) at cfg5 (FlyingChairs 384x512 -> 48x64,
        C=256, B=6, 12 lookups)
  * a4  raft_fs.CorrBlock forward at cfg2 (pyramid with scale 1 + 12 lookups), bf16
The MatchingNet that consumes a6/a8 (MIOpen convolutions, out of scope) is timed beside them.
  * f1  on-the-fly lookup (rmd_corr_otf_*) at cfg2: prepare + per-lookup time, bf16 / fp32
  * f2  flow heads at cfg2 (B=8, 55x128): rmd_up8 (+backward), rmd_softargmax L=4 r=4 (+backward),
        each beside the reference's eager torch formulation on the same GPU (raft.py:112-135, 319-331)
  * f4  input format (rmd.input: clip + range + modulo padding + NCHW) for 8 frame pairs at 436x1024,
        beside the reference's numpy path plus the host-to-device copy
  * f3  warped DICL volume (rmd_dicl_stack_int_warped) at cfg3 level 2 (B=8, C=32, 96x128, ru=rv=3) and
        rmd_warp_backwards alone, beside the reference's eager warp (warp.py:5-33)
usage: python tools/bench_components.py [reps] [fs|heads]   -> one JSON document on stdout
      ('fs' runs only the a4 / f1 part, 'heads' only f2)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-meets-dicl_amd"))
import torch  # noqa: E402

PEAK = 8000.0


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ts)
    return ms[len(ms) // 2]


def entry(ms, nbytes, **kw):
    gbs = nbytes / (ms * 1e-3) / 1e9
    return dict(ms=ms, algorithmic_bytes=nbytes, achieved_GBps=gbs, frac_of_hbm_peak=gbs / PEAK, **kw)


def main():
    import rmd
    from rmd import ops
    from rmd.blocks.dicl import MatchingNet
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    only = sys.argv[2] if len(sys.argv) > 2 else ""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {}

    def smooth_coords(b, h, w, amp=3.0):
        """grid + a smooth flow (low-res noise upsampled), as bench.py: the coordinates a flow
        network produces; per-pixel i.i.d. noise would scatter every gather and atomic."""
        ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
        low = torch.randn(b, 2, max(h // 8, 2), max(w // 8, 2), generator=g) * amp
        flow = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=True)
        return (torch.stack([xs, ys]).float()[None] + flow).to(dev)

    if only == "heads":
        heads(res, reps, dev, g)
        print(json.dumps(res, indent=1))
        return

    if only != "fs":
        # a6: DICL displacement stack, cfg4 1/8 level
        b, c, h, w, r = 8, 32, 48, 160, 4
        f1 = torch.randn(b, c, h, w, generator=g).to(dev)
        f2 = torch.randn(b, c, h, w, generator=g).to(dev)
        co = smooth_coords(b, h, w)
        d = (2 * r + 1) ** 2
        out_bytes = b * d * 2 * c * h * w * 4
        res["a6_dicl_stack_cfg4"] = entry(timed(lambda: ops.dicl_stack(f1, f2, co, r), reps),
                                          out_bytes + 2 * f1.numel() * 4 + co.numel() * 4,
                                          shape=f"B{b} C{c} {h}x{w} r{r}", output_GB=out_bytes / 1e9)
        stack = ops.dicl_stack(f1, f2, co, r)
        gst = torch.randn_like(stack)
        f1g, f2g = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)

        def stack_bwd():
            st = ops.dicl_stack(f1g, f2g, co, r)
            torch.autograd.grad(st, (f1g, f2g), gst)
        fwd_ms = res["a6_dicl_stack_cfg4"]["ms"]
        res["a6_dicl_stack_backward_cfg4"] = entry(max(timed(stack_bwd, reps) - fwd_ms, 1e-6),
                                                   out_bytes + 2 * f1.numel() * 4,
                                                   note="forward+backward time minus forward time")
        # a7: raft_dicl_ml level 1 (fmap2 at 24x80, grid scaled by (w_l - 1)/(w - 1)): general kernels
        f2l = torch.randn(b, c, h // 2, w // 2, generator=g).to(dev)
        res["a7_dicl_ml_level1_stack_cfg4"] = entry(timed(lambda: ops.dicl_stack(f1, f2l, co, r, level=1, norm_hw=(h, w)), reps),
                                                    out_bytes + f1.numel() * 4 + f2l.numel() * 4)
        stl = ops.dicl_stack(f1, f2l, co, r, level=1, norm_hw=(h, w))
        gstl = torch.randn_like(stl)
        f2lg = f2l.clone().requires_grad_(True)

        def ml_bwd():
            torch.autograd.grad(ops.dicl_stack(f1g, f2lg, co, r, level=1, norm_hw=(h, w)), (f1g, f2lg), gstl)
        res["a7_dicl_ml_level1_stack_backward_cfg4"] = entry(
            max(timed(ml_bwd, reps) - res["a7_dicl_ml_level1_stack_cfg4"]["ms"], 1e-6), out_bytes,
            note="forward+backward time minus forward time")
        del stl, gstl
        mnet = MatchingNet(2 * c).to(dev).eval()
        with torch.no_grad():
            res["a10_matchingnet_cfg4_consumer"] = {"ms": timed(lambda: mnet(stack), max(3, reps // 4)),
                                                    "note": "MIOpen convolutions, out of scope (context)"}
        del stack, gst

        # a8: DICL integer volume, cfg3 level 2
        b, c, h, w = 8, 32, 96, 128
        g1 = torch.randn(b, c, h, w, generator=g).to(dev)
        g2 = torch.randn(b, c, h, w, generator=g).to(dev)
        out_bytes = b * 49 * 2 * c * h * w * 4
        res["a8_dicl_stack_int_cfg3"] = entry(timed(lambda: ops.dicl_stack_int(g1, g2, 3, 3), reps),
                                              out_bytes + 2 * g1.numel() * 4, shape=f"B{b} C{c} {h}x{w} ru=rv=3",
                                              output_GB=out_bytes / 1e9)

        # a9: DAP
        for dd, name in ((81, "a9_dap_d81_cfg4"), (324, "a9_dap_d324_full")):
            x = torch.randn(8, dd, 48 * 160, generator=g).to(dev)
            wgt = torch.randn(dd, dd, generator=g).to(dev) / dd
            res[name] = entry(timed(lambda: ops.dap(x, wgt), reps), 2 * x.numel() * 4 + wgt.numel() * 4,
                              flop=2.0 * x.numel() * dd)

        # a11: RAFT correlation backward at cfg5 (12 lookups + pyramid backward)
        b, c, h, w = 6, 256, 48, 64
        p1 = torch.randn(b, c, h, w, generator=g).to(dev).requires_grad_(True)
        p2 = torch.randn(b, c, h, w, generator=g).to(dev).requires_grad_(True)
        cos = [smooth_coords(b, h, w) for _ in range(12)]
        gos = [torch.randn(b, 324, h, w, generator=g).to(dev) for _ in range(12)]

        def fwd():
            cb = rmd.raft.CorrBlock(p1, p2, 4, 4, precision="bf16")
            return sum((cb(cc) * gg).sum() for cc, gg in zip(cos, gos))

        def fwd_bwd():
            torch.autograd.grad(fwd(), (p1, p2))
        with torch.no_grad():
            t_f = timed(lambda: [rmd.raft.CorrBlock(p1.detach(), p2.detach(), 4, 4, precision="bf16")(cc) for cc in cos], reps)
        t_fb = timed(fwd_bwd, max(3, reps // 2))
        res["a11_corr_backward_cfg5"] = {"forward_ms": t_f, "forward_backward_ms": t_fb,
                                         "shape": f"B{b} C{c} {h}x{w}, 12 lookups",
                                         "note": "forward_backward includes the loss multiply-adds (torch)"}

    # a4: raft_fs block at cfg2
    b, c, h, w = 8, 256, 55, 128
    q1 = torch.randn(b, c, h, w, generator=g).to(dev)
    q2 = torch.randn(b, c, h, w, generator=g).to(dev)
    cq = smooth_coords(b, h, w)
    def fs_step():
        cb = rmd.raft_fs.CorrBlock(q1, q2, 4, 4, precision="bf16")
        for _ in range(12):
            cb(cq)
    with torch.no_grad():
        res["a4_raft_fs_cfg2_pyramid_plus_12_lookups_bf16"] = {"ms": timed(fs_step, reps)}
        # f1: on-the-fly lookup (no volume), bf16 and exact-f32 MFMA
        for prec in ("bf16", "fp32"):
            st = ops.otf_prepare(q1, q2, 4, prec)
            t_prep = timed(lambda: ops.otf_prepare(q1, q2, 4, prec), reps)
            t_look = timed(lambda: ops.otf_lookup(st, cq, 4), reps)
            es = 2 if prec == "bf16" else 4
            rows = b * (h * w + sum((h >> l) * (w >> l) for l in range(4))) * c * es
            out_b = b * 4 * 81 * h * w * 4
            res[f"f1_otf_cfg2_{prec}"] = dict(
                prepare_ms=t_prep, lookup_ms=t_look, step_12_lookups_ms=t_prep + 12 * t_look,
                lookup_algorithmic_bytes=rows + out_b + cq.numel() * 4,
                lookup_GBps=(rows + out_b + cq.numel() * 4) / (t_look * 1e-3) / 1e9,
                workspace_MB=st.ws.numel() / 1e6)
    print(json.dumps(res, indent=1))


def heads(res, reps, dev, g):
    """f2: per-iteration flow heads at cfg2, vs the reference's eager torch formulation (same GPU)."""
    import torch.nn.functional as F
    from rmd import ops
    b, h, w = 8, 55, 128
    n = h * w
    mask = torch.randn(b, 576, h, w, generator=g).to(dev)
    flow = torch.randn(b, 2, h, w, generator=g).to(dev)

    def up8_eager():                       # raft.py:319-331
        m = torch.softmax(mask.view(b, 1, 9, 8, 8, h, w) / 4.0, dim=2)
        u = F.unfold(8 * flow, (3, 3), padding=1).view(b, 2, 9, 1, 1, h, w)
        return torch.sum(m * u, dim=2).permute(0, 1, 4, 2, 5, 3).reshape(b, 2, h * 8, w * 8)

    with torch.no_grad():
        t = timed(lambda: ops.up8(mask, flow, 4.0), reps)
        res["f2_up8_cfg2"] = entry(t, (b * 576 * n + b * 2 * n + b * 2 * 64 * n) * 4,
                                   eager_torch_ms=timed(up8_eager, reps))
    mg, fg = mask.clone().requires_grad_(True), flow.clone().requires_grad_(True)
    go = torch.randn(b, 2, 8 * h, 8 * w, generator=g).to(dev)
    out = ops.up8(mg, fg, 4.0)
    t_b = timed(lambda: torch.autograd.grad(out, (mg, fg), go, retain_graph=True), reps)
    mge, fge = mask.clone().requires_grad_(True), flow.clone().requires_grad_(True)
    m = torch.softmax(mge.view(b, 1, 9, 8, 8, h, w) / 4.0, dim=2)
    u = F.unfold(8 * fge, (3, 3), padding=1).view(b, 2, 9, 1, 1, h, w)
    oute = torch.sum(m * u, dim=2).permute(0, 1, 4, 2, 5, 3).reshape(b, 2, h * 8, w * 8)
    t_be = timed(lambda: torch.autograd.grad(oute, (mge, fge), go, retain_graph=True), reps)
    # backward bytes: mask + grad_out read, grad_mask written, flow/q traffic (72 B/pixel x2)
    res["f2_up8_backward_cfg2"] = entry(t_b, (2 * b * 576 * n + b * 2 * 64 * n + 2 * b * 18 * n + 4 * b * n) * 4,
                                        eager_torch_ms=t_be)

    L, r = 4, 4
    cost = (3 * torch.randn(b, L * 81, h, w, generator=g)).to(dev)
    d = torch.stack(torch.meshgrid(torch.linspace(-r, r, 9), torch.linspace(-r, r, 9), indexing="ij"), -1).to(dev)

    def sam_eager():                       # raft.py:112-135
        out = []
        for lvl, c in enumerate(torch.split(cost, 81, dim=1)):
            s = F.softmax(c.reshape(b, 81, 1, h, w), dim=1)
            out.append(torch.sum(d.view(1, 81, 2, 1, 1) * 2 ** lvl * s, dim=1))
        return out

    with torch.no_grad():
        res["f2_softargmax_L4_r4_cfg2"] = entry(timed(lambda: ops.softargmax(cost, L, r), reps),
                                                (cost.numel() + L * b * 2 * n) * 4, eager_torch_ms=timed(sam_eager, reps))
    cg = cost.clone().requires_grad_(True)
    fl = ops.softargmax(cg, L, r)
    gfl = [torch.randn_like(f) for f in fl]
    # f3: warped integer volume, cfg3 level 2
    from rmd import warp as rwarp
    bb, c, hh, ww = 8, 32, 96, 128
    f1 = torch.randn(bb, c, hh, ww, generator=g).to(dev)
    f2 = torch.randn(bb, c, hh, ww, generator=g).to(dev)
    wfl = (2 * torch.randn(bb, 2, hh, ww, generator=g)).to(dev)

    def warp_eager():                      # warp.py:5-33
        gx = torch.arange(ww, device=dev).view(1, ww).expand(hh, -1)
        gy = torch.arange(hh, device=dev).view(hh, 1).expand(-1, ww)
        fpos = (torch.stack((gx, gy), 0).float() + wfl).permute(0, 2, 3, 1)
        fpos[..., 0] = 2 * fpos[..., 0] / (ww - 1) - 1
        fpos[..., 1] = 2 * fpos[..., 1] / (hh - 1) - 1
        est = F.grid_sample(f2, fpos, align_corners=True)
        m = F.grid_sample(torch.ones(f2.shape, device=dev), fpos, align_corners=True) > (1.0 - 1e-5)
        return est * m, m

    with torch.no_grad():
        nbytes = bb * c * hh * ww * 4
        res["f3_warp_backwards_cfg3_l2"] = entry(timed(lambda: rwarp.warp_backwards(f2, wfl), reps),
                                                 2 * nbytes + wfl.numel() * 4 + bb * hh * ww,
                                                 eager_torch_ms=timed(warp_eager, reps))
        vol = 49 * 2 * nbytes                # (B, 7, 7, 2C, h, w) fp32
        res["f3_dicl_stack_int_warped_cfg3_l2"] = entry(
            timed(lambda: ops.dicl_stack_int_warped(f1, f2, wfl, 3, 3), reps), vol + 3 * nbytes + wfl.numel() * 4,
            unwarped_ms=timed(lambda: ops.dicl_stack_int(f1, f2, 3, 3), reps),
            eager_warp_then_rmd_volume_ms=timed(lambda: ops.dicl_stack_int(f1, warp_eager()[0], 3, 3), reps))
    res["f2_softargmax_backward_L4_r4_cfg2"] = entry(
        timed(lambda: torch.autograd.grad(fl, cg, gfl, retain_graph=True), reps),
        (2 * cost.numel() + L * b * 2 * n) * 4)

    # f4: input format at cfg2 (8 frame pairs 436x1024 RGB -> padded 440x1024 NCHW in [-1, 1]), frames
    # already resident in HBM; beside the reference's host path (numpy clip/range/pad + permute +
    # host-to-device copy of the padded pair), input.py:208-281
    import numpy as np
    from rmd.input import InputSpec, ModuloPadding
    spec = InputSpec(padding=ModuloPadding("zeros", [8, 8]))
    fr = torch.rand(b, 436, 1024, 3, generator=g)
    fr1, fr2 = fr.to(dev), fr.flip(0).to(dev)
    nbytes = 2 * (fr.numel() * 4 + b * 3 * 440 * 1024 * 4)
    npf = fr.numpy()

    def host_ref():
        out = []
        for im in (npf, npf[::-1]):
            x = 2.0 * np.clip(im, 0.0, 1.0) - 1.0
            x = np.pad(x, ((0, 0), (0, 4), (0, 0), (0, 0)), mode="constant", constant_values=0.0)
            out.append(torch.from_numpy(x).float().permute(0, 3, 1, 2).to(dev))
        return out
    res["f4_input_pair_cfg2"] = entry(timed(lambda: spec.prepare(fr1, fr2), reps), nbytes,
                                      host_numpy_plus_copy_ms=timed(host_ref, max(3, reps // 4)))


if __name__ == "__main__":
    main()
