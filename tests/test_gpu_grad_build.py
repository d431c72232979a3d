"""rmd_corr_grad_build (corr_backward.hip): G of every lookup of a forward written in one pass must
equal, bit for bit, the sequence of rmd_corr_lookup_backward calls into a zeroed G that it replaces
(same per-lookup arithmetic, same summation order) — the sequential kernel is itself checked against
the float64 oracle (test_gpu_corr.py backward tests), so this pins the build to the same oracle.
Covers ragged query counts, widths not a multiple of 8, 1-pixel (NaN) levels, zeroed levels, every
radius, more lookups than one launch holds (the accumulate path), coordinates far outside / NaN,
accumulate = 1 into a non-zero G and the empty list."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from rmd import _lib as L
    return L


def _desc(b, h, w, levels):
    L = _lib()
    d = L.PyramidDesc()
    L.check(L.lib().rmd_pyramid_describe(b, h, w, levels, L.RMD_F32, ctypes.byref(d)), "describe")
    return d


def _inputs(b, h, w, levels, radius, n, seed, spread=3.0, wild=False):
    rng = np.random.default_rng(seed)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    grid = np.stack([xs, ys])[None].astype(np.float64)
    d = 2 * radius + 1
    out = []
    for i in range(n):
        co = grid + rng.normal(0, spread, (b, 2, h, w)) + rng.normal(0, 2.0, (b, 2, 1, 1))
        if wild:
            co.reshape(-1)[rng.integers(0, co.size, 40)] = rng.choice([1e9, -1e9, 3e5, np.nan], 40)
        go = rng.standard_normal((b, levels * d * d, h, w))
        out.append((torch.tensor(go, dtype=torch.float32, device="cuda"),
                    torch.tensor(co, dtype=torch.float32, device="cuda")))
    return out


def _sequential(d, lookups, radius, masks, init=None):
    L = _lib()
    t = L.lib().rmd_corr_grad_targets(d.height, d.width, d.levels)
    G = torch.zeros(d.batch * d.height * d.width * t, dtype=torch.float32, device="cuda") if init is None \
        else init.clone()
    for (go, co), m in zip(lookups, masks):
        L.check(L.lib().rmd_corr_lookup_backward(ctypes.c_void_p(go.data_ptr()), ctypes.byref(d),
                                                 ctypes.c_void_p(co.data_ptr()), radius, m,
                                                 ctypes.c_void_p(G.data_ptr()), None), "lookup_backward")
    return G


def _build(d, lookups, radius, masks, init=None):
    L = _lib()
    t = L.lib().rmd_corr_grad_targets(d.height, d.width, d.levels)
    G = torch.full((d.batch * d.height * d.width * t,), float("nan"), dtype=torch.float32, device="cuda") \
        if init is None else init.clone()
    n = len(lookups)
    gouts = (ctypes.c_void_p * max(n, 1))(*[go.data_ptr() for go, _ in lookups])
    cos = (ctypes.c_void_p * max(n, 1))(*[co.data_ptr() for _, co in lookups])
    ms = (ctypes.c_uint * max(n, 1))(*masks)
    L.check(L.lib().rmd_corr_grad_build(gouts, cos, ms, n, ctypes.byref(d), radius, 0 if init is None else 1,
                                        ctypes.c_void_p(G.data_ptr()), None), "grad_build")
    return G


@pytest.mark.parametrize("b,h,w,levels,radius,n", [
    (2, 19, 26, 4, 3, 3),          # 494 queries (ragged wave), widths 26 / 13 / 6 / 3
    (1, 55, 128, 4, 4, 12),        # cfg2 image, the RAFT iteration count
    (3, 9, 70, 4, 4, 5),           # level 3 is 1 x 8: the reference's NaN level, no gradient
    (1, 23, 41, 3, 1, 2),
    (1, 30, 33, 2, 8, 4),
    (2, 17, 96, 4, 4, 21),         # 21 lookups: a second launch accumulates (16 + 5)
    (1, 64, 200, 4, 2, 7),         # 25 chunks per level-0 row: four column tiles
])
def test_build_equals_sequential_lookup_backwards(b, h, w, levels, radius, n):
    d = _desc(b, h, w, levels)
    lk = _inputs(b, h, w, levels, radius, n, seed=h * w + n)
    masks = [(i * 5) % (1 << levels) if i % 3 == 2 else 0 for i in range(n)]
    ref = _sequential(d, lk, radius, masks)
    got = _build(d, lk, radius, masks)
    assert torch.isfinite(got).all()
    assert torch.equal(got, ref), float((got - ref).abs().max())


def test_build_wild_coordinates_and_accumulate():
    b, h, w, levels, radius = 2, 21, 37, 4, 4
    d = _desc(b, h, w, levels)
    lk = _inputs(b, h, w, levels, radius, 6, seed=9, spread=12.0, wild=True)
    masks = [0] * 6
    ref = _sequential(d, lk, radius, masks)
    assert torch.equal(_build(d, lk, radius, masks), ref)
    # accumulate = 1 continues a sequence: G of the first 4 lookups, then the last 2 added in order
    first = _build(d, lk[:4], radius, masks[:4])
    assert torch.equal(_build(d, lk[4:], radius, masks[4:], init=first), ref)


def test_build_of_no_lookups_is_zero_and_pads_stay_zero():
    d = _desc(1, 13, 27, 3)
    assert (_build(d, [], 4, []) == 0).all()
    # pad targets (x >= W_l in the last chunk of a row) are never written with gradient
    lk = _inputs(1, 13, 27, 3, 4, 3, seed=1, spread=20.0)
    G = _build(d, lk, 4, [0, 0, 0]).view(-1, 13 * 27, 8)          # (chunks, N, 8)
    ch = 0
    for lv in range(3):
        lh, lw = 13 >> lv, 27 >> lv
        nch = (lw + 7) // 8
        for y in range(lh):
            last = G[ch + y * nch + nch - 1]
            assert (last[:, lw - 8 * (nch - 1):] == 0).all()
        ch += lh * nch


def test_cfg2_batch8_build_equals_sequential():
    b, h, w, levels, radius, n = 8, 55, 128, 4, 4, 12
    d = _desc(b, h, w, levels)
    lk = _inputs(b, h, w, levels, radius, n, seed=3)
    masks = [0] * n
    assert torch.equal(_build(d, lk, radius, masks), _sequential(d, lk, radius, masks))


def test_autograd_path_uses_build_and_matches_sequential_path():
    """The CorrBlock backward (GRAD_BUILD, the product) and the per-lookup path give identical grads."""
    import rmd
    from rmd import ops
    rng = np.random.default_rng(11)
    b, c, h, w = 2, 64, 23, 40
    f1 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    f2 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    lk = _inputs(b, h, w, 4, 4, 5, seed=2)

    def grads(build):
        ops.GRAD_BUILD = build
        try:
            t1, t2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
            cb = rmd.raft.CorrBlock(t1, t2, 4, 4, precision="fp32")
            loss = sum((cb(co, [4] if i == 1 else []) * go).sum() for i, (go, co) in enumerate(lk))
            loss.backward()
            return t1.grad, t2.grad
        finally:
            ops.GRAD_BUILD = True

    a1, a2 = grads(True)
    s1, s2 = grads(False)
    assert torch.equal(a1, s1) and torch.equal(a2, s2)


def _build_bf16(d, lookups, radius, masks):
    L = _lib()
    t = L.lib().rmd_corr_grad_targets(d.height, d.width, d.levels)
    G = torch.full((d.batch * d.height * d.width * t,), float("nan"), dtype=torch.bfloat16, device="cuda")
    n = len(lookups)
    gouts = (ctypes.c_void_p * max(n, 1))(*[go.data_ptr() for go, _ in lookups])
    cos = (ctypes.c_void_p * max(n, 1))(*[co.data_ptr() for _, co in lookups])
    ms = (ctypes.c_uint * max(n, 1))(*masks)
    L.check(L.lib().rmd_corr_grad_build_ex(gouts, cos, ms, n, ctypes.byref(d), radius, 0, 1,
                                           ctypes.c_void_p(G.data_ptr()), None), "grad_build_ex")
    return G


@pytest.mark.parametrize("b,h,w,levels,radius,n", [(2, 19, 26, 4, 3, 3), (1, 55, 128, 4, 4, 12), (3, 9, 70, 4, 4, 5)])
def test_bf16_build_is_the_rounded_fp32_build(b, h, w, levels, radius, n):
    """bf16_out: every element is the round-to-nearest-even bfloat16 of the fp32 build's sum."""
    d = _desc(b, h, w, levels)
    lk = _inputs(b, h, w, levels, radius, n, seed=7 + n)
    masks = [0] * n
    g32 = _build(d, lk, radius, masks)
    g16 = _build_bf16(d, lk, radius, masks)
    assert torch.equal(g16.view(torch.int16), g32.to(torch.bfloat16).view(torch.int16))


def test_bf16_build_rejects_accumulation_and_long_lists():
    L = _lib()
    d = _desc(1, 9, 12, 2)
    G = torch.empty(10, dtype=torch.bfloat16, device="cuda")
    assert L.lib().rmd_corr_grad_build_ex(None, None, None, 0, ctypes.byref(d), 4, 1, 1,
                                          ctypes.c_void_p(G.data_ptr()), None) == -1
    p = (ctypes.c_void_p * 17)(*([G.data_ptr()] * 17))
    assert L.lib().rmd_corr_grad_build_ex(p, p, None, 17, ctypes.byref(d), 4, 0, 1,
                                          ctypes.c_void_p(G.data_ptr()), None) == -1


@pytest.mark.parametrize("layout", [2, 3])
@pytest.mark.parametrize("b,m,k,nc", [(2, 256, 3896, 2852), (1, 100, 37, 45), (3, 256, 1000, 9), (1, 48, 8, 1030)])
def test_bf16g_gemm_equals_fp32g_gemm_in_bf16_compute(layout, b, m, k, nc):
    """rmd_corr_grad_gemm_bf16g on the bfloat16 B == rmd_corr_grad_gemm(RMD_BF16) on the fp32 B, bitwise."""
    L = _lib()
    lib = L.lib()
    rng = np.random.default_rng(b * 1000 + k)
    a = torch.tensor(rng.standard_normal((b, m, k)), dtype=torch.float32, device="cuda")
    # B in the blocked layout: 2 = ((n/8) ldb + k) 8 + n%8 (ldb = k), 3 = ((k/8) ldb + n) 8 + k%8 (ldb = nc)
    blocks = (nc + 7) // 8 if layout == 2 else (k + 7) // 8
    ldb = k if layout == 2 else nc
    bm = torch.tensor(rng.standard_normal((b, blocks * ldb * 8)), dtype=torch.float32, device="cuda")
    bh = bm.to(torch.bfloat16)
    ws = torch.empty(max(lib.rmd_corr_grad_gemm_workspace_bytes(b, m, k, nc), 1), dtype=torch.uint8, device="cuda")
    o32 = torch.empty((b, m, nc), dtype=torch.float32, device="cuda")
    o16 = torch.empty_like(o32)
    P = ctypes.c_void_p
    L.check(lib.rmd_corr_grad_gemm(P(a.data_ptr()), k, P(bm.data_ptr()), ldb, b, m, k, nc, layout, L.RMD_BF16,
                                   P(o32.data_ptr()), P(ws.data_ptr()), None), "gemm")
    L.check(lib.rmd_corr_grad_gemm_bf16g(P(a.data_ptr()), k, P(bh.data_ptr()), ldb, b, m, k, nc, layout,
                                         P(o16.data_ptr()), P(ws.data_ptr()), None), "gemm_bf16g")
    assert torch.equal(o16, o32)


def test_autograd_bf16_mode_bf16_g_matches_fp32_g():
    """bf16 precision: the bfloat16-G backward (product) and the fp32-G backward give identical grads."""
    import rmd
    from rmd import ops
    rng = np.random.default_rng(12)
    b, c, h, w = 2, 64, 23, 40
    f1 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    f2 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    lk = _inputs(b, h, w, 4, 4, 6, seed=4)

    def grads(flag):
        ops.GRAD_BF16 = flag
        try:
            t1, t2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
            cb = rmd.raft.CorrBlock(t1, t2, 4, 4, precision="bf16")
            loss = sum((cb(co) * go).sum() for go, co in lk)
            loss.backward()
            return t1.grad, t2.grad
        finally:
            ops.GRAD_BF16 = True

    a1, a2 = grads(True)
    s1, s2 = grads(False)
    assert torch.isfinite(a1).all() and torch.equal(a1, s1) and torch.equal(a2, s2)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_autograd_pending_flush_matches_single_build(precision):
    """past ops.GRAD_PENDING_BYTES of kept lookup gradients the lookups are folded into an
    fp32 G early (accumulate launches, same lookup order).  With the threshold at one byte every lookup
    backward flushes: the gradients are bit-identical to one build at the pyramid backward (bf16 mode:
    the bfloat16 G is the rounded fp32 G, which its GEMM rounds on load, so equal there too)."""
    import rmd
    from rmd import ops
    rng = np.random.default_rng(21)
    b, c, h, w = 2, 64, 23, 40
    f1 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    f2 = torch.tensor(rng.standard_normal((b, c, h, w)), dtype=torch.float32, device="cuda")
    lk = _inputs(b, h, w, 4, 4, 5, seed=8)

    def grads(limit):
        old = ops.GRAD_PENDING_BYTES
        ops.GRAD_PENDING_BYTES = limit
        try:
            t1, t2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
            cb = rmd.raft.CorrBlock(t1, t2, 4, 4, precision=precision)
            loss = sum((cb(co) * go).sum() for go, co in lk)
            loss.backward()
            return t1.grad, t2.grad
        finally:
            ops.GRAD_PENDING_BYTES = old

    a1, a2 = grads(1 << 40)
    s1, s2 = grads(1)
    assert torch.isfinite(a1).all() and torch.equal(a1, s1) and torch.equal(a2, s2)
