// dicl.hip — DICL displacement-invariant cost-volume construction and displacement-aware projection.
//
// Replaces (qzed/raft-meets-dicl v2):
//  * corr.dicl.CorrelationModule.forward gather/expand/cat  src/models/common/corr/dicl.py:26-54
//    (same in dicl_1x1.py:51-79; dicl_emb.py:51-89 adds the 2 displacement channels) and the
//    per-level gather of raft_dicl_ml.CorrelationModule.forward (src/models/impls/raft_dicl_ml.py:294-315)
//    -> rmd_dicl_stack / rmd_dicl_stack_backward
//  * FlowLevel.compute_cost volume build + occlusion mask   src/models/impls/dicl.py:212-238
//    -> rmd_dicl_stack_int / rmd_dicl_stack_int_backward
//  * DisplacementAwareProjection 1x1 conv                    src/models/common/blocks/dicl.py:121-150
//    -> rmd_dap (forward; with transpose = 1 it is the input gradient W^T g)
//
// All of them are HBM-bound byte movers: one lane owns 4 consecutive pixels of one
// displacement plane, so every store is a 16-byte-per-lane, fully coalesced row of the contiguous
// (B, du, dv, 2C(+2), h, w) MatchingNet input; the f1 half is re-read from L2 per displacement.

#include "rmd_common.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace rmd {
namespace {

constexpr int kThreads = 256;

// bilinear, align_corners=True, zero padding per tap: the 4 taps of one sample position
struct Taps {
    int idx[4];
    float wgt[4];
};

__device__ __forceinline__ Taps make_taps(float px, float py, int hl, int wl) {
    Taps t;
    px = fminf(fmaxf(px, -1.0e6f), 1.0e6f);
    py = fminf(fmaxf(py, -1.0e6f), 1.0e6f);
    const float fx0 = floorf(px), fy0 = floorf(py);
    const float fx = px - fx0, fy = py - fy0;
    const int x0 = (int)fx0, y0 = (int)fy0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int xx = x0 + (k & 1), yy = y0 + (k >> 1);
        const bool ok = xx >= 0 && xx < wl && yy >= 0 && yy < hl;
        const float wx = (k & 1) ? fx : 1.f - fx;
        const float wy = (k >> 1) ? fy : 1.f - fy;
        t.idx[k] = ok ? yy * wl + xx : 0;
        t.wgt[k] = ok ? wx * wy : 0.f;
    }
    return t;
}

// sample position of displacement (a, bb) for pixel p: the reference adds the integer offset to
// coords/2^level, normalises with (wn-1),(hn-1) and grid_sample un-normalises with (wl-1),(hl-1)
struct StackParams {
    int B, C, h, w, hl, wl, radius, extra;     // extra = 2 adds the displacement channels (dicl_emb)
    float inv_scale;                            // 1 / 2^level
    float sx, sy;                               // (wl-1)/(wn-1), (hl-1)/(hn-1)
};

typedef __attribute__((ext_vector_type(4))) float f4_t;

template <bool NT>
__device__ __forceinline__ void st4(float* p, f4_t v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<f4_t*>(p));
    else *reinterpret_cast<f4_t*>(p) = v;
}

// grid: (pixel quads, d*d, B); one lane = 4 consecutive pixels of one displacement plane.  The
// channel loop is unrolled by U so a lane's f1 row loads and 16 U bilinear taps are in flight
// before its 2 U stores; stores are non-temporal (the volume is written once, read by MatchingNet).
template <bool NT, int U>
__global__ void __launch_bounds__(kThreads)
dicl_stack_kernel(const float* __restrict__ f1, const float* __restrict__ f2, const float* __restrict__ coords,
                  StackParams P, float* __restrict__ out) {
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int quad = blockIdx.x * kThreads + threadIdx.x;
    const int p0 = quad * 4;
    if (p0 >= n) return;
    const int d = 2 * P.radius + 1;
    const int disp = blockIdx.y;                 // a * d + bb
    const int a = disp / d, bb = disp - a * d;
    const int b = blockIdx.z;
    const int C = P.C, C2 = 2 * C + P.extra;
    const float* cx = coords + (size_t)b * 2 * n;
    const float* cy = cx + n;
    Taps t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int p = p0 + k;
        const float px = (cx[p] * P.inv_scale + (float)(a - P.radius)) * P.sx;
        const float py = (cy[p] * P.inv_scale + (float)(bb - P.radius)) * P.sy;
        t[k] = make_taps(px, py, P.hl, P.wl);
    }
    float* o = out + ((size_t)(b * d * d + disp) * C2) * n + p0;
    const float* f1b = f1 + (size_t)b * C * n + p0;
    const float* f2b = f2 + (size_t)b * C * nl;
    for (int c0 = 0; c0 < C; c0 += U) {
        f4_t a1[U], v2[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (c0 + u < C) {
                const float* f2c = f2b + (size_t)(c0 + u) * nl;
                a1[u] = *reinterpret_cast<const f4_t*>(f1b + (size_t)(c0 + u) * n);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v2[u][k] = t[k].wgt[0] * f2c[t[k].idx[0]] + t[k].wgt[1] * f2c[t[k].idx[1]] +
                               t[k].wgt[2] * f2c[t[k].idx[2]] + t[k].wgt[3] * f2c[t[k].idx[3]];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (c0 + u < C) {
                st4<NT>(o + (size_t)(c0 + u) * n, a1[u]);
                st4<NT>(o + (size_t)(C + c0 + u) * n, v2[u]);
            }
        }
    }
    if (P.extra) {       // dicl_emb.py:81-85: delta (dx = a-r, dy = bb-r) as two constant channels
        const float dx = (float)(a - P.radius), dy = (float)(bb - P.radius);
        *reinterpret_cast<float4*>(o + (size_t)(2 * C) * n) = make_float4(dx, dx, dx, dx);
        *reinterpret_cast<float4*>(o + (size_t)(2 * C + 1) * n) = make_float4(dy, dy, dy, dy);
    }
}

// Scaled-grid forward (raft_dicl_ml levels > 0, sx, sy < 1): displacement (a, bb) samples
// x = (cx + a - r) sx, y = (cy + bb - r) sy, so all (2r+1)^2 samples of a pixel lie in a K x K
// integer patch (K = floor(2 r s) + 2, rounded up to even) and the x weights depend on a only, the
// y weights on bb only.  One lane per (pixel, channel) loads the patch once (K^2 loads instead of
// 4 (2r+1)^2 gathers), interpolates along x into K row values per a, then along y with per-bb
// weight vectors held in registers; lanes whose samples leave the patch (fp32 rounding at an
// exact span bound) fall back to the per-tap formula.  Stores: wave-uniform plane base + 32-bit
// lane offset, non-temporal.  grid (pixels/256, C, B).
template <int R, int K, bool NT>
__global__ void __launch_bounds__(kThreads)
dicl_stack_sep_kernel(const float* __restrict__ f1, const float* __restrict__ f2, const float* __restrict__ coords,
                      StackParams P, float* __restrict__ out) {
    constexpr int D = 2 * R + 1;
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int c = blockIdx.y, b = blockIdx.z;
    if (p >= n) return;
    const float cxs = fminf(fmaxf(coords[(size_t)b * 2 * n + p] * P.inv_scale, -1.0e6f), 1.0e6f);
    const float cys = fminf(fmaxf(coords[(size_t)b * 2 * n + n + p] * P.inv_scale, -1.0e6f), 1.0e6f);
    const int xbase = (int)floorf((cxs - (float)R) * P.sx), ybase = (int)floorf((cys - (float)R) * P.sy);
    int rx[D], ry[D];
    float fxa[D], fyb[D];
    bool fits = true;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        const float px = fminf(fmaxf((cxs + (float)(a - R)) * P.sx, -1.0e6f), 1.0e6f);
        const float py = fminf(fmaxf((cys + (float)(a - R)) * P.sy, -1.0e6f), 1.0e6f);
        const float x0 = floorf(px), y0 = floorf(py);
        rx[a] = (int)x0 - xbase;
        ry[a] = (int)y0 - ybase;
        fxa[a] = px - x0;
        fyb[a] = py - y0;
        fits = fits && rx[a] >= 0 && rx[a] <= K - 2 && ry[a] >= 0 && ry[a] <= K - 2;
    }
    const int C = P.C, C2 = 2 * C + P.extra;
    const size_t dstride = (size_t)C2 * n;
    float* const ob = out + (size_t)b * D * D * dstride;
    const unsigned lo1 = (unsigned)(((size_t)c * n + p) * sizeof(float));
    const unsigned lo2 = lo1 + (unsigned)((size_t)C * n * sizeof(float));
    const float v1 = f1[((size_t)b * C + c) * n + p];
    const float* f2c = f2 + ((size_t)b * C + c) * nl;
    auto put = [&](int a, int bb, float v) {
        char* od = reinterpret_cast<char*>(ob + (size_t)(a * D + bb) * dstride);
        if constexpr (NT) {
            __builtin_nontemporal_store(v1, reinterpret_cast<float*>(od + lo1));
            __builtin_nontemporal_store(v, reinterpret_cast<float*>(od + lo2));
        } else {
            *reinterpret_cast<float*>(od + lo1) = v1;
            *reinterpret_cast<float*>(od + lo2) = v;
        }
    };
    if (fits) {
        float patch[K][K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int yy = ybase + j;
            const bool rok = yy >= 0 && yy < P.hl;
            const int roff = min(max(yy, 0), P.hl - 1) * P.wl;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const int xx = xbase + i;
                const float e = f2c[roff + min(max(xx, 0), P.wl - 1)];
                patch[j][i] = (rok && xx >= 0 && xx < P.wl) ? e : 0.f;
            }
        }
        float wy[D][K];                 // y weights of displacement row bb over the patch rows
#pragma unroll
        for (int bb = 0; bb < D; ++bb)
#pragma unroll
            for (int j = 0; j < K; ++j) wy[bb][j] = j == ry[bb] ? 1.f - fyb[bb] : (j == ry[bb] + 1 ? fyb[bb] : 0.f);
#pragma unroll
        for (int a = 0; a < D; ++a) {
            float col[K];               // the patch interpolated along x at displacement a, per row
#pragma unroll
            for (int j = 0; j < K; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const float wx = i == rx[a] ? 1.f - fxa[a] : (i == rx[a] + 1 ? fxa[a] : 0.f);
                    acc = fmaf(wx, patch[j][i], acc);
                }
                col[j] = acc;
            }
#pragma unroll
            for (int bb = 0; bb < D; ++bb) {
                float v = 0.f;
#pragma unroll
                for (int j = 0; j < K; ++j) v = fmaf(wy[bb][j], col[j], v);
                put(a, bb, v);
            }
        }
    } else {
        for (int a = 0; a < D; ++a)
            for (int bb = 0; bb < D; ++bb) {
                const Taps t = make_taps((cxs + (float)(a - R)) * P.sx, (cys + (float)(bb - R)) * P.sy, P.hl, P.wl);
                put(a, bb, t.wgt[0] * f2c[t.idx[0]] + t.wgt[1] * f2c[t.idx[1]] + t.wgt[2] * f2c[t.idx[2]] +
                               t.wgt[3] * f2c[t.idx[3]]);
            }
    }
    if (P.extra && c == 0) {       // dicl_emb.py:81-85: delta (dx = a-r, dy = bb-r) as two constant channels
        for (int a = 0; a < D; ++a)
            for (int bb = 0; bb < D; ++bb) {
                float* od = ob + (size_t)(a * D + bb) * dstride + p;
                od[(size_t)(2 * C) * n] = (float)(a - R);
                od[(size_t)(2 * C + 1) * n] = (float)(bb - R);
            }
    }
}

// backward: grad_f1 = sum over displacements of the f1 half (deterministic, no atomics)
__global__ void __launch_bounds__(kThreads)
dicl_stack_grad_f1_kernel(const float* __restrict__ g, StackParams P, float* __restrict__ gf1) {
    const int n = P.h * P.w;
    const int quad = blockIdx.x * kThreads + threadIdx.x;
    const int p0 = quad * 4;
    if (p0 >= n) return;
    const int c = blockIdx.y, b = blockIdx.z;
    const int d = 2 * P.radius + 1, C2 = 2 * P.C + P.extra;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* gp = g + ((size_t)b * d * d * C2 + c) * n + p0;
    for (int disp = 0; disp < d * d; ++disp) {
        const float4 v = *reinterpret_cast<const float4*>(gp + (size_t)disp * C2 * n);
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
    }
    *reinterpret_cast<float4*>(gf1 + ((size_t)b * P.C + c) * n + p0) = s;
}

// backward: grad_f2 = bilinear scatter of the f2 half (float atomics, like grid_sampler backward)
__global__ void __launch_bounds__(kThreads)
dicl_stack_grad_f2_kernel(const float* __restrict__ g, const float* __restrict__ coords, StackParams P,
                          float* __restrict__ gf2) {
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= n) return;
    const int d = 2 * P.radius + 1;
    const int disp = blockIdx.y;
    const int a = disp / d, bb = disp - a * d;
    const int b = blockIdx.z;
    const int C = P.C, C2 = 2 * C + P.extra;
    const float px = (coords[(size_t)b * 2 * n + p] * P.inv_scale + (float)(a - P.radius)) * P.sx;
    const float py = (coords[(size_t)b * 2 * n + n + p] * P.inv_scale + (float)(bb - P.radius)) * P.sy;
    const Taps t = make_taps(px, py, P.hl, P.wl);
    const float* gp = g + ((size_t)(b * d * d + disp) * C2 + C) * n + p;
    float* gb = gf2 + (size_t)b * C * nl;
    for (int c = 0; c < C; ++c) {
        const float gv = gp[(size_t)c * n];
        float* gc = gb + (size_t)c * nl;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (t.wgt[k] != 0.f) atomicAdd(gc + t.idx[k], gv * t.wgt[k]);
    }
}

// ---- unit-step fast path ---------------------------------------------------------------------
// When the sample grid has unit steps (sx = sy = 1: corr/dicl.py and every same-size call), the
// (2r+1)^2 displacements of pixel p sample (x_p + a - r, y_p + b - r) with ONE fractional weight
// set, so together they read exactly the (2r+2)^2 integer patch [x0-r, x0+r+1] x [y0-r, y0+r+1]
// (as the RAFT lookup).  One lane per pixel, all displacements, a loop over channels: per channel
// the patch is read once (instead of 4 taps x (2r+1)^2 gathers), interpolated separably (x, then y)
// and the (2r+1)^2 f2 values plus the f1 copies are stored as coalesced 256-B wave rows.
template <int PX> struct FVec;
template <> struct FVec<4> { typedef __attribute__((ext_vector_type(4))) float T; };
template <> struct FVec<2> { typedef __attribute__((ext_vector_type(2))) float T; };
template <> struct FVec<1> { typedef __attribute__((ext_vector_type(1))) float T; };

template <bool NT, typename V>
__device__ __forceinline__ void stv(float* p, V v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<V*>(p));
    else *reinterpret_cast<V*>(p) = v;
}

template <int R, int PX, bool NT>
__global__ void __launch_bounds__(kThreads)
dicl_stack_patch_kernel(const float* __restrict__ f1, const float* __restrict__ f2, const float* __restrict__ coords,
                        StackParams P, int nxb, int remap, float* __restrict__ out) {
    // PX consecutive pixels per lane (each with its own patch) so every store is a PX-float vector
    // (PX * 256 B per wave-instruction); one channel per thread: 1-D grid of (pixels / 256 PX) x C x B
    // blocks, optionally remapped so an XCD works on one batch image.  Product PX = 1: 56 VGPRs at
    // r = 4, 7 waves per SIMD, the most stores in flight (PX = 2 needs ~106 VGPRs, PX = 4 ~200).
    typedef typename FVec<PX>::T V;
    constexpr int D = 2 * R + 1, K = 2 * R + 2;
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int lid = remap ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int xb = lid % nxb, rest = lid / nxb;
    const int c = rest % P.C, b = rest / P.C;
    const int p0 = (xb * kThreads + threadIdx.x) * PX;
    if (p0 >= n) return;
    float fx[PX], fy[PX];
    int xs[PX], ys[PX];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
        float cx = coords[(size_t)b * 2 * n + p0 + k] * P.inv_scale;
        float cy = coords[(size_t)b * 2 * n + n + p0 + k] * P.inv_scale;
        cx = fminf(fmaxf(cx, -1.0e6f), 1.0e6f);
        cy = fminf(fmaxf(cy, -1.0e6f), 1.0e6f);
        const float fx0 = floorf(cx), fy0 = floorf(cy);
        fx[k] = cx - fx0;
        fy[k] = cy - fy0;
        xs[k] = (int)fx0 - R;
        ys[k] = (int)fy0 - R;
    }
    const int C = P.C, C2 = 2 * C + P.extra;
    const size_t dstride = (size_t)C2 * n;                       // next displacement plane
    float* o = out + (size_t)b * D * D * dstride + p0;
    // stores: wave-uniform plane base + one 32-bit lane offset (saddr + voffset addressing; the
    // host checks that a batch image's volume stays below 4 GiB), so the 2 D^2 store addresses
    // cost no VGPRs
    float* const ob = out + (size_t)b * D * D * dstride;
    const unsigned lo1 = (unsigned)(((size_t)c * n + p0) * sizeof(float));
    const unsigned lo2 = lo1 + (unsigned)((size_t)C * n * sizeof(float));
    const V v1 = *reinterpret_cast<const V*>(f1 + ((size_t)b * C + c) * n + p0);
    const float* f2c = f2 + ((size_t)b * C + c) * nl;
    float hprev[PX][D];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        float hcur[PX][D];
#pragma unroll
        for (int k = 0; k < PX; ++k) {
            const int yy = ys[k] + j;
            const bool rok = yy >= 0 && yy < P.hl;
            const unsigned roff = (unsigned)(min(max(yy, 0), P.hl - 1) * P.wl);
            float v[K];
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const int xx = xs[k] + i;
                const float e = f2c[roff + (unsigned)min(max(xx, 0), P.wl - 1)];
                v[i] = (rok && xx >= 0 && xx < P.wl) ? e : 0.f;
            }
#pragma unroll
            for (int a = 0; a < D; ++a) hcur[k][a] = fmaf(fx[k], v[a + 1] - v[a], v[a]);
        }
        if (j > 0) {
            const int bb = j - 1;
#pragma unroll
            for (int a = 0; a < D; ++a) {
                char* od = reinterpret_cast<char*>(ob + (size_t)(a * D + bb) * dstride);
                stv<NT>(reinterpret_cast<float*>(od + lo1), v1);
                V r;
#pragma unroll
                for (int k = 0; k < PX; ++k) r[k] = fmaf(fy[k], hcur[k][a] - hprev[k][a], hprev[k][a]);
                stv<NT>(reinterpret_cast<float*>(od + lo2), r);
            }
        }
#pragma unroll
        for (int k = 0; k < PX; ++k)
#pragma unroll
            for (int a = 0; a < D; ++a) hprev[k][a] = hcur[k][a];
    }
    if (P.extra && c == 0) {       // dicl_emb.py:81-85: delta (dx = a-r, dy = bb-r) as two constant channels
#pragma unroll
        for (int a = 0; a < D; ++a)
#pragma unroll
            for (int bb = 0; bb < D; ++bb) {
                float* od = o + (size_t)(a * D + bb) * dstride;
                const float dx = (float)(a - R), dy = (float)(bb - R);
                *reinterpret_cast<V*>(od + (size_t)(2 * C) * n) = V(dx);
                *reinterpret_cast<V*>(od + (size_t)(2 * C + 1) * n) = V(dy);
            }
    }
}

// backward of the unit-step stack: grad_f1[c,p] = sum of the (2r+1)^2 f1-half gradients (plain
// store); grad_f2 = the f2-half tap gradients spread over p's patch with the forward's separable
// weights (as rmd_corr_lookup_backward).  The patches of a workgroup's 256 consecutive pixels are
// summed in LDS (ds_add_f32) over the row window [wy0, wy0 + wrows) starting at the group's lowest
// patch row; rows past the window go straight to global float atomics; the window is then added
// to grad_f2 once per element.  grid (pixels/256, C, B).
constexpr int kWinFloats = 12288;      // 48 KiB LDS window
constexpr int kWinSmall = 4096;        // 16 KiB LDS window (narrow maps, see rmd_dicl_stack_backward)

template <int R, int WIN>
__global__ void __launch_bounds__(kThreads)
dicl_stack_patch_backward_kernel(const float* __restrict__ g, const float* __restrict__ coords, StackParams P,
                                 float* __restrict__ gf1, float* __restrict__ gf2) {
    constexpr int D = 2 * R + 1, K = 2 * R + 2;
    __shared__ float win[WIN];
    __shared__ int wmin;
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int c = blockIdx.y, b = blockIdx.z;
    const bool pv = p < n;
    float fx = 0.f, fy = 0.f;
    int xs = 0, ys = 1 << 30;
    if (pv) {
        float cx = coords[(size_t)b * 2 * n + p] * P.inv_scale;
        float cy = coords[(size_t)b * 2 * n + n + p] * P.inv_scale;
        cx = fminf(fmaxf(cx, -1.0e6f), 1.0e6f);
        cy = fminf(fmaxf(cy, -1.0e6f), 1.0e6f);
        const float fx0 = floorf(cx), fy0 = floorf(cy);
        fx = cx - fx0;
        fy = cy - fy0;
        xs = (int)fx0 - R;
        ys = (int)fy0 - R;
    }
    if (threadIdx.x == 0) wmin = 1 << 30;
    for (int k = threadIdx.x; k < WIN; k += kThreads) win[k] = 0.f;
    __syncthreads();
    if (pv) atomicMin(&wmin, max(ys, 0));
    __syncthreads();
    const int wy0 = min(wmin, P.hl);
    const int wrows = min(P.hl - wy0, WIN / P.wl);
    const int C = P.C, C2 = 2 * C + P.extra;
    const size_t dstride = (size_t)C2 * n;
    float* g2c = gf2 + ((size_t)b * C + c) * nl;
    if (pv) {
        const float* gp = g + (size_t)b * D * D * dstride + p;
        float s1 = 0.f;
        float qprev[K];
#pragma unroll
        for (int i = 0; i < K; ++i) qprev[i] = 0.f;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            float qcur[K];
            if (j < D) {
                float gr[D];
#pragma unroll
                for (int a = 0; a < D; ++a) {
                    const float* gd = gp + (size_t)(a * D + j) * dstride;
                    s1 += gd[(size_t)c * n];
                    gr[a] = gd[(size_t)(C + c) * n];
                }
#pragma unroll
                for (int i = 0; i < K; ++i)
                    qcur[i] = (i < D ? gr[i] * (1.0f - fx) : 0.f) + (i >= 1 ? gr[i - 1] * fx : 0.f);
            } else {
#pragma unroll
                for (int i = 0; i < K; ++i) qcur[i] = 0.f;
            }
            const int yy = ys + j;
            if (yy >= 0 && yy < P.hl) {
                // LDS and global targets in separate branches: a pointer selected between them is
                // generic, and flat atomics into LDS cost 4x the whole kernel (0.96 vs 0.23 ms)
                if (yy - wy0 < wrows) {
                    float* r = win + (yy - wy0) * P.wl;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const int xx = xs + i;
                        if (xx >= 0 && xx < P.wl) atomicAdd(r + xx, qcur[i] * (1.0f - fy) + qprev[i] * fy);
                    }
                } else {
                    float* r = g2c + (size_t)yy * P.wl;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const int xx = xs + i;
                        if (xx >= 0 && xx < P.wl) atomicAdd(r + xx, qcur[i] * (1.0f - fy) + qprev[i] * fy);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < K; ++i) qprev[i] = qcur[i];
        }
        gf1[((size_t)b * C + c) * n + p] = s1;
    }
    __syncthreads();
    float* gw = g2c + (size_t)wy0 * P.wl;
    for (int k = threadIdx.x; k < wrows * P.wl; k += kThreads) {
        const float v = win[k];
        if (v != 0.f) atomicAdd(gw + k, v);
    }
}


// Same backward, 2 pixels per lane, with a GENERAL merge of the lane's two patches: whenever the
// pixels' integer window origins differ by at most 1 row and 2 columns (any smooth flow), the two
// (2r+2)^2 patches are summed in registers over their joint box of (2r+3) rows x (2r+4) columns and
// every lane adds one run of 2r+4 values per joint row.  The round-1 kernel merged only origins exactly one
// column apart and sends every other lane through a per-pixel path of 2 (2r+2) adds per row; because
// a wave executes every path one of its lanes takes, a wave with both kinds paid for both (the
// cost of the LDS atomics, ~100 cycles per ds_add_f32 wave-instruction, is per instruction).  Here
// all lanes of a smooth-flow wave take one path: (2r+3) (2r+4) add instructions per wave instead of
// up to (2r+2) (2r+3) + 2 (2r+2)^2.  Lanes outside the merge condition still add per pixel.  With CH,
// lanes whose joint box continues the previous lane's two columns further on the same rows (smooth
// flow) sum the overlapping runs through DPP lane shifts, so only a chain's last lane adds more than
// its own two new columns (far fewer active lanes per add instruction).
// grid (pixels/512, C, B).
template <int R, int WIN, bool CH>
__global__ void __launch_bounds__(kThreads)
dicl_stack_patch_backward_gm_kernel(const float* __restrict__ g, const float* __restrict__ coords, StackParams P,
                                    float* __restrict__ gf1, float* __restrict__ gf2) {
    constexpr int D = 2 * R + 1, K = 2 * R + 2, PX = 2, MW = K + 2;
    __shared__ float win[WIN];
    __shared__ int wmin;
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int p0 = (blockIdx.x * kThreads + threadIdx.x) * PX;
    const int c = blockIdx.y, b = blockIdx.z;
    const bool pv = p0 < n;               // n % 4 == 0: a lane's PX pixels are all valid or all not
    float fx[PX], fy[PX];
    int xs[PX], ys[PX];
    int ymin = 1 << 30;
#pragma unroll
    for (int k = 0; k < PX; ++k) {
        fx[k] = fy[k] = 0.f;
        xs[k] = 0;
        ys[k] = 1 << 30;
        if (pv) {
            float cx = coords[(size_t)b * 2 * n + p0 + k] * P.inv_scale;
            float cy = coords[(size_t)b * 2 * n + n + p0 + k] * P.inv_scale;
            cx = fminf(fmaxf(cx, -1.0e6f), 1.0e6f);
            cy = fminf(fmaxf(cy, -1.0e6f), 1.0e6f);
            const float fx0 = floorf(cx), fy0 = floorf(cy);
            fx[k] = cx - fx0;
            fy[k] = cy - fy0;
            xs[k] = (int)fx0 - R;
            ys[k] = (int)fy0 - R;
            ymin = min(ymin, max(ys[k], 0));
        }
    }
    // joint box origin and per-pixel offsets inside it
    const int oy = min(ys[0], ys[1]), ox = min(xs[0], xs[1]);
    const int dy0 = ys[0] - oy, dy1 = ys[1] - oy, dx0 = xs[0] - ox, dx1 = xs[1] - ox;
    const bool gm = pv && dy0 + dy1 <= 1 && dx0 + dx1 <= 2;      // |dy| <= 1, |dx| <= 2
    // CH: lane l's joint box continues lane l-1's two columns further on the same rows (smooth flow)
    // -> the wave sums the overlapping runs with DPP lane shifts and each lane adds only its own two
    // new columns (a chain's last lane adds its whole tail)
    bool link = false, link_next = false;
    if constexpr (CH) {
        const int poy = __builtin_amdgcn_update_dpp((int)0x80000000, oy, 0x138, 0xf, 0xf, false);   // wave_shr:1
        const int pox = __builtin_amdgcn_update_dpp((int)0x80000000, ox, 0x138, 0xf, 0xf, false);
        const int pgm = __builtin_amdgcn_update_dpp(0, (int)gm, 0x138, 0xf, 0xf, false);
        link = gm && pgm != 0 && poy == oy && pox + PX == ox;
        link_next = __builtin_amdgcn_update_dpp(0, (int)link, 0x130, 0xf, 0xf, false) != 0;      // wave_shl:1
    }
    if (threadIdx.x == 0) wmin = 1 << 30;
    for (int k = threadIdx.x; k < WIN; k += kThreads) win[k] = 0.f;
    __syncthreads();
    if (pv) atomicMin(&wmin, ymin);
    __syncthreads();
    const int wy0 = min(wmin, P.hl);
    const int wrows = min(P.hl - wy0, WIN / P.wl);
    const int C = P.C, C2 = 2 * C + P.extra;
    const size_t dstride = (size_t)C2 * n;
    float* g2c = gf2 + ((size_t)b * C + c) * nl;
    typedef typename FVec<PX>::T v2;
    auto add = [&](int yy, int xx, float v) {        // LDS window or (rows past it) global
        if (yy - wy0 < wrows) atomicAdd(win + (yy - wy0) * P.wl + xx, v);
        else atomicAdd(g2c + (size_t)yy * P.wl + xx, v);
    };
    if (pv) {
        const char* gb = reinterpret_cast<const char*>(g + (size_t)b * D * D * dstride);
        const unsigned lo1 = (unsigned)(((size_t)c * n + p0) * sizeof(float));
        const unsigned lo2 = lo1 + (unsigned)((size_t)C * n * sizeof(float));
        v2 s1 = v2(0.f);
        float qprev[PX][K], vprev[PX][K];
#pragma unroll
        for (int k = 0; k < PX; ++k)
#pragma unroll
            for (int i = 0; i < K; ++i) qprev[k][i] = vprev[k][i] = 0.f;
#pragma unroll 1
        for (int j = 0; j <= K; ++j) {     // patch rows 0..K-1, plus the joint box's extra row K
            float qcur[PX][K];
            if (j < D) {
                v2 gr[D];
#pragma unroll
                for (int a = 0; a < D; ++a) {
                    const char* gd = gb + (size_t)(a * D + j) * dstride * sizeof(float);
                    s1 += *reinterpret_cast<const v2*>(gd + lo1);
                    gr[a] = *reinterpret_cast<const v2*>(gd + lo2);
                }
#pragma unroll
                for (int k = 0; k < PX; ++k)
#pragma unroll
                    for (int i = 0; i < K; ++i)
                        qcur[k][i] = (i < D ? gr[i][k] * (1.0f - fx[k]) : 0.f) + (i >= 1 ? gr[i - 1][k] * fx[k] : 0.f);
            } else {
#pragma unroll
                for (int k = 0; k < PX; ++k)
#pragma unroll
                    for (int i = 0; i < K; ++i) qcur[k][i] = 0.f;
            }
            float val[PX][K];              // patch row j of each pixel (0 for j == K)
#pragma unroll
            for (int k = 0; k < PX; ++k)
#pragma unroll
                for (int i = 0; i < K; ++i) val[k][i] = qcur[k][i] * (1.0f - fy[k]) + qprev[k][i] * fy[k];
            if (gm) {
                // joint row j: pixel k contributes its patch row j - dy_k (this row or the previous one)
                const int yy = oy + j;
                if (yy >= 0 && yy < P.hl) {
                    float mm[MW];
#pragma unroll
                    for (int t = 0; t < MW; ++t) {
                        float m = 0.f;
#pragma unroll
                        for (int k = 0; k < PX; ++k) {
                            const int dyk = k ? dy1 : dy0, dxk = k ? dx1 : dx0;
                            const float* row = dyk ? vprev[k] : val[k];
                            // element t - dx_k of the row, dx_k in {0, 1, 2}
                            const float e0 = t < K ? row[t] : 0.f;
                            const float e1 = (t >= 1 && t - 1 < K) ? row[t - 1] : 0.f;
                            const float e2 = (t >= 2 && t - 2 < K) ? row[t - 2] : 0.f;
                            m += dxk == 0 ? e0 : (dxk == 1 ? e1 : e2);
                        }
                        mm[t] = m;
                    }
                    if constexpr (CH) {
                        // r_t(l) = mm_l[t] + link_l r_{t+2}(l-1): column ox_l + t of the chain
#pragma unroll
                        for (int t = 0; t < MW; ++t) {
                            const int kmax = (MW - 1 - t) / PX;
                            float rr = mm[t + PX * kmax];
#pragma unroll
                            for (int k = kmax - 1; k >= 0; --k) {
                                const float up = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(rr), 0x138, 0xf, 0xf, false));
                                rr = mm[t + PX * k] + (link ? up : 0.f);
                            }
                            mm[t] = (t < PX || !link_next) ? rr : 0.f;
                        }
                    }
#pragma unroll
                    for (int t = 0; t < MW; ++t) {
                        const int xx = ox + t;
                        if (xx >= 0 && xx < P.wl && mm[t] != 0.f) add(yy, xx, mm[t]);
                    }
                }
            } else if (j < K) {
#pragma unroll
                for (int k = 0; k < PX; ++k) {
                    const int yy = ys[k] + j;
                    if (yy < 0 || yy >= P.hl) continue;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const int xx = xs[k] + i;
                        if (xx >= 0 && xx < P.wl) add(yy, xx, val[k][i]);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < PX; ++k)
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    qprev[k][i] = qcur[k][i];
                    vprev[k][i] = val[k][i];
                }
        }
        *reinterpret_cast<v2*>(gf1 + ((size_t)b * C + c) * n + p0) = s1;
    }
    __syncthreads();
    float* gw = g2c + (size_t)wy0 * P.wl;
    for (int k = threadIdx.x; k < wrows * P.wl; k += kThreads) {
        const float v = win[k];
        if (v != 0.f) atomicAdd(gw + k, v);
    }
}

// backward of the general (scaled-grid) stack, raft_dicl_ml levels > 0: every displacement has its
// own bilinear weights, so each lane (pixel p, channel c) walks the (2r+1)^2 displacements, adds its
// f1-half gradients into grad_f1 (plain store) and its 4 f2 taps into the workgroup's LDS window
// (rows [wy0, wy0 + wrows) from the group's lowest tap row; taps past it go to global atomics);
// the window is then added to grad_f2 once per element.  grid (pixels/256, C, B).
template <int WIN>
__global__ void __launch_bounds__(kThreads)
dicl_stack_general_backward_kernel(const float* __restrict__ g, const float* __restrict__ coords, StackParams P,
                                   float* __restrict__ gf1, float* __restrict__ gf2) {
    __shared__ float win[WIN];
    __shared__ int wmin;
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int c = blockIdx.y, b = blockIdx.z;
    const bool pv = p < n;
    const int d = 2 * P.radius + 1;
    float cxs = 0.f, cys = 0.f;
    if (pv) {
        cxs = coords[(size_t)b * 2 * n + p] * P.inv_scale;
        cys = coords[(size_t)b * 2 * n + n + p] * P.inv_scale;
    }
    if (threadIdx.x == 0) wmin = 1 << 30;
    for (int k = threadIdx.x; k < WIN; k += kThreads) win[k] = 0.f;
    __syncthreads();
    if (pv) {
        // lowest tap row of this pixel: y of displacement bb = 0 (sy >= 0), clamped into the level
        const float py = fminf(fmaxf((cys - (float)P.radius) * P.sy, -1.0e6f), 1.0e6f);
        atomicMin(&wmin, min(max((int)floorf(py), 0), P.hl));
    }
    __syncthreads();
    const int wy0 = min(wmin, P.hl);
    const int wrows = min(P.hl - wy0, WIN / P.wl);
    const int C = P.C, C2 = 2 * C + P.extra;
    const size_t dstride = (size_t)C2 * n;
    float* g2c = gf2 + ((size_t)b * C + c) * nl;
    if (pv) {
        const float* gp = g + (size_t)b * d * d * dstride + p;
        float s1 = 0.f;
        for (int a = 0; a < d; ++a) {
            for (int bb = 0; bb < d; ++bb) {
                const float* gd = gp + (size_t)(a * d + bb) * dstride;
                s1 += gd[(size_t)c * n];
                const float gv = gd[(size_t)(C + c) * n];
                const float px = (cxs + (float)(a - P.radius)) * P.sx;
                const float py = (cys + (float)(bb - P.radius)) * P.sy;
                const Taps t = make_taps(px, py, P.hl, P.wl);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (t.wgt[k] == 0.f) continue;
                    const int yy = t.idx[k] / P.wl;
                    if (yy >= wy0 && yy - wy0 < wrows) atomicAdd(win + (t.idx[k] - wy0 * P.wl), gv * t.wgt[k]);
                    else atomicAdd(g2c + t.idx[k], gv * t.wgt[k]);
                }
            }
        }
        gf1[((size_t)b * C + c) * n + p] = s1;
    }
    __syncthreads();
    float* gw = g2c + (size_t)wy0 * P.wl;
    for (int k = threadIdx.x; k < wrows * P.wl; k += kThreads) {
        const float v = win[k];
        if (v != 0.f) atomicAdd(gw + k, v);
    }
}

// Separable form of the general backward (scaled grids with 0 <= sx, sy <= 1, raft_dicl_ml levels > 0).
// The x-weights of displacement (a, bb) depend on a only and the y-weights on bb only, so a lane's 81
// f2-half gradients reach a K x K patch as  patch[j][i] = sum_bb wy_bb(j) * sum_a wx_a(i) * g[a][bb]:
// K FMAs per displacement plus K^2 per row bb, all in registers, then K^2 window atomics per lane
// instead of 4 per displacement (324 for r = 4).  A lane whose taps do not fit the patch (fp32
// rounding at an exact span bound) takes the per-tap path, so the result never depends on K.
template <int K, int WIN>
__global__ void __launch_bounds__(kThreads)
dicl_stack_sep_backward_kernel(const float* __restrict__ g, const float* __restrict__ coords, StackParams P,
                               float* __restrict__ gf1, float* __restrict__ gf2) {
    __shared__ float win[WIN];
    __shared__ int wmin;
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int c = blockIdx.y, b = blockIdx.z;
    const bool pv = p < n;
    const int d = 2 * P.radius + 1;
    float cxs = 0.f, cys = 0.f;
    if (pv) {
        cxs = fminf(fmaxf(coords[(size_t)b * 2 * n + p] * P.inv_scale, -1.0e6f), 1.0e6f);
        cys = fminf(fmaxf(coords[(size_t)b * 2 * n + n + p] * P.inv_scale, -1.0e6f), 1.0e6f);
    }
    if (threadIdx.x == 0) wmin = 1 << 30;
    for (int k = threadIdx.x; k < WIN; k += kThreads) win[k] = 0.f;
    __syncthreads();
    const float py0 = (cys - (float)P.radius) * P.sy, px0 = (cxs - (float)P.radius) * P.sx;
    const int ybase = (int)floorf(py0), xbase = (int)floorf(px0);
    if (pv) atomicMin(&wmin, min(max(ybase, 0), P.hl));
    __syncthreads();
    const int wy0 = min(wmin, P.hl);
    const int wrows = min(P.hl - wy0, WIN / P.wl);
    const int C = P.C, C2 = 2 * C + P.extra;
    const size_t dstride = (size_t)C2 * n;
    float* g2c = gf2 + ((size_t)b * C + c) * nl;
    if (pv) {
        const float* gp = g + (size_t)b * d * d * dstride + p;
        // does every tap land inside the K x K patch?
        const float pxl = (cxs + (float)P.radius) * P.sx, pyl = (cys + (float)P.radius) * P.sy;
        const bool fits = (int)floorf(pxl) - xbase <= K - 2 && (int)floorf(pyl) - ybase <= K - 2;
        float s1 = 0.f;
        if (fits) {
            float patch[K][K];
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
                for (int i = 0; i < K; ++i) patch[j][i] = 0.f;
            for (int bb = 0; bb < d; ++bb) {
                float row[K];
#pragma unroll
                for (int i = 0; i < K; ++i) row[i] = 0.f;
                for (int a = 0; a < d; ++a) {
                    const float* gd = gp + (size_t)(a * d + bb) * dstride;
                    s1 += gd[(size_t)c * n];
                    const float gv = gd[(size_t)(C + c) * n];
                    const float px = (cxs + (float)(a - P.radius)) * P.sx;
                    const float fx0 = floorf(px);
                    const int rx = (int)fx0 - xbase;
                    const float w1 = (px - fx0) * gv, w0 = gv - w1;
#pragma unroll
                    for (int i = 0; i < K; ++i) row[i] += i == rx ? w0 : (i == rx + 1 ? w1 : 0.f);
                }
                const float py = (cys + (float)(bb - P.radius)) * P.sy;
                const float fy0 = floorf(py);
                const int ry = (int)fy0 - ybase;
                const float fy = py - fy0;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const float wy = j == ry ? 1.f - fy : (j == ry + 1 ? fy : 0.f);
#pragma unroll
                    for (int i = 0; i < K; ++i) patch[j][i] = fmaf(wy, row[i], patch[j][i]);
                }
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const int yy = ybase + j;
                if (yy < 0 || yy >= P.hl) continue;
                if (yy >= wy0 && yy - wy0 < wrows) {        // LDS / global in separate branches (no flat atomics)
                    float* r = win + (yy - wy0) * P.wl;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const int xx = xbase + i;
                        if (xx >= 0 && xx < P.wl && patch[j][i] != 0.f) atomicAdd(r + xx, patch[j][i]);
                    }
                } else {
                    float* r = g2c + (size_t)yy * P.wl;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const int xx = xbase + i;
                        if (xx >= 0 && xx < P.wl && patch[j][i] != 0.f) atomicAdd(r + xx, patch[j][i]);
                    }
                }
            }
        } else {
            for (int a = 0; a < d; ++a) {
                for (int bb = 0; bb < d; ++bb) {
                    const float* gd = gp + (size_t)(a * d + bb) * dstride;
                    s1 += gd[(size_t)c * n];
                    const float gv = gd[(size_t)(C + c) * n];
                    const Taps t = make_taps((cxs + (float)(a - P.radius)) * P.sx, (cys + (float)(bb - P.radius)) * P.sy,
                                             P.hl, P.wl);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (t.wgt[k] == 0.f) continue;
                        const int yy = t.idx[k] / P.wl;
                        if (yy >= wy0 && yy - wy0 < wrows) atomicAdd(win + (t.idx[k] - wy0 * P.wl), gv * t.wgt[k]);
                        else atomicAdd(g2c + t.idx[k], gv * t.wgt[k]);
                    }
                }
            }
        }
        gf1[((size_t)b * C + c) * n + p] = s1;
    }
    __syncthreads();
    float* gw = g2c + (size_t)wy0 * P.wl;
    for (int k = threadIdx.x; k < wrows * P.wl; k += kThreads) {
        const float v = win[k];
        if (v != 0.f) atomicAdd(gw + k, v);
    }
}

// Separable backward, two pixels per lane with the unit-step kernel's merge: when both pixels' K x K
// patches fit and their origins differ by <= 1 row and <= 2 columns (any smooth flow; at level-1
// scale adjacent pixels' origins move half a column), the patches are summed in registers over their
// joint (K+1) x (K+2) box and, where lane l's box sits one column right of lane l-1's on the same rows
// (the common step: 2 pixels x 0.5), the overlapping runs are summed through DPP lane shifts so each
// lane adds only its one new column (a chain's last lane its whole tail).  Other lanes add per pixel
// (or per tap).  grid (pixels / 512, C, B).
template <int K, int WIN>
__global__ void __launch_bounds__(kThreads)
dicl_stack_sep_backward2_kernel(const float* __restrict__ g, const float* __restrict__ coords, StackParams P,
                                float* __restrict__ gf1, float* __restrict__ gf2) {
    constexpr int PX = 2, MW = K + 2, MH = K + 1;
    __shared__ float win[WIN];
    __shared__ int wmin;
    const int n = P.h * P.w, nl = P.hl * P.wl;
    const int p0 = (blockIdx.x * kThreads + threadIdx.x) * PX;
    const int c = blockIdx.y, b = blockIdx.z;
    const bool pv = p0 < n;                       // n % 4 == 0: both pixels valid or neither
    const int d = 2 * P.radius + 1;
    float cxs[PX], cys[PX];
    int xbase[PX], ybase[PX];
    bool fits[PX];
    int ymin = 1 << 30;
#pragma unroll
    for (int k = 0; k < PX; ++k) {
        cxs[k] = cys[k] = 0.f;
        if (pv) {
            cxs[k] = fminf(fmaxf(coords[(size_t)b * 2 * n + p0 + k] * P.inv_scale, -1.0e6f), 1.0e6f);
            cys[k] = fminf(fmaxf(coords[(size_t)b * 2 * n + n + p0 + k] * P.inv_scale, -1.0e6f), 1.0e6f);
        }
        ybase[k] = (int)floorf((cys[k] - (float)P.radius) * P.sy);
        xbase[k] = (int)floorf((cxs[k] - (float)P.radius) * P.sx);
        const float pxl = (cxs[k] + (float)P.radius) * P.sx, pyl = (cys[k] + (float)P.radius) * P.sy;
        fits[k] = (int)floorf(pxl) - xbase[k] <= K - 2 && (int)floorf(pyl) - ybase[k] <= K - 2;
        if (pv) ymin = min(ymin, max(ybase[k], 0));
    }
    const int oy = min(ybase[0], ybase[1]), ox = min(xbase[0], xbase[1]);
    const int dy0 = ybase[0] - oy, dy1 = ybase[1] - oy, dx0 = xbase[0] - ox, dx1 = xbase[1] - ox;
    const bool gm = pv && fits[0] && fits[1] && dy0 + dy1 <= 1 && dx0 + dx1 <= 2;
    const int pys = __builtin_amdgcn_update_dpp((int)0x80000000, oy, 0x138, 0xf, 0xf, false);   // wave_shr:1
    const int pxs = __builtin_amdgcn_update_dpp((int)0x80000000, ox, 0x138, 0xf, 0xf, false);
    const int pgm = __builtin_amdgcn_update_dpp(0, (int)gm, 0x138, 0xf, 0xf, false);
    const bool link = gm && pgm != 0 && pys == oy && pxs + 1 == ox;
    const bool link_next = __builtin_amdgcn_update_dpp(0, (int)link, 0x130, 0xf, 0xf, false) != 0;   // wave_shl:1
    if (threadIdx.x == 0) wmin = 1 << 30;
    for (int k = threadIdx.x; k < WIN; k += kThreads) win[k] = 0.f;
    __syncthreads();
    if (pv) atomicMin(&wmin, ymin);
    __syncthreads();
    const int wy0 = min(wmin, P.hl);
    const int wrows = min(P.hl - wy0, WIN / P.wl);
    const int C = P.C, C2 = 2 * C + P.extra;
    const size_t dstride = (size_t)C2 * n;
    float* g2c = gf2 + ((size_t)b * C + c) * nl;
    auto add = [&](int yy, int xx, float v) {            // LDS window or (rows past it) global
        if (yy >= wy0 && yy - wy0 < wrows) atomicAdd(win + (yy - wy0) * P.wl + xx, v);
        else atomicAdd(g2c + (size_t)yy * P.wl + xx, v);
    };
    typedef typename FVec<PX>::T v2;
    if (pv) {
        const char* gb = reinterpret_cast<const char*>(g + (size_t)b * d * d * dstride);
        const unsigned lo1 = (unsigned)(((size_t)c * n + p0) * sizeof(float));
        const unsigned lo2 = lo1 + (unsigned)((size_t)C * n * sizeof(float));
        v2 s1 = v2(0.f);
        float patch[PX][K][K];
#pragma unroll
        for (int k = 0; k < PX; ++k)
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
                for (int i = 0; i < K; ++i) patch[k][j][i] = 0.f;
        const bool any_fit = fits[0] || fits[1];
        for (int bb = 0; bb < d; ++bb) {
            float row[PX][K];
#pragma unroll
            for (int k = 0; k < PX; ++k)
#pragma unroll
                for (int i = 0; i < K; ++i) row[k][i] = 0.f;
            for (int a = 0; a < d; ++a) {
                const char* gd = gb + (size_t)(a * d + bb) * dstride * sizeof(float);
                s1 += *reinterpret_cast<const v2*>(gd + lo1);
                const v2 gv = *reinterpret_cast<const v2*>(gd + lo2);
#pragma unroll
                for (int k = 0; k < PX; ++k) {
                    if (fits[k]) {
                        const float px = (cxs[k] + (float)(a - P.radius)) * P.sx;
                        const float fx0 = floorf(px);
                        const int rx = (int)fx0 - xbase[k];
                        const float w1 = (px - fx0) * gv[k], w0 = gv[k] - w1;
#pragma unroll
                        for (int i = 0; i < K; ++i) row[k][i] += i == rx ? w0 : (i == rx + 1 ? w1 : 0.f);
                    } else {                           // per-tap path (fp32 rounding at a span bound)
                        const Taps t = make_taps((cxs[k] + (float)(a - P.radius)) * P.sx,
                                                 (cys[k] + (float)(bb - P.radius)) * P.sy, P.hl, P.wl);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (t.wgt[q] != 0.f) add(t.idx[q] / P.wl, t.idx[q] % P.wl, gv[k] * t.wgt[q]);
                    }
                }
            }
            if (any_fit) {
#pragma unroll
                for (int k = 0; k < PX; ++k) {
                    const float py = (cys[k] + (float)(bb - P.radius)) * P.sy;
                    const float fy0 = floorf(py);
                    const int ry = (int)fy0 - ybase[k];
                    const float fy = py - fy0;
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        const float wy = j == ry ? 1.f - fy : (j == ry + 1 ? fy : 0.f);
#pragma unroll
                        for (int i = 0; i < K; ++i) patch[k][j][i] = fmaf(wy, row[k][i], patch[k][j][i]);
                    }
                }
            }
        }
        if (gm) {
#pragma unroll
            for (int r = 0; r < MH; ++r) {
                const int yy = oy + r;
                if (yy < 0 || yy >= P.hl) continue;
                float mm[MW];
#pragma unroll
                for (int t = 0; t < MW; ++t) {
                    float m = 0.f;
#pragma unroll
                    for (int k = 0; k < PX; ++k) {
                        // element (r - dy_k, t - dx_k) of pixel k's patch: select among the compile-time
                        // candidates rows {r, r-1} x columns {t, t-1, t-2}
                        const int dyk = k ? dy1 : dy0, dxk = k ? dx1 : dx0;
                        float e[3];
#pragma unroll
                        for (int q = 0; q < 3; ++q) {
                            const int i = t - q;
                            const float a0 = (i >= 0 && i < K && r < K) ? patch[k][r < K ? r : 0][i >= 0 && i < K ? i : 0] : 0.f;
                            const float a1 = (i >= 0 && i < K && r >= 1 && r - 1 < K)
                                                 ? patch[k][r >= 1 && r - 1 < K ? r - 1 : 0][i >= 0 && i < K ? i : 0] : 0.f;
                            e[q] = dyk ? a1 : a0;
                        }
                        m += dxk == 0 ? e[0] : (dxk == 1 ? e[1] : e[2]);
                    }
                    mm[t] = m;
                }
                // r_t(l) = mm_l[t] + link_l r_{t+1}(l-1): column ox_l + t of the chain
#pragma unroll
                for (int t = 0; t < MW; ++t) {
                    const int kmax = MW - 1 - t;
                    float rr = mm[t + kmax];
#pragma unroll
                    for (int q = kmax - 1; q >= 0; --q) {
                        const float up = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(rr), 0x138, 0xf, 0xf, false));
                        rr = mm[t + q] + (link ? up : 0.f);
                    }
                    mm[t] = (t < 1 || !link_next) ? rr : 0.f;
                }
#pragma unroll
                for (int t = 0; t < MW; ++t) {
                    const int xx = ox + t;
                    if (xx >= 0 && xx < P.wl && mm[t] != 0.f) add(yy, xx, mm[t]);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < PX; ++k) {
                if (!fits[k]) continue;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const int yy = ybase[k] + j;
                    if (yy < 0 || yy >= P.hl) continue;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const int xx = xbase[k] + i;
                        if (xx >= 0 && xx < P.wl && patch[k][j][i] != 0.f) add(yy, xx, patch[k][j][i]);
                    }
                }
            }
        }
        *reinterpret_cast<v2*>(gf1 + ((size_t)b * C + c) * n + p0) = s1;
    }
    __syncthreads();
    float* gw = g2c + (size_t)wy0 * P.wl;
    for (int k = threadIdx.x; k < wrows * P.wl; k += kThreads) {
        const float v = win[k];
        if (v != 0.f) atomicAdd(gw + k, v);
    }
}

// ---- DICL baseline integer volume ------------------------------------------------------------
struct IntParams {
    int B, C, h, w, ru, rv;
};

// occlusion mask of dicl.py:236-237 depends only on the displaced f2 pixel: nz = sum_c f2 != 0
__global__ void __launch_bounds__(kThreads)
dicl_nz_kernel(const float* __restrict__ f2, IntParams P, unsigned char* __restrict__ nz) {
    const int n = P.h * P.w;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= n) return;
    const int b = blockIdx.y;
    const float* f = f2 + (size_t)b * P.C * n + p;
    float s = 0.f;
    for (int c = 0; c < P.C; ++c) s += f[(size_t)c * n];
    nz[(size_t)b * n + p] = s != 0.f;
}

// Integer volume (impls/dicl.py:212-238), written for the write stream: a 1-D grid remapped per
// XCD (one batch image's f1/f2 — 2 x 1.5 MB at cfg3 level 2 — stay in that XCD's L2 while its 49
// displacement planes re-read them), the channel loop unrolled by U so a lane's loads of U channels
// are all in flight before its 2U stores, and optionally non-temporal stores (the 1.2 GB volume is
// written once and read by the next kernel, never by this one).
template <int CT, bool NT, int WPE = 1>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(WPE)))
dicl_stack_int_v2_kernel(const float* __restrict__ f1, const float* __restrict__ f2,
                         const unsigned char* __restrict__ nz, IntParams P, int nqb, int remap,
                         float* __restrict__ out) {
    constexpr int U = 8;
    const int n = P.h * P.w;
    const int dv = 2 * P.rv + 1, ndisp = (2 * P.ru + 1) * dv;
    const int lid = remap ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int xb = lid % nqb, rest = lid / nqb;
    const int disp = rest % ndisp, b = rest / ndisp;
    const int p0 = (xb * kThreads + threadIdx.x) * 4;
    if (p0 >= n) return;
    const int i = disp / dv, jj = disp - i * dv;
    const int di = i - P.ru, dj = jj - P.rv;
    int src[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int p = p0 + k;
        const int y = p / P.w, x = p - y * P.w;
        const int xx = x + di, yy = y + dj;
        const bool inb = xx >= 0 && xx < P.w && yy >= 0 && yy < P.h;
        src[k] = inb ? yy * P.w + xx : 0;
        ok[k] = inb && nz[(size_t)b * n + src[k]];
    }
    const int C = CT ? CT : P.C;
    float* o = out + ((size_t)(b * ndisp + disp) * 2 * C) * n + p0;
    const float* f1b = f1 + (size_t)b * C * n + p0;
    const float* f2b = f2 + (size_t)b * C * n;
#pragma unroll 4
    for (int c0 = 0; c0 < C; c0 += U) {
        f4_t a[U], v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (CT || c0 + u < C) {
                const float* f2c = f2b + (size_t)(c0 + u) * n;
                a[u] = *reinterpret_cast<const f4_t*>(f1b + (size_t)(c0 + u) * n);
                v[u] = f4_t{f2c[src[0]], f2c[src[1]], f2c[src[2]], f2c[src[3]]};
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (CT || c0 + u < C) {
                const f4_t m1{ok[0] ? a[u].x : 0.f, ok[1] ? a[u].y : 0.f, ok[2] ? a[u].z : 0.f, ok[3] ? a[u].w : 0.f};
                const f4_t m2{ok[0] ? v[u].x : 0.f, ok[1] ? v[u].y : 0.f, ok[2] ? v[u].z : 0.f, ok[3] ? v[u].w : 0.f};
                st4<NT>(o + (size_t)(c0 + u) * n, m1);
                st4<NT>(o + (size_t)(C + c0 + u) * n, m2);
            }
        }
    }
}

// launch the integer volume (nz already computed).  Measured at cfg3 (profiles/dicl_ab_r01.json): 0.366 ms
// for the first formulation (3-D grid, rolled channel loop) -> 0.234 ms (unrolled, non-temporal stores,
// no XCD remap); 8 waves per SIMD forced is slower (0.235 ms, profiles/dicl_int_wpe_ab_r02.json)
int launch_stack_int(const float* fmap1, const float* fmap2, const unsigned char* nz, const IntParams& P,
                     float* out, hipStream_t st) {
    const int n = P.h * P.w;
    const int ndisp = (2 * P.ru + 1) * (2 * P.rv + 1);
    const int nqb = (n / 4 + kThreads - 1) / kThreads;
    const long long nwg = (long long)nqb * ndisp * P.B;
    RMD_REQUIRE(nwg < (1ll << 31), RMD_ERR_SHAPE, "rmd_dicl_stack_int: grid too large");
    const bool remap = false;
    if (P.C == 32) {
        dicl_stack_int_v2_kernel<32, true><<<(unsigned)nwg, kThreads, 0, st>>>(fmap1, fmap2, nz, P, nqb, remap, out);
    } else {
        dicl_stack_int_v2_kernel<0, true><<<(unsigned)nwg, kThreads, 0, st>>>(fmap1, fmap2, nz, P, nqb, remap, out);
    }
    return check_launch("rmd_dicl_stack_int");
}

// backward (deterministic gathers, no atomics):
//   grad_f1[c, p] = sum_{i,j} ok_ij(p) g[i,j,c,p];   grad_f2[c, q] = sum_{i,j} ok_ij(q-d_ij) g[i,j,C+c,q-d_ij]
__global__ void __launch_bounds__(kThreads)
dicl_stack_int_backward_kernel(const float* __restrict__ g, const unsigned char* __restrict__ nz, IntParams P,
                               float* __restrict__ gf1, float* __restrict__ gf2) {
    const int n = P.h * P.w;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= n) return;
    const int c = blockIdx.y, b = blockIdx.z;
    const int C = P.C;
    const int du = 2 * P.ru + 1, dv = 2 * P.rv + 1;
    const int y = p / P.w, x = p - y * P.w;
    const unsigned char* nzb = nz + (size_t)b * n;
    const bool nzp = nzb[p];
    const float* gb = g + (size_t)b * du * dv * 2 * C * n;
    float s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < du; ++i) {
        for (int jj = 0; jj < dv; ++jj) {
            const int di = i - P.ru, dj = jj - P.rv;
            const size_t plane = (size_t)(i * dv + jj) * 2 * C;
            // this pixel as the query: its f1 half (needs target p + d in bounds and non-zero)
            const int xx = x + di, yy = y + dj;
            if (xx >= 0 && xx < P.w && yy >= 0 && yy < P.h && nzb[yy * P.w + xx]) s1 += gb[(plane + c) * n + p];
            // this pixel as the target of query p - d: its f2 half
            const int qx = x - di, qy = y - dj;
            if (nzp && qx >= 0 && qx < P.w && qy >= 0 && qy < P.h) s2 += gb[(plane + C + c) * n + qy * P.w + qx];
        }
    }
    gf1[((size_t)b * C + c) * n + p] = s1;
    gf2[((size_t)b * C + c) * n + p] = s2;
}

// ---- displacement-aware projection: out[b, o, p] = sum_i W[o, i] x[b, i, p] ------------------
// One lane per pixel, 16 output channels per pass held in registers; W rows broadcast from LDS.
constexpr int kDapOB = 16;

template <bool LDS_W>
__global__ void __launch_bounds__(kThreads)
dap_kernel(const float* __restrict__ x, const float* __restrict__ wgt, int D, int n, int transpose,
           float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float sw[];     // D x D (row o, col i)
    if constexpr (LDS_W) {
        for (int k = threadIdx.x; k < D * D; k += kThreads) {
            const int o = k / D, i = k - o * D;
            sw[k] = transpose ? wgt[i * D + o] : wgt[k];
        }
        __syncthreads();
    }
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y;
    if (p >= n) return;
    const float* xb = x + (size_t)b * D * n + p;
    float* ob = out + (size_t)b * D * n + p;
    for (int o0 = 0; o0 < D; o0 += kDapOB) {
        float acc[kDapOB];
#pragma unroll
        for (int k = 0; k < kDapOB; ++k) acc[k] = 0.f;
        for (int i = 0; i < D; ++i) {
            const float xv = xb[(size_t)i * n];
#pragma unroll
            for (int k = 0; k < kDapOB; ++k) {
                const int o = min(o0 + k, D - 1);
                float wv;
                if constexpr (LDS_W) wv = sw[o * D + i];
                else wv = transpose ? wgt[i * D + o] : wgt[o * D + i];     // wave-uniform: scalar loads
                acc[k] = fmaf(wv, xv, acc[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < kDapOB; ++k)
            if (o0 + k < D) ob[(size_t)(o0 + k) * n] = acc[k];
    }
}

typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 dbf16x8_t;
typedef __attribute__((ext_vector_type(4))) __bf16 dbf16x4_t;

// ---- DAP as a split-bf16 (x3) MFMA GEMM (product form) -----------------------------------------
// out_b (D x n) = W (D x D) . x_b (D x n), fp32 accuracy from three bf16 products per k-step,
// v = hi + lo, hi = bf16(v), lo = bf16(v - hi):  acc += W_lo.x_hi + W_hi.x_lo + W_hi.x_hi  (the
// dropped lo.lo term is ~2^-16 relative; same split as the fp32-mode correlation GEMM).  The exact
// f32 MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate and held the round-1 kernel at
// ~25 % of even that peak (0.27 ms at D = 324); here the 3 bf16 products cost 3/16.
// Geometry: a workgroup owns an M-block of MT x 32 output displacements (all of them when D <= 128)
// and one chunk of the batch image's 32-pixel tiles.  The block's W rows (or W^T rows, transpose)
// are split once into hi / lo bf16 in LDS — rows of 2 Kp + 16 bytes, an odd number of 16-B slots,
// so a ds_read_b128 lane group hits distinct bank slots; each wave then sweeps its tiles: x is read
// straight from HBM as the MFMA B operand (lane (r, h) holds rows 8h..8h+7 of k-step s at pixel r:
// eight coalesced 128-B row segments), split in registers, KC k-steps per chunk with the next chunk
// (or the next tile's first) in flight during the current chunk's MFMAs.  Rows >= D and pixels >= n
// fall outside the per-image buffer range (loads read 0, stores are dropped).  The M-blocks of one
// pixel chunk are consecutive workgroup ids (one XCD), so x is fetched from HBM once for all blocks.
// Output stores are non-temporal.  Measured (profiles/dap_ab_r02.json, b8): D = 49 10.1 us, D = 81
// 12.1 us, D = 324 62 us, vs 16.8 / 23.2 / 317 us for the exact-f32 MFMA form; error vs float64
// 1.5e-5 max-normalised.  At D = 324 the MFMA floor is ~19 us and the HBM floor ~27 us; PMC shows x
// fetched from HBM once (84 MB) and the x ring depth (3-8 chunks of prefetch) changes nothing, so the
// gap is in the per-CU issue of the 4x L2 re-reads of x and the single 8-wave workgroup per CU.
constexpr int kDapSG = 4;     // W staging: 4-element groups per thread in flight
constexpr int kDapStoreAux = 2;   // output store cache policy (gfx950 cpol: 2 = nt): 10-15 % at D <= 81
constexpr int kDapKC = 8, kDapNB = 2;   // x ring: NB buffers of KC k-steps

__device__ __forceinline__ void dap_split8(const float* v, dbf16x8_t& hi, dbf16x8_t& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        hi[j] = (__bf16)v[j];
        lo[j] = (__bf16)(v[j] - (float)hi[j]);
    }
}

template <int MT, int NW, int AUX, int KC, int NB>
__global__ void __launch_bounds__(NW * 64, 2)
dap_x3_kernel(const float* __restrict__ x, const float* __restrict__ wgt, int D, int n, int transpose,
              int mblocks, int per, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
    const int Kp = (D + 15) & ~15, nks = Kp >> 4;
    const int RB = 2 * Kp + 16;
    unsigned char* const sh = sm;                       // hi rows
    unsigned char* const sl = sm + MT * 32 * RB;        // lo rows
    int id = xcd_block(blockIdx.x, gridDim.x);
    const int mb = id % mblocks;
    id /= mblocks;
    const int pc = id % per, b = id / per;
    const int o0 = mb * 32 * MT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int ntile = (n + 31) >> 5;
    auto rsrc = [&](const void* base) {
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)base);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)base >> 32));
        return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo), (short)0,
                                                 (int)((unsigned)D * (unsigned)n * 4u), 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t xr = rsrc(x + (size_t)b * D * n);
    const __amdgpu_buffer_rsrc_t orr = rsrc(out + (size_t)b * D * n);
    const unsigned rowb = (unsigned)n * 4u;
    const unsigned aoff = (unsigned)(r * RB + 16 * h);
    const int nch = (nks + KC - 1) / KC;

    // x chunks stream through a ring of NB register buffers: step i = (tile t0 + (i / nch) tstride,
    // chunk i % nch) lives in buffer i % NB and is loaded NB - 1 steps before its use
    float xb[NB][KC * 8];
    // chunk c of tile tt: rows 16 (KC c + u) + 8 h + j at pixel 32 tt + r (out of range past n / D)
    auto load = [&](float (&v)[KC * 8], int tt, int c) {
        const int p = tt * 32 + r;
        const unsigned base = p < n ? (unsigned)(8 * h + 16 * KC * c) * rowb + (unsigned)p * 4u : 0x80000000u;
#pragma unroll
        for (int u = 0; u < KC; ++u)
            if (KC * c + u < nks)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    v[u * 8 + j] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        xr, (int)(base + (unsigned)(16 * u + j) * rowb), 0, 0));
    };

    const int t0 = pc * NW + w, tstride = per * NW;
    const int mytiles = t0 < ntile ? (ntile - 1 - t0) / tstride + 1 : 0;
    const int nsteps = mytiles * nch;
#pragma unroll
    for (int u = 0; u < NB - 1; ++u)        // in flight while the workgroup stages W
        if (u < nsteps) load(xb[u], t0 + (u / nch) * tstride, u % nch);

    // stage the block's W rows as hi / lo bf16 (4 consecutive k per thread; W^T reads run along o),
    // kDapSG groups' loads in flight per thread before any is converted
    {
        constexpr int rows = MT * 32;
        const int kq = Kp >> 2, total = rows * kq;
        for (int e0 = tid; e0 < total; e0 += NW * 64 * kDapSG) {
            float v[kDapSG][4];
            int ro[kDapSG];
#pragma unroll
            for (int g = 0; g < kDapSG; ++g) {
                const int e = e0 + g * NW * 64;
                int rr, k;
                if (transpose) { rr = e % rows; k = 4 * (e / rows); }
                else { rr = e / kq; k = 4 * (e - rr * kq); }
                const int o = o0 + rr;
                ro[g] = e < total ? rr * RB + 2 * k : -1;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int i = k + q;
                    v[g][q] = (e < total && o < D && i < D) ? (transpose ? wgt[(size_t)i * D + o] : wgt[(size_t)o * D + i])
                                                            : 0.f;
                }
            }
#pragma unroll
            for (int g = 0; g < kDapSG; ++g) {
                if (ro[g] < 0) continue;
                dbf16x4_t hi, lo;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    hi[q] = (__bf16)v[g][q];
                    lo[q] = (__bf16)(v[g][q] - (float)hi[q]);
                }
                *reinterpret_cast<dbf16x4_t*>(sh + ro[g]) = hi;
                *reinterpret_cast<dbf16x4_t*>(sl + ro[g]) = lo;
            }
        }
    }
    __syncthreads();

    f32x16_t acc[MT];
    for (int i0 = 0; i0 < nsteps; i0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int i = i0 + u;
            if (i >= nsteps) break;
            const int ip = i + NB - 1;
            if (ip < nsteps) load(xb[(u + NB - 1) % NB], t0 + (ip / nch) * tstride, ip % nch);
            const int c = i % nch;
            if (c == 0) {
#pragma unroll
                for (int m = 0; m < MT; ++m) acc[m] = f32x16_t{};
            }
#pragma unroll
            for (int uu = 0; uu < KC; ++uu) {
                const int s = c * KC + uu;
                if (s < nks) {
                    dbf16x8_t bh, bl;
                    dap_split8(xb[u] + uu * 8, bh, bl);
#pragma unroll
                    for (int m = 0; m < MT; ++m) {
                        const unsigned a = aoff + (unsigned)(m * 32 * RB + 32 * s);
                        const dbf16x8_t ah = *reinterpret_cast<const dbf16x8_t*>(sh + a);
                        const dbf16x8_t al = *reinterpret_cast<const dbf16x8_t*>(sl + a);
                        f32x16_t cacc = acc[m];
                        cacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, cacc, 0, 0, 0);
                        cacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, cacc, 0, 0, 0);
                        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, cacc, 0, 0, 0);
                    }
                }
            }
            if (c == nch - 1) {
                // C tile: lane (r, h) holds rows 8 (e >> 2) + 4 h + (e & 3) of pixel column r
                const int p = (t0 + (i / nch) * tstride) * 32 + r;
                const unsigned so = p < n ? (unsigned)(4 * h) * rowb + (unsigned)p * 4u : 0x80000000u;
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        const unsigned row = (unsigned)(o0 + m * 32 + 8 * (e >> 2) + (e & 3));
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(acc[m][e]), orr, (int)(so + row * rowb),
                                                              0, AUX);
                    }
            }
        }
    }
}


int stack_params(StackParams& P, int B, int C, int h, int w, int hl, int wl, int radius, int level, int nh, int nw,
                 int extra) {
    RMD_REQUIRE(B > 0 && C > 0 && h > 0 && w > 0 && hl > 0 && wl > 0, RMD_ERR_SHAPE, "rmd_dicl_stack: bad sizes");
    RMD_REQUIRE(radius >= 0 && radius <= 32, RMD_ERR_SHAPE, "rmd_dicl_stack: radius %d out of range", radius);
    RMD_REQUIRE((h * w) % 4 == 0, RMD_ERR_SHAPE, "rmd_dicl_stack: h*w must be a multiple of 4 (MatchingNet needs even h, w)");
    RMD_REQUIRE(level >= 0 && level < 16, RMD_ERR_SHAPE, "rmd_dicl_stack: bad level");
    P.B = B; P.C = C; P.h = h; P.w = w; P.hl = hl; P.wl = wl; P.radius = radius; P.extra = extra ? 2 : 0;
    P.inv_scale = 1.0f / (float)(1 << level);
    // (wl-1)/(wn-1): 0/0 -> NaN exactly as the reference's normalisation does for 1-pixel maps
    P.sx = (float)(wl - 1) / (float)(nw - 1);
    P.sy = (float)(hl - 1) / (float)(nh - 1);
    return RMD_OK;
}

// ---- backward warping (common/warp.py:5-33), alone or fused into the occlusion pass of the integer
// volume (impls/dicl.py:178-181 -> 212-238) ---------------------------------------------------------
// warped[c, p] = mask(p) * bilinear(img2[c], x + fx, y + fy) with zero padding, where mask(p) = the
// in-bounds bilinear weight > 1 - eps (grid_sample of a ones tensor, warp.py:28-30).  One lane per pixel
// loops over the channels; with NZ it also writes the occlusion flag sum_c warped[c, p] != 0 that
// integer-volume kernel consumes, so the warp costs no extra pass over the warped map.
struct WarpTaps {
    int idx[4];
    float wgt[4];
    bool valid;
};

__device__ __forceinline__ WarpTaps warp_taps(const float* __restrict__ flow, int b, int p, int h, int w, float eps) {
    const int n = h * w;
    const int y = p / w, x = p - y * w;
    const float ix = (float)x + flow[((size_t)b * 2 + 0) * n + p];
    const float iy = (float)y + flow[((size_t)b * 2 + 1) * n + p];
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const float ax = ix - fx0, ay = iy - fy0;
    WarpTaps t;
    float wsum = 0.f;
    // far-away positions: clamp before the int conversion (their taps are all out of bounds anyway)
    const int x0 = (int)fminf(fmaxf(fx0, -2.f), (float)w + 1.f), y0 = (int)fminf(fmaxf(fy0, -2.f), (float)h + 1.f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int dx = k & 1, dy = k >> 1;
        const int xx = x0 + dx, yy = y0 + dy;
        const bool in = xx >= 0 && xx < w && yy >= 0 && yy < h;
        const float wk = (dx ? ax : 1.f - ax) * (dy ? ay : 1.f - ay);
        t.idx[k] = in ? yy * w + xx : 0;
        t.wgt[k] = in ? wk : 0.f;
        wsum += t.wgt[k];
    }
    t.valid = wsum > 1.0f - eps;
    return t;
}

template <bool NZ>
__global__ void __launch_bounds__(kThreads)
warp_kernel(const float* __restrict__ img2, const float* __restrict__ flow, int C, int h, int w, float eps,
            float* __restrict__ out, unsigned char* __restrict__ mask, unsigned char* __restrict__ nz) {
    const int n = h * w;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y;
    if (p >= n) return;
    const WarpTaps t = warp_taps(flow, b, p, h, w, eps);
    const float* src = img2 + (size_t)b * C * n;
    float* o = out + (size_t)b * C * n + p;
    float s = 0.f;
    for (int c = 0; c < C; ++c) {
        const float* sc = src + (size_t)c * n;
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) v = fmaf(t.wgt[k], sc[t.idx[k]], v);
        v = t.valid ? v : 0.f;
        o[(size_t)c * n] = v;
        s += v;
    }
    if (mask) mask[(size_t)b * n + p] = t.valid;
    if (NZ) nz[(size_t)b * n + p] = s != 0.f;
}

// d img2 += bilinear^T (mask * grad): float atomics onto the 4 taps (as ATen's grid_sampler_2d_backward)
__global__ void __launch_bounds__(kThreads)
warp_backward_kernel(const float* __restrict__ grad, const float* __restrict__ flow, int C, int h, int w, float eps,
                     float* __restrict__ grad_img2) {
    const int n = h * w;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y;
    if (p >= n) return;
    const WarpTaps t = warp_taps(flow, b, p, h, w, eps);
    if (!t.valid) return;
    const float* g = grad + (size_t)b * C * n + p;
    float* d = grad_img2 + (size_t)b * C * n;
    for (int c = 0; c < C; ++c) {
        const float gv = g[(size_t)c * n];
        if (gv == 0.f) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (t.wgt[k] != 0.f) atomicAdd(d + (size_t)c * n + t.idx[k], t.wgt[k] * gv);
    }
}

}  // namespace
}  // namespace rmd

using namespace rmd;

extern "C" int rmd_dicl_stack(const float* fmap1, const float* fmap2, const float* coords, int batch, int channels,
                              int height, int width, int level_height, int level_width, int radius, int level,
                              int norm_height, int norm_width, int extra_delta, float* out, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && coords && out, RMD_ERR_ARG, "rmd_dicl_stack: null pointer");
    StackParams P;
    int rc = stack_params(P, batch, channels, height, width, level_height, level_width, radius, level, norm_height,
                          norm_width, extra_delta);
    if (rc) return rc;
    const int d = 2 * radius + 1;
    const double image_bytes = 4.0 * d * d * (2.0 * channels + P.extra) * height * width;
    if (P.sx == 1.0f && P.sy == 1.0f && radius >= 1 && radius <= 4 && image_bytes < 4294967296.0) {
        // Measured at cfg4 (profiles/dicl_ab_r01.json, dicl_px_ab_r02.json): non-temporal stores are the
        // win (0.33 -> 0.26 ms); one pixel per lane (56 VGPRs, 7 waves per SIMD instead of 4 with 2 or 4
        // pixels per lane) keeps more stores in flight: 0.238 vs 0.256 ms; an XCD remap changes nothing
        constexpr int px = 1;
        const int nxb = (height * width / px + kThreads - 1) / kThreads;
        const long long nwg = (long long)nxb * channels * batch;
        RMD_REQUIRE(nwg < (1ll << 31), RMD_ERR_SHAPE, "rmd_dicl_stack: grid too large");
        constexpr int remap = 0;
        hipStream_t st = as_stream(stream);
        switch (radius) {
#define RMD_CASE(RR) case RR: \
            dicl_stack_patch_kernel<RR, px, true><<<(unsigned)nwg, kThreads, 0, st>>>(fmap1, fmap2, coords, P, nxb, remap, out); \
            break;
            RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4)
#undef RMD_CASE
        }
        return check_launch("rmd_dicl_stack/patch");
    }
    dim3 grid((height * width / 4 + kThreads - 1) / kThreads, d * d, batch);
    if ((radius == 3 || radius == 4) && std::isfinite(P.sx) && std::isfinite(P.sy) && P.sx >= 0.f &&
        P.sy >= 0.f && P.sx <= 1.f && P.sy <= 1.f && image_bytes < 4294967296.0) {
        const float span = 2.0f * radius * std::max(P.sx, P.sy);
        const int k = ((int)std::floor(span * (1.0f + 1e-5f) + 1e-4f) + 3 + 1) & ~1;
        dim3 g1((height * width + kThreads - 1) / kThreads, channels, batch);
        hipStream_t st = as_stream(stream);
        bool launched = true;
        switch (radius * 100 + k) {
#define RMD_SCASE(RR, KK) case RR * 100 + KK: dicl_stack_sep_kernel<RR, KK, true><<<g1, kThreads, 0, st>>>(fmap1, fmap2, coords, P, out); break;
            RMD_SCASE(3, 4) RMD_SCASE(3, 6) RMD_SCASE(3, 8) RMD_SCASE(4, 4) RMD_SCASE(4, 6) RMD_SCASE(4, 8)
#undef RMD_SCASE
            default: launched = false;
        }
        if (launched) return check_launch("rmd_dicl_stack/separable");
    }
    dicl_stack_kernel<true, 1><<<grid, kThreads, 0, as_stream(stream)>>>(fmap1, fmap2, coords, P, out);
    return check_launch("rmd_dicl_stack");
}

extern "C" int rmd_dicl_stack_backward(const float* grad_stack, const float* coords, int batch, int channels,
                                       int height, int width, int level_height, int level_width, int radius,
                                       int level, int norm_height, int norm_width, int extra_delta,
                                       float* grad_fmap1, float* grad_fmap2, void* stream) {
    RMD_REQUIRE(grad_stack && coords && grad_fmap1 && grad_fmap2, RMD_ERR_ARG, "rmd_dicl_stack_backward: null pointer");
    StackParams P;
    int rc = stack_params(P, batch, channels, height, width, level_height, level_width, radius, level, norm_height,
                          norm_width, extra_delta);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    const int d = 2 * radius + 1;
    // LDS window: a workgroup's 256 pixels cover ~256/w + 1 rows; with the patch (<= 2r+2 rows at
    // unit steps) and some flow spread, 4096 floats (16 KiB) hold them for w up to ~170 and leave
    // room for 9 workgroups per CU instead of 3 (48 KiB); rows past the window still go to global
    // atomics, so the choice only affects speed.
    const float rows_est = 2.0f * radius * std::max(P.sy, 1.0f) + 256.0f / width * std::max(P.sy, 0.5f) + 10.0f;
    const bool small_win = rows_est * level_width <= (float)kWinSmall;
    const double image_bytes = 4.0 * d * d * (2.0 * channels + P.extra) * height * width;
    if (P.sx == 1.0f && P.sy == 1.0f && radius >= 1 && radius <= 4) {
        (void)hipMemsetAsync(grad_fmap2, 0, sizeof(float) * (size_t)batch * channels * level_height * level_width, st);
        dim3 grid((height * width + kThreads - 1) / kThreads, channels, batch);
        // two pixels per lane: the general two-pixel merge over the joint patch box + the cross-lane chain
        // (0.55 vs 0.75 ms smooth flow, 0.77 vs 0.96 ms steep flow at cfg4 against the round-1 per-pixel
        // adds, profiles/dicl_bwd_ab_r02.json); one pixel per lane for images past 4 GiB of stack
        if (image_bytes < 4294967296.0) {
            const float rows2 = 2.0f * radius + 512.0f / width + 10.0f;
            const bool small2 = rows2 * level_width <= (float)kWinSmall;
            dim3 grid2((height * width / 2 + kThreads - 1) / kThreads, channels, batch);
            switch (radius) {
#define RMD_CASE(RR) case RR: \
                if (small2) dicl_stack_patch_backward_gm_kernel<RR, kWinSmall, true><<<grid2, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
                else dicl_stack_patch_backward_gm_kernel<RR, kWinFloats, true><<<grid2, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
                break;
                RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4)
#undef RMD_CASE
            }
            return check_launch("rmd_dicl_stack_backward/patch2");
        }
        switch (radius) {
#define RMD_CASE(RR) case RR: \
            if (small_win) dicl_stack_patch_backward_kernel<RR, kWinSmall><<<grid, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
            else dicl_stack_patch_backward_kernel<RR, kWinFloats><<<grid, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
            break;
            RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4)
#undef RMD_CASE
        }
        return check_launch("rmd_dicl_stack_backward/patch");
    }
    (void)hipMemsetAsync(grad_fmap2, 0, sizeof(float) * (size_t)batch * channels * level_height * level_width, st);
    if (level_width <= kWinFloats && std::isfinite(P.sx) && std::isfinite(P.sy) && P.sy >= 0.f && P.sx >= 0.f &&
        P.sx <= 1.f && P.sy <= 1.f) {
        // patch edge: floor(span) + 1 tap offsets + 1 for the right/bottom tap + 1 for fp32 rounding, even
        const float span = 2.0f * radius * std::max(P.sx, P.sy);
        const int k = ((int)std::floor(span * (1.0f + 1e-5f) + 1e-4f) + 3 + 1) & ~1;
        dim3 grid((height * width + kThreads - 1) / kThreads, channels, batch);
        // two pixels per lane with the merged / chained patch adds (K <= 8: 0.50 vs 0.68 ms smooth, 0.52 vs
        // 0.61 ms steep flow at cfg4 level 1 against one pixel per lane); K > 8 one pixel per lane
        if (k <= 8) {
            const float rows2 = 2.0f * radius * std::max(P.sy, 1.0f) + 512.0f / width * std::max(P.sy, 0.5f) + 10.0f;
            const bool small2 = rows2 * level_width <= (float)kWinSmall;
            dim3 grid2((height * width / 2 + kThreads - 1) / kThreads, channels, batch);
            switch (k) {
#define RMD_KCASE2(KK) case KK: \
                if (small2) dicl_stack_sep_backward2_kernel<KK, kWinSmall><<<grid2, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
                else dicl_stack_sep_backward2_kernel<KK, kWinFloats><<<grid2, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
                return check_launch("rmd_dicl_stack_backward/separable2");
                RMD_KCASE2(4) RMD_KCASE2(6) RMD_KCASE2(8)
#undef RMD_KCASE2
                default: break;
            }
        }
        switch (k) {
#define RMD_KCASE(KK) case KK: \
            if (small_win) dicl_stack_sep_backward_kernel<KK, kWinSmall><<<grid, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
            else dicl_stack_sep_backward_kernel<KK, kWinFloats><<<grid, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2); \
            return check_launch("rmd_dicl_stack_backward/separable");
            RMD_KCASE(4) RMD_KCASE(6) RMD_KCASE(8) RMD_KCASE(10)
#undef RMD_KCASE
            default: break;
        }
    }
    if (level_width <= kWinFloats && std::isfinite(P.sx) && std::isfinite(P.sy) && P.sy >= 0.f) {
        dim3 grid((height * width + kThreads - 1) / kThreads, channels, batch);
        if (small_win) dicl_stack_general_backward_kernel<kWinSmall><<<grid, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2);
        else dicl_stack_general_backward_kernel<kWinFloats><<<grid, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap1, grad_fmap2);
        return check_launch("rmd_dicl_stack_backward/general");
    }
    dim3 g1((height * width / 4 + kThreads - 1) / kThreads, channels, batch);
    dicl_stack_grad_f1_kernel<<<g1, kThreads, 0, st>>>(grad_stack, P, grad_fmap1);
    dim3 g2((height * width + kThreads - 1) / kThreads, d * d, batch);
    dicl_stack_grad_f2_kernel<<<g2, kThreads, 0, st>>>(grad_stack, coords, P, grad_fmap2);
    return check_launch("rmd_dicl_stack_backward");
}

extern "C" size_t rmd_dicl_stack_int_workspace_bytes(int batch, int height, int width) {
    return (size_t)batch * height * width;
}

extern "C" int rmd_dicl_stack_int(const float* fmap1, const float* fmap2, int batch, int channels, int height,
                                  int width, int ru, int rv, float* out, void* workspace, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && out && workspace, RMD_ERR_ARG, "rmd_dicl_stack_int: null pointer");
    RMD_REQUIRE(batch > 0 && channels > 0 && height > 0 && width > 0 && ru >= 0 && rv >= 0, RMD_ERR_SHAPE,
                "rmd_dicl_stack_int: bad sizes");
    RMD_REQUIRE((height * width) % 4 == 0, RMD_ERR_SHAPE, "rmd_dicl_stack_int: h*w must be a multiple of 4");
    IntParams P{batch, channels, height, width, ru, rv};
    hipStream_t st = as_stream(stream);
    const int n = height * width;
    unsigned char* nz = reinterpret_cast<unsigned char*>(workspace);
    dicl_nz_kernel<<<dim3((n + kThreads - 1) / kThreads, batch), kThreads, 0, st>>>(fmap2, P, nz);
    return launch_stack_int(fmap1, fmap2, nz, P, out, st);
}

extern "C" int rmd_dicl_stack_int_backward(const float* grad_mvol, const float* fmap2, int batch, int channels,
                                           int height, int width, int ru, int rv, float* grad_fmap1,
                                           float* grad_fmap2, void* workspace, void* stream) {
    RMD_REQUIRE(grad_mvol && fmap2 && grad_fmap1 && grad_fmap2 && workspace, RMD_ERR_ARG,
                "rmd_dicl_stack_int_backward: null pointer");
    RMD_REQUIRE(batch > 0 && channels > 0 && height > 0 && width > 0 && ru >= 0 && rv >= 0, RMD_ERR_SHAPE,
                "rmd_dicl_stack_int_backward: bad sizes");
    IntParams P{batch, channels, height, width, ru, rv};
    hipStream_t st = as_stream(stream);
    const int n = height * width;
    unsigned char* nz = reinterpret_cast<unsigned char*>(workspace);
    dicl_nz_kernel<<<dim3((n + kThreads - 1) / kThreads, batch), kThreads, 0, st>>>(fmap2, P, nz);
    dim3 grid((n + kThreads - 1) / kThreads, channels, batch);
    dicl_stack_int_backward_kernel<<<grid, kThreads, 0, st>>>(grad_mvol, nz, P, grad_fmap1, grad_fmap2);
    return check_launch("rmd_dicl_stack_int_backward");
}

namespace rmd {
namespace {

// ---- DAP weight gradient ------------------------------------------------------------------------
// dW[o][i] = sum_b sum_p g[b][o][p] x[b][i][p]: the weight gradient of the 1x1 convolution
// (blocks/dicl.py:137,147; autograd of F.conv2d w.r.t. its weight).  M = N = D (tiny), K = B * pixels
// (large): K is split over workgroups (one image's pixel chunk each), every workgroup computes the
// full D x D partial with v_mfma_f32_32x32x16_bf16 on split operands (g = hi + lo, x = hi + lo:
// lo.hi + hi.lo + hi.hi, the forward DAP's split), a second kernel sums the partials in split order
// (deterministic).  Wave w of a workgroup owns a 2 x 2 block of 32 x 32 output tiles; A / B fragments
// are 8 consecutive pixels of one row (two float4 loads) split in registers.
constexpr int kWgPx = 16;                        // pixels per MFMA k-step

__device__ __forceinline__ void wg_frag(const float* __restrict__ row, bool rok, int p, int n, dbf16x8_t& hi, dbf16x8_t& lo) {
    float v[8];
    if (rok && p + 7 < n && ((reinterpret_cast<uintptr_t>(row + p) & 15) == 0)) {
        *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(row + p);
        *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(row + p + 4);
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (rok && p + e < n) ? row[p + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        hi[e] = (__bf16)v[e];
        lo[e] = (__bf16)(v[e] - (float)hi[e]);
    }
}

// grid (B * nchunk, tile groups); 256 threads; part (splits, Dp, Dp)
__global__ void __launch_bounds__(256)
dap_wgrad_kernel(const float* __restrict__ g, const float* __restrict__ x, int D, int n, int nchunk, int pchunk,
                 int Dp, float* __restrict__ part) {
    const int s = blockIdx.x, b = s / nchunk, c = s % nchunk;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 31, h = lane >> 5;
    const int Dt = Dp / 32, Db = (Dt + 1) / 2;                   // 32-row tiles, 2x2 tile blocks per side
    const int tb = blockIdx.y * 4 + w;
    if (tb >= Db * Db) return;                                   // no barriers in this kernel
    const int ot0 = 2 * (tb / Db), it0 = 2 * (tb % Db);
    const int p0 = c * pchunk, p1 = min(n, p0 + pchunk);
    const float* gb = g + (size_t)b * D * n;
    const float* xb = x + (size_t)b * D * n;
    f32x16_t acc[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) acc[u][v] = f32x16_t{};
    const int o[2] = {32 * ot0 + j, 32 * (ot0 + 1) + j}, i[2] = {32 * it0 + j, 32 * (it0 + 1) + j};
    for (int p = p0; p < p1; p += kWgPx) {
        dbf16x8_t ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            wg_frag(gb + (size_t)min(o[u], D - 1) * n, o[u] < D, p + 8 * h, p1, ah[u], al[u]);
            wg_frag(xb + (size_t)min(i[u], D - 1) * n, i[u] < D, p + 8 * h, p1, bh[u], bl[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[u], bh[v], acc[u][v], 0, 0, 0);
                acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[u], bl[v], acc[u][v], 0, 0, 0);
                acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[u], bh[v], acc[u][v], 0, 0, 0);
            }
    }
    // lane (column j, half h): register 4r + k is row 8r + 4h + k of the tile
    float* ps = part + (size_t)s * Dp * Dp;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            if (ot0 + u >= Dt || it0 + v >= Dt) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 32 * (ot0 + u) + 8 * (r >> 2) + 4 * h + (r & 3);
                ps[(size_t)row * Dp + 32 * (it0 + v) + j] = acc[u][v][r];
            }
        }
}

// dW[o][i] = the sum over splits (fixed order: deterministic)
__global__ void __launch_bounds__(512)
dap_wgrad_reduce(const float* __restrict__ part, int splits, int D, int Dp, float* __restrict__ dw) {
    // 32 consecutive outputs x 16 split groups per 512-thread workgroup: thread (g, i) sums splits
    // g, g + 16, ... in order, then the 16 group sums are added in fixed order from LDS — the same
    // result for every launch (deterministic), with D^2 / 32 workgroups and coalesced 128-B reads
    __shared__ float red[16][33];
    const int t = threadIdx.x, i32 = t & 31, gsp = t >> 5;
    const int idx = blockIdx.x * 32 + i32;
    const bool ok = idx < D * D;
    const int o = ok ? idx / D : 0, i = ok ? idx % D : 0;
    const float* pp = part + (size_t)o * Dp + i;
    const size_t mat = (size_t)Dp * Dp;
    // the group's partials are summed in split order, 8 loads in flight at a time (the plain loop waited
    // for each strided load before the next add: latency-bound at ~20 splits per group)
    float s = 0.f;
    int k = gsp;
    for (; k + 16 * 7 < splits; k += 16 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = pp[(size_t)(k + 16 * u) * mat];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < splits; k += 16) s += pp[(size_t)k * mat];
    red[gsp][i32] = s;
    __syncthreads();
    if (gsp == 0 && ok) {
        float r = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) r += red[g][i32];
        dw[idx] = r;
    }
}

struct WgPlan {
    int Dp, groups, nchunk, pchunk, splits;
};

WgPlan wgrad_plan(int batch, int D, int n) {
    WgPlan w{};
    w.Dp = (D + 31) / 32 * 32;
    const int Db = (w.Dp / 32 + 1) / 2;
    w.groups = (Db * Db + 3) / 4;
    // about 256 workgroups in all (one per CU), at least 4 k-steps per split
    const int want = std::max(1, 256 / (w.groups * batch));
    const int steps = (n + kWgPx - 1) / kWgPx;
    const int per = std::max(4, (steps + want - 1) / want);
    w.pchunk = per * kWgPx;
    w.nchunk = (n + w.pchunk - 1) / w.pchunk;
    w.splits = batch * w.nchunk;
    return w;
}

}  // namespace
}  // namespace rmd

extern "C" size_t rmd_dap_weight_grad_workspace_bytes(int batch, int disp, int pixels) {
    if (batch <= 0 || disp <= 0 || pixels <= 0) return 0;
    const rmd::WgPlan w = rmd::wgrad_plan(batch, disp, pixels);
    return (size_t)w.splits * w.Dp * w.Dp * sizeof(float);
}

extern "C" int rmd_dap_weight_grad(const float* grad_out, const float* x, int batch, int disp, int pixels,
                                   float* grad_weight, void* workspace, void* stream) {
    RMD_REQUIRE(grad_out && x && grad_weight && workspace, RMD_ERR_ARG, "rmd_dap_weight_grad: null pointer");
    RMD_REQUIRE(batch > 0 && disp > 0 && pixels > 0, RMD_ERR_SHAPE, "rmd_dap_weight_grad: bad sizes");
    const rmd::WgPlan w = rmd::wgrad_plan(batch, disp, pixels);
    RMD_REQUIRE((long long)w.splits * w.groups < (1ll << 31) && w.groups < 65536, RMD_ERR_SHAPE,
                "rmd_dap_weight_grad: grid too large");
    hipStream_t st = rmd::as_stream(stream);
    float* part = static_cast<float*>(workspace);
    rmd::dap_wgrad_kernel<<<dim3(w.splits, w.groups), 256, 0, st>>>(grad_out, x, disp, pixels, w.nchunk, w.pchunk,
                                                                    w.Dp, part);
    int rc = rmd::check_launch("rmd_dap_weight_grad");
    if (rc) return rc;
    rmd::dap_wgrad_reduce<<<(disp * disp + 31) / 32, 512, 0, st>>>(part, w.splits, disp, w.Dp, grad_weight);
    return rmd::check_launch("rmd_dap_weight_grad reduce");
}

extern "C" int rmd_dap(const float* x, const float* weight, int batch, int disp, int pixels, int transpose,
                       float* out, void* stream) {
    RMD_REQUIRE(x && weight && out, RMD_ERR_ARG, "rmd_dap: null pointer");
    RMD_REQUIRE(batch > 0 && disp > 0 && pixels > 0, RMD_ERR_SHAPE, "rmd_dap: bad sizes");
    const int Kp = (disp + 15) & ~15;
    if (disp <= 1024 && (long long)(Kp + 16) * pixels * 4 < (1ll << 31)) {
        // split-bf16 MFMA form: M-block of MT row tiles = the largest (<= 4) whose hi / lo W rows fit in
        // 160 KB of LDS; 8 waves per workgroup when the block leaves room for only one workgroup per CU
        const int mt_all = (disp + 31) / 32;
        const size_t rowb = 2 * (size_t)(2 * Kp + 16);       // hi + lo bytes per W row
        int mt = mt_all < 4 ? mt_all : 4;
        while (mt > 1 && (size_t)32 * mt * rowb > 160 * 1024) --mt;
        const size_t lds = (size_t)32 * mt * rowb;
        constexpr int nw = 8;
        const int mblocks = (mt_all + mt - 1) / mt;
        const int ntile = (pixels + 31) / 32;
        // one round of workgroups over the chip: ~256 x (workgroups per CU) in all, at least one
        // 32-pixel tile per wave.  At 171-227 VGPRs a SIMD holds 2 waves, so a CU holds one 8-wave
        // workgroup (measured against 4-wave workgroups, 2-3 per CU: 11.5 vs 13.2 us at D = 49, 13.1 vs
        // 15.1 at D = 81, 62 vs 87 at D = 324 — fewer W stagings; profiles/dap_ab_r02.json)
        const int occ = 1;
        const long long units = (long long)mblocks * batch;
        int per = (int)std::min<long long>((256LL * occ + units - 1) / units, (ntile + nw - 1) / nw);
        per = std::max(per, 1);
        const long long nwg = units * per;
        RMD_REQUIRE(nwg < (1LL << 31), RMD_ERR_SHAPE, "rmd_dap: grid too large");
        hipStream_t st = as_stream(stream);
#define RMD_DAPX3_R(MT, NW, AUX, KC, NB)                                                                    \
        do {                                                                                                \
            /* the >64 KB LDS opt-in is per device: set before every launch */                           \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dap_x3_kernel<MT, NW, AUX, KC, NB>),     \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);               \
            dap_x3_kernel<MT, NW, AUX, KC, NB><<<(unsigned)nwg, NW * 64, lds, st>>>(x, weight, disp, pixels, \
                                                                                  transpose, mblocks, per, out); \
        } while (0)
#define RMD_DAPX3(MT, NW) RMD_DAPX3_R(MT, NW, kDapStoreAux, kDapKC, kDapNB)
        switch (mt) {
            case 1: RMD_DAPX3(1, 8); break;
            case 2: RMD_DAPX3(2, 8); break;
            case 3: RMD_DAPX3(3, 8); break;
            default: RMD_DAPX3(4, 8); break;
        }
#undef RMD_DAPX3
#undef RMD_DAPX3_R
        return check_launch("rmd_dap/x3");
    }
    const size_t lds = sizeof(float) * (size_t)disp * disp;
    dim3 grid((pixels + kThreads - 1) / kThreads, batch);
    if (lds <= 64 * 1024) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dap_kernel<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        dap_kernel<true><<<grid, kThreads, lds, as_stream(stream)>>>(x, weight, disp, pixels, transpose, out);
    } else {   // e.g. the 324x324 'full' DAP of raft_dicl_ml: W streamed through the scalar cache
        dap_kernel<false><<<grid, kThreads, 0, as_stream(stream)>>>(x, weight, disp, pixels, transpose, out);
    }
    return check_launch("rmd_dap");
}

extern "C" int rmd_warp_backwards(const float* img2, const float* flow, int batch, int channels, int height,
                                  int width, float eps, float* out, unsigned char* mask, void* stream) {
    RMD_REQUIRE(img2 && flow && out, RMD_ERR_ARG, "rmd_warp_backwards: null pointer");
    RMD_REQUIRE(batch > 0 && batch <= 65535 && channels > 0 && height > 0 && width > 0, RMD_ERR_SHAPE,
                "rmd_warp_backwards: bad sizes");
    const int n = height * width;
    warp_kernel<false><<<dim3((n + kThreads - 1) / kThreads, batch), kThreads, 0, as_stream(stream)>>>(
        img2, flow, channels, height, width, eps, out, mask, nullptr);
    return check_launch("rmd_warp_backwards");
}

extern "C" int rmd_warp_backwards_backward(const float* grad_out, const float* flow, int batch, int channels,
                                           int height, int width, float eps, float* grad_img2, void* stream) {
    RMD_REQUIRE(grad_out && flow && grad_img2, RMD_ERR_ARG, "rmd_warp_backwards_backward: null pointer");
    RMD_REQUIRE(batch > 0 && batch <= 65535 && channels > 0 && height > 0 && width > 0, RMD_ERR_SHAPE,
                "rmd_warp_backwards_backward: bad sizes");
    const int n = height * width;
    hipStream_t st = as_stream(stream);
    (void)hipMemsetAsync(grad_img2, 0, sizeof(float) * (size_t)batch * channels * n, st);
    warp_backward_kernel<<<dim3((n + kThreads - 1) / kThreads, batch), kThreads, 0, st>>>(
        grad_out, flow, channels, height, width, eps, grad_img2);
    return check_launch("rmd_warp_backwards_backward");
}

extern "C" size_t rmd_dicl_stack_int_warped_workspace_bytes(int batch, int channels, int height, int width) {
    if (batch < 1 || channels < 1 || height < 1 || width < 1) return 0;
    const size_t n = (size_t)height * width;
    return ((size_t)batch * channels * n * sizeof(float) + 2 * (size_t)batch * n + 255) & ~(size_t)255;
}

extern "C" int rmd_dicl_stack_int_warped(const float* fmap1, const float* fmap2, const float* flow, int batch,
                                         int channels, int height, int width, int ru, int rv, float* out,
                                         void* workspace, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && flow && out && workspace, RMD_ERR_ARG, "rmd_dicl_stack_int_warped: null pointer");
    RMD_REQUIRE(batch > 0 && batch <= 65535 && channels > 0 && height > 0 && width > 0 && ru >= 0 && rv >= 0,
                RMD_ERR_SHAPE, "rmd_dicl_stack_int_warped: bad sizes");
    RMD_REQUIRE((height * width) % 4 == 0, RMD_ERR_SHAPE, "rmd_dicl_stack_int_warped: h*w must be a multiple of 4");
    IntParams P{batch, channels, height, width, ru, rv};
    hipStream_t st = as_stream(stream);
    const int n = height * width;
    float* warped = static_cast<float*>(workspace);
    unsigned char* nz = reinterpret_cast<unsigned char*>(warped + (size_t)batch * channels * n);
    warp_kernel<true><<<dim3((n + kThreads - 1) / kThreads, batch), kThreads, 0, st>>>(
        fmap2, flow, channels, height, width, 1e-5f, warped, nullptr, nz);
    const int rc = launch_stack_int(fmap1, warped, nz, P, out, st);
    return rc ? rc : check_launch("rmd_dicl_stack_int_warped");
}

extern "C" int rmd_dicl_stack_int_warped_backward(const float* grad_mvol, const float* fmap2, const float* flow,
                                                  int batch, int channels, int height, int width, int ru, int rv,
                                                  float* grad_fmap1, float* grad_fmap2, void* workspace,
                                                  void* stream) {
    RMD_REQUIRE(grad_mvol && fmap2 && flow && grad_fmap1 && grad_fmap2 && workspace, RMD_ERR_ARG,
                "rmd_dicl_stack_int_warped_backward: null pointer");
    RMD_REQUIRE(batch > 0 && batch <= 65535 && channels > 0 && height > 0 && width > 0 && ru >= 0 && rv >= 0,
                RMD_ERR_SHAPE, "rmd_dicl_stack_int_warped_backward: bad sizes");
    IntParams P{batch, channels, height, width, ru, rv};
    hipStream_t st = as_stream(stream);
    const int n = height * width;
    float* warped = static_cast<float*>(workspace);
    unsigned char* nz = reinterpret_cast<unsigned char*>(warped + (size_t)batch * channels * n);
    const dim3 pix((n + kThreads - 1) / kThreads, batch);
    // recompute the occlusion flags; the warped map's buffer then receives d warped
    warp_kernel<true><<<pix, kThreads, 0, st>>>(fmap2, flow, channels, height, width, 1e-5f, warped, nullptr, nz);
    dicl_stack_int_backward_kernel<<<dim3((n + kThreads - 1) / kThreads, channels, batch), kThreads, 0, st>>>(
        grad_mvol, nz, P, grad_fmap1, warped);
    (void)hipMemsetAsync(grad_fmap2, 0, sizeof(float) * (size_t)batch * channels * n, st);
    warp_backward_kernel<<<pix, kThreads, 0, st>>>(warped, flow, channels, height, width, 1e-5f, grad_fmap2);
    return check_launch("rmd_dicl_stack_int_warped_backward");
}
