// corr_backward.hip — gradients of the RAFT correlation pyramid and its windowed lookup.
//
// Replaces the autograd of raft.CorrBlock (qzed/raft-meets-dicl src/models/impls/raft.py:18-95):
// grid_sampler_2d_backward of the lookup (:80; coordinates are detached at raft.py:402, so only the
// volume receives a gradient), avg_pool2d_backward of the pyramid (:45) and the bmm transposes of
// the all-pairs product (:30-33).
//
// Decomposition (backward):
//   level l of the pyramid equals fmap1 . P_l with P_l = avg-pooled fmap2 / sqrt(C) (the pooling
//   commutes with the product), so with G_l = dL/d(level l):
//     dfmap1[p]  = sum_l sum_t G_l[p, t] P_l[t]                         (GEMM, K = sum_l T_l)
//     dP_l[t]    = sum_p G_l[p, t] fmap1[p]                              (GEMM, K = N)
//     dfmap2     = sum_l unpool_l(dP_l) / sqrt(C)                        (this file)
//   G (all levels, all lookups of a forward) is accumulated densely in float32 in the forward
//   pyramid's chunked query-minor order with 8-target chunks: target row (l, y) is cut into
//   ceil(W_l / 8) chunks, chunk index ch = coff(l) + y * ceil(W_l / 8) + x / 8 over all levels, and
//   element (b, t, p) sits at ((b * TC + ch) * N + p) * 8 + x % 8.  As a matrix over the padded
//   targets t' = 8 ch + x % 8 (T' = 8 TC, pad columns stay zero) both GEMMs read it with 8-element
//   blocked operand layouts (rmd_corr_grad_gemm layouts 2 / 3), so no transpose pass is needed.
//   rmd_corr_lookup_backward: lanes are consecutive queries; at a tap, query p + 1's target is one
//   column right of query p's (smooth flow), so in the chunked order 8 neighbouring lanes touch
//   3 128-B lines (36-B lane stride) instead of 8 lines of the plain (B, T, N) order (N + 1 floats
//   apart).  Each lane owns column (b, p) of G for its level: it spreads the (2r+1)^2 tap gradients
//   over its (2r+2)^2 integer patch with the forward's bilinear weights (separable: x then y) and
//   read-modify-writes the patch — no atomics: the patch rows are split over 3 lanes (parts) that
//   write disjoint rows, no other lane touches column p, and successive lookups are ordered by the
//   stream.  Since the lane owns every (chunk, p) piece its rows touch, it reads, adds to and writes
//   whole 32-B pieces as two 16-B vectors (the row's values barrel-shifted to their slots): 77 vs 143 us
//   per cfg2 b8 lookup backward for one float per target (profiles/raft_bwd_vec_ab_r04.json).

#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 256;

constexpr int kGcw = 8;                // targets per G chunk
// lookup backward: 1 = read-modify-write whole 32-B chunk pieces as 16-B vectors, 0 = one float per target
#ifndef RMD_BWD_VEC
#define RMD_BWD_VEC 1
#endif

struct GradGeom {
    int batch, height, width, levels;
    int lh[RMD_MAX_LEVELS], lw[RMD_MAX_LEVELS];
    int nch[RMD_MAX_LEVELS];          // chunks per target row of level l: ceil(W_l / 8)
    long long coff[RMD_MAX_LEVELS];   // first chunk of level l
    long long TC;                     // chunks per image (all levels); T' = 8 TC padded targets
};

inline GradGeom make_grad_geom(int batch, int h, int w, int levels) {
    GradGeom g{};
    g.batch = batch;
    g.height = h;
    g.width = w;
    g.levels = levels;
    long long c = 0;
    for (int l = 0; l < levels; ++l) {
        g.lh[l] = h >> l;
        g.lw[l] = w >> l;
        g.nch[l] = (g.lw[l] + kGcw - 1) / kGcw;
        g.coff[l] = c;
        c += (long long)g.lh[l] * g.nch[l];
    }
    g.TC = c;
    return g;
}

// grid: (query blocks of 64, batch, level + levels * part); one lane per (query, level, part), part k
// producing patch rows [k*PR, min(K, (k+1)*PR)) from tap rows k*PR - 1 .. (k+1)*PR - 1
constexpr int kBwdThreads = 64, kBwdParts = 3;

template <int R>
__global__ void __launch_bounds__(kBwdThreads)
corr_lookup_backward_kernel(const float* __restrict__ gout, GradGeom g, const float* __restrict__ coords,
                            unsigned zmask, float* __restrict__ grad) {
    constexpr int D = 2 * R + 1, K = 2 * R + 2, PR = (K + kBwdParts - 1) / kBwdParts;
    const int N = g.height * g.width;
    const int p = blockIdx.x * kBwdThreads + threadIdx.x;
    const int b = blockIdx.y;
    const int L = (int)blockIdx.z % g.levels, part = (int)blockIdx.z / g.levels;
    if (p >= N) return;
    if ((zmask >> L) & 1u) return;                       // zeroed level (raft.py:86-87): no gradient
    const int lh = g.lh[L], lw = g.lw[L];
    if (lh < 2 || lw < 2) return;                        // NaN level of the reference: no gradient
    const float inv = 1.0f / (float)(1 << L);
    float cx = coords[((size_t)b * 2 + 0) * N + p] * inv;
    float cy = coords[((size_t)b * 2 + 1) * N + p] * inv;
    cx = fminf(fmaxf(cx, -1.0e6f), 1.0e6f);
    cy = fminf(fmaxf(cy, -1.0e6f), 1.0e6f);
    const float fx0 = floorf(cx), fy0 = floorf(cy);
    const float fx = cx - fx0, fy = cy - fy0;
    const int xs = (int)fx0 - R, ys = (int)fy0 - R;

    const float* go = gout + ((size_t)b * g.levels + L) * D * D * (size_t)N + p;
    // G element (y, x) of this lane: chunk coff + y nch + x / 8, query p, slot x % 8
    float* col = grad + (((size_t)b * g.TC + g.coff[L]) * N + p) * kGcw;
    const size_t chs = (size_t)N * kGcw;                                       // one chunk step

    // x pass of tap row j: Q[j][i] = g[i][j](1-fx) + g[i-1][j] fx, i = 0..K-1 (zero for j outside 0..D-1)
    auto qrow = [&](int j, float (&q)[K]) {
        if (j >= 0 && j < D) {
            float gr[D];
#pragma unroll
            for (int a = 0; a < D; ++a) gr[a] = go[(size_t)(a * D + j) * N];   // channel a*D + j
#pragma unroll
            for (int i = 0; i < K; ++i) q[i] = (i < D ? gr[i] * (1.0f - fx) : 0.f) + (i >= 1 ? gr[i - 1] * fx : 0.f);
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) q[i] = 0.f;
        }
    };
    // y pass: patch row j = Q[j](1-fy) + Q[j-1] fy
    const int j0 = part * PR, j1 = min(K, j0 + PR);
    float qprev[K];
    qrow(j0 - 1, qprev);
#pragma unroll
    for (int jj = 0; jj < PR; ++jj) {
        const int j = j0 + jj;
        if (j >= j1) break;
        float qcur[K];
        qrow(j, qcur);
        const int y = ys + j;
        if (y >= 0 && y < lh) {
            float* r = col + (size_t)y * g.nch[L] * chs;
            if constexpr (RMD_BWD_VEC) {
                // whole 32-B chunk pieces: the row's K values shifted to their in-chunk slots (a 3-stage
                // barrel shift by xs mod 8), then each chunk the row touches read, added to and written as
                // two 16-B vectors (the lane owns (chunk, query) for this launch: no other lane writes it);
                // slots outside the window or past the level's width add 0
                constexpr int NC = (K + 14) / 8, NW = 8 * NC;
                float wv[NW];
#pragma unroll
                for (int i = 0; i < NW; ++i) wv[i] = i < K ? qcur[i] * (1.0f - fy) + qprev[i] * fy : 0.f;
                const int sh = xs & 7;
#pragma unroll
                for (int st = 1; st < 8; st <<= 1) {
                    const bool on = (sh & st) != 0;
#pragma unroll
                    for (int i = NW - 1; i >= 0; --i) wv[i] = on ? (i >= st ? wv[i - st] : 0.f) : wv[i];
                }
                const int c0 = xs >> 3, nch = g.nch[L];
                const int nc = (sh + K + 7) >> 3;                       // chunks this row spans (2 or 3 at r = 4)
#pragma unroll
                for (int k = 0; k < NC; ++k) {
                    const int c = c0 + k;
                    if (k >= nc || c < 0 || c >= nch) continue;
                    float4* pc = reinterpret_cast<float4*>(r + (size_t)c * chs);
                    float4 a = pc[0], b = pc[1];
                    const int lim = lw - 8 * c;                         // slots e < lim are on the level
                    a.x += 0 < lim ? wv[8 * k + 0] : 0.f;
                    a.y += 1 < lim ? wv[8 * k + 1] : 0.f;
                    a.z += 2 < lim ? wv[8 * k + 2] : 0.f;
                    a.w += 3 < lim ? wv[8 * k + 3] : 0.f;
                    b.x += 4 < lim ? wv[8 * k + 4] : 0.f;
                    b.y += 5 < lim ? wv[8 * k + 5] : 0.f;
                    b.z += 6 < lim ? wv[8 * k + 6] : 0.f;
                    b.w += 7 < lim ? wv[8 * k + 7] : 0.f;
                    pc[0] = a;
                    pc[1] = b;
                }
            } else {
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const int x = xs + i;
                    if (x >= 0 && x < lw) r[(size_t)(x >> 3) * chs + (x & 7)] += qcur[i] * (1.0f - fy) + qprev[i] * fy;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < K; ++i) qprev[i] = qcur[i];
    }
}

// P (B, C, T') = avg-pooled fmap2 * scale, all levels, in G's padded target order t' = 8 ch + x % 8
// (pad targets x >= W_l are 0), one launch per level: level 0 is fmap2 * scale, level l the 2x2
// average of level l - 1 in P (avg_pool2d(k=2, s=2) of the previous level, raft.py:45-46, floor
// sizes: every 2x2 window of level l - 1 exists).  grid (level-l padded targets / 256, B * C): one
// thread per (b, c, target), x fastest within a chunk row (a wave reads and writes contiguous runs;
// 32-bit index math only).
__global__ void __launch_bounds__(kThreads)
pool_targets_kernel(const float* __restrict__ f, GradGeom g, int l, float scale, float* __restrict__ P) {
    const int per = g.lh[l] * g.nch[l] * kGcw;                    // padded targets of level l
    const int tl = blockIdx.x * kThreads + threadIdx.x;
    if (tl >= per) return;
    const size_t bc = blockIdx.y;
    const int rowp = g.nch[l] * kGcw;
    const int y = tl / rowp, x = tl - y * rowp;
    const size_t Tp = (size_t)g.TC * kGcw;
    float v = 0.f;
    if (x < g.lw[l]) {
        if (l == 0) {
            v = f[bc * g.height * g.width + (size_t)y * g.width + x] * scale;
        } else {
            const float* q = P + bc * Tp;
            const int pl = l - 1, np = g.nch[pl];
            auto at = [&](int yy, int xx) {
                return q[(size_t)(g.coff[pl] + (long long)yy * np + (xx >> 3)) * kGcw + (xx & 7)];
            };
            v = (at(2 * y, 2 * x) + at(2 * y, 2 * x + 1) + at(2 * y + 1, 2 * x) + at(2 * y + 1, 2 * x + 1)) * 0.25f;
        }
    }
    P[bc * Tp + (size_t)g.coff[l] * kGcw + tl] = v;
}

// dfmap2 (B, C, H, W) = sum_l unpool_l(dP_l) * scale / 4^l, dP (B, C, T') in G's padded target order.
// grid (H W / 256, B * C): one thread per output element, 32-bit index math only.
__global__ void __launch_bounds__(kThreads)
unpool_targets_kernel(const float* __restrict__ dP, GradGeom g, float scale, float* __restrict__ df) {
    const int HW = g.height * g.width;
    const int px = blockIdx.x * kThreads + threadIdx.x;
    if (px >= HW) return;
    const size_t bc = blockIdx.y;
    const int y = px / g.width, x = px - y * g.width;
    const float* base = dP + bc * (size_t)g.TC * kGcw;
    float acc = 0.f;
#pragma unroll
    for (int l = 0; l < RMD_MAX_LEVELS; ++l) {
        if (l >= g.levels) break;
        const int yl = y >> l, xl = x >> l;
        if (yl < g.lh[l] && xl < g.lw[l])
            acc += base[(size_t)(g.coff[l] + (long long)yl * g.nch[l] + (xl >> 3)) * kGcw + (xl & 7)] *
                   (1.0f / (float)(1 << (2 * l)));
    }
    df[bc * HW + px] = acc * scale;
}

int check_grad_args(int batch, int channels, int h, int w, int levels) {
    RMD_REQUIRE(batch >= 1 && channels >= 1 && h >= 1 && w >= 1, RMD_ERR_SHAPE, "rmd corr backward: bad sizes");
    RMD_REQUIRE(levels >= 1 && levels <= RMD_MAX_LEVELS, RMD_ERR_SHAPE, "rmd corr backward: bad levels");
    RMD_REQUIRE((h >> (levels - 1)) >= 1 && (w >> (levels - 1)) >= 1, RMD_ERR_SHAPE,
                "rmd corr backward: level %d of a %dx%d map is empty", levels - 1, h, w);
    return RMD_OK;
}

}  // namespace
}  // namespace rmd

extern "C" long long rmd_corr_grad_targets(int height, int width, int levels) {
    if (height < 1 || width < 1 || levels < 1 || levels > RMD_MAX_LEVELS) return -1;
    return rmd::make_grad_geom(1, height, width, levels).TC * rmd::kGcw;
}

extern "C" int rmd_corr_lookup_backward(const float* grad_out, const rmd_pyramid_desc* d, const float* coords,
                                        int radius, unsigned zero_level_mask, float* grad_levels, void* stream) {
    RMD_REQUIRE(grad_out && d && coords && grad_levels, RMD_ERR_ARG, "rmd_corr_lookup_backward: null pointer");
    int rc = rmd::check_grad_args(d->batch, 1, d->height, d->width, d->levels);
    if (rc) return rc;
    const rmd::GradGeom g = rmd::make_grad_geom(d->batch, d->height, d->width, d->levels);
    const int N = d->height * d->width;
    dim3 grid((N + rmd::kBwdThreads - 1) / rmd::kBwdThreads, d->batch, d->levels * rmd::kBwdParts);
    hipStream_t st = rmd::as_stream(stream);
    switch (radius) {
#define RMD_CASE(RR) \
    case RR: rmd::corr_lookup_backward_kernel<RR><<<grid, rmd::kBwdThreads, 0, st>>>(grad_out, g, coords, zero_level_mask, grad_levels); break;
        RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4) RMD_CASE(5) RMD_CASE(6) RMD_CASE(7) RMD_CASE(8)
#undef RMD_CASE
        default:
            rmd::set_error("rmd_corr_lookup_backward: radius %d not in 1..8", radius);
            return RMD_ERR_SHAPE;
    }
    return rmd::check_launch("rmd_corr_lookup_backward");
}

extern "C" int rmd_corr_pool_targets(const float* fmap2, int batch, int channels, int height, int width, int levels,
                                     float scale, float* pooled, void* stream) {
    RMD_REQUIRE(fmap2 && pooled, RMD_ERR_ARG, "rmd_corr_pool_targets: null pointer");
    int rc = rmd::check_grad_args(batch, channels, height, width, levels);
    if (rc) return rc;
    const rmd::GradGeom g = rmd::make_grad_geom(batch, height, width, levels);
    RMD_REQUIRE((long long)batch * channels <= 65535, RMD_ERR_SHAPE, "rmd_corr_pool_targets: batch * channels > 65535");
    for (int l = 0; l < levels; ++l) {          // level l reads level l - 1 (same stream: ordered)
        const int per = g.lh[l] * g.nch[l] * rmd::kGcw;
        const dim3 grid((per + rmd::kThreads - 1) / rmd::kThreads, batch * channels);
        rmd::pool_targets_kernel<<<grid, rmd::kThreads, 0, rmd::as_stream(stream)>>>(fmap2, g, l, scale, pooled);
    }
    return rmd::check_launch("rmd_corr_pool_targets");
}

extern "C" int rmd_corr_unpool_targets(const float* grad_pooled, int batch, int channels, int height, int width,
                                       int levels, float scale, float* grad_fmap2, void* stream) {
    RMD_REQUIRE(grad_pooled && grad_fmap2, RMD_ERR_ARG, "rmd_corr_unpool_targets: null pointer");
    int rc = rmd::check_grad_args(batch, channels, height, width, levels);
    if (rc) return rc;
    const rmd::GradGeom g = rmd::make_grad_geom(batch, height, width, levels);
    RMD_REQUIRE((long long)batch * channels <= 65535, RMD_ERR_SHAPE, "rmd_corr_unpool_targets: batch * channels > 65535");
    const dim3 grid((height * width + rmd::kThreads - 1) / rmd::kThreads, batch * channels);
    rmd::unpool_targets_kernel<<<grid, rmd::kThreads, 0, rmd::as_stream(stream)>>>(grad_pooled, g, scale, grad_fmap2);
    return rmd::check_launch("rmd_corr_unpool_targets");
}

