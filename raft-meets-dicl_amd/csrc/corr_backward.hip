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

// a (1 - f) + b f as one explicit fma over a rounded product: both G kernels (sequential and build)
// then round identically whatever the compiler's contraction choices (bit-equal G)
__device__ __forceinline__ float xlerp(float a, float b, float f) { return __builtin_fmaf(a, 1.0f - f, b * f); }

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
            for (int i = 0; i < K; ++i) q[i] = xlerp(i < D ? gr[i] : 0.f, i >= 1 ? gr[i - 1] : 0.f, fx);
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
                for (int i = 0; i < NW; ++i) wv[i] = i < K ? xlerp(qcur[i], qprev[i], fy) : 0.f;
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

// ---- G build: every lookup of a forward in one pass that writes G once -------------------------
//
// rmd_corr_grad_build replaces (zero-fill G) + (one rmd_corr_lookup_backward per lookup): 2.09 GB
// of zeros plus 12 read-modify-write passes (0.35 + 12 x 0.065 ms at cfg2 b8) become one write of G.
// One wave per segment = (image b, 64 consecutive queries, level L, kBuildSegRows target rows,
// kBuildChunks chunk columns); lane = query p.  The lanes' patch origins for every lookup are staged in
// LDS once per segment; the segment's target rows are then built kBuildRows at a time in an LDS tile
// laid out [row][slot][query] (slot = a target column of the tile, plus a trash slot at each end), so
// a lane adds its patch values at per-lane columns without bank conflicts, shifts or selects.
// Lookups go in groups of kBuildGroup: a lane whose (2r+2)^2 patch meets the tile loads its
// coordinates and the kBuildRows + 1 tap rows it needs, for the whole group in one batch of buffer
// loads (tap rows outside 0 .. 2r, and lanes / lookups that miss the tile, go to an out-of-range
// offset: zeros, no traffic); it forms the patch rows with the x-then-y bilinear arithmetic of
// corr_lookup_backward_kernel (xlerp) and adds them into the tile in lookup order.  Columns left or
// right of the tile land in the trash slots.  The wave then stores the tile — lane l writes the 16 B
// at byte 16 l of each 1-KB half of a (row, chunk)'s 2 KB, read across lanes, so every store
// instruction covers 8 whole 128-B lines, non-temporal (G is 2 GB, read next by the GEMMs) — with pad
// targets x >= W_l as 0, and clears it.  Each G element thus receives 0 + v_0 + v_1 + ... in lookup
// order: the sum the sequential kernels form, bit for bit.  ACC: a tile starts from G's current
// values (launches after the first when a forward holds more than kBuildMax lookups).
// Measured variants (profiles/grad_build_r05.json): register tiles with select-shifted accumulation,
// one unit per wave, 1-row / 4-row tiles, lookup-at-a-time loads, a producer / consumer wave pair.
#ifndef RMD_BUILD_ROWS
#define RMD_BUILD_ROWS 2
#endif
#ifndef RMD_BUILD_CHUNKS
#define RMD_BUILD_CHUNKS 4
#endif
// 1: G stores non-temporal (streamed past L2, which then keeps the grad_out / coordinate reads)
#ifndef RMD_BUILD_NT
#define RMD_BUILD_NT 1
#endif
// A/B ablations only: bit 0 sends every grad_out load out of range (no memory traffic, zeros)
#ifndef RMD_BUILD_ABL
#define RMD_BUILD_ABL 0
#endif
#ifndef RMD_BUILD_SEG
#define RMD_BUILD_SEG 8
#endif
constexpr int kBuildMax = 16, kBuildRows = RMD_BUILD_ROWS, kBuildChunks = RMD_BUILD_CHUNKS, kBuildThreads = 64;
constexpr int kBuildSegRows = RMD_BUILD_SEG * kBuildRows;     // target rows per wave (tiles in sequence)
#ifndef RMD_BUILD_GROUP
#define RMD_BUILD_GROUP 4
#endif
constexpr int kBuildGroup = RMD_BUILD_GROUP;                 // lookups per batch of loads
constexpr int kBuildSlots = 8 * kBuildChunks + 2;            // tile columns + 2 trash slots
constexpr unsigned kBuildOOB = 0x80000000u;                  // buffer offset past any slab: loads return 0

struct BuildArgs {
    const float* gout[kBuildMax];
    const float* coords[kBuildMax];
    unsigned zmask[kBuildMax];
    int n;                              // lookups in this launch (0 .. kBuildMax)
    int ufirst[RMD_MAX_LEVELS + 1];     // first unit of level l (per image and query block)
    int nct[RMD_MAX_LEVELS];            // chunk-column tiles of level l
};

// query coordinate at level L, clamped to +-30000 (beyond it no patch meets a level, H, W < 2^15;
// the sequential kernel's +-1e6 clamp differs only where neither adds anything)
__device__ __forceinline__ float build_coord(float c, float inv) { return fminf(fmaxf(c * inv, -30000.f), 30000.f); }

template <int R, bool ACC, bool BF>
__global__ void __launch_bounds__(kBuildThreads)
corr_grad_build_kernel(BuildArgs a, GradGeom g, float* __restrict__ grad) {
    static_assert(!(ACC && BF), "a bfloat16 G is written by one launch (no accumulation)");
    constexpr int D = 2 * R + 1, K = 2 * R + 2;
    constexpr int RB = kBuildRows, CB = kBuildChunks, TS = kBuildSlots, TILE = RB * TS * kBuildThreads;
    __shared__ float tile[TILE];                             // [row][slot][query]
    __shared__ int sxy[kBuildMax * kBuildThreads];           // [lookup][query] patch origin (xs | ys << 16)
    const int N = g.height * g.width;
    const int lane = threadIdx.x;
    const int p0 = blockIdx.x * kBuildThreads;
    const int pc = p0 + lane < N ? p0 + lane : N - 1;        // lanes past N compute on a valid query, store nothing
    const int b = blockIdx.y;
    int u = blockIdx.z, L = 0;
    while (L + 1 < g.levels && u >= a.ufirst[L + 1]) ++L;
    u -= a.ufirst[L];
    const int lh = g.lh[L], lw = g.lw[L], nch = g.nch[L];
    const int ys0 = (u / a.nct[L]) * kBuildSegRows, ys1 = min(lh, ys0 + kBuildSegRows);
    const int clo = (u % a.nct[L]) * CB, ncol = min(nch - clo, CB);
    const bool lok = lh >= 2 && lw >= 2;                      // 1-pixel levels: NaN in the reference, no gradient
    const float inv = 1.0f / (float)(1 << L);
    const size_t chs = (size_t)N * kGcw;                      // one chunk step
    const int ntile = (ys1 - ys0 + RB - 1) / RB;

    for (int t = lane; t < TILE; t += kBuildThreads) tile[t] = 0.f;
#pragma unroll
    for (int i = 0; i < kBuildMax; ++i) {
        if (i < a.n) {
            const float* co = a.coords[i] + (size_t)b * 2 * N + pc;
            const int xs = (int)floorf(build_coord(co[0], inv)) - R, ys = (int)floorf(build_coord(co[N], inv)) - R;
            sxy[i * kBuildThreads + lane] = (xs & 0xffff) | (ys << 16);
        }
    }

    // the segment's tiles in turn (the lookup state above serves all of them): build, store, clear
    for (int st = 0; st < ntile; ++st) {
        float* __restrict__ tb = tile;
        const int y0 = ys0 + st * RB, nr = min(ys1 - y0, RB);
        {
            if constexpr (ACC) {
                const float* col = grad + (((size_t)b * g.TC + g.coff[L]) * N + pc) * kGcw + ((size_t)y0 * nch + clo) * chs;
#pragma unroll
                for (int r = 0; r < RB; ++r)
#pragma unroll
                    for (int k = 0; k < CB; ++k) {
                        if (r >= nr || k >= ncol) continue;
                        const float4* sp = reinterpret_cast<const float4*>(col + ((size_t)r * nch + k) * chs);
                        const float4 va = sp[0], vb = sp[1];
                        const float v[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
#pragma unroll
                        for (int e = 0; e < 8; ++e) tb[(r * TS + 1 + 8 * k + e) * kBuildThreads + lane] = v[e];
                    }
            }
            const unsigned slab = (unsigned)(D * D * N) * 4u;                  // one (b, level) gout block
            // lookups in groups of BG: the tap rows and coordinates of a whole group are one batch of
            // loads (lanes / lookups that do not meet the tile load from an out-of-range offset: no
            // traffic), so a tile waits for memory once per group instead of once per lookup
            constexpr int BG = kBuildGroup;
            for (int i0 = 0; i0 < a.n; i0 += BG) {
                bool act[BG];
                int xsg[BG], j0g[BG];
                bool any = false;
#pragma unroll
                for (int q = 0; q < BG; ++q) {
                    const int i = i0 + q;
                    act[q] = false;
                    xsg[q] = j0g[q] = 0;
                    if (i < a.n) {
                        const int xy = sxy[i * kBuildThreads + lane];
                        const int xs = (int)(short)(xy & 0xffff), ys = xy >> 16;
                        const int j0 = y0 - ys;             // patch row of tile row 0
                        const int c0 = xs >> 3, nc = ((xs & 7) + K + 7) >> 3;
                        const bool on = lok && !((a.zmask[i] >> L) & 1u);
                        act[q] = on && j0 < K && j0 + nr > 0 && c0 < clo + ncol && c0 + nc > clo;
                        xsg[q] = xs;
                        j0g[q] = j0;
                        any = any || act[q];
                    }
                }
                if (!__any(any)) continue;
                float gt[BG][RB + 1][D], cxg[BG], cyg[BG];
#pragma unroll
                for (int q = 0; q < BG; ++q) {
                    const int i = i0 + q;
                    cxg[q] = cyg[q] = 0.f;
                    if (i >= a.n) continue;
                    const float* co = a.coords[i] + (size_t)b * 2 * N + pc;
                    cxg[q] = co[0];
                    cyg[q] = co[N];
                    // tap rows j0 - 1 .. j0 + RB - 1 of lookup i, rows outside 0 .. D-1 -> 0
                    const float* blk = a.gout[i] + ((size_t)b * g.levels + L) * D * D * (size_t)N;
                    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)blk);
                    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)blk >> 32));
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo), (short)0, (int)slab, 0x00020000);
#pragma unroll
                    for (int r = 0; r <= RB; ++r) {
                        const int jt = j0g[q] - 1 + r;
                        const unsigned vo = act[q] && jt >= 0 && jt < D && !(RMD_BUILD_ABL & 1)
                                                ? (unsigned)(jt * N + pc) * 4u : kBuildOOB;
#pragma unroll
                        for (int t = 0; t < D; ++t)
                            gt[q][r][t] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                rs, (int)vo, (int)__builtin_amdgcn_readfirstlane((unsigned)(t * D * N) * 4u), 0));
                    }
                }
#pragma unroll
                for (int q = 0; q < BG; ++q) {
                    if (!act[q]) continue;
                    const float cx = build_coord(cxg[q], inv), cy = build_coord(cyg[q], inv);
                    const float fx = cx - floorf(cx), fy = cy - floorf(cy);
                    const int j0 = j0g[q];
                    float qprev[K];
#pragma unroll
                    for (int t = 0; t < K; ++t)
                        qprev[t] = xlerp(t < D ? gt[q][0][t] : 0.f, t >= 1 ? gt[q][0][t - 1] : 0.f, fx);
                    const int sb = xsg[q] - 8 * clo + 1;    // tile slot of patch column 0
#pragma unroll
                    for (int r = 0; r < RB; ++r) {
                        float qcur[K];
#pragma unroll
                        for (int t = 0; t < K; ++t)
                            qcur[t] = xlerp(t < D ? gt[q][r + 1][t] : 0.f, t >= 1 ? gt[q][r + 1][t - 1] : 0.f, fx);
                        const int jr = j0 + r;              // patch row of tile row r
                        if (r < nr && jr >= 0 && jr < K) {
                            float* trow = tb + r * TS * kBuildThreads + lane;
                            float w[K];
                            int at[K];
#pragma unroll
                            for (int t = 0; t < K; ++t) {
                                at[t] = min(max(sb + t, 0), TS - 1) * kBuildThreads;
                                w[t] = trow[at[t]];
                            }
#pragma unroll
                            for (int t = 0; t < K; ++t) w[t] += xlerp(qcur[t], qprev[t], fy);
#pragma unroll
                            for (int t = 0; t < K; ++t) trow[at[t]] = w[t];
                        }
#pragma unroll
                        for (int t = 0; t < K; ++t) qprev[t] = qcur[t];
                    }
                }
            }
        }
        __syncthreads();                                    // (one wave) the tile is read across lanes below
        {
            // per (row, chunk) the 64 queries' 32-B pieces are 2 KB contiguous; lane l stores the 16 B at
            // byte 16 l of each 1-KB half (query 32 h + l / 2, slots 4 (l & 1) ..), so every store
            // instruction writes 8 whole 128-B lines; the tile is cleared for the next one on the way.
            // BF: G in bfloat16 (round to nearest even of the fp32 sums): a piece is 16 B, lane l stores
            // query l's (1 KB contiguous per row and chunk)
            typedef __attribute__((ext_vector_type(4))) float f32x4;
#pragma unroll
            for (int r = 0; r < RB; ++r)
#pragma unroll
                for (int k = 0; k < CB; ++k) {
                    if (r >= nr || k >= ncol) continue;
                    const int lim = lw - 8 * (clo + k);     // slots e < lim are on the level (pads stay 0)
                    const size_t piece = (((size_t)b * g.TC + g.coff[L] + (size_t)(y0 + r) * nch + clo + k) * N + p0);
                    if constexpr (BF) {
                        float v[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            float* at = tb + (r * TS + 1 + 8 * k + e) * kBuildThreads + lane;
                            v[e] = e < lim ? *at : 0.f;
                            *at = 0.f;
                        }
                        if (p0 + lane < N) {
                            unsigned w[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const __bf16 lo = (__bf16)v[2 * e], hi = (__bf16)v[2 * e + 1];
                                w[e] = (unsigned)__builtin_bit_cast(unsigned short, lo) |
                                       ((unsigned)__builtin_bit_cast(unsigned short, hi) << 16);
                            }
                            f32x4* d = reinterpret_cast<f32x4*>(reinterpret_cast<unsigned short*>(grad) +
                                                                (piece + lane) * kGcw);
                            const f32x4 o{__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                                          __uint_as_float(w[3])};
                            if constexpr (RMD_BUILD_NT) __builtin_nontemporal_store(o, d);
                            else *d = o;
                        }
                    } else {
                        const int e0 = 4 * (lane & 1);
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int q = 32 * h + (lane >> 1);
                            float v[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                float* at = tb + (r * TS + 1 + 8 * k + e0 + j) * kBuildThreads + q;
                                v[j] = e0 + j < lim ? *at : 0.f;
                                *at = 0.f;
                            }
                            if (p0 + q < N) {
                                f32x4* d = reinterpret_cast<f32x4*>(grad + (piece + q) * kGcw + e0);
                                if constexpr (RMD_BUILD_NT) __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, d);
                                else *d = f32x4{v[0], v[1], v[2], v[3]};
                            }
                        }
                    }
                }
        }
        __syncthreads();
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

extern "C" int rmd_corr_grad_build(const float* const* grad_outs, const float* const* coords,
                                   const unsigned* zero_level_masks, int nlookups, const rmd_pyramid_desc* d,
                                   int radius, int accumulate, float* grad_levels, void* stream) {
    return rmd_corr_grad_build_ex(grad_outs, coords, zero_level_masks, nlookups, d, radius, accumulate, 0, grad_levels,
                                  stream);
}

extern "C" int rmd_corr_grad_build_ex(const float* const* grad_outs, const float* const* coords,
                                      const unsigned* zero_level_masks, int nlookups, const rmd_pyramid_desc* d,
                                      int radius, int accumulate, int bf16_out, void* grad_levels, void* stream) {
    RMD_REQUIRE(!bf16_out || (!accumulate && nlookups <= rmd::kBuildMax), RMD_ERR_ARG,
                "rmd_corr_grad_build: a bfloat16 G takes at most %d lookups and no accumulation", rmd::kBuildMax);
    RMD_REQUIRE(d && grad_levels && nlookups >= 0 && (nlookups == 0 || (grad_outs && coords)), RMD_ERR_ARG,
                "rmd_corr_grad_build: null pointer or negative lookup count");
    RMD_REQUIRE(radius >= 1 && radius <= 8, RMD_ERR_SHAPE, "rmd_corr_grad_build: radius %d not in 1..8", radius);
    int rc = rmd::check_grad_args(d->batch, 1, d->height, d->width, d->levels);
    if (rc) return rc;
    for (int i = 0; i < nlookups; ++i)
        RMD_REQUIRE(grad_outs[i] && coords[i], RMD_ERR_ARG, "rmd_corr_grad_build: null pointer (lookup %d)", i);
    // the kernel clamps coordinates to +-30000 (patch origins in 16 bits) and addresses one (image,
    // level) block of grad_out with 32-bit buffer offsets
    RMD_REQUIRE(d->height < 16384 && d->width < 16384, RMD_ERR_SHAPE, "rmd_corr_grad_build: %dx%d map (< 16384)",
                d->height, d->width);
    RMD_REQUIRE((long long)(2 * radius + 1) * (2 * radius + 1) * d->height * d->width * 4 < (1LL << 31), RMD_ERR_SHAPE,
                "rmd_corr_grad_build: grad_out level block >= 2 GiB");
    const rmd::GradGeom g = rmd::make_grad_geom(d->batch, d->height, d->width, d->levels);
    const int N = d->height * d->width;
    rmd::BuildArgs a{};
    int units = 0;
    for (int l = 0; l < d->levels; ++l) {
        a.ufirst[l] = units;
        a.nct[l] = (g.nch[l] + rmd::kBuildChunks - 1) / rmd::kBuildChunks;
        units += (g.lh[l] + rmd::kBuildSegRows - 1) / rmd::kBuildSegRows * a.nct[l];
    }
    a.ufirst[d->levels] = units;
    RMD_REQUIRE(units <= 65535 && d->batch <= 65535, RMD_ERR_SHAPE, "rmd_corr_grad_build: %d units x %d images",
                units, d->batch);
    const dim3 grid((N + rmd::kBuildThreads - 1) / rmd::kBuildThreads, d->batch, units);
    hipStream_t st = rmd::as_stream(stream);
    float* gl = static_cast<float*>(grad_levels);
    // one launch per kBuildMax lookups; after the first, each launch adds to G in lookup order
    for (int i0 = 0; i0 < nlookups || (i0 == 0 && !accumulate); i0 += rmd::kBuildMax) {
        a.n = nlookups - i0 < rmd::kBuildMax ? nlookups - i0 : rmd::kBuildMax;
        for (int i = 0; i < a.n; ++i) {
            a.gout[i] = grad_outs[i0 + i];
            a.coords[i] = coords[i0 + i];
            a.zmask[i] = zero_level_masks ? zero_level_masks[i0 + i] : 0u;
        }
        const bool acc = accumulate || i0 > 0;
        switch (radius) {
#define RMD_CASE(RR)                                                                                              \
    case RR:                                                                                                      \
        if (acc) rmd::corr_grad_build_kernel<RR, true, false><<<grid, rmd::kBuildThreads, 0, st>>>(a, g, gl);      \
        else if (bf16_out) rmd::corr_grad_build_kernel<RR, false, true><<<grid, rmd::kBuildThreads, 0, st>>>(a, g, gl); \
        else rmd::corr_grad_build_kernel<RR, false, false><<<grid, rmd::kBuildThreads, 0, st>>>(a, g, gl);        \
        break;
            RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4) RMD_CASE(5) RMD_CASE(6) RMD_CASE(7) RMD_CASE(8)
#undef RMD_CASE
        }
        rc = rmd::check_launch("rmd_corr_grad_build");
        if (rc != RMD_OK) return rc;
        if (nlookups == 0) break;
    }
    return RMD_OK;
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

