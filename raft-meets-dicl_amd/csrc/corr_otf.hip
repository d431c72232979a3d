// corr_otf.hip — on-the-fly windowed correlation lookup: no all-pairs volume in HBM.
//
// Replaces raft_fs.CorrBlock (qzed/raft-meets-dicl src/models/impls/raft_fs.py:13-87) — pooled
// fmap2 levels sampled on the (2r+1)^2 window of each query and dotted with fmap1, no 1/sqrt(C) —
// and, with one level and scale 1/sqrt(C), the window dot of corr/dot.py:25-57.  SURVEY.md §8(f)
// rank 1: memory O(B*C*N) instead of O(B*N^2).
//
// Operand layout (rmd_corr_otf_prepare): every map row is cut into segments of 16 pixels; a segment
// holds Cp channels of its 16 pixels as Cp/LSC load steps of exactly the 1 KiB one wave-instruction
// loads (16 B per lane), already in the lane order of the 16x16 MFMA operand (lane = 16*g + pixel):
//   bf16  16x16x32: lane (g, i) holds channels 32*ls + 8*g + e, e < 8           (one MFMA per step)
//   f32   16x16x4 : lane (g, i) holds channels 16*ls + 4*m + g, m < 4           (four MFMAs per step)
// so operand loads are whole 128-B lines (the row-per-lane gather of a pixel-major layout touches 32
// lines per instruction and halves the L1 rate).  Query rows (fmap1 * scale) use the same layout.
// compute RMD_BF16X3 (the fp32 precision mode) stores every value as a split bf16 pair v = hi + lo
// (hi = bf16(v), lo = bf16(v - hi)): each bf16 load step is followed by its lo step, and a task
// accumulates lo.hi + hi.lo + hi.hi with the 16x16x32 bf16 MFMA (the dropped lo.lo term is ~2^-16
// relative; same split as the fp32-mode GEMM), in the workspace bytes of f32 operands.  RMD_F32 keeps
// the exact f32 MFMA (fp32-exact).
//
// Lookup: one 256-thread block per (16 x 2 query block, batch), looping over the levels.  The 32 queries' (2r+2)^2
// integer patches at level l are bounded by one box (clipped to the map, widened to whole segments),
// processed in bands of whole rows of at most kMaxT targets: S = band targets x queries, one 16x16
// MFMA tile per (target segment, query segment), into LDS.  Each (query, x-offset) thread keeps its
// window rows x-interpolated in registers across bands and finally y-interpolates exactly as
// rmd_corr_lookup does (shared bilinear weights, zero padding per tap, NaN for 1-pixel levels, zeroed
// masked levels).  A box wider than kMaxT (flow differing by hundreds of pixels inside one block)
// takes a per-query VALU patch path.
#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 256;                        // prepare kernels
constexpr int kLookThreads = 256, kWaves = kLookThreads / 64;
constexpr int kBX = 16, kBY = 2, kQ = kBX * kBY;     // query block = 2 query segments
#ifndef RMD_OTF_MAXT
#define RMD_OTF_MAXT 384
#endif
constexpr int kMaxT = RMD_OTF_MAXT;                  // targets of one band
constexpr int kLd = kMaxT + 5;                       // S row stride (spreads queries over banks)
// diagnostic variant (RMD_OTF_PF=1): the next band task's target fragments in flight during this task's
// MFMAs; needs 256 VGPRs (2 waves/SIMD, spills) and measured slower: 123 vs 100 us at cfg2 bf16
// (profiles/otf_ablate_r02.json)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <typename T> struct Seg;
template <> struct Seg<__bf16> {
    static constexpr int LE = 8, LSC = 32;           // elements per lane, channels per load step
    typedef bf16x8 frag;
    static __device__ __forceinline__ void mma(f32x4& acc, const frag& a, const frag& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
    // (lane, element) of channel c within a load step
    static __host__ __device__ constexpr int lane_g(int c) { return (c >> 3) & 3; }
    static __host__ __device__ constexpr int elem(int c) { return c & 7; }
};
template <> struct Seg<float> {
    static constexpr int LE = 4, LSC = 16;
    typedef f32x4 frag;
    static __device__ __forceinline__ void mma(f32x4& acc, const frag& a, const frag& b) {
#pragma unroll
        for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], b[m], acc, 0, 0, 0);
    }
    static __host__ __device__ constexpr int lane_g(int c) { return c & 3; }
    static __host__ __device__ constexpr int elem(int c) { return (c >> 2) & 3; }
};

struct OtfGeom {
    int B, C, Cp, H, W, L;
    int lh[RMD_MAX_LEVELS], lw[RMD_MAX_LEVELS], nsx[RMD_MAX_LEVELS];
    long long soff[RMD_MAX_LEVELS], TS;               // target segments: level offsets, per batch
    int qnsx;
    long long QS;                                     // query segments per batch
};

// operand channel padding: one of the compiled channel counts, else a multiple of 128
int otf_cp(int C) {
    for (int c : {32, 64, 128, 256})
        if (C <= c) return c;
    return (C + 127) / 128 * 128;
}

OtfGeom make_otf_geom(int B, int C, int H, int W, int L) {
    OtfGeom g{};
    g.B = B;
    g.C = C;
    g.Cp = otf_cp(C);
    g.H = H;
    g.W = W;
    g.L = L;
    long long s = 0;
    for (int l = 0; l < L; ++l) {
        g.lh[l] = H >> l;
        g.lw[l] = W >> l;
        g.nsx[l] = (g.lw[l] + 15) / 16;
        g.soff[l] = s;
        s += (long long)g.lh[l] * g.nsx[l];
    }
    g.TS = s;
    g.qnsx = (W + 15) / 16;
    g.QS = (long long)H * g.qnsx;
    return g;
}

// workspace: query segments (B, QS) | target segments (B, TS) | f32 scratch of levels 1.. (B, C, lh, lw)
size_t otf_query_elems(const OtfGeom& g) { return (size_t)g.B * g.QS * 16 * g.Cp; }
size_t otf_scratch_elems(const OtfGeom& g) {
    size_t n = 0;
    for (int l = 1; l < g.L; ++l) n += (size_t)g.B * g.C * g.lh[l] * g.lw[l];
    return n;
}
size_t otf_scratch_offset(const OtfGeom& g, size_t es) {
    return ((size_t)g.B * (g.QS + g.TS) * 16 * g.Cp * es + 255) / 256 * 256;
}

// Level l of fmap2 as the reference builds it (raft_fs.py:27-30): F.avg_pool2d(k=2, s=2) of level l-1.
// src / dst are (B, C, h, w) / (B, C, h/2, w/2) float32; one thread per output element.
__global__ void __launch_bounds__(kThreads)
otf_pool2_kernel(const float* __restrict__ src, int BC, int h, int w, float* __restrict__ dst) {
    const int h2 = h >> 1, w2 = w >> 1;
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= (long long)BC * h2 * w2) return;
    const int x = (int)(idx % w2);
    const long long r = idx / w2;
    const int y = (int)(r % h2);
    const long long bc = r / h2;
    const float* p = src + (size_t)bc * h * w + (size_t)(2 * y) * w + 2 * x;
    dst[idx] = (p[0] + p[1] + p[w] + p[w + 1]) * 0.25f;
}

struct LevelSrc {
    const float* p[RMD_MAX_LEVELS];      // (B, C, lh, lw) float32 per level
};

// Segment operands: one thread per 16-B lane chunk (segment, load step, lane); a wave writes one
// contiguous 1-KiB load step, its reads run along x within each channel.
// levels = 1 and scale = s give the query operand (fmap1 * s).
template <typename T, bool X3>
__global__ void __launch_bounds__(kThreads)
otf_segments_kernel(LevelSrc src, OtfGeom g, float scale, T* __restrict__ seg) {
    static_assert(!X3 || sizeof(T) == 2, "split pairs are bf16");
    using S = Seg<T>;
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    const int nls = g.Cp / S::LSC;
    const long long total = (long long)g.B * g.TS * nls * 64;
    if (idx >= total) return;
    const int lane = (int)(idx & 63), gq = lane >> 4, i = lane & 15;
    const long long r = idx >> 6;
    const int ls = (int)(r % nls);
    const long long bs = r / nls;
    const long long s = bs % g.TS;
    const int b = (int)(bs / g.TS);
    int l = 0;
#pragma unroll
    for (int k = 1; k < RMD_MAX_LEVELS; ++k)
        if (k < g.L && s >= g.soff[k]) l = k;
    const int sl = (int)(s - g.soff[l]);
    const int y = sl / g.nsx[l], x = (sl - y * g.nsx[l]) * 16 + i;
    const size_t plane = (size_t)g.lh[l] * g.lw[l];
    const float* base = src.p[l] + (size_t)b * g.C * plane + (size_t)y * g.lw[l] + x;
    typedef __attribute__((ext_vector_type(S::LE))) T frag_t;
    frag_t v, vl;
#pragma unroll
    for (int e = 0; e < S::LE; ++e) {
        // channel of element e of lane group gq (inverse of Seg::lane_g / Seg::elem)
        const int c = S::LE == 8 ? ls * 32 + gq * 8 + e : ls * 16 + 4 * e + gq;
        const float f = x < g.lw[l] && c < g.C ? base[(size_t)c * plane] * scale : 0.f;
        v[e] = (T)f;
        if constexpr (X3) vl[e] = (T)(f - (float)v[e]);
    }
    if constexpr (X3) {
        // load step (r, hi) then (r, lo): r = idx >> 6 counts (segment, step) pairs
        T* o = seg + ((size_t)(idx >> 6) * 128 + lane) * S::LE;
        *reinterpret_cast<frag_t*>(o) = v;
        *reinterpret_cast<frag_t*>(o + 64 * S::LE) = vl;
    } else {
        (void)vl;
        *reinterpret_cast<frag_t*>(seg + (size_t)idx * S::LE) = v;
    }
}

// element (pixel i of segment, channel c) of a segment operand (X3: hi + lo)
template <typename T, bool X3>
__device__ __forceinline__ float seg_elem(const T* segbase, int i, int c) {
    using S = Seg<T>;
    constexpr int NP = X3 ? 2 : 1;
    const T* p = segbase + (c / S::LSC) * NP * 64 * S::LE + (S::lane_g(c) * 16 + i) * S::LE + S::elem(c);
    if constexpr (X3) return (float)p[0] + (float)p[64 * S::LE];
    return (float)p[0];
}

// one 16x16 tile's products of one load step: t / q point at the step's fragment(s)
template <typename T, bool X3>
__device__ __forceinline__ void seg_mma(f32x4& acc, const typename Seg<T>::frag* t, const typename Seg<T>::frag* q) {
    if constexpr (X3) {
        Seg<T>::mma(acc, t[1], q[0]);        // lo.hi, hi.lo first, hi.hi last
        Seg<T>::mma(acc, t[0], q[1]);
        Seg<T>::mma(acc, t[0], q[0]);
    } else {
        Seg<T>::mma(acc, t[0], q[0]);
    }
}

// 1-D grid over (batch, query block), XCD-aware: adjacent query blocks, whose target boxes overlap,
// run on the same XCD and share its L2.  One block runs every level of its 32 queries, so the query
// staging, the coords load and the block's fixed start-up cost are paid once, not once per level.
// CPT = compiled Cp (0: runtime multiple of 128).
template <typename T, bool X3, int R, int CPT, bool PF>
__global__ void __launch_bounds__(kLookThreads, PF ? 2 : 1)
otf_lookup_kernel(const T* __restrict__ qseg, const T* __restrict__ tseg, OtfGeom g,
                  const float* __restrict__ coords, unsigned zmask, float* __restrict__ out, int ablate) {
    using SG = Seg<T>;
    using frag = typename SG::frag;
    constexpr int D = 2 * R + 1, K = 2 * R + 2, KK = K * K;
    extern __shared__ float S[];                       // [kQ][kLd]: band (boxed) or patch (per query)
    // every level's window origins / fractions and the block's bounding box per level, computed once
    // before the level loop (no per-level reduction barriers)
    __shared__ int box[RMD_MAX_LEVELS][4];             // x0, x1, y0, y1 (min / max)
    __shared__ int sxs[RMD_MAX_LEVELS][kQ], sys[RMD_MAX_LEVELS][kQ];
    __shared__ float sfx[RMD_MAX_LEVELS][kQ], sfy[RMD_MAX_LEVELS][kQ];
    const int nbx = (g.W + kBX - 1) / kBX, nqb = nbx * ((g.H + kBY - 1) / kBY);
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int qb = lid % nqb, b = lid / nqb;
    const int qx0 = (qb % nbx) * kBX, qy0 = (qb / nbx) * kBY;
    const int N = g.H * g.W;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int NP = X3 ? 2 : 1;                      // load steps per channel step (X3: hi, lo)
    const int cp = CPT > 0 ? CPT : g.Cp;
    const int nls = cp / SG::LSC;
    const size_t segsz = (size_t)16 * cp * NP;
    const T* qsb = qseg + ((size_t)b * g.QS + (size_t)qy0 * g.qnsx + (qx0 >> 4)) * segsz;
    const T* qsb1 = qseg + ((size_t)b * g.QS + (size_t)min(qy0 + 1, g.H - 1) * g.qnsx + (qx0 >> 4)) * segsz;

    // the block's two query segments (CPT > 0): one coalesced copy into LDS, overlapping the coords
    // load; each wave then keeps its register fragments for every level and target segment
    constexpr int NLS = CPT > 0 ? CPT / SG::LSC * NP : 1;                 // load steps per segment
    constexpr int QV = CPT > 0 ? 16 * CPT * NP * (int)sizeof(T) / 16 : 0;     // 16-B vectors per segment
    static_assert(2 * QV * 16 <= kQ * kLd * 4, "two query segments must fit the S buffer");
    if constexpr (CPT > 0) {
        const uint4* s0 = reinterpret_cast<const uint4*>(qsb);
        const uint4* s1 = reinterpret_cast<const uint4*>(qsb1);
        uint4* dst = reinterpret_cast<uint4*>(S);
        for (int v = tid; v < QV; v += kLookThreads) {
            dst[v] = s0[v];
            dst[QV + v] = s1[v];
        }
    }
    // thread (level tid / kQ, query tid % kQ)
    float cx0 = 0.f, cy0 = 0.f;
    if (tid < kQ * g.L) {
        const int q = tid % kQ;
        const int y = min(qy0 + q / kBX, g.H - 1), x = min(qx0 + q % kBX, g.W - 1);
        cx0 = coords[((size_t)b * 2 + 0) * N + y * g.W + x];
        cy0 = coords[((size_t)b * 2 + 1) * N + y * g.W + x];
    }
    static_assert(kQ * RMD_MAX_LEVELS <= kLookThreads, "one thread per (level, query)");
    if (tid < RMD_MAX_LEVELS * 4) box[tid >> 2][tid & 3] = (tid & 1) ? -(1 << 30) : (1 << 30);
    __syncthreads();
    frag q0[NLS], q1[NLS];
    if constexpr (CPT > 0) {
        const frag* qs = reinterpret_cast<const frag*>(S);
#pragma unroll
        for (int ls = 0; ls < NLS; ++ls) {
            q0[ls] = qs[ls * 64 + lane];
            q1[ls] = qs[(NLS + ls) * 64 + lane];
        }
    }
    if (tid < kQ * g.L) {
        // query's window origin at level L (coords clamped as rmd_corr_lookup does)
        const int q = tid % kQ, L = tid / kQ;
        const float inv = 1.0f / (float)(1 << L);
        const float rx = cx0 * inv, ry = cy0 * inv;
        const float cx = fminf(fmaxf(rx, -1.0e6f), 1.0e6f);
        const float cy = fminf(fmaxf(ry, -1.0e6f), 1.0e6f);
        const float fx0 = floorf(cx), fy0 = floorf(cy);
        const int xs = (int)fx0 - R, ys = (int)fy0 - R;
        sxs[L][q] = xs;
        sys[L][q] = ys;
        sfx[L][q] = rx - floorf(rx);                // NaN / inf coordinate -> NaN window (grid_sample)
        sfy[L][q] = ry - floorf(ry);
        atomicMin(&box[L][0], xs);
        atomicMax(&box[L][1], xs + K - 1);
        atomicMin(&box[L][2], ys);
        atomicMax(&box[L][3], ys + K - 1);
    }
    __syncthreads();                                   // boxes complete; the query fragments are read: S is free
    // thread items (q, a): query q, window x-offset a; hx[i][jj] = row jj of the window, x-interpolated
    constexpr int ITEMS = (kQ * D + kLookThreads - 1) / kLookThreads;

    for (int L = 0; L < g.L; ++L) {
        const int lh = g.lh[L], lw = g.lw[L];
        float* ob = out + ((size_t)b * g.L + L) * D * D * (size_t)N;
        // masked / degenerate level: constant output (raft_fs.py:77-78; 1-pixel levels divide by zero)
        const bool masked = (zmask >> L) & 1u;
        if (masked || lh < 2 || lw < 2) {
            const float v = masked ? 0.f : __builtin_nanf("");
            for (int idx = tid; idx < kQ * D * D; idx += kLookThreads) {
                const int q = idx % kQ, c = idx / kQ;
                const int y = qy0 + q / kBX, x = qx0 + q % kBX;
                if (y < g.H && x < g.W) ob[(size_t)c * N + y * g.W + x] = v;
            }
            continue;
        }
        const int bx0 = max(box[L][0], 0), bx1 = min(box[L][1], lw - 1);
        const int by0 = max(box[L][2], 0), by1 = min(box[L][3], lh - 1);
        const int th = max(by1 - by0 + 1, 0);
        const int sa = bx0 >> 4, nseg = bx1 >= bx0 ? (bx1 >> 4) - sa + 1 : 0, sw = nseg * 16;
        const T* tlev = tseg + ((size_t)b * g.TS + g.soff[L]) * segsz;

        float hx[ITEMS][K];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
#pragma unroll
            for (int jj = 0; jj < K; ++jj) hx[i][jj] = 0.f;

        if (sw <= kMaxT) {
            const int bh = sw > 0 ? kMaxT / sw : 1;
            for (int ry0 = by0; ry0 < by0 + th; ry0 += bh) {
                const int nrow = min(bh, by0 + th - ry0), ntask = nrow * nseg;
                // C[target 4*(lane>>4)+e][query lane&15] -> S[query][band target]
                auto store = [&](const f32x4& a0, const f32x4& a1, int task) {
                    const int col = (task / nseg) * sw + (task % nseg) * 16 + 4 * (lane >> 4), j = lane & 15;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        S[j * kLd + col + e] = a0[e];
                        S[(16 + j) * kLd + col + e] = a1[e];
                    }
                };
                auto tptr = [&](int task) {
                    return tlev + ((size_t)(ry0 + task / nseg) * g.nsx[L] + sa + task % nseg) * segsz +
                           (size_t)lane * SG::LE;
                };
                if constexpr (CPT > 0) {
                    // the next task's target fragments load while this task's MFMAs run
                    auto tload = [&](frag (&t)[NLS], int task) {
                        const T* tsb = tptr(task);
#pragma unroll
                        for (int ls = 0; ls < NLS; ++ls) t[ls] = *reinterpret_cast<const frag*>(tsb + (size_t)ls * 64 * SG::LE);
                    };
                    frag tc[NLS], tn[NLS];
                    if (PF && w < ntask && !(ablate & 2)) tload(tc, w);
                    for (int task = w; task < ntask; task += kWaves) {
                        if (ablate & 2) break;
                        if (!PF) tload(tc, task);
                        else if (task + kWaves < ntask) tload(tn, task + kWaves);
                        f32x4 a0 = {}, a1 = {};
#pragma unroll
                        for (int ls = 0; ls < NLS; ls += NP) {
                            seg_mma<T, X3>(a0, tc + ls, q0 + ls);
                            seg_mma<T, X3>(a1, tc + ls, q1 + ls);
                        }
                        store(a0, a1, task);
                        if (PF) {
#pragma unroll
                            for (int ls = 0; ls < NLS; ++ls) tc[ls] = tn[ls];
                        }
                    }
                } else {
                    for (int task = w; task < ntask; task += kWaves) {
                        const T* tsb = tptr(task);
                        f32x4 a0 = {}, a1 = {};
                        for (int ls = 0; ls < nls * NP; ls += NP) {
                            frag t[NP], u0[NP], u1[NP];
#pragma unroll
                            for (int p = 0; p < NP; ++p) {
                                t[p] = *reinterpret_cast<const frag*>(tsb + (size_t)(ls + p) * 64 * SG::LE);
                                u0[p] = *reinterpret_cast<const frag*>(qsb + ((size_t)(ls + p) * 64 + lane) * SG::LE);
                                u1[p] = *reinterpret_cast<const frag*>(qsb1 + ((size_t)(ls + p) * 64 + lane) * SG::LE);
                            }
                            seg_mma<T, X3>(a0, t, u0);
                            seg_mma<T, X3>(a1, t, u1);
                        }
                        store(a0, a1, task);
                    }
                }
                __syncthreads();
#pragma unroll
                for (int i = 0; i < ITEMS; ++i) {
                    const int idx = tid + i * kLookThreads;
                    if (idx >= kQ * D) break;
                    const int q = idx % kQ, a = idx / kQ;
                    const int xs = sxs[L][q], ys = sys[L][q];
                    const float fx = sfx[L][q];
                    const float* Sq = S + q * kLd;
#pragma unroll
                    for (int jj = 0; jj < K; ++jj) {
                        const int ty = ys + jj;
                        if (ty >= ry0 && ty < ry0 + nrow) {
                            float v[2];
#pragma unroll
                            for (int u = 0; u < 2; ++u) {
                                const int tx = xs + a + u;
                                v[u] = (tx >= 0 && tx < lw) ? Sq[(ty - ry0) * sw + (tx - sa * 16)] : 0.f;
                            }
                            hx[i][jj] = fmaf(fx, v[1] - v[0], v[0]);
                        }
                    }
                }
                __syncthreads();
            }
        } else {
            // box wider than kMaxT: each query's own (2r+2)^2 patch, one dot product per thread
            for (int idx = tid; idx < kQ * KK; idx += kLookThreads) {
                const int q = idx / KK, r = idx - q * KK;
                const int ty = sys[L][q] + r / K, tx = sxs[L][q] + r % K;
                float acc = 0.f;
                if (ty >= 0 && ty < lh && tx >= 0 && tx < lw) {
                    const T* qs = q < kBX ? qsb : qsb1;
                    const T* ts = tlev + ((size_t)ty * g.nsx[L] + (tx >> 4)) * segsz;
                    for (int c = 0; c < g.C; ++c)
                        acc = fmaf(seg_elem<T, X3>(qs, q % kBX, c), seg_elem<T, X3>(ts, tx & 15, c), acc);
                }
                S[q * kLd + r] = acc;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const int idx = tid + i * kLookThreads;
                if (idx >= kQ * D) break;
                const int q = idx % kQ, a = idx / kQ;
                const float fx = sfx[L][q];
                const float* Sq = S + q * kLd;
#pragma unroll
                for (int jj = 0; jj < K; ++jj) hx[i][jj] = fmaf(fx, Sq[jj * K + a + 1] - Sq[jj * K + a], Sq[jj * K + a]);
            }
            __syncthreads();                           // S is free for the next level
        }

        // y-interpolation and the (a, b)-major output planes
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const int idx = tid + i * kLookThreads;
            if (idx >= kQ * D) break;
            const int q = idx % kQ, a = idx / kQ;
            const int y = qy0 + q / kBX, x = qx0 + q % kBX;
            if (y >= g.H || x >= g.W) continue;
            const float fy = sfy[L][q] + (sfx[L][q] - sfx[L][q]);   // a NaN x weight reaches rows outside the band too
            if (ablate & 1) {
                if (hx[i][0] == 123.f) ob[0] = fy;       // keep the sums live
                continue;
            }
            float* o = ob + (size_t)(a * D) * N + y * g.W + x;
#pragma unroll
            for (int bb = 0; bb < D; ++bb) o[(size_t)bb * N] = fmaf(fy, hx[i][bb + 1] - hx[i][bb], hx[i][bb]);
        }
    }
}

int check_otf(int batch, int channels, int height, int width, int levels, int compute) {
    RMD_REQUIRE(batch > 0 && channels > 0 && height > 0 && width > 0, RMD_ERR_SHAPE, "rmd_corr_otf: bad sizes");
    RMD_REQUIRE(levels >= 1 && levels <= RMD_MAX_LEVELS, RMD_ERR_SHAPE, "rmd_corr_otf: bad levels");
    RMD_REQUIRE((height >> (levels - 1)) >= 1 && (width >> (levels - 1)) >= 1, RMD_ERR_SHAPE,
                "rmd_corr_otf: level %d of a %dx%d map is empty", levels - 1, height, width);
    RMD_REQUIRE(compute == RMD_F32 || compute == RMD_BF16 || compute == RMD_BF16X3, RMD_ERR_ARG,
                "rmd_corr_otf: compute must be F32, BF16 or BF16X3");
    return RMD_OK;
}

template <typename T, bool X3>
void launch_segments(const LevelSrc& src, const OtfGeom& g, float scale, T* seg, hipStream_t st) {
    const long long n = (long long)g.B * g.TS * (g.Cp / Seg<T>::LSC) * 64;
    otf_segments_kernel<T, X3><<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, st>>>(src, g, scale, seg);
}

}  // namespace
}  // namespace rmd

using namespace rmd;

extern "C" size_t rmd_corr_otf_workspace_bytes(int batch, int channels, int height, int width, int levels,
                                               int compute) {
    if (check_otf(batch, channels, height, width, levels, compute)) return 0;
    const OtfGeom g = make_otf_geom(batch, channels, height, width, levels);
    const size_t es = compute == RMD_BF16 ? 2 : 4;        // BF16X3: (hi, lo) bf16 pairs
    return otf_scratch_offset(g, es) + otf_scratch_elems(g) * 4;
}

extern "C" int rmd_corr_otf_prepare(const float* fmap1, const float* fmap2, int batch, int channels, int height,
                                    int width, int levels, float scale, int compute, void* workspace, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && workspace, RMD_ERR_ARG, "rmd_corr_otf_prepare: null pointer");
    int rc = check_otf(batch, channels, height, width, levels, compute);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    const OtfGeom g = make_otf_geom(batch, channels, height, width, levels);
    const OtfGeom g1 = make_otf_geom(batch, channels, height, width, 1);   // query segments: TS = QS
    const size_t es = compute == RMD_BF16 ? 2 : 4;
    LevelSrc lq{}, lt{};
    lq.p[0] = fmap1;
    lt.p[0] = fmap2;
    float* scratch = reinterpret_cast<float*>(static_cast<char*>(workspace) + otf_scratch_offset(g, es));
    for (int l = 1; l < levels; ++l) {
        const long long n = (long long)batch * channels * g.lh[l] * g.lw[l];
        otf_pool2_kernel<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, st>>>(
            lt.p[l - 1], batch * channels, g.lh[l - 1], g.lw[l - 1], scratch);
        lt.p[l] = scratch;
        scratch += n;
    }
    const size_t qn = otf_query_elems(g);
    if (compute == RMD_BF16) {
        __bf16* q = reinterpret_cast<__bf16*>(workspace);
        launch_segments<__bf16, false>(lq, g1, scale, q, st);
        launch_segments<__bf16, false>(lt, g, 1.0f, q + qn, st);
    } else if (compute == RMD_BF16X3) {
        __bf16* q = reinterpret_cast<__bf16*>(workspace);          // split pairs: 2 x qn bf16 = qn floats
        launch_segments<__bf16, true>(lq, g1, scale, q, st);
        launch_segments<__bf16, true>(lt, g, 1.0f, q + 2 * qn, st);
    } else {
        float* q = reinterpret_cast<float*>(workspace);
        launch_segments<float, false>(lq, g1, scale, q, st);
        launch_segments<float, false>(lt, g, 1.0f, q + qn, st);
    }
    return check_launch("rmd_corr_otf_prepare");
}

extern "C" int rmd_corr_otf_lookup(const void* workspace, int batch, int channels, int height, int width, int levels,
                                   int compute, const float* coords, int radius, unsigned zero_level_mask, float* out,
                                   void* stream) {
    RMD_REQUIRE(workspace && coords && out, RMD_ERR_ARG, "rmd_corr_otf_lookup: null pointer");
    int rc = check_otf(batch, channels, height, width, levels, compute);
    if (rc) return rc;
    RMD_REQUIRE(radius >= 1 && radius <= 8, RMD_ERR_SHAPE, "rmd_corr_otf_lookup: radius %d not in 1..8", radius);
    hipStream_t st = as_stream(stream);
    const OtfGeom g = make_otf_geom(batch, channels, height, width, levels);
    const long long nblk = (long long)((width + kBX - 1) / kBX) * ((height + kBY - 1) / kBY) * batch;
    RMD_REQUIRE(nblk < (1ll << 31), RMD_ERR_SHAPE, "rmd_corr_otf_lookup: grid too large");
    const size_t lds = sizeof(float) * kQ * kLd;
    const size_t qn = otf_query_elems(g);
    // compiled channel counts keep the query segments in registers; f32 operands of >= 128 channels
    // would not fit and take the runtime loop (RMD_OTF_RUNTIME=1 forces it in the diagnostic build)
    // RMD_OTF_ABLATE (diagnostic build only, results invalid): bits 1 = skip output stores, 2 = skip the MFMA
    // phase
    const int ablate = env_knob("RMD_OTF_ABLATE", 0);           // always 0 outside librmd_diag.so
    const bool force_rt = env_knob("RMD_OTF_RUNTIME", 0) != 0;
#ifdef RMD_DIAG
    const bool pf = env_knob("RMD_OTF_PF", 0) != 0;
#define RMD_OTF_K(T, RR, CC) (pf ? otf_lookup_kernel<T, XS, RR, CC, true> : otf_lookup_kernel<T, XS, RR, CC, false>)
#else
#define RMD_OTF_K(T, RR, CC) otf_lookup_kernel<T, XS, RR, CC, false>
#endif
    const bool exact = compute == RMD_F32;
    const bool x3 = compute == RMD_BF16X3;
    const int cpt = force_rt || (exact && g.Cp >= 128) || g.Cp > 256 ? 0 : g.Cp;
#define RMD_OTF(T, RR, CC)                                                                                     \
    do {                                                                                                       \
        auto k = RMD_OTF_K(T, RR, CC);                                                                         \
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)lds);                                                                   \
        const T* q = reinterpret_cast<const T*>(workspace);                                                    \
        k<<<(unsigned)nblk, kLookThreads, lds, st>>>(q, q + qn * XN, g, coords, zero_level_mask, out, ablate);   \
    } while (0)
#define RMD_OTF_C(T, RR)                                 \
    switch (cpt) {                                       \
        case 32: RMD_OTF(T, RR, 32); break;              \
        case 64: RMD_OTF(T, RR, 64); break;              \
        case 128: RMD_OTF(T, RR, 128); break;            \
        case 256: RMD_OTF(T, RR, 256); break;            \
        default: RMD_OTF(T, RR, 0); break;               \
    }
#define RMD_OTF_R(T)                                     \
    switch (radius) {                                    \
        case 1: RMD_OTF_C(T, 1); break;                  \
        case 2: RMD_OTF_C(T, 2); break;                  \
        case 3: RMD_OTF_C(T, 3); break;                  \
        case 4: RMD_OTF_C(T, 4); break;                  \
        case 5: RMD_OTF_C(T, 5); break;                  \
        case 6: RMD_OTF_C(T, 6); break;                  \
        case 7: RMD_OTF_C(T, 7); break;                  \
        default: RMD_OTF_C(T, 8); break;                 \
    }
    if (compute == RMD_BF16) {
        constexpr bool XS = false;
        constexpr size_t XN = 1;
        RMD_OTF_R(__bf16)
    } else if (x3) {
        constexpr bool XS = true;
        constexpr size_t XN = 2;                    // query segments: qn split pairs
        RMD_OTF_R(__bf16)
    } else {
        constexpr bool XS = false;
        constexpr size_t XN = 1;
        RMD_OTF_R(float)
    }
#undef RMD_OTF_R
#undef RMD_OTF_C
#undef RMD_OTF
#undef RMD_OTF_K
    return check_launch("rmd_corr_otf_lookup");
}
