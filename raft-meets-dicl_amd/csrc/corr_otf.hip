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
// Lookup: one 256-thread block per (query block of QSX x QSY segments of 16 x 1 pixels, batch), looping
// over the levels.  The block's queries' (2r+2)^2 integer patches at level l are bounded by one box
// (clipped to the map, widened to whole segments); every (box row, target segment) is one task: one
// 16x16 MFMA tile per query segment (16 targets x 16 queries), of whose products each lane keeps only
// those inside its query's own patch, in an LDS patch buffer per query (zero for targets off the map:
// zero padding per tap).  Each (query, x-offset) thread then interpolates its window exactly as
// rmd_corr_lookup does (shared bilinear weights, NaN for 1-pixel levels, zeroed masked levels).  A box
// of more than kMaxTasks segments (flow differing by hundreds of pixels inside one block) takes a
// per-query VALU patch path.
#include "rmd_common.h"

#include <algorithm>
#include <type_traits>

namespace rmd {
namespace {

constexpr int kThreads = 256;                        // prepare kernels
// lookup workgroup size per compute (-D knobs)
#ifndef RMD_OTF_NT_B
#define RMD_OTF_NT_B 256
#endif
#ifndef RMD_OTF_NT_X
#define RMD_OTF_NT_X 512
#endif
// wide-map bf16 query block (16 x WQY), workgroup size and occupancy hint (-D knobs for A/B builds)
#ifndef RMD_OTF_WQY
#define RMD_OTF_WQY 4
#endif
#ifndef RMD_OTF_WNT
#define RMD_OTF_WNT 512
#endif
#ifndef RMD_OTF_WOCC
#define RMD_OTF_WOCC 2
#endif
constexpr long long kWideBlocks = 4096;              // bf16: 16x4 query blocks from this many 16x2 blocks
constexpr int kMaxTasks = 1024;                      // box segments of the MFMA path (more: per-query VALU)
// Query block, occupancy and query-fragment placement per compute (-D knobs for A/B builds,
// tools/_gpu_r03k.sh).  cfg2 bf16, one box per comparison (profiles/otf_patch_ab_r03.jsonl,
// otf_ql_ab_r03.jsonl): 16x2 blocks with the query fragments in LDS (QL) 77.7 us; 16x1 with them in
// registers 87.5; 16x4 in registers 84.8; 16x4 QL 100.7 at 256 threads, 77.2 at 512.  Round 4, with the
// interleaved MFMA order (profiles/otf_put_ab_r04.json): bf16 16x2 QL 256 threads 69-71 us (16x4 at 512
// 73-74, 16x1 88-91, 16x2 at 512 / 384 / 128 threads 75 / 86 / 83); split-bf16 16x2 QL 512 threads
// 115-119 us (256 threads 136-139, register fragments 145-147).
#ifndef RMD_OTF_QSX_B
#define RMD_OTF_QSX_B 1
#endif
#ifndef RMD_OTF_QSY_B
#define RMD_OTF_QSY_B 2
#endif
#ifndef RMD_OTF_QSX_X
#define RMD_OTF_QSX_X 1
#endif
#ifndef RMD_OTF_QSY_X
#define RMD_OTF_QSY_X 2
#endif
#ifndef RMD_OTF_OCC_B
#define RMD_OTF_OCC_B 2
#endif
#ifndef RMD_OTF_OCC_X
#define RMD_OTF_OCC_X 2
#endif
#ifndef RMD_OTF_QL_B
#define RMD_OTF_QL_B 1
#endif
#ifndef RMD_OTF_QL_X
#define RMD_OTF_QL_X 1
#endif
// LDS write of a task's products (put): 1 = every lane writes its 4 products, those outside its query's
// patch into a pad slot (no branches), 0 = only the products inside, under per-element branches.
// cfg2 A/B (profiles/otf_put_ab_r04.json): bf16 70.8-73.2 us with 1 vs 75.9-78.5 with 0; split-bf16
// (two waves per SIMD) 150 with 0 vs 170 with 1
#ifndef RMD_OTF_PUTSEL_B
#define RMD_OTF_PUTSEL_B 1
#endif
#ifndef RMD_OTF_PUTSEL_X
#define RMD_OTF_PUTSEL_X 0
#endif
// MFMA order in a task: 1 = load step outer, query segments inner (independent chains interleaved)
#ifndef RMD_OTF_ILV
#define RMD_OTF_ILV 1
#endif
// backward ablation for A/B timing only (wrong results): 1 = the dP atomic adds are skipped, 2 = the G
// build reads no record weights (constants instead)
#ifndef RMD_OTF_BWD_ABL
#define RMD_OTF_BWD_ABL 0
#endif
// pad slots per query patch in LDS (odd patch stride): 1, or 4 = one per lane group (put's pad writes of
// the 4 lane groups of a query go to distinct addresses)
#ifndef RMD_OTF_PADS
#define RMD_OTF_PADS 1
#endif
// ablation for A/B timing only (wrong results): 1 = no output stores, 2 = no MFMA tasks, 3 = tasks
// without MFMAs (operand loads and puts), 4 = tasks without operand loads (MFMAs on one task's operands)
#ifndef RMD_OTF_ABL
#define RMD_OTF_ABL 0
#endif

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

struct LevelOff {
    long long o[RMD_MAX_LEVELS];
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

// Query block = QSX x QSY query segments (16 x 1 pixels each): 16 QSX x QSY queries.  Larger blocks
// load each target segment of their box once for more queries (the L2 -> CU operand traffic is the
// bound: every block re-reads its box), at the cost of MFMA tiles for targets outside a query's own
// window.  A 16 x 4 block (bf16) reads 2.5x fewer target bytes per query than 16 x 2.
// LDS floats per query patch: the (2r+2)^2 products, then RMD_OTF_PADS pad slots, rounded to an odd stride
constexpr int otf_patch_stride(int R) { return ((2 * R + 2) * (2 * R + 2) + RMD_OTF_PADS) | 1; }

template <int QSX, int QSY> struct QBlock {
    static constexpr int kQS = QSX * QSY, kBX = 16 * QSX, kBY = QSY, kQ = kBX * kBY;
};

// 1-D grid over (batch, query block), XCD-aware: adjacent query blocks, whose target boxes overlap,
// run on the same XCD and share its L2.  One block runs every level of its queries, so the query
// staging, the coords load and the block's fixed start-up cost are paid once, not once per level.
// CPT = compiled Cp (0: runtime multiple of 128).
template <typename T, bool X3, int R, int CPT, int QSX, int QSY, int OCC, bool QL, int kLookThreads>
__global__ void __launch_bounds__(kLookThreads, OCC)
otf_lookup_kernel(const T* __restrict__ qseg, const T* __restrict__ tseg, OtfGeom g,
                  const float* __restrict__ coords, unsigned zmask, float* __restrict__ out) {
    using SG = Seg<T>;
    using frag = typename SG::frag;
    using QB = QBlock<QSX, QSY>;
    constexpr int kQS = QB::kQS, kBX = QB::kBX, kBY = QB::kBY, kQ = QB::kQ;
    constexpr int kWaves = kLookThreads / 64;
    constexpr int D = 2 * R + 1, K = 2 * R + 2, KK = K * K, KKp = otf_patch_stride(R);   // odd: queries spread over banks
    constexpr bool kPutSel = sizeof(T) == 2 && !X3 ? RMD_OTF_PUTSEL_B != 0 : RMD_OTF_PUTSEL_X != 0;
    extern __shared__ float S[];                       // [kQ][KKp]: every query's (2r+2)^2 patch
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
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);      // wave-uniform: task indices in SGPRs
    constexpr int NP = X3 ? 2 : 1;                      // load steps per channel step (X3: hi, lo)
    const int cp = CPT > 0 ? CPT : g.Cp;
    const int nls = cp / SG::LSC;
    const size_t segsz = (size_t)16 * cp * NP;
    // query segment s = (row sy, column sx) of the block: its operand rows (clamped at the map edge)
    const T* qsb[kQS];
#pragma unroll
    for (int s = 0; s < kQS; ++s)
        qsb[s] = qseg + ((size_t)b * g.QS + (size_t)min(qy0 + s / QSX, g.H - 1) * g.qnsx +
                         min((qx0 >> 4) + s % QSX, g.qnsx - 1)) * segsz;

    // the block's query fragments (CPT > 0): each wave keeps them in registers for every level and
    // target segment (a load step is one coalesced 1-KiB read per instruction), or (QL) one copy in
    // LDS behind the patch buffers, read per MFMA (fewer VGPRs: more waves and target loads in flight)
    constexpr int NLS = CPT > 0 ? CPT / SG::LSC * NP : 1;                 // load steps per segment
    constexpr bool QREG = CPT > 0 && !QL;
    frag qf[QREG ? kQS : 1][QREG ? NLS : 1];
    const frag* qlds = reinterpret_cast<const frag*>(S + kQ * KKp);
    if constexpr (QREG) {
#pragma unroll
        for (int s = 0; s < kQS; ++s)
#pragma unroll
            for (int ls = 0; ls < NLS; ++ls) qf[s][ls] = *reinterpret_cast<const frag*>(qsb[s] + ((size_t)ls * 64 + lane) * SG::LE);
    } else if constexpr (CPT > 0) {
        constexpr int QV = 16 * CPT * NP * (int)sizeof(T) / 16;            // 16-B vectors per segment
        uint4* dst = reinterpret_cast<uint4*>(S + kQ * KKp);
#pragma unroll
        for (int s = 0; s < kQS; ++s) {
            const uint4* src = reinterpret_cast<const uint4*>(qsb[s]);
            for (int v = tid; v < QV; v += kLookThreads) dst[s * QV + v] = src[v];
        }
    }
    // query fragments (s, load steps ls .. ls + NP - 1) of this lane
    auto qget = [&](frag (&u)[NP], int s, int ls) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if constexpr (QREG) u[p] = qf[s][ls + p];
            else u[p] = qlds[(s * NLS + ls + p) * 64 + lane];
        }
    };
    if (tid < RMD_MAX_LEVELS * 4) box[tid >> 2][tid & 3] = (tid & 1) ? -(1 << 30) : (1 << 30);
    __syncthreads();
    // thread (level, query) items: every level's window origin (coords clamped as rmd_corr_lookup does)
    for (int it = tid; it < kQ * g.L; it += kLookThreads) {
        const int q = it % kQ, L = it / kQ;
        const int y = min(qy0 + q / kBX, g.H - 1), x = min(qx0 + q % kBX, g.W - 1);
        const float cx0 = coords[((size_t)b * 2 + 0) * N + y * g.W + x];
        const float cy0 = coords[((size_t)b * 2 + 1) * N + y * g.W + x];
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
    __syncthreads();                                   // boxes complete
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
        const int sa = bx0 >> 4, nseg = bx1 >= bx0 ? (bx1 >> 4) - sa + 1 : 0;
        const int ntask = th * nseg;                   // (box row, target segment) MFMA tasks
        const T* tlev = tseg + ((size_t)b * g.TS + g.soff[L]) * segsz;

        float hx[ITEMS][K];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
#pragma unroll
            for (int jj = 0; jj < K; ++jj) hx[i][jj] = 0.f;

        if (ntask > 0 && ntask <= kMaxTasks) {
            // every query's (2r+2)^2 patch in LDS, zero where the target is off the map (zero padding)
            for (int i = tid; i < kQ * KKp; i += kLookThreads) S[i] = 0.f;
            // the lane's query in each query segment: its window origin at this level
            int wx[kQS], wy[kQS], wq[kQS];
#pragma unroll
            for (int s = 0; s < kQS; ++s) {
                wq[s] = (s / QSX) * kBX + (s % QSX) * 16 + (lane & 15);
                wx[s] = sxs[L][wq[s]];
                wy[s] = sys[L][wq[s]];
            }
            __syncthreads();
            // C[target 4*(lane>>4)+e][query lane&15] of task (box row r, target segment column c): keep the
            // products inside the query's own patch (kPutSel: the others go to a pad slot of the query,
            // never read, so the four LDS writes carry no branches)
            auto put = [&](const f32x4& acc, int s, int r, int c) {
                const int dy = by0 + r - wy[s];
                const int dx0 = c * 16 + 4 * (lane >> 4) - wx[s];
                const bool rok = (unsigned)dy < (unsigned)K;
                float* P = S + wq[s] * KKp;
                if constexpr (kPutSel) {
                    const int pad = KK + (RMD_OTF_PADS > 1 ? (lane >> 4) % RMD_OTF_PADS : 0);
#pragma unroll
                    for (int e = 0; e < 4; ++e) P[rok && (unsigned)(dx0 + e) < (unsigned)K ? dy * K + dx0 + e : pad] = acc[e];
                } else if (rok) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if ((unsigned)(dx0 + e) < (unsigned)K) P[dy * K + dx0 + e] = acc[e];
                }
            };
            auto tptr = [&](int r, int c) {
                return tlev + ((size_t)(by0 + r) * g.nsx[L] + c) * segsz + (size_t)lane * SG::LE;
            };
            // the wave's tasks w, w + kWaves, ... as (box row, segment column), advanced without division
            int tr = w / nseg, tcol = sa + w - tr * nseg;
            auto advance = [&](int& r, int& c) {
                c += kWaves;
                while (c >= sa + nseg) {
                    c -= nseg;
                    ++r;
                }
            };
            if constexpr (CPT > 0) {
                frag tc[NLS];
                if constexpr (RMD_OTF_ABL == 4) {          // ablation: one task's operands for all tasks
                    const T* tsb = tptr(by0, sa);
#pragma unroll
                    for (int ls = 0; ls < NLS; ++ls) tc[ls] = *reinterpret_cast<const frag*>(tsb + (size_t)ls * 64 * SG::LE);
                }
                for (int task = w; task < (RMD_OTF_ABL == 2 ? 0 : ntask); task += kWaves, advance(tr, tcol)) {
                    if constexpr (RMD_OTF_ABL != 4) {
                        const T* tsb = tptr(tr, tcol);
#pragma unroll
                        for (int ls = 0; ls < NLS; ++ls) tc[ls] = *reinterpret_cast<const frag*>(tsb + (size_t)ls * 64 * SG::LE);
                    }
                    if constexpr (RMD_OTF_ILV && RMD_OTF_ABL != 3) {
                        // load step outer, query segment inner: kQS independent accumulator chains interleave
                        f32x4 acc[kQS];
#pragma unroll
                        for (int s = 0; s < kQS; ++s) acc[s] = f32x4{};
#pragma unroll
                        for (int ls = 0; ls < NLS; ls += NP)
#pragma unroll
                            for (int s = 0; s < kQS; ++s) {
                                frag u[NP];
                                qget(u, s, ls);
                                seg_mma<T, X3>(acc[s], tc + ls, u);
                            }
#pragma unroll
                        for (int s = 0; s < kQS; ++s) put(acc[s], s, tr, tcol);
                    } else {
#pragma unroll
                    for (int s = 0; s < kQS; ++s) {
                        f32x4 acc = {};
                        if constexpr (RMD_OTF_ABL == 3) {      // ablation: operand loads and puts, no MFMA
#pragma unroll
                            for (int ls = 0; ls < NLS; ++ls) acc[ls & 3] += (float)tc[ls][s & 7];
                        } else {
#pragma unroll
                            for (int ls = 0; ls < NLS; ls += NP) {
                                frag u[NP];
                                qget(u, s, ls);
                                seg_mma<T, X3>(acc, tc + ls, u);
                            }
                        }
                        put(acc, s, tr, tcol);
                    }
                    }
                }
            } else {
                for (int task = w; task < ntask; task += kWaves, advance(tr, tcol)) {
                    const T* tsb = tptr(tr, tcol);
                    f32x4 acc[kQS];
#pragma unroll
                    for (int s = 0; s < kQS; ++s) acc[s] = f32x4{};
                    for (int ls = 0; ls < nls * NP; ls += NP) {
                        frag t[NP];
#pragma unroll
                        for (int p = 0; p < NP; ++p) t[p] = *reinterpret_cast<const frag*>(tsb + (size_t)(ls + p) * 64 * SG::LE);
#pragma unroll
                        for (int s = 0; s < kQS; ++s) {
                            frag u[NP];
#pragma unroll
                            for (int p = 0; p < NP; ++p)
                                u[p] = *reinterpret_cast<const frag*>(qsb[s] + ((size_t)(ls + p) * 64 + lane) * SG::LE);
                            seg_mma<T, X3>(acc[s], t, u);
                        }
                    }
#pragma unroll
                    for (int s = 0; s < kQS; ++s) put(acc[s], s, tr, tcol);
                }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const int idx = tid + i * kLookThreads;
                if (idx >= kQ * D) break;
                const int q = idx % kQ, a = idx / kQ;
                const float fx = sfx[L][q];
                const float* P = S + q * KKp + a;
#pragma unroll
                for (int jj = 0; jj < K; ++jj) hx[i][jj] = fmaf(fx, P[jj * K + 1] - P[jj * K], P[jj * K]);
            }
            __syncthreads();                           // S is free for the next level
        } else if (ntask > 0) {
            // a box of more than kMaxTasks segments (flow differing by hundreds of pixels inside one
            // block): each query's own (2r+2)^2 patch, one dot product per thread
            for (int idx = tid; idx < kQ * KK; idx += kLookThreads) {
                const int q = idx / KK, r = idx - q * KK;
                const int ty = sys[L][q] + r / K, tx = sxs[L][q] + r % K;
                float acc = 0.f;
                if (ty >= 0 && ty < lh && tx >= 0 && tx < lw) {
                    const int qr = q / kBX, qc = q % kBX;
                    const T* qs = qsb[qr * QSX + qc / 16];
                    const T* ts = tlev + ((size_t)ty * g.nsx[L] + (tx >> 4)) * segsz;
                    for (int c = 0; c < g.C; ++c)
                        acc = fmaf(seg_elem<T, X3>(qs, qc % 16, c), seg_elem<T, X3>(ts, tx & 15, c), acc);
                }
                S[q * KKp + r] = acc;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const int idx = tid + i * kLookThreads;
                if (idx >= kQ * D) break;
                const int q = idx % kQ, a = idx / kQ;
                const float fx = sfx[L][q];
                const float* P = S + q * KKp + a;
#pragma unroll
                for (int jj = 0; jj < K; ++jj) hx[i][jj] = fmaf(fx, P[jj * K + 1] - P[jj * K], P[jj * K]);
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
            if (RMD_OTF_ABL == 1 && fy != 12345.f) continue;
            float* o = ob + (size_t)(a * D) * N + y * g.W + x;
#pragma unroll
            for (int bb = 0; bb < D; ++bb) o[(size_t)bb * N] = fmaf(fy, hx[i][bb + 1] - hx[i][bb], hx[i][bb]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Backward (training).  With G_l the gradient of the level-l window products w.r.t. the pooled targets
// (per query the (2r+2)^2 bilinear patch weights of its grad_out window, raft_fs.py:68-74 transposed),
//   d q~ = sum_l G_l . P_l      (q~ = fmap1 * scale, the query operand)
//   d P_l = G_l^T . q~          (P_l the level-l pooled fmap2, raft_fs.py:25-31)
// and d fmap2 = sum_l avgpool_l^T(d P_l).  Coordinates carry no gradient (raft.py:402).
//
// Every lookup of a block records its patch weights (otf_record_kernel: origin + K*K weights per
// (level, query), no volume); one launch after the last lookup backward turns all records into the
// two products, so the box of target rows a query tile touches is swept once for all iterations:
//  * one 512-thread workgroup per 32 x 4 query tile; per level the target rows some record patch covers,
//    each over its covered column extent (per-row extents: a divergent flow costs its patches' rows);
//  * those rows' 16-column target segments are packed in order into bands of up to 8 segments (128
//    targets, possibly spanning several rows): fewer, longer MFMA phases than one band per row;
//  * per band the dense G (128 queries x 128 band targets, fp32) is built in LDS by owner threads:
//    thread (query q, p) owns the band columns = p (mod 4) of its query's row and adds, record by
//    record in order, the patch weights that land there (deterministic; a wave's loads run along the
//    queries of its own patch column: coalesced);
//  * d q~ (128 queries x C) += G . P_band: v_mfma_f32_32x32x16_bf16 with A = G rows from LDS and B =
//    the band's target segments in the "T layout" (lane c + 32h holds pixels 8h..8h+7 of channel c of a
//    16-pixel segment), the next segment's fragments loaded while the current one's MFMAs run;
//  * d P_band = G^T . q~: A = G columns from LDS, B = the tile's query segments (bf16: copied to LDS
//    once per workgroup; split-bf16: from L2, one k-step ahead); every fp32 32 x 32 result tile is added
//    to d P as 64-bit fixed point with integer atomics.  Integer addition is associative, so d P is
//    bitwise independent of the order the workgroups add in — with no premise on the contributions'
//    dynamic range.  The scale 2^s is a power of two chosen per backward from the largest |weight|
//    (recorded by otf_record_kernel) and |q~| (otf_tlayout_kernel) so that no sum can exceed 2^62:
//    |d P| <= records * N * max|w| * max|q~|; the fixed-point step 2^-s is ~2^-40 of that bound,
//    far below the fp32 ulp of any element the bound lets reach 2^-15 of it.  Non-finite contributions
//    go to a float side buffer instead (NaN / inf propagate as through the reference's autograd).
// fp32 modes split G and both operands into bf16 hi + lo and accumulate lo.hi + hi.lo + hi.hi (the
// forward x3 split); bf16 mode uses one product.
constexpr int kBwdQX = 32, kBwdQY = 4, kBwdQ = kBwdQX * kBwdQY;
constexpr int kBwdSeg = 8;                           // 16-target segments per band
constexpr int kBwdTB = 16 * kBwdSeg;                 // band width (targets)
constexpr int kBwdRows = 4;                          // distinct target rows per band (G-build registers)
constexpr int kBwdLd = kBwdTB + 4;                   // G row stride (floats): conflict-free row and column reads
constexpr int kBwdThreads = 512;
constexpr int kMaxRec = 16;                          // records per launch (more: several launches)
constexpr int kFar = -(1 << 29);                     // origin of a masked / degenerate level

typedef __attribute__((ext_vector_type(16))) float f32x16;

struct OtfRecords {
    const int2* org[kMaxRec];                       // (L, B, N) patch origins (x0, y0) at level l
    const float* wp[kMaxRec];                       // (L, B, K*K, N) patch weights
    int n;
};

size_t otf_record_org_bytes(int B, int H, int W, int L) {
    return ((size_t)L * B * H * W * sizeof(int2) + 255) / 256 * 256;
}
size_t otf_record_wp_bytes(int B, int H, int W, int L, int K) {
    return ((size_t)L * B * H * W * K * K * sizeof(float) + 255) / 256 * 256;
}

// |v| as ordered integer bits for an atomicMax of finite magnitudes (non-finite values are skipped);
// dst is an array of kMaxSlots words, each workgroup adds into slot blockIdx % kMaxSlots (one
// address per thousands of waves would serialise the atomics)
constexpr int kMaxSlots = 64;
__device__ __forceinline__ void max_abs_finite(unsigned* dst, float v) {
    unsigned m = __builtin_isfinite(v) ? (__float_as_uint(v) & 0x7fffffffu) : 0u;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(dst + blockIdx.x % kMaxSlots, m);
}

// per (level, batch, query): origin and the (2r+2)^2 patch weights of grad_out's window
//   wp[j][k] = (1-fy) hx(k, j) + fy hx(k, j-1),  hx(k, bb) = (1-fx) g[k][bb] + fx g[k-1][bb]
// (g[a][bb] = grad_out channel l*D*D + a*D + bb; out-of-range a / bb -> 0).  Masked and 1-pixel levels
// record kFar (no contribution); a non-finite coordinate clamps far off the map (no contribution).
// The largest finite |weight| goes to *wmax (the record's header word, zeroed by the launcher).
template <int R>
__global__ void __launch_bounds__(kThreads)
otf_record_kernel(const float* __restrict__ gout, const float* __restrict__ coords, OtfGeom g, unsigned zmask,
                  int2* __restrict__ org, float* __restrict__ wp, unsigned* __restrict__ wmax) {
    constexpr int D = 2 * R + 1, K = 2 * R + 2;
    const long long N = (long long)g.H * g.W;
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    const bool in = idx < (long long)g.L * g.B * N;
    const long long id = in ? idx : 0;
    const int q = (int)(id % N);
    const int b = (int)((id / N) % g.B);
    const int l = (int)(id / (N * g.B));
    const int lh = g.lh[l], lw = g.lw[l];
    const float x = coords[((size_t)b * 2 + 0) * N + q], y = coords[((size_t)b * 2 + 1) * N + q];
    const float inv = 1.0f / (float)(1 << l);
    const float rx = x * inv, ry = y * inv;
    const float cx = fminf(fmaxf(rx, -1.0e6f), 1.0e6f), cy = fminf(fmaxf(ry, -1.0e6f), 1.0e6f);
    const bool dead = !in || ((zmask >> l) & 1u) || lh < 2 || lw < 2 || !(rx == rx) || !(ry == ry);
    if (in) org[id] = dead ? make_int2(kFar, kFar) : make_int2((int)floorf(cx) - R, (int)floorf(cy) - R);
    const float fx = rx - floorf(rx), fy = ry - floorf(ry);
    const float* gp = gout + ((size_t)b * g.L + l) * D * D * N + q;
    float gv[D][D];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
        for (int bb = 0; bb < D; ++bb) gv[a][bb] = dead ? 0.f : gp[(size_t)(a * D + bb) * N];
    float* w = wp + ((size_t)l * g.B + b) * K * K * N + q;
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            auto hx = [&](int bb) {
                if (bb < 0 || bb >= D) return 0.f;
                const float v0 = k < D ? gv[k][bb] : 0.f, v1 = k >= 1 ? gv[k - 1][bb] : 0.f;
                return (1.f - fx) * v0 + fx * v1;
            };
            const float v = dead ? 0.f : (1.f - fy) * hx(j) + fy * hx(j - 1);
            if (in) w[(size_t)(j * K + k) * N] = v;
            m = __builtin_isfinite(v) ? fmaxf(m, fabsf(v)) : m;
        }
    }
    max_abs_finite(wmax, m);
}

// T layout of a planar (B, C, h, w) fp32 map (times s): unit (b, level segment row/seg, channel group cg)
// = 64 lanes x 8 elements, lane c + 32h = pixels 8h..8h+7 of channel 32cg + c (zero past the map / C);
// X3: the unit's lo half follows its hi half.  One thread per (unit, lane).  vmax (optional): the
// largest finite |value| (the query operand's, for the fixed-point scale of d P).
template <bool X3>
__global__ void __launch_bounds__(kThreads)
otf_tlayout_kernel(LevelSrc src, OtfGeom g, float s, __bf16* __restrict__ dst, unsigned* __restrict__ vmax) {
    constexpr int NP = X3 ? 2 : 1;
    const int ncg = g.Cp / 32;
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    const bool in = idx < (long long)g.B * g.TS * ncg * 64;
    const long long id = in ? idx : 0;
    const int lane = (int)(id & 63), c32 = lane & 31, h = lane >> 5;
    const long long u = id >> 6;
    const int cg = (int)(u % ncg);
    const long long bs = u / ncg;
    const long long sg = bs % g.TS;
    const int b = (int)(bs / g.TS);
    int l = 0;
#pragma unroll
    for (int k = 1; k < RMD_MAX_LEVELS; ++k)
        if (k < g.L && sg >= g.soff[k]) l = k;
    const int sl = (int)(sg - g.soff[l]);
    const int y = sl / g.nsx[l], x0 = (sl - y * g.nsx[l]) * 16 + 8 * h;
    const int c = 32 * cg + c32;
    const size_t plane = (size_t)g.lh[l] * g.lw[l];
    const float* row = src.p[l] + ((size_t)b * g.C + (c < g.C ? c : 0)) * plane + (size_t)y * g.lw[l];
    bf16x8 hi, lo;
    float m = 0.f;
    float xv[8];
    const bool cin = in && c < g.C;
    if (cin && x0 + 8 <= g.lw[l] && ((((uintptr_t)(row + x0)) & 15) == 0)) {
        // whole 8-pixel run: two 16-B loads (the per-element path below is the map's right edge)
        *reinterpret_cast<float4*>(xv) = *reinterpret_cast<const float4*>(row + x0);
        *reinterpret_cast<float4*>(xv + 4) = *reinterpret_cast<const float4*>(row + x0 + 4);
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = (cin && x0 + e < g.lw[l]) ? row[x0 + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float v = cin ? xv[e] * s : 0.f;
        hi[e] = (__bf16)v;
        lo[e] = (__bf16)(v - (float)hi[e]);
        m = __builtin_isfinite(v) ? fmaxf(m, fabsf(v)) : m;
    }
    if (in) {
        __bf16* o = dst + ((size_t)u * NP * 64 + lane) * 8;
        *reinterpret_cast<bf16x8*>(o) = hi;
        if constexpr (X3) *reinterpret_cast<bf16x8*>(o + 64 * 8) = lo;
    }
    if (vmax) max_abs_finite(vmax, m);
}

__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        hi[e] = (__bf16)v[e];
        lo[e] = (__bf16)(v[e] - (float)hi[e]);
    }
}

template <bool X3>
__device__ __forceinline__ void mma3(f32x16& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                     const bf16x8& bl) {
    if constexpr (X3) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

struct BwdArgs {
    OtfGeom g;                  // targets (all levels); g.QS / g.qnsx: query segments
    const __bf16* pt;           // targets, T layout (B, TS, ncg units)
    const __bf16* qt;           // queries (fmap1 * scale), T layout (B, QS, ncg units)
    OtfRecords rec;
    long long* dP;              // (B, PT, C) pixel-major fixed point (2^-s units), += G^T q~
    float* dPnf;                // (B, PT, C) non-finite contributions (float atomics; zero otherwise)
    long long pT;               // pooled pixels per batch (all levels)
    long long poff[RMD_MAX_LEVELS];
    float* gq;                  // (B, C, H, W) fp32, += scale * G P
    float scale;
    const int* sexp;            // fixed-point exponent s of d P (otf_fixed_exp_kernel)
    int* nf;                    // set when any contribution went to dPnf
};

struct BwdWmax {                // header words of up to kMaxRecAll records (the scale's bound)
    const unsigned* p[64];
};

// fixed-point exponent s: 2^s * bound <= 2^62 with bound = nrec * N * max|w| * max|q~| (a power of two
// scale, the same for every workgroup: deterministic).  The bound is formed in double: the maxima are
// finite floats, so it stays finite (<= 2^64 * FLT_MAX^2) where a float product would overflow to inf
// (ADVICE r05); a zero bound (no nonzero contribution) takes any exponent, and a non-finite one — not
// reachable from finite maxima — the smallest, so no sum can overflow.
__device__ __forceinline__ int fixed_exp(double bound) {
    if (!__builtin_isfinite(bound)) return -960;
    if (!(bound > 0.0)) return 60;
    int e;
    (void)frexp(bound, &e);                          // bound < 2^e
    return max(-960, min(960, 62 - e));
}

template <bool X3, int R>
__global__ void __launch_bounds__(kBwdThreads, 1)
otf_backward_kernel(BwdArgs a) {
    constexpr int K = 2 * R + 2;
    constexpr int NP = X3 ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    float* G = reinterpret_cast<float*>(dyn);                              // [kBwdQ][kBwdLd]
    __bf16* qimg = reinterpret_cast<__bf16*>(dyn + sizeof(float) * kBwdQ * kBwdLd);   // bf16: [8][ncg][64][8]
    __shared__ int2 sorg[kMaxRec][kBwdQ];
    __shared__ int box[4];
    __shared__ int bseg_row[kBwdSeg], bseg_x[kBwdSeg];
    __shared__ int bnseg, bcur_row, bcur_x, bnrow;
    __shared__ int brow_y[kBwdRows], brow_s0[kBwdRows], brow_x0[kBwdRows], brow_n[kBwdRows];
    __shared__ const int2* s_org[kMaxRec];
    __shared__ const float* s_wp[kMaxRec];
    const OtfGeom& g = a.g;
    const int N = g.H * g.W;
    const int ncg = g.Cp / 32;
    const int nbx = (g.W + kBwdQX - 1) / kBwdQX, nqb = nbx * ((g.H + kBwdQY - 1) / kBwdQY);
    const int lid = xcd_block(blockIdx.x, gridDim.x);
    const int qb = lid % nqb, b = lid / nqb;
    const int qx0 = (qb % nbx) * kBwdQX, qy0 = (qb / nbx) * kBwdQY;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j32 = lane & 31, h = lane >> 5;
    const int mt = w & 3;                                            // query row / target tile of this wave
    const int nt0 = (w >> 2) * 4;                                    // first channel tile of this wave
    const int ntn = max(0, min(4, ncg - nt0));
    const size_t unit = (size_t)64 * 8 * NP;                         // elements per T-layout unit
    int2* rowext = reinterpret_cast<int2*>(dyn + sizeof(float) * kBwdQ * kBwdLd + (X3 ? 0 : (size_t)8 * ncg * 1024));
    // G build ownership: thread (query gq_, class p) owns band columns = p (mod 4); the 4 classes of a
    // query are adjacent lanes, so a wave's weight load reads 16 consecutive queries of 4 patch columns
    const int gq_ = tid >> 2, p = tid & 3;
    const int gy = qy0 + gq_ / kBwdQX, gx = qx0 + gq_ % kBwdQX;
    const bool gvalid = gy < g.H && gx < g.W;
    const size_t qoff = gvalid ? (size_t)gy * g.W + gx : 0;

    // bf16: the tile's query segments (8 x ncg units) -> LDS once (the B operand of every d P phase)
    if constexpr (!X3) {
        for (int i = tid; i < 8 * ncg * 64; i += kBwdThreads) {
            const int un = i >> 6, ln = i & 63;
            const int qs = un / ncg, cg = un % ncg;
            const int qrow = qy0 + (qs >> 1), qsx = (qx0 >> 4) + (qs & 1);
            uint4 v = make_uint4(0, 0, 0, 0);
            if (qrow < g.H && qsx < g.qnsx)
                v = *reinterpret_cast<const uint4*>(a.qt + ((size_t)(b * g.QS + qrow * g.qnsx + qsx) * ncg + cg) * unit + ln * 8);
            *reinterpret_cast<uint4*>(qimg + (size_t)i * 8) = v;
        }
    }

    // record pointers to LDS (runtime-indexed kernel-argument arrays would sit in SGPRs and spill)
    if (tid < kMaxRec) {
        s_org[tid] = tid < a.rec.n ? a.rec.org[tid] : nullptr;
        s_wp[tid] = tid < a.rec.n ? a.rec.wp[tid] : nullptr;
    }
    const int nrec = a.rec.n;
    f32x16 accq[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) accq[t] = f32x16{};
    const double fscale = ldexp(1.0, *a.sexp);

    for (int l = 0; l < g.L; ++l) {
        const int lh = g.lh[l], lw = g.lw[l];
        // ---- origins of every record for the tile's queries, and their union box at this level ----
        __syncthreads();                                             // previous level's G / sorg reads done
        if (tid < 4) box[tid] = (tid & 1) ? -(1 << 30) : (1 << 30);
        __syncthreads();
        for (int i = tid; i < nrec * kBwdQ; i += kBwdThreads) {
            const int r = i / kBwdQ, q = i % kBwdQ;
            const int y = qy0 + q / kBwdQX, x = qx0 + q % kBwdQX;
            int2 o = make_int2(kFar, kFar);
            if (y < g.H && x < g.W) o = s_org[r][((size_t)l * g.B + b) * N + y * g.W + x];
            // patches entirely off the map contribute nothing
            if (o.x + K - 1 < 0 || o.x >= lw || o.y + K - 1 < 0 || o.y >= lh) o = make_int2(kFar, kFar);
            sorg[r][q] = o;
            if (o.x != kFar) {
                atomicMin(&box[0], max(o.x, 0));
                atomicMax(&box[1], min(o.x + K - 1, lw - 1));
                atomicMin(&box[2], max(o.y, 0));
                atomicMax(&box[3], min(o.y + K - 1, lh - 1));
            }
        }
        __syncthreads();
        const int bx0 = box[0], bx1 = box[1], by0 = box[2], by1 = box[3];
        if (bx0 > bx1) continue;                                     // uniform: nothing at this level
        // per target row of the box, the column extent of the record patches that cover it
        for (int i = tid; i <= by1 - by0; i += kBwdThreads) rowext[i] = make_int2(1 << 30, -(1 << 30));
        if (tid == 0) {
            bcur_row = by0;
            bcur_x = -1;
        }
        __syncthreads();
        for (int i = tid; i < nrec * kBwdQ; i += kBwdThreads) {
            const int2 o = sorg[i / kBwdQ][i % kBwdQ];
            if (o.x == kFar) continue;
            const int x0 = max(o.x, 0), x1 = min(o.x + K - 1, lw - 1);
            for (int j = max(o.y, 0); j <= min(o.y + K - 1, lh - 1); ++j) {
                atomicMin(&rowext[j - by0].x, x0);
                atomicMax(&rowext[j - by0].y, x1);
            }
        }
        const __bf16* plev = a.pt + ((size_t)b * g.TS + g.soff[l]) * ncg * unit;
        for (;;) {
            // ---- next band: up to kBwdSeg segments (row, 16-column segment) in row-major order -------
            __syncthreads();                                         // rowext ready / previous band's G reads done
            if (tid == 0) {
                // segments join in row-major order; a band holds at most kBwdSeg segments in at most
                // kBwdRows rows (consecutive segment columns within a row)
                int n = 0, nr = 0, ty = bcur_row, sx = bcur_x;   // sx < 0: start of row ty
                while (n < kBwdSeg && ty <= by1) {
                    const int2 e = rowext[ty - by0];
                    if (e.x > e.y) { ++ty; sx = -1; continue; }
                    if (sx < 0) sx = e.x >> 4;
                    if (sx > (e.y >> 4)) { ++ty; sx = -1; continue; }
                    if (nr == 0 || brow_y[nr - 1] != ty) {
                        if (nr == kBwdRows) break;
                        brow_y[nr] = ty;
                        brow_s0[nr] = n;
                        brow_x0[nr] = sx;
                        brow_n[nr] = 0;
                        ++nr;
                    }
                    bseg_row[n] = ty;
                    bseg_x[n] = sx;
                    ++brow_n[nr - 1];
                    ++n;
                    ++sx;
                }
                bnseg = n;
                bnrow = nr;
                bcur_row = ty;
                bcur_x = sx;
            }
            __syncthreads();
            const int nseg = bnseg, bnrow_ = bnrow;                  // uniform
            if (nseg == 0) break;
            // ---- G (queries x band targets): owner threads, records in order ----------------------
            // zero this thread's columns (band columns = p mod 4 of row gq_), then add every record's
            // patch weights that land in them
            float* grow = G + gq_ * kBwdLd;
            for (int c = p; c < kBwdTB; c += 4) grow[c] = 0.f;
            if (gvalid) {
                // records in batches of kRB: every weight load of a batch is issued before the first
                // add (one memory latency per batch, not one per record and row), then the adds in record
                // order (each G element receives at most one weight per record)
                constexpr int kRB = 4, KM = (K + 3) / 4;
                const size_t lofs = ((size_t)l * g.B + b) * K * K * N + qoff;
                for (int r0 = 0; r0 < nrec; r0 += kRB) {
                    float v[kRB][kBwdRows][KM];
#pragma unroll
                    for (int ri = 0; ri < kRB; ++ri) {
                        const int r = r0 + ri;
                        const int2 o = r < nrec ? sorg[r][gq_] : make_int2(kFar, kFar);
                        const float* wq = s_wp[r < nrec ? r : 0] + lofs;
                        const int k0 = (p - o.x) & 3;
#pragma unroll
                        for (int br = 0; br < kBwdRows; ++br) {
                            const int jr = brow_y[br] - o.y;
                            const bool rok = br < bnrow_ && o.x != kFar && jr >= 0 && jr < K;
#pragma unroll
                            for (int m = 0; m < KM; ++m) {
                                const int k = k0 + 4 * m;
                                const int tx = o.x + k;
                                const int si = (tx >> 4) - brow_x0[br];
                                const bool ok = rok && k < K && tx >= 0 && tx < lw && si >= 0 && si < brow_n[br];
                                v[ri][br][m] = ok ? (RMD_OTF_BWD_ABL == 2 ? 1e-3f * (float)(k + jr)
                                                                          : wq[(size_t)(jr * K + k) * N])
                                                  : 0.f;
                            }
                        }
                    }
#pragma unroll
                    for (int ri = 0; ri < kRB; ++ri) {
                        const int r = r0 + ri;
                        const int2 o = r < nrec ? sorg[r][gq_] : make_int2(kFar, kFar);
                        const int k0 = (p - o.x) & 3;
#pragma unroll
                        for (int br = 0; br < kBwdRows; ++br) {
                            const int jr = brow_y[br] - o.y;
                            const bool rok = br < bnrow_ && o.x != kFar && jr >= 0 && jr < K;
#pragma unroll
                            for (int m = 0; m < KM; ++m) {
                                const int k = k0 + 4 * m;
                                const int tx = o.x + k;
                                const int si = (tx >> 4) - brow_x0[br];
                                if (rok && k < K && tx >= 0 && tx < lw && si >= 0 && si < brow_n[br])
                                    grow[16 * (brow_s0[br] + si) + (tx & 15)] += v[ri][br][m];
                            }
                        }
                    }
                }
            }
            __syncthreads();
            // ---- d q~ += G . P_band (query tile mt, channel tiles nt0..nt0+ntn-1) ------------------
            // rolling fragment ring: channel tile t's fragments of segment s + 1 are loaded right after
            // its MFMAs of segment s (one buffer of 4 (x2) fragments, each load covered by the other
            // tiles' MFMAs)
            if (ntn > 0) {
                bf16x8 bh[4], bl[4];
                const size_t seg_unit = (size_t)ncg * unit;
                auto seg_ptr = [&](int s) {
                    return plev + (size_t)(bseg_row[s] * g.nsx[l] + bseg_x[s]) * seg_unit + lane * 8;
                };
                const __bf16* pu = seg_ptr(0);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const __bf16* pp = pu + (size_t)(nt0 + min(t, ntn - 1)) * unit;
                    bh[t] = *reinterpret_cast<const bf16x8*>(pp);
                    bl[t] = X3 ? *reinterpret_cast<const bf16x8*>(pp + 64 * 8) : bh[t];
                }
                for (int s = 0; s < nseg; ++s) {
                    const float* gr = G + (mt * 32 + j32) * kBwdLd + s * 16 + 8 * h;
                    float v[8];
                    *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(gr);
                    *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(gr + 4);
                    bf16x8 ah, al;
                    split8(v, ah, al);
                    const __bf16* pn = seg_ptr(min(s + 1, nseg - 1));
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (t < ntn) mma3<X3>(accq[t], ah, al, bh[t], bl[t]);
                        const __bf16* pp = pn + (size_t)(nt0 + min(t, ntn - 1)) * unit;
                        bh[t] = *reinterpret_cast<const bf16x8*>(pp);
                        bl[t] = X3 ? *reinterpret_cast<const bf16x8*>(pp + 64 * 8) : bh[t];
                    }
                }
            }
            // ---- d P_band = G^T . q~ (target tile mt = segments 2mt, 2mt+1), fixed-point atomics ----
            // in two passes of two channel tiles (32 accumulator registers instead of 64 beside accq)
            if (2 * mt < nseg) {
                for (int tp = 0; tp < 2; ++tp) {
                    const int t0 = 2 * tp;
                    if (t0 >= ntn) break;                            // uniform
                    f32x16 accp[2] = {f32x16{}, f32x16{}};
                    bf16x8 qh[2], ql[2];
                    auto load_q = [&](int qs, int t) {
                        const int cg = nt0 + min(t0 + t, ntn - 1);
                        if constexpr (X3) {
                            const int qrow = qy0 + (qs >> 1), qsx = (qx0 >> 4) + (qs & 1);
                            const bool ok = qrow < g.H && qsx < g.qnsx;
                            const __bf16* pp =
                                a.qt + ((size_t)(b * g.QS + (ok ? qrow * g.qnsx + qsx : 0)) * ncg + cg) * unit + lane * 8;
                            const bf16x8 z = {};
                            qh[t] = ok ? *reinterpret_cast<const bf16x8*>(pp) : z;
                            ql[t] = ok ? *reinterpret_cast<const bf16x8*>(pp + 64 * 8) : z;
                        } else {
                            qh[t] = *reinterpret_cast<const bf16x8*>(qimg + ((size_t)(qs * ncg + cg) * 64 + lane) * 8);
                            ql[t] = qh[t];
                        }
                    };
                    load_q(0, 0);
                    load_q(0, 1);
                    for (int ks = 0; ks < kBwdQ / 16; ++ks) {
                        float v[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] = G[(ks * 16 + 8 * h + e) * kBwdLd + mt * 32 + j32];
                        bf16x8 ah, al;
                        split8(v, ah, al);
#pragma unroll
                        for (int t = 0; t < 2; ++t) {
                            if (t0 + t < ntn) mma3<X3>(accp[t], ah, al, qh[t], ql[t]);
                            load_q(min(ks + 1, kBwdQ / 16 - 1), t);
                        }
                    }
                    // lane (channel j32, half h): register 4i + k is band target mt*32 + 8i + 4h + k
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int ch = (nt0 + t0 + t) * 32 + j32;
                        if (t0 + t >= ntn || ch >= g.C) continue;
#pragma unroll
                        for (int v = 0; v < 16; ++v) {
                            const int jt = mt * 32 + 8 * (v >> 2) + 4 * h + (v & 3);
                            const int s = jt >> 4;
                            if (s >= nseg) continue;
                            const int tx = bseg_x[s] * 16 + (jt & 15);
                            const float val = accp[t][v];
                            if (tx >= lw || val == 0.f || RMD_OTF_BWD_ABL == 1) continue;
                            const size_t e = ((size_t)b * a.pT + a.poff[l] + (size_t)bseg_row[s] * lw + tx) * g.C + ch;
                            if (__builtin_isfinite(val))
                                atomicAdd(reinterpret_cast<unsigned long long*>(a.dP + e),
                                          (unsigned long long)(long long)__builtin_rint((double)val * fscale));
                            else {
                                atomicAdd(a.dPnf + e, val);
                                *a.nf = 1;
                            }
                        }
                    }
                }
            }
        }
    }
    // ---- d fmap1 (planar) += scale * d q~: lane (channel j32, half h), register 4i + k = query x 8i+4h+k ----
    const int y = qy0 + mt;
    if (y < g.H) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (t >= ntn) break;
            const int ch = (nt0 + t) * 32 + j32;
            if (ch >= g.C) continue;
            float* o = a.gq + ((size_t)b * g.C + ch) * N + (size_t)y * g.W + qx0;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int x = 8 * (v >> 2) + 4 * h + (v & 3);
                if (qx0 + x < g.W) o[x] += a.scale * accq[t][v];
            }
        }
    }
}

// the largest recorded |weight| of up to 64 records (their kMaxSlots header words) -> *acc (one wave)
__global__ void otf_wmax_kernel(BwdWmax wm, int n, unsigned* __restrict__ acc) {
    unsigned m = 0;
    for (int i = 0; i < n; ++i) m = max(m, wm.p[i][threadIdx.x]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
    if (threadIdx.x == 0) atomicMax(acc, m);
}

// the fixed-point exponent of this backward's d P from the maxima (one wave)
__global__ void otf_fixed_exp_kernel(const unsigned* __restrict__ wmax, const unsigned* __restrict__ qmax, int nrec,
                                     long long N, int* __restrict__ sexp) {
    unsigned mq = qmax[threadIdx.x];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mq = max(mq, (unsigned)__shfl_xor((int)mq, o));
    const double bound = (double)nrec * (double)N * (double)__uint_as_float(*wmax) * (double)__uint_as_float(mq);
    if (threadIdx.x == 0) *sexp = fixed_exp(bound * 1.0001);
}

// d fmap2[b, c, y, x] = sum_l d P_l[b, (y >> l, x >> l), c] / 4^l over the floor-cropped part of each level
// (the transpose of l successive 2x2 average pools).  d P: fixed point in 2^-s units plus the
// non-finite side buffer (read only when *nf is set).  A 256-thread block takes 64 pixels x 64
// channels: reads run along the channels of d P's pixel-major rows, the transposed writes along the
// pixels of the planar output (through an LDS tile).
__global__ void __launch_bounds__(256)
otf_unpool_kernel(const long long* __restrict__ dP, const float* __restrict__ dPnf, const int* __restrict__ sexp,
                  const int* __restrict__ nf, OtfGeom g, long long pT, LevelOff po, float* __restrict__ gf2) {
    __shared__ float tile[64][65];
    const long long N = (long long)g.H * g.W;
    const long long p0 = (long long)blockIdx.x * 64;
    const int c0 = blockIdx.y * 64, b = blockIdx.z;
    const double inv = ldexp(1.0, -*sexp);
    const bool anynf = *nf != 0;
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int px = i >> 6, c = c0 + (i & 63);
        const long long p = p0 + px;
        float s = 0.f;
        if (p < N && c < g.C) {
            const int y = (int)(p / g.W), x = (int)(p % g.W);
#pragma unroll
            for (int l = 0; l < RMD_MAX_LEVELS; ++l) {
                if (l >= g.L) break;
                const int yy = y >> l, xx = x >> l;
                if (yy < g.lh[l] && xx < g.lw[l]) {
                    const size_t e = ((size_t)b * pT + po.o[l] + (size_t)yy * g.lw[l] + xx) * g.C + c;
                    const float v = (float)((double)dP[e] * inv) + (anynf ? dPnf[e] : 0.f);
                    s += v * (1.0f / (float)(1 << (2 * l)));
                }
            }
        }
        tile[px][i & 63] = s;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int c = c0 + (i >> 6), px = i & 63;
        const long long p = p0 + px;
        if (p < N && c < g.C) gf2[((size_t)b * g.C + c) * N + p] = tile[px][i >> 6];
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
    const size_t qn = otf_query_elems(g);
    // compiled channel counts keep the query segments in registers; f32 operands of >= 128 channels
    // would not fit and take the runtime loop
    const bool exact = compute == RMD_F32;
    const bool x3 = compute == RMD_BF16X3;
    const int cpt = (exact && g.Cp >= 128) || g.Cp > 256 ? 0 : g.Cp;
    // query block per compute: bf16 QSX_B x QSY_B segments, split-bf16 / f32 QSX_X x QSY_X (query
    // fragments in registers: 8 (bf16) / 16 (x3) load steps per segment at C = 256)
#define RMD_OTF(T, RR, CC, QX, QY, OC)                                                                         \
    do {                                                                                                       \
        using QB = QBlock<QX, QY>;                                                                             \
        auto k = otf_lookup_kernel<T, XS, RR, CC, QX, QY, OC, QLK, NTK>;                                        \
        const long long nblk = (long long)((width + QB::kBX - 1) / QB::kBX) * ((height + QB::kBY - 1) / QB::kBY) * batch; \
        RMD_REQUIRE(nblk < (1ll << 31), RMD_ERR_SHAPE, "rmd_corr_otf_lookup: grid too large");                  \
        const size_t lds = sizeof(float) * QB::kQ * otf_patch_stride(RR) +                      \
                           (QLK && CC > 0 ? (size_t)QB::kQS * 16 * CC * XN * sizeof(T) : 0);                    \
        RMD_REQUIRE(lds <= 160 * 1024, RMD_ERR_SHAPE, "rmd_corr_otf_lookup: %zu B of LDS per block", lds);      \
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)lds);                                                                   \
        const T* q = reinterpret_cast<const T*>(workspace);                                                    \
        k<<<(unsigned)nblk, NTK, lds, st>>>(q, q + qn * XN, g, coords, zero_level_mask, out);                   \
    } while (0)
#define RMD_OTF_C(T, RR, QX, QY, OC)                                 \
    switch (cpt) {                                                   \
        case 32: RMD_OTF(T, RR, 32, QX, QY, OC); break;              \
        case 64: RMD_OTF(T, RR, 64, QX, QY, OC); break;              \
        case 128: RMD_OTF(T, RR, 128, QX, QY, OC); break;            \
        case 256: RMD_OTF(T, RR, 256, QX, QY, OC); break;            \
        default: RMD_OTF(T, RR, 0, QX, QY, OC); break;               \
    }
#define RMD_OTF_R(T, QX, QY, OC)                                     \
    switch (radius) {                                                \
        case 1: RMD_OTF_C(T, 1, QX, QY, OC); break;                  \
        case 2: RMD_OTF_C(T, 2, QX, QY, OC); break;                  \
        case 3: RMD_OTF_C(T, 3, QX, QY, OC); break;                  \
        case 4: RMD_OTF_C(T, 4, QX, QY, OC); break;                  \
        case 5: RMD_OTF_C(T, 5, QX, QY, OC); break;                  \
        case 6: RMD_OTF_C(T, 6, QX, QY, OC); break;                  \
        case 7: RMD_OTF_C(T, 7, QX, QY, OC); break;                  \
        default: RMD_OTF_C(T, 8, QX, QY, OC); break;                 \
    }
    // bf16 on wide maps (at least kWideBlocks 16x2 query blocks): 16x4 blocks at 512 threads read 45 %
    // fewer target bytes per query; at the 4K map (b2, 270x480) 362 us vs 396 us per lookup, at cfg2
    // (1,792 blocks) 77 vs 73 us (profiles/otf_put_ab_r04.json, box r04t)
    const long long blocks16x2 = (long long)((width + 15) / 16) * ((height + 1) / 2) * batch;
    if (compute == RMD_BF16 && blocks16x2 >= kWideBlocks) {
        constexpr bool XS = false;
        constexpr size_t XN = 1;
        constexpr bool QLK = true;
        constexpr int NTK = RMD_OTF_WNT;
        RMD_OTF_R(__bf16, 1, RMD_OTF_WQY, RMD_OTF_WOCC)
    } else if (compute == RMD_BF16) {
        constexpr bool XS = false;
        constexpr size_t XN = 1;
        constexpr bool QLK = RMD_OTF_QL_B != 0;
        constexpr int NTK = RMD_OTF_NT_B;
        RMD_OTF_R(__bf16, RMD_OTF_QSX_B, RMD_OTF_QSY_B, RMD_OTF_OCC_B)
    } else if (x3) {
        constexpr bool XS = true;
        constexpr size_t XN = 2;                    // query segments: qn split pairs
        constexpr bool QLK = RMD_OTF_QL_X != 0;
        constexpr int NTK = RMD_OTF_NT_X;
        RMD_OTF_R(__bf16, RMD_OTF_QSX_X, RMD_OTF_QSY_X, RMD_OTF_OCC_X)
    } else {
        constexpr bool XS = false;
        constexpr size_t XN = 1;
        constexpr bool QLK = false;
        constexpr int NTK = 256;
        RMD_OTF_R(float, RMD_OTF_QSX_X, RMD_OTF_QSY_X, 1)
    }
#undef RMD_OTF_R
#undef RMD_OTF_C
#undef RMD_OTF
    return check_launch("rmd_corr_otf_lookup");
}

// ---- backward entry points -------------------------------------------------------------------------

namespace {

struct BwdLayout {
    OtfGeom g, gq;              // targets (all levels) / queries (level 0 of fmap1)
    size_t pt_off, qt_off, dp_off, nf_off, sc_off, total;
    long long pT;
    long long poff[RMD_MAX_LEVELS];
};

// workspace: target T layout | query T layout | d P fixed point (int64) | d P non-finite (float) |
// scalars (qmax, wmax, s)
BwdLayout bwd_layout(int B, int C, int H, int W, int L, int compute) {
    BwdLayout y{};
    y.g = make_otf_geom(B, C, H, W, L);
    y.gq = make_otf_geom(B, C, H, W, 1);
    y.g.Cp = y.gq.Cp = (C + 31) / 32 * 32;                // T layout: 32-channel groups
    y.g.QS = y.gq.TS;
    y.g.qnsx = y.gq.nsx[0];
    const size_t np = compute == RMD_BF16 ? 1 : 2;
    const size_t ncg = (size_t)y.g.Cp / 32;
    const size_t tbytes = (size_t)B * y.g.TS * ncg * 512 * np * 2, qbytes = (size_t)B * y.gq.TS * ncg * 512 * np * 2;
    long long p = 0;
    for (int l = 0; l < L; ++l) {
        y.poff[l] = p;
        p += (long long)y.g.lh[l] * y.g.lw[l];
    }
    y.pT = p;
    auto up = [](size_t v) { return (v + 255) / 256 * 256; };
    y.pt_off = 0;
    y.qt_off = up(tbytes);
    y.dp_off = y.qt_off + up(qbytes);
    y.nf_off = y.dp_off + up((size_t)B * p * C * sizeof(long long));
    y.sc_off = y.nf_off + up((size_t)B * p * C * sizeof(float));
    y.total = y.sc_off + 512;
    return y;
}

// LDS of otf_backward_kernel: dynamic (G, bf16 query image, per-row extents) + static (origins, box, band)
size_t bwd_lds_dynamic(int ncg, bool x3, int height) {
    return sizeof(float) * kBwdQ * kBwdLd + (x3 ? 0 : (size_t)8 * ncg * 1024) + sizeof(int2) * (size_t)height;
}
constexpr size_t kBwdLdsStatic = sizeof(int2) * kMaxRec * kBwdQ + sizeof(int) * (4 + 2 * kBwdSeg + 4 * kBwdRows + 4) +
                                 2 * sizeof(void*) * kMaxRec;

}  // namespace

extern "C" size_t rmd_corr_otf_record_bytes(int batch, int height, int width, int levels, int radius) {
    if (batch <= 0 || height <= 0 || width <= 0 || levels < 1 || levels > RMD_MAX_LEVELS || radius < 1 || radius > 8)
        return 0;
    const int K = 2 * radius + 2;
    // origins | weights | 256-B header (largest |weight|, for the fixed-point scale of the backward)
    return otf_record_org_bytes(batch, height, width, levels) + otf_record_wp_bytes(batch, height, width, levels, K) + 256;
}

extern "C" int rmd_corr_otf_record(const float* grad_out, const float* coords, int batch, int height, int width,
                                   int levels, int radius, unsigned zero_level_mask, void* record, void* stream) {
    RMD_REQUIRE(grad_out && coords && record, RMD_ERR_ARG, "rmd_corr_otf_record: null pointer");
    RMD_REQUIRE(rmd_corr_otf_record_bytes(batch, height, width, levels, radius) > 0, RMD_ERR_SHAPE,
                "rmd_corr_otf_record: bad sizes or radius %d not in 1..8", radius);
    const OtfGeom g = make_otf_geom(batch, 1, height, width, levels);
    const int K = 2 * radius + 2;
    int2* org = static_cast<int2*>(record);
    char* base = static_cast<char*>(record) + otf_record_org_bytes(batch, height, width, levels);
    float* wp = reinterpret_cast<float*>(base);
    unsigned* wmax = reinterpret_cast<unsigned*>(base + otf_record_wp_bytes(batch, height, width, levels, K));
    const long long n = (long long)levels * batch * height * width;
    const unsigned blocks = (unsigned)((n + kThreads - 1) / kThreads);
    hipStream_t st = as_stream(stream);
    if (hipMemsetAsync(wmax, 0, sizeof(unsigned) * kMaxSlots, st) != hipSuccess) {
        set_error("rmd_corr_otf_record: hipMemsetAsync failed");
        return RMD_ERR_LAUNCH;
    }
    switch (radius) {
#define RMD_CASE(RR) case RR: otf_record_kernel<RR><<<blocks, kThreads, 0, st>>>(grad_out, coords, g, zero_level_mask, org, wp, wmax); break;
        RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4) RMD_CASE(5) RMD_CASE(6) RMD_CASE(7) RMD_CASE(8)
#undef RMD_CASE
    }
    return check_launch("rmd_corr_otf_record");
}

extern "C" size_t rmd_corr_otf_backward_workspace_bytes(int batch, int channels, int height, int width, int levels,
                                                        int compute) {
    if (check_otf(batch, channels, height, width, levels, compute) || channels > 256) return 0;
    return bwd_layout(batch, channels, height, width, levels, compute).total;
}

extern "C" int rmd_corr_otf_backward(const float* fmap1, const float* fmap2, const void* otf_workspace, int batch,
                                     int channels, int height, int width, int levels, float scale, int compute,
                                     int radius, int nrecords, const void* const* records, float* grad_fmap1,
                                     float* grad_fmap2, void* workspace, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && otf_workspace && grad_fmap1 && grad_fmap2 && workspace && (records || nrecords == 0),
                RMD_ERR_ARG, "rmd_corr_otf_backward: null pointer");
    int rc = check_otf(batch, channels, height, width, levels, compute);
    if (rc) return rc;
    RMD_REQUIRE(channels <= 256, RMD_ERR_SHAPE, "rmd_corr_otf_backward: channels %d > 256", channels);
    RMD_REQUIRE(radius >= 1 && radius <= 8, RMD_ERR_SHAPE, "rmd_corr_otf_backward: radius %d not in 1..8", radius);
    for (int i = 0; i < nrecords; ++i)
        RMD_REQUIRE(records[i], RMD_ERR_ARG, "rmd_corr_otf_backward: null record %d", i);
    hipStream_t st = as_stream(stream);
    const BwdLayout y = bwd_layout(batch, channels, height, width, levels, compute);
    const bool x3 = compute != RMD_BF16;
    const int ncg = y.g.Cp / 32;
    // LDS per block (dynamic + static) against the 160 KiB of a CU, checked before any launch
    const size_t lds = bwd_lds_dynamic(ncg, x3, height);
    RMD_REQUIRE(lds + kBwdLdsStatic <= 160 * 1024, RMD_ERR_SHAPE,
                "rmd_corr_otf_backward: a %d-row map needs %zu B of LDS per block (dynamic %zu + static %zu) > 160 KiB",
                height, lds + kBwdLdsStatic, lds, kBwdLdsStatic);
    char* ws = static_cast<char*>(workspace);
    __bf16* pt = reinterpret_cast<__bf16*>(ws + y.pt_off);
    __bf16* qt = reinterpret_cast<__bf16*>(ws + y.qt_off);
    long long* dP = reinterpret_cast<long long*>(ws + y.dp_off);
    float* dPnf = reinterpret_cast<float*>(ws + y.nf_off);
    unsigned* qmax = reinterpret_cast<unsigned*>(ws + y.sc_off);     // kMaxSlots partial maxima
    unsigned* wmax = qmax + kMaxSlots;
    int* sexp = reinterpret_cast<int*>(qmax + kMaxSlots + 1);
    int* nf = sexp + 1;
    const size_t N = (size_t)height * width;
    if (hipMemsetAsync(grad_fmap1, 0, (size_t)batch * channels * N * sizeof(float), st) != hipSuccess ||
        hipMemsetAsync(dP, 0, (size_t)batch * y.pT * channels * sizeof(long long), st) != hipSuccess ||
        hipMemsetAsync(dPnf, 0, (size_t)batch * y.pT * channels * sizeof(float), st) != hipSuccess ||
        hipMemsetAsync(qmax, 0, 512, st) != hipSuccess) {
        set_error("rmd_corr_otf_backward: hipMemsetAsync failed");
        return RMD_ERR_LAUNCH;
    }
    // operands in the T layout: pooled targets from the forward workspace's fp32 levels, queries = fmap1 * scale
    {
        const OtfGeom gf = make_otf_geom(batch, channels, height, width, levels);
        const size_t es = compute == RMD_BF16 ? 2 : 4;
        const float* scratch = reinterpret_cast<const float*>(static_cast<const char*>(otf_workspace) +
                                                              otf_scratch_offset(gf, es));
        LevelSrc lt{}, lq{};
        lt.p[0] = fmap2;
        for (int l = 1; l < levels; ++l) {
            lt.p[l] = scratch;
            scratch += (size_t)batch * channels * gf.lh[l] * gf.lw[l];
        }
        lq.p[0] = fmap1;
        const long long nt = (long long)batch * y.g.TS * (y.g.Cp / 32) * 64;
        const long long nq = (long long)batch * y.gq.TS * (y.gq.Cp / 32) * 64;
        if (x3) {
            otf_tlayout_kernel<true><<<(unsigned)((nt + kThreads - 1) / kThreads), kThreads, 0, st>>>(lt, y.g, 1.0f, pt, nullptr);
            otf_tlayout_kernel<true><<<(unsigned)((nq + kThreads - 1) / kThreads), kThreads, 0, st>>>(lq, y.gq, scale, qt, qmax);
        } else {
            otf_tlayout_kernel<false><<<(unsigned)((nt + kThreads - 1) / kThreads), kThreads, 0, st>>>(lt, y.g, 1.0f, pt, nullptr);
            otf_tlayout_kernel<false><<<(unsigned)((nq + kThreads - 1) / kThreads), kThreads, 0, st>>>(lq, y.gq, scale, qt, qmax);
        }
        rc = check_launch("rmd_corr_otf_backward (operands)");
        if (rc) return rc;
    }
    // fixed-point exponent of d P from the largest recorded |weight| and |q~|
    const size_t obytes = otf_record_org_bytes(batch, height, width, levels);
    const size_t wbytes = otf_record_wp_bytes(batch, height, width, levels, 2 * radius + 2);
    for (int r0 = 0; r0 < nrecords; r0 += 64) {
        BwdWmax wm{};
        const int n = std::min(64, nrecords - r0);
        for (int i = 0; i < n; ++i)
            wm.p[i] = reinterpret_cast<const unsigned*>(static_cast<const char*>(records[r0 + i]) + obytes + wbytes);
        otf_wmax_kernel<<<1, kMaxSlots, 0, st>>>(wm, n, wmax);
    }
    otf_fixed_exp_kernel<<<1, kMaxSlots, 0, st>>>(wmax, qmax, std::max(nrecords, 1), (long long)N, sexp);
    rc = check_launch("rmd_corr_otf_backward (scale)");
    if (rc) return rc;
    const long long nblk = (long long)((width + kBwdQX - 1) / kBwdQX) * ((height + kBwdQY - 1) / kBwdQY) * batch;
    RMD_REQUIRE(nblk < (1ll << 31), RMD_ERR_SHAPE, "rmd_corr_otf_backward: grid too large");
    for (int r0 = 0; r0 < nrecords; r0 += kMaxRec) {
        BwdArgs a{};
        a.g = y.g;
        a.pt = pt;
        a.qt = qt;
        a.dP = dP;
        a.dPnf = dPnf;
        a.pT = y.pT;
        for (int l = 0; l < RMD_MAX_LEVELS; ++l) a.poff[l] = y.poff[l];
        a.gq = grad_fmap1;
        a.scale = scale;
        a.sexp = sexp;
        a.nf = nf;
        a.rec.n = std::min(kMaxRec, nrecords - r0);
        for (int i = 0; i < a.rec.n; ++i) {
            a.rec.org[i] = static_cast<const int2*>(records[r0 + i]);
            a.rec.wp[i] = reinterpret_cast<const float*>(static_cast<const char*>(records[r0 + i]) + obytes);
        }
#define RMD_BWD(XX, RR)                                                                                          \
        do {                                                                                                     \
            auto k = otf_backward_kernel<XX, RR>;                                                                \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                      (int)lds);                                                                 \
            k<<<(unsigned)nblk, kBwdThreads, lds, st>>>(a);                                                      \
        } while (0)
#define RMD_BWD_R(XX)                                                                                            \
        switch (radius) {                                                                                        \
            case 1: RMD_BWD(XX, 1); break;                                                                       \
            case 2: RMD_BWD(XX, 2); break;                                                                       \
            case 3: RMD_BWD(XX, 3); break;                                                                       \
            case 4: RMD_BWD(XX, 4); break;                                                                       \
            case 5: RMD_BWD(XX, 5); break;                                                                       \
            case 6: RMD_BWD(XX, 6); break;                                                                       \
            case 7: RMD_BWD(XX, 7); break;                                                                       \
            default: RMD_BWD(XX, 8); break;                                                                      \
        }
        if (x3) { RMD_BWD_R(true) } else { RMD_BWD_R(false) }
#undef RMD_BWD_R
#undef RMD_BWD
        rc = check_launch("rmd_corr_otf_backward");
        if (rc) return rc;
    }
    LevelOff po{};
    for (int l = 0; l < RMD_MAX_LEVELS; ++l) po.o[l] = y.poff[l];
    const dim3 ugrid((unsigned)((N + 63) / 64), (unsigned)((channels + 63) / 64), (unsigned)batch);
    otf_unpool_kernel<<<ugrid, 256, 0, st>>>(dP, dPnf, sexp, nf, y.g, y.pT, po, grad_fmap2);
    return check_launch("rmd_corr_otf_backward (unpool)");
}
