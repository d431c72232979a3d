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
// backward ablation for A/B timing only (wrong results): 1 = the dP atomic adds are skipped
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
//  * one 512-thread workgroup per 32 x 4 query tile; per level the union box of the tile's patches
//    over all records, swept in bands of one target row x kBwdTB columns;
//  * only the target rows some record patch covers are swept, each over its covered column extent;
//  * per band the dense G (128 queries x kBwdTB targets, fp32) is built in LDS, one thread per (query,
//    column) summing the records in order (deterministic);
//  * d q~ (128 queries x C) += G . P_band: v_mfma_f32_32x32x16_bf16 with A = G rows from LDS and B =
//    the band's targets in the "T layout" (lane c + 32h holds pixels 8h..8h+7 of channel c of a 16-pixel
//    segment: the B fragment of a 16-target k-step), accumulated in registers over all bands;
//  * d P_band (kBwdTB targets x C) = G^T . q~: A = G columns from LDS, B = the tile's queries in the T
//    layout; the 32 x 32 result tiles (fp32) are added to a pixel-major fp64 d P with float64 atomics:
//    the fp64 sum of fp32 tile sums is exact — so independent of the order the workgroups add in — as
//    long as a target's contributions span less than 2^29 in magnitude, and below that the fp64
//    rounding (2^-53) stays far under the fp32 result's ulp (run-to-run equal in the tests).
// fp32 modes split G and both operands into bf16 hi + lo and accumulate lo.hi + hi.lo + hi.hi (the
// forward x3 split); bf16 mode uses one product.
constexpr int kBwdQX = 32, kBwdQY = 4, kBwdQ = kBwdQX * kBwdQY;
constexpr int kBwdTB = 128;                          // band width (targets)
constexpr int kBwdLd = kBwdTB + 4;                   // G row stride (floats): conflict-free row and column reads
constexpr int kBwdThreads = 512;
constexpr int kMaxRec = 32;                          // records per launch (more: several launches)
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

// per (level, batch, query): origin and the (2r+2)^2 patch weights of grad_out's window
//   wp[j][k] = (1-fy) hx(k, j) + fy hx(k, j-1),  hx(k, bb) = (1-fx) g[k][bb] + fx g[k-1][bb]
// (g[a][bb] = grad_out channel l*D*D + a*D + bb; out-of-range a / bb -> 0).  Masked and 1-pixel levels
// record kFar (no contribution); a non-finite coordinate clamps far off the map (no contribution).
template <int R>
__global__ void __launch_bounds__(kThreads)
otf_record_kernel(const float* __restrict__ gout, const float* __restrict__ coords, OtfGeom g, unsigned zmask,
                  int2* __restrict__ org, float* __restrict__ wp) {
    constexpr int D = 2 * R + 1, K = 2 * R + 2;
    const long long N = (long long)g.H * g.W;
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= (long long)g.L * g.B * N) return;
    const int q = (int)(idx % N);
    const int b = (int)((idx / N) % g.B);
    const int l = (int)(idx / (N * g.B));
    const int lh = g.lh[l], lw = g.lw[l];
    const float x = coords[((size_t)b * 2 + 0) * N + q], y = coords[((size_t)b * 2 + 1) * N + q];
    const float inv = 1.0f / (float)(1 << l);
    const float rx = x * inv, ry = y * inv;
    const float cx = fminf(fmaxf(rx, -1.0e6f), 1.0e6f), cy = fminf(fmaxf(ry, -1.0e6f), 1.0e6f);
    const bool dead = ((zmask >> l) & 1u) || lh < 2 || lw < 2 || !(rx == rx) || !(ry == ry);
    org[idx] = dead ? make_int2(kFar, kFar) : make_int2((int)floorf(cx) - R, (int)floorf(cy) - R);
    const float fx = rx - floorf(rx), fy = ry - floorf(ry);
    const float* gp = gout + ((size_t)b * g.L + l) * D * D * N + q;
    float gv[D][D];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
        for (int bb = 0; bb < D; ++bb) gv[a][bb] = dead ? 0.f : gp[(size_t)(a * D + bb) * N];
    float* w = wp + ((size_t)l * g.B + b) * K * K * N + q;
#pragma unroll
    for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            auto hx = [&](int bb) {
                if (bb < 0 || bb >= D) return 0.f;
                const float v0 = k < D ? gv[k][bb] : 0.f, v1 = k >= 1 ? gv[k - 1][bb] : 0.f;
                return (1.f - fx) * v0 + fx * v1;
            };
            const float v = (1.f - fy) * hx(j) + fy * hx(j - 1);
            w[(size_t)(j * K + k) * N] = dead ? 0.f : v;
        }
    }
}

// T layout of a planar (B, C, h, w) fp32 map (times s): unit (b, level segment row/seg, channel group cg)
// = 64 lanes x 8 elements, lane c + 32h = pixels 8h..8h+7 of channel 32cg + c (zero past the map / C);
// X3: the unit's lo half follows its hi half.  One thread per (unit, lane).
template <bool X3>
__global__ void __launch_bounds__(kThreads)
otf_tlayout_kernel(LevelSrc src, OtfGeom g, float s, __bf16* __restrict__ dst) {
    constexpr int NP = X3 ? 2 : 1;
    const int ncg = g.Cp / 32;
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= (long long)g.B * g.TS * ncg * 64) return;
    const int lane = (int)(idx & 63), c32 = lane & 31, h = lane >> 5;
    const long long u = idx >> 6;
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
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float v = (c < g.C && x0 + e < g.lw[l]) ? row[x0 + e] * s : 0.f;
        hi[e] = (__bf16)v;
        lo[e] = (__bf16)(v - (float)hi[e]);
    }
    __bf16* o = dst + ((size_t)u * NP * 64 + lane) * 8;
    *reinterpret_cast<bf16x8*>(o) = hi;
    if constexpr (X3) *reinterpret_cast<bf16x8*>(o + 64 * 8) = lo;
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
    double* dP;                 // (B, PT, C) pixel-major fp64, += G^T q~ (fp32 tile sums added in fp64)
    long long pT;               // pooled pixels per batch (all levels)
    long long poff[RMD_MAX_LEVELS];
    float* gq;                  // (B, C, H, W) fp32, += scale * G P
    float scale;
};

template <bool X3, int R>
__global__ void __launch_bounds__(kBwdThreads, 1)
otf_backward_kernel(BwdArgs a) {
    constexpr int K = 2 * R + 2;
    constexpr int NP = X3 ? 2 : 1;
    extern __shared__ float G[];                                     // [kBwdQ][kBwdLd], then rowext
    int2* rowext = reinterpret_cast<int2*>(G + kBwdQ * kBwdLd);      // [level-0 rows]
    __shared__ int2 sorg[kMaxRec][kBwdQ];
    __shared__ int box[4];
    const OtfGeom& g = a.g;
    const int N = g.H * g.W;
    const int nbx = (g.W + kBwdQX - 1) / kBwdQX, nqb = nbx * ((g.H + kBwdQY - 1) / kBwdQY);
    const int lid = xcd_block(blockIdx.x, gridDim.x);
    const int qb = lid % nqb, b = lid / nqb;
    const int qx0 = (qb % nbx) * kBwdQX, qy0 = (qb / nbx) * kBwdQY;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j32 = lane & 31, h = lane >> 5;
    const int ncg = g.Cp / 32;
    const int mt = w & 3;                                            // query row / target tile of this wave
    const int nt0 = (w >> 2) * 4;                                    // first channel tile of this wave
    const int ntn = max(0, min(4, ncg - nt0));
    const size_t unit = (size_t)64 * 8 * NP;                         // elements per T-layout unit

    f32x16 accq[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) accq[t] = f32x16{};

    for (int l = 0; l < g.L; ++l) {
        const int lh = g.lh[l], lw = g.lw[l];
        // ---- origins of every record for the tile's queries, and their union box at this level ----
        __syncthreads();                                             // previous level's G / sorg reads done
        if (tid < 4) box[tid] = (tid & 1) ? -(1 << 30) : (1 << 30);
        __syncthreads();
        for (int i = tid; i < a.rec.n * kBwdQ; i += kBwdThreads) {
            const int r = i / kBwdQ, q = i % kBwdQ;
            const int y = qy0 + q / kBwdQX, x = qx0 + q % kBwdQX;
            int2 o = make_int2(kFar, kFar);
            if (y < g.H && x < g.W) o = a.rec.org[r][((size_t)l * g.B + b) * N + y * g.W + x];
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
        // per target row of the box, the column extent of the record patches that cover it: bands of
        // rows (and columns) no patch touches are skipped, so a divergent flow costs its patches' rows,
        // not the whole union box
        for (int i = tid; i <= by1 - by0; i += kBwdThreads) rowext[i] = make_int2(1 << 30, -(1 << 30));
        __syncthreads();
        for (int i = tid; i < a.rec.n * kBwdQ; i += kBwdThreads) {
            const int2 o = sorg[i / kBwdQ][i % kBwdQ];
            if (o.x == kFar) continue;
            const int x0 = max(o.x, 0), x1 = min(o.x + K - 1, lw - 1);
            for (int j = max(o.y, 0); j <= min(o.y + K - 1, lh - 1); ++j) {
                atomicMin(&rowext[j - by0].x, x0);
                atomicMax(&rowext[j - by0].y, x1);
            }
        }
        __syncthreads();
        const __bf16* plev = a.pt + ((size_t)b * g.TS + g.soff[l]) * ncg * unit;
        for (int ty = by0; ty <= by1; ++ty) {
            const int2 ext = rowext[ty - by0];                       // uniform
            if (ext.x > ext.y) continue;
            for (int cx = ext.x & ~15; cx <= ext.y; cx += kBwdTB) {
                const int ncols = min(kBwdTB, ((ext.y - cx + 1) + 15) & ~15);
                // ---- G (queries x band targets) from every record's patch row ty -----------------------
                // one thread per (query, column) sums the records in order: deterministic, no atomics;
                // columns up to the next multiple of 32 are written (zero) for the 32-wide dP tiles
                __syncthreads();                                     // previous band's G reads done
                const int ncols32 = (ncols + 31) & ~31;
                for (int i = tid; i < kBwdQ * ncols32; i += kBwdThreads) {
                    const int col = i % ncols32, q = i / ncols32;
                    const int tx = cx + col;
                    float sum = 0.f;
                    if (col < ncols && tx < lw) {
                        const size_t qoff = (size_t)(qy0 + q / kBwdQX) * g.W + qx0 + q % kBwdQX;
                        for (int r = 0; r < a.rec.n; ++r) {
                            const int2 o = sorg[r][q];
                            const int j = ty - o.y, k = tx - o.x;
                            if (o.x != kFar && j >= 0 && j < K && k >= 0 && k < K)
                                sum += a.rec.wp[r][(((size_t)l * g.B + b) * K * K + j * K + k) * N + qoff];
                        }
                    }
                    G[q * kBwdLd + col] = sum;
                }
                __syncthreads();
                // ---- d q~ += G . P_band (query tile mt, channel tiles nt0..nt0+ntn-1) ------------------
                for (int ks = 0; ks < ncols / 16; ++ks) {
                    const float* gr = G + (mt * 32 + j32) * kBwdLd + ks * 16 + 8 * h;
                    float v[8];
                    *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(gr);
                    *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(gr + 4);
                    bf16x8 ah, al;
                    split8(v, ah, al);
                    const __bf16* pu = plev + ((size_t)(ty * g.nsx[l] + (cx >> 4) + ks) * ncg) * unit + lane * 8;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (t >= ntn) break;
                        const __bf16* pp = pu + (size_t)(nt0 + t) * unit;
                        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(pp);
                        const bf16x8 bl = X3 ? *reinterpret_cast<const bf16x8*>(pp + 64 * 8) : bh;
                        mma3<X3>(accq[t], ah, al, bh, bl);
                    }
                }
                // ---- d P_band = G^T . q~ (target tile mt, channel tiles nt0..), float atomics ------------
                if (mt * 32 < ncols && ntn > 0) {
                    f32x16 accp[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) accp[t] = f32x16{};
                    for (int ks = 0; ks < kBwdQ / 16; ++ks) {
                        const int qrow = qy0 + (ks >> 1);
                        if (qrow >= g.H) break;                      // uniform
                        float v[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] = G[(ks * 16 + 8 * h + e) * kBwdLd + mt * 32 + j32];
                        bf16x8 ah, al;
                        split8(v, ah, al);
                        const int qsx = (qx0 >> 4) + (ks & 1);
                        if (qsx >= g.qnsx) continue;                 // uniform: a segment past the map's width
                        const __bf16* qu = a.qt + ((size_t)(b * g.QS + qrow * g.qnsx + qsx) * ncg) * unit + lane * 8;
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            if (t >= ntn) break;
                            const __bf16* pp = qu + (size_t)(nt0 + t) * unit;
                            const bf16x8 bh = *reinterpret_cast<const bf16x8*>(pp);
                            const bf16x8 bl = X3 ? *reinterpret_cast<const bf16x8*>(pp + 64 * 8) : bh;
                            mma3<X3>(accp[t], ah, al, bh, bl);
                        }
                    }
                    // lane (channel j32, half h): register 4i + k is target column mt*32 + 8i + 4h + k
                    double* drow = a.dP + ((size_t)b * a.pT + a.poff[l] + (size_t)ty * lw) * g.C;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (t >= ntn) break;
                        const int ch = (nt0 + t) * 32 + j32;
#pragma unroll
                        for (int v = 0; v < 16; ++v) {
                            const int col = mt * 32 + 8 * (v >> 2) + 4 * h + (v & 3);
                            const int tx = cx + col;
                            if (col < ncols && tx <= ext.y && ch < g.C &&
                                (RMD_OTF_BWD_ABL == 0 || accp[t][v] == 1.2345e30f))      // ablation: no adds
                                atomicAdd(drow + (size_t)tx * g.C + ch, (double)accp[t][v]);
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

// d fmap2[b, c, y, x] = sum_l d P_l[b, (y >> l, x >> l), c] / 4^l over the floor-cropped part of each level
// (the transpose of l successive 2x2 average pools); one thread per (b, y, x, c), channel fastest.
__global__ void __launch_bounds__(kThreads)
otf_unpool_kernel(const double* __restrict__ dP, OtfGeom g, long long pT, LevelOff po, float* __restrict__ gf2) {
    const long long N = (long long)g.H * g.W;
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= (long long)g.B * N * g.C) return;
    const int c = (int)(idx % g.C);
    const long long p = (idx / g.C) % N;
    const int b = (int)(idx / ((long long)g.C * N));
    const int y = (int)(p / g.W), x = (int)(p % g.W);
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < RMD_MAX_LEVELS; ++l) {
        if (l >= g.L) break;
        const int yy = y >> l, xx = x >> l;
        if (yy < g.lh[l] && xx < g.lw[l])
            s += (float)dP[((size_t)b * pT + po.o[l] + (size_t)yy * g.lw[l] + xx) * g.C + c] * (1.0f / (float)(1 << (2 * l)));
    }
    gf2[((size_t)b * g.C + c) * N + p] = s;
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
    size_t pt_off, qt_off, dp_off, total;
    long long pT;
    long long poff[RMD_MAX_LEVELS];
};

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
    y.pt_off = 0;
    y.qt_off = (tbytes + 255) / 256 * 256;
    y.dp_off = y.qt_off + (qbytes + 255) / 256 * 256;
    y.total = y.dp_off + (size_t)B * p * C * sizeof(double);
    return y;
}

}  // namespace

extern "C" size_t rmd_corr_otf_record_bytes(int batch, int height, int width, int levels, int radius) {
    if (batch <= 0 || height <= 0 || width <= 0 || levels < 1 || levels > RMD_MAX_LEVELS || radius < 1 || radius > 8)
        return 0;
    const size_t K = 2 * radius + 2;
    return otf_record_org_bytes(batch, height, width, levels) + (size_t)levels * batch * height * width * K * K * sizeof(float);
}

extern "C" int rmd_corr_otf_record(const float* grad_out, const float* coords, int batch, int height, int width,
                                   int levels, int radius, unsigned zero_level_mask, void* record, void* stream) {
    RMD_REQUIRE(grad_out && coords && record, RMD_ERR_ARG, "rmd_corr_otf_record: null pointer");
    RMD_REQUIRE(rmd_corr_otf_record_bytes(batch, height, width, levels, radius) > 0, RMD_ERR_SHAPE,
                "rmd_corr_otf_record: bad sizes or radius %d not in 1..8", radius);
    const OtfGeom g = make_otf_geom(batch, 1, height, width, levels);
    int2* org = static_cast<int2*>(record);
    float* wp = reinterpret_cast<float*>(static_cast<char*>(record) + otf_record_org_bytes(batch, height, width, levels));
    const long long n = (long long)levels * batch * height * width;
    const unsigned blocks = (unsigned)((n + kThreads - 1) / kThreads);
    hipStream_t st = as_stream(stream);
    switch (radius) {
#define RMD_CASE(RR) case RR: otf_record_kernel<RR><<<blocks, kThreads, 0, st>>>(grad_out, coords, g, zero_level_mask, org, wp); break;
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
    hipStream_t st = as_stream(stream);
    const BwdLayout y = bwd_layout(batch, channels, height, width, levels, compute);
    const bool x3 = compute != RMD_BF16;
    char* ws = static_cast<char*>(workspace);
    __bf16* pt = reinterpret_cast<__bf16*>(ws + y.pt_off);
    __bf16* qt = reinterpret_cast<__bf16*>(ws + y.qt_off);
    double* dP = reinterpret_cast<double*>(ws + y.dp_off);
    const size_t N = (size_t)height * width;
    if (hipMemsetAsync(grad_fmap1, 0, (size_t)batch * channels * N * sizeof(float), st) != hipSuccess ||
        hipMemsetAsync(dP, 0, (size_t)batch * y.pT * channels * sizeof(double), st) != hipSuccess) {
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
            otf_tlayout_kernel<true><<<(unsigned)((nt + kThreads - 1) / kThreads), kThreads, 0, st>>>(lt, y.g, 1.0f, pt);
            otf_tlayout_kernel<true><<<(unsigned)((nq + kThreads - 1) / kThreads), kThreads, 0, st>>>(lq, y.gq, scale, qt);
        } else {
            otf_tlayout_kernel<false><<<(unsigned)((nt + kThreads - 1) / kThreads), kThreads, 0, st>>>(lt, y.g, 1.0f, pt);
            otf_tlayout_kernel<false><<<(unsigned)((nq + kThreads - 1) / kThreads), kThreads, 0, st>>>(lq, y.gq, scale, qt);
        }
        rc = check_launch("rmd_corr_otf_backward (operands)");
        if (rc) return rc;
    }
    const long long nblk = (long long)((width + kBwdQX - 1) / kBwdQX) * ((height + kBwdQY - 1) / kBwdQY) * batch;
    RMD_REQUIRE(nblk < (1ll << 31), RMD_ERR_SHAPE, "rmd_corr_otf_backward: grid too large");
    const size_t lds = sizeof(float) * kBwdQ * kBwdLd + sizeof(int2) * height;     // G + per-row extents
    const size_t obytes = otf_record_org_bytes(batch, height, width, levels);
    for (int r0 = 0; r0 < nrecords; r0 += kMaxRec) {
        BwdArgs a{};
        a.g = y.g;
        a.pt = pt;
        a.qt = qt;
        a.dP = dP;
        a.pT = y.pT;
        for (int l = 0; l < RMD_MAX_LEVELS; ++l) a.poff[l] = y.poff[l];
        a.gq = grad_fmap1;
        a.scale = scale;
        a.rec.n = std::min(kMaxRec, nrecords - r0);
        for (int i = 0; i < a.rec.n; ++i) {
            RMD_REQUIRE(records[r0 + i], RMD_ERR_ARG, "rmd_corr_otf_backward: null record %d", r0 + i);
            a.rec.org[i] = static_cast<const int2*>(records[r0 + i]);
            a.rec.wp[i] = reinterpret_cast<const float*>(static_cast<const char*>(records[r0 + i]) + obytes);
        }
#define RMD_BWD(XX, RR)                                                                                          \
        do {                                                                                                     \
            auto k = otf_backward_kernel<XX, RR>;                                                                \
            RMD_REQUIRE(lds <= 160 * 1024, RMD_ERR_SHAPE, "rmd_corr_otf_backward: %zu B of LDS per block", lds);    \
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
    const long long n2 = (long long)batch * N * channels;
    otf_unpool_kernel<<<(unsigned)((n2 + kThreads - 1) / kThreads), kThreads, 0, st>>>(dP, y.g, y.pT, po, grad_fmap2);
    return check_launch("rmd_corr_otf_backward (unpool)");
}
