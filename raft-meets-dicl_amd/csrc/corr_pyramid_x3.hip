// corr_pyramid_x3.hip — fp32-accurate correlation GEMM + fused pooled pyramid from split-bf16 MFMAs.
//
// Replaces raft.CorrBlock.__init__ (qzed/raft-meets-dicl src/models/impls/raft.py:18-47) in the
// fp32 parity mode.  The reference computes the volume in fp32 (raft.py:31-33, fmaps .float() at
// :381); exact f32 MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate, so each operand is
// split x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (16 significant bits together) and
//   corr = A_hi.B_hi + A_hi.B_lo + A_lo.B_hi        (the dropped lo.lo term is ~2^-16 relative)
// runs as three v_mfma_f32_32x32x16_bf16 per k-step into one fp32 accumulator: 3/16 of the exact-
// f32 MFMA cost.  The 1/sqrt(C) scale is folded into fmap2 before the split (fp32 multiply).
//
// Geometry: one workgroup (8 waves, two per SIMD) owns an 8 x 16 block of target
// pixels — both split halves of its A operand sit in LDS as one 1072-B row per target (hi 512 B,
// lo 512 B, 48 B pad; 1072 = 67 x 16 B, so a ds_read_b128 lane group's 16 consecutive rows hit 16
// distinct 16-B bank slots, see w8::pad_row in corr_pyramid.hip) — and each wave sweeps its own
// 32-query tiles: 4 MFMA tiles (4 x 8 targets each) x 16 k-steps x 3 products = 192 MFMAs, then
// pools in-lane and stores all four fp32 levels straight from the accumulators with range-checked
// buffer stores (rows past the level fall outside the descriptor, chunks past the row get a 1 GiB
// bias).  fp32 level-0 chunks are 32 B per query, so lane h of a query writes bytes 16h..16h+15 and
// every level-0 store instruction is one contiguous 1 KiB run without a lane exchange.

#include "rmd_common.h"
#include "corr_x3.h"

namespace rmd {
namespace x3 {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) float f32x8;
#ifndef RMD_X3_S16TEST
#define RMD_X3_S16TEST 0
#endif
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(2))) int i32x2;

constexpr int kRow = 1072;                  // LDS bytes per target row: hi 512 + lo 512 + 48 pad
constexpr int kBlockRows = 8, kBlockCols = 16;
constexpr unsigned kBig = 0x40000000u;      // offset bias beyond every level's range

// LDS row of block target (y 0..7, x 0..15): tile (rg = y>>2, cg = x>>3) holds rows
// cg*64 + rg*32 + (y&3)*8 + (x&7), i.e. lane j of an MFMA tile reads row base + j.
__device__ __forceinline__ int lds_row(int y, int x) { return ((x >> 3) << 6) + (y << 3) + (x & 7); }

__device__ __forceinline__ __bf16 hi_part(float v) { return (__bf16)v; }
__device__ __forceinline__ __bf16 lo_part(float v) { return (__bf16)(v - (float)(__bf16)v); }

// ---- operand prep: both feature maps, split, in one launch ------------------------------------
// grid (128-pixel tiles, B, 2).  z = 0: fmap2 * scale -> A hi / lo, pixel-major (B, N, 256);
// z = 1: fmap1 -> B hi / lo in MFMA B-fragment order o[b][qt][s][lane][8] (lane = j + 32h: channels
// 16s + 8h .. +7 of query min(32 qt + j, N - 1)).  Read phase as prep_pair (float4 per channel row),
// hi and lo tiles staged in LDS, one 16-B chunk per lane-store on the write side.
constexpr int kPx = 128, kStride = 256 * 2 + 16;

template <bool S16>
__global__ void __launch_bounds__(512)
prep_split(const float* __restrict__ f1, const float* __restrict__ f2, __bf16* __restrict__ aHi,
           __bf16* __restrict__ aLo, __bf16* __restrict__ bHi, __bf16* __restrict__ bLo, int C, int N, int nqt,
           float scale) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned char* tHi = lds;
    unsigned char* tLo = lds + kPx * kStride;
    const int b = blockIdx.y, which = blockIdx.z;
    const float* f = which ? f1 : f2;
    const float s = which ? 1.0f : scale;
    const int t = threadIdx.x;
    const int p0 = blockIdx.x * kPx;
    const bool full = p0 + kPx <= N && (N & 3) == 0;
    const int pl = N - 1 - p0;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int item = it * 512 + t;               // (channel octet cg, pixel quad q), q fastest
        const int q = item & 31, cg = item >> 5;
        float v[8][4];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = cg * 8 + e;
            const float* src = f + ((size_t)b * C + c) * N + p0 + 4 * q;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (c < C) {
                if (full) {
                    x = *reinterpret_cast<const float4*>(src);
                } else {
                    x.x = src[min(4 * q + 0, pl) - 4 * q];
                    x.y = src[min(4 * q + 1, pl) - 4 * q];
                    x.z = src[min(4 * q + 2, pl) - 4 * q];
                    x.w = src[min(4 * q + 3, pl) - 4 * q];
                }
            }
            v[e][0] = x.x * s;
            v[e][1] = x.y * s;
            v[e][2] = x.z * s;
            v[e][3] = x.w * s;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bf16x8 hi, lo;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                hi[e] = hi_part(v[e][i]);
                lo[e] = lo_part(v[e][i]);
            }
            *reinterpret_cast<bf16x8*>(tHi + (size_t)(4 * q + i) * kStride + cg * 16) = hi;
            *reinterpret_cast<bf16x8*>(tLo + (size_t)(4 * q + i) * kStride + cg * 16) = lo;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int k = it * 512 + t;                  // 16-B output chunk of the tile's 64 KiB block
        int px, c0;
        if (which && S16) {
            // 16x16x32 B fragments: 16-query tile t16 = k >> 9, k-step (32 channels) st, lane n + 16 g
            const int L = k & 63, st = (k >> 6) & 7;
            px = (k >> 9) * 16 + (L & 15);
            c0 = 32 * st + 8 * (L >> 4);
        } else if (which) {
            const int L = k & 63, st = (k >> 6) & 15;
            px = (k >> 10) * 32 + (L & 31);
            c0 = 16 * st + 8 * (L >> 5);
        } else {
            px = k >> 5;
            c0 = (k & 31) * 8;
        }
        const bf16x8 hi = *reinterpret_cast<const bf16x8*>(tHi + (size_t)px * kStride + c0 * 2);
        const bf16x8 lo = *reinterpret_cast<const bf16x8*>(tLo + (size_t)px * kStride + c0 * 2);
        if (which && S16) {
            const int t16 = blockIdx.x * 8 + (k >> 9);
            if (t16 < 2 * nqt) {
                const size_t o = (((size_t)b * 2 * nqt + t16) * 512 + (k & 511)) * 8;
                *reinterpret_cast<bf16x8*>(bHi + o) = hi;
                *reinterpret_cast<bf16x8*>(bLo + o) = lo;
            }
        } else if (which) {
            const int qt = blockIdx.x * 4 + (k >> 10);
            if (qt < nqt) {
                const size_t o = (((size_t)b * nqt + qt) * 1024 + (k & 1023)) * 8;
                *reinterpret_cast<bf16x8*>(bHi + o) = hi;
                *reinterpret_cast<bf16x8*>(bLo + o) = lo;
            }
        } else if (p0 + px < N) {
            const size_t o = ((size_t)b * N + p0) * 256 + (size_t)k * 8;
            *reinterpret_cast<bf16x8*>(aHi + o) = hi;
            *reinterpret_cast<bf16x8*>(aLo + o) = lo;
        }
    }
}

// ---- store descriptors -------------------------------------------------------------------------
struct Lvl {
    __amdgpu_buffer_rsrc_t rsrc;
    unsigned rs;      // row stride (bytes)
    unsigned cs;      // chunk stride (bytes)
    int rows;         // valid rows of this block on the level
    int chunks;       // valid chunks of this block's rows (level 0: 0..2, others 0..1)
    unsigned a;       // base address mod 4 (S24 level 3 aligns its word store with it)
};

__device__ __forceinline__ unsigned soff(const Lvl& L, int row, int chunk) {
    return (row < L.rows && chunk < L.chunks) ? (unsigned)row * L.rs + (unsigned)chunk * L.cs : kBig;
}

__device__ __forceinline__ void swap32(unsigned& x, unsigned& y) {
    auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    x = r[0];
    y = r[1];
}

__device__ __forceinline__ void swapf(float& x, float& y) {
    unsigned a = __float_as_uint(x), b = __float_as_uint(y);
    swap32(a, b);
    x = __uint_as_float(a);
    y = __uint_as_float(b);
}

constexpr int AUX_NT = 2;     // non-temporal stores: the pyramid is re-read a whole GEMM later

typedef __attribute__((ext_vector_type(3))) int i32x3;
// RMD_S24 (include/rmd.h): a float rounded to its top 24 bits (round half away from zero on the
// magnitude; a NaN stays a quiet NaN), kept in bytes 1..3 of the returned word
__device__ __forceinline__ unsigned s24_round(float v) {
    const unsigned u = __float_as_uint(v);
    return (u & 0x7fffffffu) > 0x7f800000u ? (u | 0x00400000u) : u + 0x80u;
}
// 4 floats -> the 12 bytes of their S24 values (3 words)
__device__ __forceinline__ i32x3 pack24(float a, float b, float c, float d) {
    const unsigned v0 = s24_round(a), v1 = s24_round(b), v2 = s24_round(c), v3 = s24_round(d);
    return i32x3{(int)__builtin_amdgcn_perm(v1, v0, 0x05030201u), (int)__builtin_amdgcn_perm(v2, v1, 0x06050302u),
                 (int)__builtin_amdgcn_perm(v3, v2, 0x07060503u)};
}

// Epilogue of one 32-query tile (32x32x16 form, F32 storage): acc[ti] (ti = 2 rg + cg) holds, for
// lane (j, h), the targets (row 4 rg + k, col 8 cg + 4 h + e) at acc[ti][4k + e].
__device__ __forceinline__ void epilogue(const f32x16 (&acc)[4], const Lvl (&L)[4], int q, int h) {
    const unsigned qo[4] = {(unsigned)q * 32u + 16u * h, (unsigned)q * 32u + 16u * h, (unsigned)q * 16u + 8u * h,
                            (unsigned)q * 8u + 4u * h};
    // level 0: 16 stores of 16 B (row 4rg + k, chunk cg, bytes 16h..)
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const i32x4 d = {__float_as_int(acc[ti][4 * k + 0]), __float_as_int(acc[ti][4 * k + 1]),
                             __float_as_int(acc[ti][4 * k + 2]), __float_as_int(acc[ti][4 * k + 3])};
            __builtin_amdgcn_raw_buffer_store_b128(d, L[0].rsrc, (int)(qo[0] + soff(L[0], 4 * (ti >> 1) + k, ti & 1)),
                                                   0, AUX_NT);
        }
    // level 1: tile rows (2m, 2m+1) -> level-1 row 2rg + m; lane pair u -> block col 4cg + 2h + u
    float s2[2][2];      // level-2 sums [rg][cg] (16 level-0 values each)
#pragma unroll
    for (int rg = 0; rg < 2; ++rg) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            float p[2][2];       // [cg][u]
#pragma unroll
            for (int cg = 0; cg < 2; ++cg)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const f32x16& a = acc[2 * rg + cg];
                    p[cg][u] = (a[4 * (2 * m) + 2 * u] + a[4 * (2 * m) + 2 * u + 1]) +
                               (a[4 * (2 * m + 1) + 2 * u] + a[4 * (2 * m + 1) + 2 * u + 1]);
                }
#pragma unroll
            for (int cg = 0; cg < 2; ++cg) {
                const float t = p[cg][0] + p[cg][1];
                s2[rg][cg] = m == 0 ? t : s2[rg][cg] + t;
            }
            // lower lanes keep cols {0,1} and receive {2,3}; upper lanes receive {4,5}, keep {6,7}
            float x0 = p[0][0], x1 = p[0][1], y0 = p[1][0], y1 = p[1][1];
            swapf(x0, y0);
            swapf(x1, y1);
            const i32x4 d = {__float_as_int(0.25f * x0), __float_as_int(0.25f * x1), __float_as_int(0.25f * y0),
                             __float_as_int(0.25f * y1)};
            __builtin_amdgcn_raw_buffer_store_b128(d, L[1].rsrc, (int)(qo[1] + soff(L[1], 2 * rg + m, 0)), 0, AUX_NT);
        }
    }
    // level 2: row rg, lane holds col h (cg 0) and 2 + h (cg 1); after the swap lower = {0,1}, upper = {2,3}
#pragma unroll
    for (int rg = 0; rg < 2; ++rg) {
        float x = s2[rg][0], y = s2[rg][1];
        swapf(x, y);
        const i32x2 d = {__float_as_int(0.0625f * x), __float_as_int(0.0625f * y)};
        __builtin_amdgcn_raw_buffer_store_b64(d, L[2].rsrc, (int)(qo[2] + soff(L[2], rg, 0)), 0, AUX_NT);
    }
    // level 3: one row, col cg = both tile rows and both lane halves of column group cg
    {
        float x = s2[0][0] + s2[1][0], y = s2[0][1] + s2[1][1];
        swapf(x, y);         // lower: own + upper's col-0 partial; upper: lower's + own col-1 partial
        const float v = (1.0f / 64.0f) * (x + y);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v), L[3].rsrc, (int)(qo[3] + soff(L[3], 0, 0)), 0,
                                              AUX_NT);
    }
}

// A/B knobs (tools/build_variant.sh -D...; the product build uses the defaults): RMD_X3_ABL = the
// kernel's ABL, RMD_X3_PP = ping-pong phases, RMD_X3_BHOT = 1 reads every B fragment from query tile 0
// (an L2-resident B stream; wrong results, timing only)
#ifndef RMD_X3_ABL
#define RMD_X3_ABL 0
#endif
#ifndef RMD_X3_PP
#define RMD_X3_PP 1
#endif
#ifndef RMD_X3_BHOT
#define RMD_X3_BHOT 0
#endif
#define X3_TILE(t) (RMD_X3_BHOT ? (size_t)0 : (size_t)(t) * 8192)

constexpr int kEpiStores = 24;  // buffer stores of one epilogue (23 in the .s), for vmcnt_pad_n
constexpr int kRing = 8;     // B ring slots (16 % kRing == 0: k-step s of every tile maps to slot s % kRing)

// A fragments (hi in [2ti], lo in [2ti+1]) of k-step S for the 4 target tiles
template <int S>
__device__ __forceinline__ void read_a(bf16x8 (&a)[8], const unsigned char* smem, unsigned b0, unsigned b1) {
#pragma unroll
    for (int ti = 0; ti < 4; ++ti) {
        const unsigned base = ((ti & 1) ? b1 : b0) + (unsigned)((ti >> 1) * 32 * kRow + 32 * S);
        a[2 * ti] = *reinterpret_cast<const bf16x8*>(smem + base);
        a[2 * ti + 1] = *reinterpret_cast<const bf16x8*>(smem + base + 512);
    }
}

template <int S>
__device__ __forceinline__ void ksteps(f32x16 (&acc)[4], bf16x8 (&acur)[8], bf16x8 (&anext)[8], bf16x8 (&rh)[kRing],
                                       bf16x8 (&rl)[kRing], const unsigned char* smem, unsigned b0, unsigned b1,
                                       const __bf16* curH, const __bf16* curL, const __bf16* nxtH,
                                       const __bf16* nxtL) {
    if constexpr (S < 16) {
        if constexpr (S + 1 < 16) read_a<S + 1>(anext, smem, b0, b1);
        {   // B fragment of k-step S + kRing - 1 (this tile) or of the next tile's k-step S + kRing - 1 - 16
            constexpr int T = S + kRing - 1, slot = T % kRing;
            const __bf16* ph = T < 16 ? curH : nxtH;
            const __bf16* pl = T < 16 ? curL : nxtL;
            rh[slot] = *reinterpret_cast<const bf16x8*>(ph + 512 * (T & 15));
            rl[slot] = *reinterpret_cast<const bf16x8*>(pl + 512 * (T & 15));
        }
        const f32x16 zero = {};
        const bf16x8 bh = rh[S % kRing], bl = rl[S % kRing];
#pragma unroll
        for (int ti = 0; ti < 4; ++ti) {
            f32x16 c = S == 0 ? zero : acc[ti];
#if RMD_X3_S16TEST
            // timing only (wrong results): each 32x32x16 product as two 16x16x32 MFMAs of the same cycles
            typedef __attribute__((ext_vector_type(4))) float f32x4;
            f32x4 p0 = __builtin_shufflevector(c, c, 0, 1, 2, 3), p1 = __builtin_shufflevector(c, c, 4, 5, 6, 7);
            f32x4 p2 = __builtin_shufflevector(c, c, 8, 9, 10, 11), p3 = __builtin_shufflevector(c, c, 12, 13, 14, 15);
            p0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * ti + 1], bh, p0, 0, 0, 0);
            p1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * ti + 1], bh, p1, 0, 0, 0);
            p2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * ti], bl, p2, 0, 0, 0);
            p3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * ti], bl, p3, 0, 0, 0);
            p0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * ti], bh, p0, 0, 0, 0);
            p3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * ti], bh, p3, 0, 0, 0);
            const f32x8 lo8 = __builtin_shufflevector(p0, p1, 0, 1, 2, 3, 4, 5, 6, 7);
            const f32x8 hi8 = __builtin_shufflevector(p2, p3, 0, 1, 2, 3, 4, 5, 6, 7);
            acc[ti] = __builtin_shufflevector(lo8, hi8, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
#else
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[2 * ti + 1], bh, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[2 * ti], bl, c, 0, 0, 0);
            acc[ti] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[2 * ti], bh, c, 0, 0, 0);
#endif
        }
        // order inside the region: k-step S+1's 8 LDS reads and the 2 ring loads first, then 12 MFMAs
        if constexpr (S + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, RMD_X3_S16TEST ? 24 : 12, 0);
        __builtin_amdgcn_sched_barrier(0);      // one scheduling region per k-step
        ksteps<S + 1>(acc, anext, acur, rh, rl, smem, b0, b1, curH, curL, nxtH, nxtL);
    }
}

// Persistent schedule: the work is cut into units = (image, quarter of the query tiles, target block)
// — `quarters` tile ranges of tq tiles per block — and workgroup lid (one per CU) runs units lid,
// lid + nwg, lid + 2 nwg, ...  Ordered image-major, then quarter, then block, a time slot of nwg
// consecutive units keeps each XCD's workgroups on one or two (image, quarter) tile ranges, whose
// B fragments (55 tiles x 32 KB = 1.8 MB at cfg2) then stay in that XCD's L2.  At cfg2, 448
// one-block workgroups take 2 rounds on 256 CUs (the second 3/4 full); 1792 quarter units take 7
// even slots.  Each unit re-stages its block's A (128 KB) — quarters = 1 and nwg = units is the
// one-block-per-workgroup launch.
//
// ABL (diagnostic build only): 1 = drop every store (descriptor range 0), 2 = no k-loop (epilogue only)
// PAD: vmcnt_pad after the ring prologue (product; the diagnostic build's RMD_X3_PAD=0 drops it for A/B)
template <bool PP, int ABL = 0, bool PAD = true>
__global__ void __launch_bounds__(512, 1)
corr_pyramid_x3(const __bf16* __restrict__ aHi, const __bf16* __restrict__ aLo, const __bf16* __restrict__ bHi,
                const __bf16* __restrict__ bLo, PyrGeom g, int units, int quarters, int tq,
                float* __restrict__ pyr) {
    constexpr int WAVES = 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int H = g.height, W = g.width, N = H * W;
    const int ncb = (W + kBlockCols - 1) / kBlockCols;
    const int nblk = ((H + kBlockRows - 1) / kBlockRows) * ncb;
    const int nqt = (N + 31) >> 5;
    const int nwg = gridDim.x;
    const int lid = xcd_block(blockIdx.x, nwg);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 31, h = lane >> 5;

    for (int u = lid; u < units; u += nwg) {            // uniform per workgroup
        const int per_img = nblk * quarters;
        const int b = u / per_img;
        const int r = u - b * per_img;
        const int qd = r / nblk;
        const int tb = r - qd * nblk;
        const int t_lo = qd * tq, t_hi = min(nqt, t_lo + tq);
        const int rb = tb / ncb, cb = tb - rb * ncb;
        const int ty0 = rb * kBlockRows, tx0 = cb * kBlockCols;

        // ---- A block (hi and lo) -> LDS, zero rows for targets outside the image ----------------
        __syncthreads();                                // the previous unit's fragment reads are done
        const size_t abase = (size_t)b * N * 256;
        // 16 pieces per thread, all 16 loads in flight before the first LDS store (a load-store loop
        // pays one HBM round trip per piece: ~16 latencies before the first MFMA)
        constexpr int kPieces = kBlockRows * kBlockCols * 64 / (64 * WAVES);
        uint4 v[kPieces];
#pragma unroll
        for (int i = 0; i < kPieces; ++i) {
            const int id = tid + i * 64 * WAVES;
            const int row = id >> 6, c = id & 63;                 // c < 32: hi chunk c, else lo chunk c - 32
            const int ty = ty0 + (row >> 4), tx = tx0 + (row & 15);
            const __bf16* src = c < 32 ? aHi : aLo;
            v[i] = make_uint4(0, 0, 0, 0);
            if (ty < H && tx < W) v[i] = *reinterpret_cast<const uint4*>(src + abase + (size_t)(ty * W + tx) * 256 + (c & 31) * 8);
        }
#pragma unroll
        for (int i = 0; i < kPieces; ++i) {
            const int id = tid + i * 64 * WAVES;
            const int row = id >> 6, c = id & 63;
            *reinterpret_cast<uint4*>(smem + (size_t)lds_row(row >> 4, row & 15) * kRow + (c < 32 ? 0 : 512) + (c & 31) * 16) = v[i];
        }
        __syncthreads();

        // ---- per-level store descriptors of this block (wave-uniform) ---------------------------
        Lvl L[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const int span = kBlockRows >> l, nch = l == 0 ? 2 : 1;
            const int y0 = rb * span, xc0 = cb * nch;
            const bool lv = l < g.levels;
            const int cw = g.tw[l];
            const int rows = lv ? max(0, min(span, g.ty[l] - y0)) : 0;
            const unsigned rs = lv ? (unsigned)g.tx[l] * (unsigned)N * cw * 4u : 0u;
            const size_t base = lv ? ((size_t)g.off[l] + (((size_t)b * g.ty[l] + y0) * g.tx[l] + xc0) * N * cw) : 0;
            float* bp = pyr + base;
            const unsigned lo32 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)bp);
            const unsigned hi32 = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)bp >> 32));
            L[l].rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi32 << 32) | lo32), (short)0,
                                                          (int)__builtin_amdgcn_readfirstlane(ABL == 1 ? 0u : (unsigned)rows * rs),
                                                          0x00020000);
            L[l].rs = __builtin_amdgcn_readfirstlane(rs);
            L[l].cs = __builtin_amdgcn_readfirstlane((unsigned)N * cw * 4u);
            L[l].rows = __builtin_amdgcn_readfirstlane(rows);
            L[l].chunks = __builtin_amdgcn_readfirstlane(lv ? max(0, min(nch, g.tx[l] - xc0)) : 0);
        }

        // A fragment of tile ti = 2 rg + cg, k-step s, half p: base[cg] + rg*32*kRow + 32 s + 512 p
        unsigned b0 = (unsigned)j * kRow + 16u * h, b1 = b0 + 64u * kRow;
        asm volatile("" : "+v"(b0), "+v"(b1));

        const size_t bb = ((size_t)b * nqt * 1024 + lane) * 8;
        const int stride = WAVES;
        int qt = t_lo + w;
        // B fragments stream through an 8-slot register ring: k-step s of a tile lives in slot s % 8
        // and is loaded at k-step s - 7 (the previous tile's k-steps 9-15 load this tile's 0-6), 7
        // k-steps (84 MFMAs) ahead; A fragments of k-step s + 1 are read from LDS at the top of k-step
        // s.  Each k-step is one scheduling region, so neither set of loads drifts to just before its
        // MFMAs.
        bf16x8 rh[kRing], rl[kRing];
        if (qt < t_hi) {
            const __bf16* pb = bHi + bb + X3_TILE(qt);
            const __bf16* pbl = bLo + bb + X3_TILE(qt);
#pragma unroll
            for (int s = 0; s < kRing - 1; ++s) {
                rh[s] = *reinterpret_cast<const bf16x8*>(pb + 512 * s);
                rl[s] = *reinterpret_cast<const bf16x8*>(pbl + 512 * s);
            }
        }
        if constexpr (PAD) vmcnt_pad_n<kEpiStores>(pyr);
        if constexpr (PP) {
            // ping-pong phases (as corr_pyramid_w8): waves w and w + 4 of each SIMD alternate between
            // the MFMA phase and the epilogue phase, separated by workgroup barriers; 2 nmax + 1 per
            // wave and unit
            const int nmax = t_lo < t_hi ? (t_hi - t_lo + stride - 1) / stride : 0;
            const int nw = qt < t_hi ? (t_hi - qt + stride - 1) / stride : 0;
            const bool late = w >= 4;
            if (late) __builtin_amdgcn_s_barrier();
            for (int k = 0; k < nmax; ++k) {
                const int qn = qt + stride;
                // one wave-uniform branch holds both phases, so every path that loads ring fragments
                // also issues the epilogue stores after them (see vmcnt_pad_n)
                if (k < nw) {
                    f32x16 acc[4];
                    if constexpr (ABL == 2) {
#pragma unroll
                        for (int ti = 0; ti < 4; ++ti)
#pragma unroll
                            for (int e = 0; e < 16; ++e) acc[ti][e] = (float)(j + ti + e + k);
                    } else {
                        const size_t pn = X3_TILE(min(qn, nqt - 1));
                        bf16x8 a0[8], a1[8];
                        read_a<0>(a0, smem, b0, b1);
                        ksteps<0>(acc, a0, a1, rh, rl, smem, b0, b1, bHi + bb + X3_TILE(qt),
                                  bLo + bb + X3_TILE(qt), bHi + bb + pn, bLo + bb + pn);
                    }
                    __builtin_amdgcn_s_barrier();
                    epilogue(acc, L, min(qt * 32 + j, N - 1), h);
                    __builtin_amdgcn_s_barrier();
                } else {
                    __builtin_amdgcn_s_barrier();
                    __builtin_amdgcn_s_barrier();
                }
                qt = qn;
            }
            if (!late) __builtin_amdgcn_s_barrier();
        } else {
            while (qt < t_hi) {
                f32x16 acc[4];
                const int qn = qt + stride;
                const size_t pn = X3_TILE(min(qn, nqt - 1));
                bf16x8 a0[8], a1[8];
                read_a<0>(a0, smem, b0, b1);
                ksteps<0>(acc, a0, a1, rh, rl, smem, b0, b1, bHi + bb + X3_TILE(qt), bLo + bb + X3_TILE(qt),
                          bHi + bb + pn, bLo + bb + pn);
                epilogue(acc, L, min(qt * 32 + j, N - 1), h);
                qt = qn;
            }
        }
    }
}


// ---- 16x16x32 form (the product since round 5) -------------------------------------------------
// The same 8 x 16 target block, ping-pong phases and B ring, with v_mfma_f32_16x16x32_bf16 tiles:
// a wave's 32-query tile is 2 N-tiles of 16 queries against 8 M-tiles of 16 targets (M-tile mt = 2 rp
// + ch: rows 2rp, 2rp+1 x cols 8ch..8ch+7 of the block), 8 k-steps of 32 channels, each k-step in two
// halves of 4 M-tiles (8 A fragments double-buffered, 24 MFMAs per half).  On random operands the chip
// holds a higher clock under this shape than under 32x32x16 at the same MFMA cycles
// (MI355X_MICROARCH.md 'DVFS give-back' item 7; profiles/x3_ab_r05.json: the kernel is power-bound,
// its cycles do not change when its stores are dropped but its clock does).
//
// A in LDS, k-major: the 16-B piece of (part p = hi/lo, channel chunk cc = 0..31, LDS row r) sits at
// ((p * 32 + cc) * 128 + r) * 16, row r = 16 mt + 8 (row in pair) + col in half.  A fragment read
// (lane n + 16 g: row 16 mt + n, chunk 4 s + g) gives every 16-lane ds_read_b128 group 16 distinct rows
// = 16 distinct 16-B bank slots (no padding, 128 KiB).
#ifndef RMD_X3_SHAPE
#define RMD_X3_SHAPE 16
#endif
typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int kLds16 = 2 * 32 * 128 * 16;
constexpr int kDR16 = 4;                     // B ring depth (k-steps of 32 channels; divides 8)
constexpr int kEpiStores16 = 30;             // buffer stores of one epilogue16 (16 + 8 + 4 + 2)

__device__ __forceinline__ int s16_row(int y, int x) { return (((y >> 1) * 2 + (x >> 3)) << 4) + ((y & 1) << 3) + (x & 7); }

// A fragments of half-step (k-step S, M-tiles 4M..4M+3): hi in [2i], lo in [2i+1]
template <int S, int M>
__device__ __forceinline__ void read_a16(bf16x8 (&a)[8], const unsigned char* smem, unsigned bhi, unsigned blo) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const unsigned off = (unsigned)(S * 8192 + (4 * M + i) * 256);
        a[2 * i] = *reinterpret_cast<const bf16x8*>(smem + bhi + off);
        a[2 * i + 1] = *reinterpret_cast<const bf16x8*>(smem + blo + off);
    }
}

template <int HS>      // half-step HS = 2 S + M
__device__ __forceinline__ void ksteps16(f32x4 (&acc)[8][2], bf16x8 (&acur)[8], bf16x8 (&anext)[8],
                                         bf16x8 (&rh)[kDR16][2], bf16x8 (&rl)[kDR16][2], const unsigned char* smem,
                                         unsigned bhi, unsigned blo, const __bf16* cur, const __bf16* nxt,
                                         size_t lo_off) {
    if constexpr (HS < 16) {
        constexpr int S = HS >> 1, M = HS & 1;
        constexpr int SN = (HS + 1) / 2, MN = (HS + 1) % 2;
        if constexpr (HS + 1 < 16) read_a16<SN, MN>(anext, smem, bhi, blo);
        {   // N-tile M's B fragments of k-step S + kDR16 - 1 (this tile) or of the next tile's
            constexpr int T = S + kDR16 - 1, slot = T % kDR16;
            const __bf16* p = (T < 8 ? cur : nxt) + M * 4096 + 512 * (T & 7);
            rh[slot][M] = *reinterpret_cast<const bf16x8*>(p);
            rl[slot][M] = *reinterpret_cast<const bf16x8*>(p + lo_off);
        }
        const f32x4 zero = {};
        // (product-outer order, 8 independent accumulators between dependent MFMAs: same cycles,
        // profiles/x3_ab_r05.json ord1)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const bf16x8 bh = rh[S % kDR16][u], bl = rl[S % kDR16][u];
                f32x4 c = S == 0 ? zero : acc[4 * M + i][u];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * i + 1], bh, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * i], bl, c, 0, 0, 0);
                acc[4 * M + i][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[2 * i], bh, c, 0, 0, 0);
            }
        if constexpr (HS + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 24, 0);
        __builtin_amdgcn_sched_barrier(0);
        ksteps16<HS + 1>(acc, anext, acur, rh, rl, smem, bhi, blo, cur, nxt, lo_off);
    }
}

// Epilogue of one 32-query tile in the 16x16 layout: acc[mt][u][e] is, for lane (n, g) and query
// 16 u + n, the target (row 2 rp + (g >> 1), col 8 ch + 4 (g & 1) + e) with mt = 2 rp + ch.
// S24: RMD_S24 storage (3 bytes per element; the Lvl strides are in those bytes): lanes gather whole
// 12-byte pieces (4 values) before each store.
template <bool S24>
__device__ __forceinline__ void epilogue16(const f32x4 (&acc)[8][2], const Lvl (&L)[4], int qt, int N, int n, int g) {
    constexpr unsigned E = S24 ? 3u : 4u;                  // bytes per element
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const unsigned q = (unsigned)min(qt * 32 + 16 * u + n, N - 1);
        // level 0: 1 x 8 chunks (8E bytes per query); lanes g = 2 r', 2 r' + 1 write row r' halves
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
            const unsigned o = q * 8u * E + 4u * E * (g & 1) + soff(L[0], 2 * (mt >> 1) + (g >> 1), mt & 1);
            if constexpr (S24) {
                __builtin_amdgcn_raw_buffer_store_b96(pack24(acc[mt][u][0], acc[mt][u][1], acc[mt][u][2], acc[mt][u][3]),
                                                      L[0].rsrc, (int)o, 0, AUX_NT);
            } else {
                const i32x4 d = {__float_as_int(acc[mt][u][0]), __float_as_int(acc[mt][u][1]),
                                 __float_as_int(acc[mt][u][2]), __float_as_int(acc[mt][u][3])};
                __builtin_amdgcn_raw_buffer_store_b128(d, L[0].rsrc, (int)o, 0, AUX_NT);
            }
        }
        // level 1: horizontal pairs in-lane, vertical pairs across the lane halves (ch 0 lands in the lower,
        // ch 1 in the upper half): lane g then holds level-1 cols 2g, 2g+1 of level-1 row rp
        float t2[2];
#pragma unroll
        for (int rp = 0; rp < 4; ++rp) {
            const f32x4& a = acc[2 * rp][u];
            const f32x4& c = acc[2 * rp + 1][u];
            float x0 = a[0] + a[1], x1 = a[2] + a[3], y0 = c[0] + c[1], y1 = c[2] + c[3];
            swapf(x0, y0);
            swapf(x1, y1);
            const float s0 = x0 + y0, s1 = x1 + y1;
            if constexpr (S24) {
                // even g takes its odd neighbour's two columns (lane + 16): cols 2g .. 2g + 3 in one piece
                const float s2 = __shfl_xor(s0, 16), s3 = __shfl_xor(s1, 16);
                __builtin_amdgcn_raw_buffer_store_b96(
                    pack24(0.25f * s0, 0.25f * s1, 0.25f * s2, 0.25f * s3), L[1].rsrc,
                    (int)((g & 1) ? kBig : q * 8u * E + 6u * (g >> 1) * 2u + soff(L[1], rp, 0)), 0, AUX_NT);
            } else {
                const i32x2 d = {__float_as_int(0.25f * s0), __float_as_int(0.25f * s1)};
                __builtin_amdgcn_raw_buffer_store_b64(d, L[1].rsrc, (int)(q * 32u + 8u * g + soff(L[1], rp, 0)), 0,
                                                      AUX_NT);
            }
            const float t = s0 + s1;
            t2[rp >> 1] = (rp & 1) ? t2[rp >> 1] + t : t;
        }
        // level 2: lane g holds level-2 col g of rows 0 and 1
#pragma unroll
        for (int y2 = 0; y2 < 2; ++y2) {
            if constexpr (S24) {
                // lane g = 0 collects cols 0..3 (lanes + 16, + 32, + 48) and writes the 12-byte chunk
                const int l = threadIdx.x & 63;
                const float v = 0.0625f * t2[y2];
                const float v1 = __shfl(v, (l + 16) & 63), v2 = __shfl(v, (l + 32) & 63), v3 = __shfl(v, (l + 48) & 63);
                __builtin_amdgcn_raw_buffer_store_b96(pack24(v, v1, v2, v3), L[2].rsrc,
                                                      (int)(g ? kBig : q * 4u * E + soff(L[2], y2, 0)), 0, AUX_NT);
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(0.0625f * t2[y2]), L[2].rsrc,
                                                      (int)(q * 16u + 4u * g + soff(L[2], y2, 0)), 0, AUX_NT);
            }
        }
        // level 3: col x3 = level-2 cols 2 x3, 2 x3 + 1 (lanes g, g ^ 1 = lane ^ 16); even g hold col g >> 1
        float t3 = t2[0] + t2[1];
        t3 += __shfl_xor(t3, 16);
        const float v3 = (1.0f / 64.0f) * t3;
        if constexpr (S24) {
            // lane g = 0 takes col 1 from lane + 32 and writes the block's 6-byte half of the 12-byte chunk as
            // a naturally aligned word + short
            const float w1 = __shfl_xor(v3, 32);
            const unsigned r0 = s24_round(v3), r1 = s24_round(w1);
            const unsigned base = q * 12u + soff(L[3], 0, 0);          // 1 x 4 chunks: 2-aligned half chunk
            const bool odd = ((base + L[3].a) & 2u) != 0;
            // even: word = bytes 0-3, short = bytes 4-5; odd: short = bytes 0-1, word = bytes 2-5
            const unsigned word = odd ? __builtin_amdgcn_perm(r1, r0, 0x07060503u) : __builtin_amdgcn_perm(r1, r0, 0x05030201u);
            const unsigned shrt = odd ? ((r0 >> 8) & 0xffffu) : (r1 >> 16);
            __builtin_amdgcn_raw_buffer_store_b32((int)word, L[3].rsrc, (int)(g ? kBig : base + (odd ? 2u : 0u)), 0, AUX_NT);
            __builtin_amdgcn_raw_buffer_store_b16((short)shrt, L[3].rsrc, (int)(g ? kBig : base + (odd ? 0u : 4u)), 0,
                                                  AUX_NT);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v3), L[3].rsrc,
                                                  (int)((g & 1) ? kBig : q * 8u + 4u * (g >> 1) + soff(L[3], 0, 0)), 0,
                                                  AUX_NT);
        }
    }
}

template <int ABL = 0, bool S24 = false>
__global__ void __launch_bounds__(512, 1)
corr_pyramid_x3s(const __bf16* __restrict__ aHi, const __bf16* __restrict__ aLo, const __bf16* __restrict__ bHi,
                 const __bf16* __restrict__ bLo, PyrGeom g, int units, unsigned char* __restrict__ pyr) {
    constexpr unsigned E = S24 ? 3u : 4u;                  // bytes per stored element
    constexpr int WAVES = 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int H = g.height, W = g.width, N = H * W;
    const int ncb = (W + kBlockCols - 1) / kBlockCols;
    const int nblk = ((H + kBlockRows - 1) / kBlockRows) * ncb;
    const int nqt = (N + 31) >> 5;
    const int u = xcd_block(blockIdx.x, gridDim.x);
    if (u >= units) return;                                        // uniform per workgroup
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, gq = lane >> 4;
    const int b = u / nblk, tb = u - b * nblk;
    const int rb = tb / ncb, cb = tb - rb * ncb;
    const int ty0 = rb * kBlockRows, tx0 = cb * kBlockCols;

    // ---- A block (hi and lo) -> LDS (k-major image), zero rows for targets outside the image -------
    // piece id = tid + 512 i: lanes of an 8-lane group take 8 consecutive LDS rows of one chunk
    // (conflict-free ds_write_b128), 8 such groups the 8 consecutive chunks of those pixels (128-B
    // global segments)
    const size_t abase = (size_t)b * N * 256;
    constexpr int kPieces = 2 * 32 * 128 / 512;                    // 16 per thread
    uint4 v[kPieces];
#pragma unroll
    for (int i = 0; i < kPieces; ++i) {
        const int id = tid + i * 512;
        const int r = (id & 7) + ((id >> 6) & 15) * 8;             // LDS row 0..127
        const int cc = ((id >> 3) & 7) + ((id >> 10) & 3) * 8;     // channel chunk 0..31
        const int part = id >> 12;
        const int mt = r >> 4, ii = r & 15;
        const int ty = ty0 + 2 * (mt >> 1) + (ii >> 3), tx = tx0 + 8 * (mt & 1) + (ii & 7);
        v[i] = make_uint4(0, 0, 0, 0);
        if (ty < H && tx < W)
            v[i] = *reinterpret_cast<const uint4*>((part ? aLo : aHi) + abase + (size_t)(ty * W + tx) * 256 + cc * 8);
    }
#pragma unroll
    for (int i = 0; i < kPieces; ++i) {
        const int id = tid + i * 512;
        const int r = (id & 7) + ((id >> 6) & 15) * 8;
        const int cc = ((id >> 3) & 7) + ((id >> 10) & 3) * 8;
        const int part = id >> 12;
        *reinterpret_cast<uint4*>(smem + (size_t)((part * 32 + cc) * 128 + r) * 16) = v[i];
    }
    __syncthreads();

    Lvl L[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const int span = kBlockRows >> l, nch = l == 0 ? 2 : 1;
        // S24 level 3: 1 x 4 chunks, two blocks per chunk (this block's 2 columns at byte 6 (cb & 1))
        const bool c4 = S24 && l == 3;
        const int y0 = rb * span, xc0 = c4 ? cb >> 1 : cb * nch;
        const bool lv = l < g.levels;
        const int cw = g.tw[l];
        const int rows = lv ? max(0, min(span, g.ty[l] - y0)) : 0;
        const unsigned rs = lv ? (unsigned)g.tx[l] * (unsigned)N * cw * E : 0u;
        const size_t base = lv ? ((size_t)g.off[l] + (((size_t)b * g.ty[l] + y0) * g.tx[l] + xc0) * N * cw) : 0;
        unsigned char* bp = pyr + base * E + (c4 && lv ? 6u * (cb & 1) : 0u);
        const unsigned lo32 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)bp);
        const unsigned hi32 = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)bp >> 32));
        L[l].rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi32 << 32) | lo32), (short)0,
                                                      (int)__builtin_amdgcn_readfirstlane(ABL == 1 ? 0u : (unsigned)rows * rs),
                                                      0x00020000);
        L[l].rs = __builtin_amdgcn_readfirstlane(rs);
        L[l].cs = __builtin_amdgcn_readfirstlane((unsigned)N * cw * E);
        L[l].rows = __builtin_amdgcn_readfirstlane(rows);
        L[l].chunks = __builtin_amdgcn_readfirstlane(lv ? max(0, min(nch, g.tx[l] - xc0)) : 0);
        L[l].a = lo32 & 3u;
    }

    unsigned bhi = (unsigned)(gq * 128 + n) * 16u, blo = bhi + 65536u;
    asm volatile("" : "+v"(bhi), "+v"(blo));
    // B of 32-query tile qt: 16-query tiles 2 qt, 2 qt + 1 at bq + qt * 8192 (+ 4096 for the second)
    const __bf16* bq = bHi + ((size_t)b * 2 * nqt * 512 + lane) * 8;
    const size_t lo_off = (size_t)(bLo - bHi);
    int qt = w;
    bf16x8 rh[kDR16][2], rl[kDR16][2];
    if (qt < nqt) {
        const __bf16* p = bq + (size_t)qt * 8192;
#pragma unroll
        for (int s = 0; s < kDR16 - 1; ++s)
#pragma unroll
            for (int uu = 0; uu < 2; ++uu) {
                rh[s][uu] = *reinterpret_cast<const bf16x8*>(p + uu * 4096 + 512 * s);
                rl[s][uu] = *reinterpret_cast<const bf16x8*>(p + uu * 4096 + 512 * s + lo_off);
            }
    }
    vmcnt_pad_n<S24 ? kEpiStores16 + 1 : kEpiStores16>(pyr);
    // ping-pong phases as corr_pyramid_x3: waves w and w + 4 of each SIMD alternate MFMA and epilogue
    const int nmax = (nqt + WAVES - 1) / WAVES;
    const int nw = qt < nqt ? (nqt - qt + WAVES - 1) / WAVES : 0;
    const bool late = w >= 4;
    if (late) __builtin_amdgcn_s_barrier();
    for (int k = 0; k < nmax; ++k) {
        const int qn = qt + WAVES;
        if (k < nw) {
            f32x4 acc[8][2];
            bf16x8 a0[8], a1[8];
            read_a16<0, 0>(a0, smem, bhi, blo);
            ksteps16<0>(acc, a0, a1, rh, rl, smem, bhi, blo, bq + (size_t)qt * 8192, bq + (size_t)min(qn, nqt - 1) * 8192,
                        lo_off);
            __builtin_amdgcn_s_barrier();
            epilogue16<S24>(acc, L, qt, N, n, gq);
            __builtin_amdgcn_s_barrier();
        } else {
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_s_barrier();
        }
        qt = qn;
    }
    if (!late) __builtin_amdgcn_s_barrier();
}

}  // namespace

bool eligible(const rmd_pyramid_desc& d, int C) {
    if (C > 256 || (d.storage != RMD_F32 && d.storage != RMD_S24) || d.levels < 1 || d.layout != RMD_LAYOUT_ROWS)
        return false;
    // every block's per-level store range (rows x row stride, bytes) plus the 1 GiB chunk bias must
    // stay inside 32-bit buffer offsets
    const double N = (double)d.height * d.width;
    const double span0 = 8.0 * d.tiles_x[0] * N * 8 * 4;
    if (span0 >= (double)(1u << 30)) return false;
    if (d.storage == RMD_S24) {
        // the lookup reads S24 through per-image level buffers only: every slab below 2^31 bytes
        for (int l = 0; l < d.levels; ++l)
            if ((double)d.tiles_y[l] * d.tiles_x[l] * d.query_slots * d.tile_h[l] * d.tile_w[l] * 3.0 >= 2147483648.0)
                return false;
    }
    return true;
}

size_t workspace_bytes(const rmd_pyramid_desc& d) {
    const size_t N = (size_t)d.height * d.width, Npad = (N + 31) / 32 * 32;
    return (size_t)d.batch * (N + Npad) * 256 * 2 * 2;
}

int prepare(const float* f1, const float* f2, int C, float scale, const rmd_pyramid_desc& d, void* ws,
            hipStream_t st) {
    const int N = d.height * d.width, nqt = (N + 31) / 32;
    __bf16* aHi = reinterpret_cast<__bf16*>(ws);
    __bf16* aLo = aHi + (size_t)d.batch * N * 256;
    __bf16* bHi = aLo + (size_t)d.batch * N * 256;
    __bf16* bLo = bHi + (size_t)d.batch * nqt * 32 * 256;
    const int lds = 2 * kPx * kStride;
    auto kp = prep_split<RMD_X3_SHAPE == 16>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kp), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kp<<<dim3((N + kPx - 1) / kPx, d.batch, 2), 512, lds, st>>>(f1, f2, aHi, aLo, bHi, bLo, C, N, nqt, scale);
    return check_launch("rmd_corr_prepare/x3");
}

int pyramid(const rmd_pyramid_desc& d, void* pyr, void* ws, hipStream_t st) {
    const int N = d.height * d.width, nqt = (N + 31) / 32;
    const __bf16* aHi = reinterpret_cast<const __bf16*>(ws);
    const __bf16* aLo = aHi + (size_t)d.batch * N * 256;
    const __bf16* bHi = aLo + (size_t)d.batch * N * 256;
    const __bf16* bLo = bHi + (size_t)d.batch * nqt * 32 * 256;
    const int nblk = ((d.height + kBlockRows - 1) / kBlockRows) * ((d.width + kBlockCols - 1) / kBlockCols);
#if RMD_X3_SHAPE == 16
    {
        const int units = nblk * d.batch;
        auto kern = d.storage == RMD_S24 ? corr_pyramid_x3s<RMD_X3_ABL, true> : corr_pyramid_x3s<RMD_X3_ABL, false>;
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, kLds16);
        kern<<<units, 512, kLds16, st>>>(aHi, aLo, bHi, bLo, make_geom(d), units, reinterpret_cast<unsigned char*>(pyr));
        return check_launch("rmd_corr_pyramid/gemm-x3");
    }
#endif
    if (d.storage != RMD_F32) return RMD_ERR_ARG;       // the 32x32x16 form stores F32 only
    // schedule (32x32x16 form, -DRMD_X3_SHAPE=32) (see corr_pyramid_x3): quarters Q in {1, 2, 4, 8} minimising slots x rounds per unit,
    // slots = ceil(B nblk Q / CUs) (one 137-KB-LDS workgroup per CU), rounds = ceil(nqt / Q / 8); a
    // unit re-stages A, charged as 0.3 round.  Q = 1 with one workgroup per unit is the plain launch
    // (the only one when the grid is already several CU-loads deep).
    static int ncu = 0;
    if (ncu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
            ncu = n;
        if (ncu <= 0) ncu = 256;
    }
    int quarters = 1;
    double best = 1e30;
    // product: Q = 1.  Measured at cfg2 (profiles/x3_ab_r02_persist.json), bitwise identical:
    // Q = 1 0.632 ms, Q <= 2 0.619, Q = 4 (7 even slots) 0.627 — like the w8 GEMM, the kernel is
    // bound chip-wide (2.09 GB fp32 pyramid stream + the MFMA phases' overlap), not by CU balance
    constexpr int qmax = 1;
    for (int q = 1; q <= qmax && q * 8 <= nqt; q *= 2) {
        const long long units = (long long)nblk * d.batch * q;
        const int tq = (nqt + q - 1) / q;
        const double slots = (double)((units + ncu - 1) / ncu);
        const double cost = slots * ((tq + 7) / 8 + 0.3);
        if (cost < best - 1e-9) {
            best = cost;
            quarters = q;
        }
    }
    const int tq = (nqt + quarters - 1) / quarters;
    const long long units = (long long)nblk * d.batch * quarters;
    const int nwg = (int)(units < ncu ? units : (quarters == 1 ? units : ncu));
    const int lds = kBlockRows * kBlockCols * kRow;
    // ping-pong phases (free-running waves measured slower, profiles/x3_ab_r02.json)
    auto kern = corr_pyramid_x3<RMD_X3_PP != 0, RMD_X3_ABL>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kern<<<nwg, 512, lds, st>>>(aHi, aLo, bHi, bLo, make_geom(d), (int)units, quarters, tq, reinterpret_cast<float*>(pyr));
    return check_launch("rmd_corr_pyramid/gemm-x3");
}

}  // namespace x3
}  // namespace rmd
