// corr_pyramid_x3.hip — fp32-accurate correlation GEMM + fused pooled pyramid from split-bf16 MFMAs.
//
// Replaces raft.CorrBlock.__init__ (qzed/raft-meets-dicl src/models/impls/raft.py:18-47) in the
// fp32 parity mode.  The reference computes the volume in fp32 (raft.py:31-33, fmaps .float() at
// :381); exact f32 MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate, so each operand is
// split x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (16 significant bits together) and
//   corr = A_hi.B_hi + A_hi.B_lo + A_lo.B_hi        (the dropped lo.lo term is ~2^-16 relative)
// runs as three v_mfma_f32_16x16x32_bf16 per k-step into one fp32 accumulator: 3/16 of the exact-
// f32 MFMA cost.  The 1/sqrt(C) scale is folded into fmap2 before the split (fp32 multiply).
//
// Geometry: one workgroup (8 waves, two per SIMD, free-running) owns an 8 x 16
// block of target pixels — both split halves of its A operand sit in LDS as a k-major image — and
// each wave sweeps its own 32-query tiles (8 M-tiles of 16 targets x 2 N-tiles of 16 queries x 8
// k-steps x 3 products), then pools in-lane and stores all four levels straight from the
// accumulators with range-checked buffer stores (rows past the level fall outside the descriptor,
// chunks past the row get a 1 GiB bias), as fp32 or as RMD_S24 (3-byte) values (epilogue16_s24, round
// 6).  Partial last rounds of one-CU workgroups are balanced by splitting the remaining blocks' query
// tiles (X3Sched).  The 32x32x16 form of rounds 2-4 is in git history (commit db30b41 and before;
// profiles/x3_ab_r05.json compares them).

#include "rmd_common.h"
#include "corr_x3.h"

namespace rmd {
namespace x3 {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(2))) int i32x2;

constexpr int kBlockRows = 8, kBlockCols = 16;
constexpr unsigned kBig = 0x40000000u;      // offset bias beyond every level's range

__device__ __forceinline__ __bf16 hi_part(float v) { return (__bf16)v; }
__device__ __forceinline__ __bf16 lo_part(float v) { return (__bf16)(v - (float)(__bf16)v); }

// ---- operand prep: both feature maps, split, in one launch ------------------------------------
// grid (128-pixel tiles, B, 2).  z = 0: fmap2 * scale -> A hi / lo, pixel-major (B, N, 256);
// z = 1: fmap1 -> B hi / lo in 16x16x32 MFMA B-fragment order o[b][t16][s][lane][8] (lane = n + 16g:
// channels 32s + 8g .. +7 of query min(16 t16 + n, N - 1)).  Read phase as prep_pair (float4 per channel row),
// hi and lo tiles staged in LDS, one 16-B chunk per lane-store on the write side.
constexpr int kPx = 128, kStride = 256 * 2 + 16;

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
        if (which) {
            // 16x16x32 B fragments: 16-query tile t16 = k >> 9, k-step (32 channels) st, lane n + 16 g
            const int L = k & 63, st = (k >> 6) & 7;
            px = (k >> 9) * 16 + (L & 15);
            c0 = 32 * st + 8 * (L >> 4);
        } else {
            px = k >> 5;
            c0 = (k & 31) * 8;
        }
        const bf16x8 hi = *reinterpret_cast<const bf16x8*>(tHi + (size_t)px * kStride + c0 * 2);
        const bf16x8 lo = *reinterpret_cast<const bf16x8*>(tLo + (size_t)px * kStride + c0 * 2);
        if (which) {
            const int t16 = blockIdx.x * 8 + (k >> 9);
            if (t16 < 2 * nqt) {
                const size_t o = (((size_t)b * 2 * nqt + t16) * 512 + (k & 511)) * 8;
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
    unsigned long long base;    // descriptor base address and byte range (epilogue16_s24 rebases them
    unsigned range;             // per query tile)
};

// L's descriptor moved `delta` bytes forward (range shrunk to match): SALU work per tile, so the stores
// keep a zero soffset — with an SGPR soffset the compiler omits the wait state a > 8-byte store needs
// before a VALU overwrites its data VGPRs (LLVM's MUBUF store-data hazard rule exempts register soffsets),
// and on gfx950 that corrupted the last lanes of the store whose data registers the next VALU reused
// (round-6 debug: tools/s24_debug.py)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rebase(const Lvl& L, unsigned delta) {
    const unsigned long long p = L.base + delta;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p), hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
    const unsigned r = __builtin_amdgcn_readfirstlane(L.range > delta ? L.range - delta : 0u);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo), (short)0, (int)r,
                                             0x00020000);
}

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

// RMD_S24 rounding of a value the x3 GEMM produces: u + 0x80, top 24 bits.  The general rule
// (s24_round) keeps a NaN a NaN by OR-ing the quiet bit; here every NaN is an MFMA result from bf16
// operands (payload = a bf16 NaN's, low 16 bits zero, quiet) or the default quiet NaN, passed through
// v_add / v_mul of the pooling (which keep an input NaN's payload) — so the + 0x80 never carries out of
// the low byte and u + 0x80 has the same top 24 bits as u | 0x00400000: one VALU op instead of five
// (test_s24_pyramid_is_rounded_f32_pyramid checks a NaN query row bit for bit).
__device__ __forceinline__ unsigned s24_gemm(float v) { return __float_as_uint(v) + 0x80u; }
__device__ __forceinline__ i32x3 pack24g(unsigned a, unsigned b, unsigned c, unsigned d) {
    const unsigned v0 = s24_gemm(__uint_as_float(a)), v1 = s24_gemm(__uint_as_float(b)),
                   v2 = s24_gemm(__uint_as_float(c)), v3 = s24_gemm(__uint_as_float(d));
    return i32x3{(int)__builtin_amdgcn_perm(v1, v0, 0x05030201u), (int)__builtin_amdgcn_perm(v2, v1, 0x06050302u),
                 (int)__builtin_amdgcn_perm(v3, v2, 0x07060503u)};
}

// v_permlane16_swap: the odd 16-lane rows of x are exchanged with the even rows of y (x.row1 <-> y.row0,
// x.row3 <-> y.row2)
__device__ __forceinline__ void swap16(unsigned& x, unsigned& y) {
    auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
}

// A/B knob (tools/build_variant.sh -D...; the product build uses the default): RMD_X3_ABL = the
// kernel's ablation (1 = drop every store through a zero descriptor range; 2 = no epilogue, the
// phase barriers kept; 3 = no epilogue and no barriers: timing only)
#ifndef RMD_X3_ABL
#define RMD_X3_ABL 0
#endif
// RMD_X3_FREE: 1 (product since round 6) = no ping-pong phase barriers, the two waves of a SIMD run
// free; 0 = waves w and w + 4 alternate MFMA and epilogue phases between workgroup barriers.  With the
// round-5 epilogue (~875 VALU per tile) the phases had to be separated; with epilogue16_s24 (~280) the
// barriers cost more than they hide: cfg2 0.464-0.466 vs 0.477-0.479 ms in the bench step, GRBM cycles
// 6.89M vs 7.42M, MFMA busy 0.69 vs 0.64 (profiles/x3_free_ab_r06.json)
#ifndef RMD_X3_FREE
#define RMD_X3_FREE 1
#endif
// RMD_X3_S24_R05 = 1: the round-5 S24 epilogue (epilogue16<true>) instead of epilogue16_s24 (A/B only)
#ifndef RMD_X3_S24_R05
#define RMD_X3_S24_R05 0
#endif

// ---- GEMM kernel (16x16x32 MFMA) ------------------------------------------------------------------
// One workgroup (8 waves, two per SIMD, free-running: RMD_X3_FREE) owns an 8 x 16 target block; its waves
// sweep their own 32-query tiles through a B-fragment register ring, with v_mfma_f32_16x16x32_bf16 tiles:
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
typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int kLds16 = 2 * 32 * 128 * 16;
constexpr int kDR16 = 4;                     // B ring depth (k-steps of 32 channels; divides 8)
constexpr int kEpiStores16 = 30;             // buffer stores of one epilogue16 (16 + 8 + 4 + 2)
constexpr int kEpiStoresS24 = 23;            // buffer stores of one epilogue16_s24 (16 + 4 + 1 + 2)

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

// S24 epilogue (round 6).  The F32-style epilogue above spent ~875 VALU instructions per 32-query tile
// (the NaN-safe rounding, per-store address arithmetic and ds_bpermute gathers) against the partner wave's
// 384 MFMAs, whose issue gaps hold ~2 VALU each, so it stretched the MFMA phase and held the clock down
// (profiles/x3_epi_r06.json).  This one computes the same values in the same order and stores the same
// bytes with ~1/3 of the VALU and 23 instead of 32 stores:
//  * every store's byte offset is a per-lane constant (S24Off, computed once per kernel) from a descriptor
//    rebased by the tile's uniform qt * 32 * stride (SALU: rebase);
//  * level 1: the two 16-query halves (u) go out in ONE store: lane row g holds level-1 cols 2g, 2g+1 of
//    both halves; one v_permlane16_swap per value pair hands row 0 the u = 0 cols 2, 3 of row 1 and row 1
//    the u = 1 cols 0, 1 of row 0 (rows 2, 3 likewise for cols 4-7), so row g writes half u = g & 1, piece
//    g >> 1 of the 24-byte chunk;
//  * level 2: the 4 (u, row) chunks of 4 columns, one column per lane row, are a 4 x 4 transpose over the
//    lane rows (2 permlane32 + 2 permlane16 swaps): lane row r writes chunk r in ONE store;
//  * level 3: one permlane16 swap sums the column pairs of both halves, one permlane32 swap brings col 1
//    next to col 0 in rows 0 (u = 0) and 1 (u = 1): one word + short store pair.
// TAIL (the last, partial query tile only, a uniform branch with the same stores): lanes whose query
// is past the map add kBig to their offsets (dropped by the range check).
struct S24Off {
    unsigned o0[8];            // level 0 M-tile mt, half u = 0 (u = 1: + 16 queries x 24 B)
    unsigned o1[4];            // level 1 row rp
    unsigned o2;               // level 2
    unsigned o3w, o3s;         // level 3 word / short
    bool odd;                  // level-3 half chunk 2-aligned: short first (uniform)
};

template <bool TAIL>
__device__ __forceinline__ void epilogue16_s24(const f32x4 (&acc)[8][2], const Lvl (&L)[4], const S24Off& o, int qt,
                                               int N, int n, int g) {
    const int q0 = qt * 32;
    const unsigned d24 = (unsigned)q0 * 24u, d12 = (unsigned)q0 * 12u;
    const __amdgpu_buffer_rsrc_t r0 = rebase(L[0], d24), r1 = rebase(L[1], d24), r2 = rebase(L[2], d12),
                                 r3 = rebase(L[3], d12);
    unsigned adj[2] = {0u, 0u}, adj1 = 0u, adj2 = 0u, adj3 = 0u;
    if constexpr (TAIL) {
        adj[0] = q0 + n < N ? 0u : kBig;
        adj[1] = q0 + 16 + n < N ? 0u : kBig;
        adj1 = adj[g & 1];
        adj2 = adj[g >> 1];
        adj3 = adj[g & 1];
    }
    // level 0: lane (n, g) holds cols 8 ch + 4 (g & 1) .. + 3 of row 2 rp + (g >> 1): one 12-byte piece
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
            __builtin_amdgcn_raw_buffer_store_b96(
                pack24g(__float_as_uint(acc[mt][u][0]), __float_as_uint(acc[mt][u][1]), __float_as_uint(acc[mt][u][2]),
                        __float_as_uint(acc[mt][u][3])),
                r0, (int)(o.o0[mt] + adj[u] + 384u * u), 0, AUX_NT);
    // level 1 (values and summation order as epilogue16)
    float t2[2][2];
#pragma unroll
    for (int rp = 0; rp < 4; ++rp) {
        float s0[2], s1[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const f32x4& a = acc[2 * rp][u];
            const f32x4& c = acc[2 * rp + 1][u];
            float x0 = a[0] + a[1], x1 = a[2] + a[3], y0 = c[0] + c[1], y1 = c[2] + c[3];
            swapf(x0, y0);
            swapf(x1, y1);
            s0[u] = x0 + y0;
            s1[u] = x1 + y1;
            const float t = s0[u] + s1[u];
            t2[u][rp >> 1] = (rp & 1) ? t2[u][rp >> 1] + t : t;
        }
        unsigned a0 = __float_as_uint(0.25f * s0[0]), b0 = __float_as_uint(0.25f * s0[1]);
        unsigned a1 = __float_as_uint(0.25f * s1[0]), b1 = __float_as_uint(0.25f * s1[1]);
        swap16(a0, b0);
        swap16(a1, b1);
        __builtin_amdgcn_raw_buffer_store_b96(pack24g(a0, a1, b0, b1), r1, (int)(o.o1[rp] + adj1), 0, AUX_NT);
    }
    // level 2: chunk c = 2 u + y2, lane row g holds its col g -> lane row r holds cols 0..3 of chunk r
    {
        unsigned v0 = __float_as_uint(0.0625f * t2[0][0]), v1 = __float_as_uint(0.0625f * t2[0][1]);
        unsigned v2 = __float_as_uint(0.0625f * t2[1][0]), v3 = __float_as_uint(0.0625f * t2[1][1]);
        swap32(v0, v2);
        swap32(v1, v3);
        swap16(v0, v1);
        swap16(v2, v3);
        __builtin_amdgcn_raw_buffer_store_b96(pack24g(v0, v1, v2, v3), r2, (int)(o.o2 + adj2), 0, AUX_NT);
    }
    // level 3: col x3 of half u = level-2 cols 2 x3, 2 x3 + 1 (lane rows); rows 0 / 1 write halves 0 / 1
    {
        unsigned a = __float_as_uint(t2[0][0] + t2[0][1]), b = __float_as_uint(t2[1][0] + t2[1][1]);
        swap16(a, b);          // row 0: (u0 col-pair of rows 0, 1), row 1: u1 .., row 2 / 3: rows 2, 3
        const unsigned v = __float_as_uint((1.0f / 64.0f) * (__uint_as_float(a) + __uint_as_float(b)));
        unsigned c0 = v, c1 = v;
        swap32(c0, c1);        // c1 of rows 0, 1 = v of rows 2, 3 (col 1)
        const unsigned r0 = s24_gemm(__uint_as_float(v)), r1 = s24_gemm(__uint_as_float(c1));
        const bool odd = o.odd;
        const unsigned word = odd ? __builtin_amdgcn_perm(r1, r0, 0x07060503u) : __builtin_amdgcn_perm(r1, r0, 0x05030201u);
        const unsigned shrt = odd ? ((r0 >> 8) & 0xffffu) : (r1 >> 16);
        __builtin_amdgcn_raw_buffer_store_b32((int)word, r3, (int)(o.o3w + adj3), 0, AUX_NT);
        __builtin_amdgcn_raw_buffer_store_b16((short)shrt, r3, (int)(o.o3s + adj3), 0, AUX_NT);
    }
}

// One segment of a workgroup's work: target block tb of image b against query tiles [qlo, qhi).  Every
// wave runs 2 ceil((qhi - qlo) / 8) + 1 barriers; after the last one no wave reads LDS any more, so the
// next segment may restage A at once.
template <int ABL, bool S24>
__device__ __forceinline__ void x3_segment(const __bf16* __restrict__ aHi, const __bf16* __restrict__ aLo,
                                           const __bf16* __restrict__ bHi, const __bf16* __restrict__ bLo,
                                           const PyrGeom& g, unsigned char* __restrict__ pyr, unsigned char* smem,
                                           int b, int tb, int qlo, int qhi) {
    constexpr unsigned E = S24 ? 3u : 4u;                  // bytes per stored element
    constexpr int WAVES = 8;
    const int H = g.height, W = g.width, N = H * W;
    const int ncb = (W + kBlockCols - 1) / kBlockCols;
    const int nqt = (N + 31) >> 5;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, gq = lane >> 4;
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
        L[l].base = ((unsigned long long)hi32 << 32) | lo32;
        L[l].range = __builtin_amdgcn_readfirstlane(ABL == 1 ? 0u : (unsigned)rows * rs);
    }

    S24Off so;
    if constexpr (S24) {
        // the per-lane parts of every S24 store offset (epilogue16_s24): query 16 u + n of the tile
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
            so.o0[mt] = (unsigned)n * 24u + 12u * (gq & 1) + soff(L[0], 2 * (mt >> 1) + (gq >> 1), mt & 1);
#pragma unroll
        for (int rp = 0; rp < 4; ++rp)
            so.o1[rp] = (unsigned)(16 * (gq & 1) + n) * 24u + 12u * (gq >> 1) + soff(L[1], rp, 0);
        so.o2 = (unsigned)(16 * (gq >> 1) + n) * 12u + soff(L[2], gq & 1, 0);
        const unsigned b3 = soff(L[3], 0, 0);
        const bool odd = ((b3 + L[3].a) & 2u) != 0;                // uniform: 12 q is a multiple of 4
        const unsigned l3 = gq < 2 ? (unsigned)(16 * gq + n) * 12u + b3 : kBig;
        so.o3w = l3 + (odd ? 2u : 0u);
        so.o3s = l3 + (odd ? 0u : 4u);
        so.odd = odd;
    }
    unsigned bhi = (unsigned)(gq * 128 + n) * 16u, blo = bhi + 65536u;
    asm volatile("" : "+v"(bhi), "+v"(blo));
    // B of 32-query tile qt: 16-query tiles 2 qt, 2 qt + 1 at bq + qt * 8192 (+ 4096 for the second)
    const __bf16* bq = bHi + ((size_t)b * 2 * nqt * 512 + lane) * 8;
    const size_t lo_off = (size_t)(bLo - bHi);
    int qt = qlo + w;
    bf16x8 rh[kDR16][2], rl[kDR16][2];
    if (qt < qhi) {
        const __bf16* p = bq + (size_t)qt * 8192;
#pragma unroll
        for (int s = 0; s < kDR16 - 1; ++s)
#pragma unroll
            for (int uu = 0; uu < 2; ++uu) {
                rh[s][uu] = *reinterpret_cast<const bf16x8*>(p + uu * 4096 + 512 * s);
                rl[s][uu] = *reinterpret_cast<const bf16x8*>(p + uu * 4096 + 512 * s + lo_off);
            }
    }
    vmcnt_pad_n<S24 ? (RMD_X3_S24_R05 ? kEpiStores16 + 1 : kEpiStoresS24) : kEpiStores16>(pyr);
    // free-running waves (RMD_X3_FREE), or ping-pong phases: waves w and w + 4 of each SIMD alternate MFMA
    // and epilogue
    const int nmax = (qhi - qlo + WAVES - 1) / WAVES;
    const int nw = qt < qhi ? (qhi - qt + WAVES - 1) / WAVES : 0;
    const bool late = w >= 4;
    if (late && ABL < 3 && !RMD_X3_FREE) __builtin_amdgcn_s_barrier();
    for (int k = 0; k < nmax; ++k) {
        const int qn = qt + WAVES;
        if (k < nw) {
            f32x4 acc[8][2];
            bf16x8 a0[8], a1[8];
            read_a16<0, 0>(a0, smem, bhi, blo);
            ksteps16<0>(acc, a0, a1, rh, rl, smem, bhi, blo, bq + (size_t)qt * 8192, bq + (size_t)min(qn, nqt - 1) * 8192,
                        lo_off);
            if (ABL < 3 && !RMD_X3_FREE) __builtin_amdgcn_s_barrier();
            if constexpr (ABL >= 2) {
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) asm volatile("" ::"v"(acc[mt][0]), "v"(acc[mt][1]));
            } else if constexpr (S24 && !RMD_X3_S24_R05) {
                if (qt * 32 + 32 <= N)
                    epilogue16_s24<false>(acc, L, so, qt, N, n, gq);
                else
                    epilogue16_s24<true>(acc, L, so, qt, N, n, gq);
            } else {
                epilogue16<S24>(acc, L, qt, N, n, gq);
            }
            if (ABL < 3 && !RMD_X3_FREE) __builtin_amdgcn_s_barrier();
        } else if (ABL < 3 && !RMD_X3_FREE) {
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_s_barrier();
        }
        qt = qn;
    }
    if (!late && ABL < 3 && !RMD_X3_FREE) __builtin_amdgcn_s_barrier();
}

// Balanced schedule (round 6).  At cfg2 the 448 (image, block) workgroups of one-CU size run 1.75
// rounds on 256 CUs: XCD x's 56 blocks take two full workgroup times on its 32 CUs while 8 of them idle
// half the time.  With bal the grid holds, per XCD, first `full` x wpx whole-block workgroups (one round
// when full = 1) and then the remaining `rest` blocks cut into `parts` query-tile ranges each, rest x
// parts a multiple of wpx: hardware dispatch hands each CU that frees up the next workgroup in index
// order, so every CU runs the same tile count (cfg2: 220 + 3 x 55) and the query tiles in flight on an
// XCD stay within `parts` offsets (B fragments L2-shared).  A part restages its block's A (from L2).
struct X3Sched {
    int bal;      // 0: one workgroup per (image, block), all query tiles
    int ipx;      // images per XCD
    int nfull;    // whole-block workgroups per XCD (wpx x full)
    int parts;    // query-tile parts of each remaining block
};

template <int ABL = 0, bool S24 = false>
__global__ void __launch_bounds__(512, 1)
corr_pyramid_x3s(const __bf16* __restrict__ aHi, const __bf16* __restrict__ aLo, const __bf16* __restrict__ bHi,
                 const __bf16* __restrict__ bLo, PyrGeom g, int units, X3Sched sc, unsigned char* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ncb = (g.width + kBlockCols - 1) / kBlockCols;
    const int nblk = ((g.height + kBlockRows - 1) / kBlockRows) * ncb;
    const int nqt = (g.height * g.width + 31) >> 5;
    int b, tb, q0 = 0, q1 = nqt;
    if (!sc.bal) {
        const int u = xcd_block(blockIdx.x, gridDim.x);
        if (u >= units) return;                                    // uniform per workgroup
        b = u / nblk;
        tb = u - b * nblk;
    } else {
        // dispatch deals workgroups round-robin over the 8 XCDs (speed only: every workgroup index
        // maps to its own piece of work, whatever CU runs it)
        const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
        int j = k;
        if (k >= sc.nfull) {
            const int kk = k - sc.nfull, part = kk % sc.parts;
            j = sc.nfull + kk / sc.parts;
            q0 = part * nqt / sc.parts;
            q1 = (part + 1) * nqt / sc.parts;
        }
        const int jb = j / nblk;
        b = x * sc.ipx + jb;
        tb = j - jb * nblk;
    }
    x3_segment<ABL, S24>(aHi, aLo, bHi, bLo, g, pyr, smem, b, tb, q0, q1);
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
    auto kp = prep_split;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kp), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kp<<<dim3((N + kPx - 1) / kPx, d.batch, 2), 512, lds, st>>>(f1, f2, aHi, aLo, bHi, bLo, C, N, nqt, scale);
    return check_launch("rmd_corr_prepare/x3");
}

// RMD_X3_BAL = 0 (A/B builds): always one workgroup per (image, block)
#ifndef RMD_X3_BAL
#define RMD_X3_BAL 1
#endif

// the balanced schedule when every XCD holds the same whole images and one workgroup per (image, block)
// would leave a partial last round (X3Sched)
X3Sched schedule(const rmd_pyramid_desc& d, int nblk, int& grid) {
    X3Sched sc{0, 0, 0, 0};
    const int units = nblk * d.batch;
    grid = units;
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
            cus = v;
        else
            cus = -1;
    }
    if (!RMD_X3_BAL || cus <= 0 || cus % 8 != 0 || d.batch % 8 != 0) return sc;
    if (units <= cus || units % cus == 0) return sc;
    const int wpx = cus / 8, nbx = d.batch / 8 * nblk;
    const int full = nbx / wpx, rest = nbx - full * wpx;
    int parts = 1;
    while ((rest * parts) % wpx != 0) ++parts;
    const int nqt = (d.height * d.width + 31) / 32;
    if (parts > 8 || nqt < 8 * parts) return sc;              // pieces too small to pay their A restage
    sc.bal = 1;
    sc.ipx = d.batch / 8;
    sc.nfull = full * wpx;
    sc.parts = parts;
    grid = 8 * (sc.nfull + rest * parts);
    return sc;
}

int pyramid(const rmd_pyramid_desc& d, void* pyr, void* ws, hipStream_t st) {
    const int N = d.height * d.width, nqt = (N + 31) / 32;
    const __bf16* aHi = reinterpret_cast<const __bf16*>(ws);
    const __bf16* aLo = aHi + (size_t)d.batch * N * 256;
    const __bf16* bHi = aLo + (size_t)d.batch * N * 256;
    const __bf16* bLo = bHi + (size_t)d.batch * nqt * 32 * 256;
    const int nblk = ((d.height + kBlockRows - 1) / kBlockRows) * ((d.width + kBlockCols - 1) / kBlockCols);
    const int units = nblk * d.batch;
    int grid = units;
    const X3Sched sc = schedule(d, nblk, grid);
    auto kern = d.storage == RMD_S24 ? corr_pyramid_x3s<RMD_X3_ABL, true> : corr_pyramid_x3s<RMD_X3_ABL, false>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, kLds16);
    kern<<<grid, 512, kLds16, st>>>(aHi, aLo, bHi, bLo, make_geom(d), units, sc,
                                                          reinterpret_cast<unsigned char*>(pyr));
    return check_launch("rmd_corr_pyramid/gemm-x3");
}

}  // namespace x3
}  // namespace rmd
