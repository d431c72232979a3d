// corr_pyramid.hip — all-pairs correlation GEMM with the pooled pyramid fused into its epilogue.
//
// Replaces raft.CorrBlock.__init__ (qzed/raft-meets-dicl src/models/impls/raft.py:18-47):
//   corr0[b,p,q] = sum_c f1[b,c,p] f2[b,c,q] / sqrt(C);  level l = avg_pool2d(level l-1, 2, 2)
//
// gfx950 design.  Targets (fmap2 pixels) are the MFMA row side, queries (fmap1
// pixels) the column side, and one 32-target MFMA tile is a 4 x 8 block of target pixels.  In the
// 32x32 accumulator layout lane (h = lane>>5, j = lane&31) then holds, for query j, a 4-row x
// 4-column patch of targets (columns 4h..4h+3) per tile, so the 2x2 average pools of levels 1-2
// are in-lane adds and level 3 needs one xor-32 lane exchange.  Every level is written from the
// f32 accumulators straight from registers into the query-minor row-chunk layout of rmd.h: the
// lanes of a store instruction are consecutive queries, so each instruction writes whole
// contiguous 512 B runs.
//
// Two kernels:
//  * corr_pyramid_stationary — performance path (bf16 operands, fp16 pyramid, C = 256): a
//    16x16 target block's A operand stays in LDS while 4 waves (one per SIMD, 512-register
//    budget) sweep 32-query tiles; the next tile's B fragments load during the epilogue.
//  * corr_pyramid_tiled — general path (exact f32 MFMA for parity, any C, f32 or fp16 storage):
//    64 queries x 256 targets per workgroup, K staged through LDS in 64-deep chunks.
// Operands are first transposed to pixel-major, channel-contiguous (B, N, Cp) by prep_operand.

#include "rmd_common.h"
#include "corr_x3.h"

#include <cstdlib>
#include <cstring>

namespace rmd {
namespace {

constexpr int kThreads = 256;
constexpr int kBQ = 64;      // queries per workgroup (tiled kernel)
constexpr int kNT = 256;     // targets per workgroup (16 x 16 block)
constexpr int kKC = 64;      // K chunk staged in LDS (tiled kernel)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <bool F32> struct Operand { using T = __bf16; static constexpr int S = 2; };
template <> struct Operand<true> { using T = float; static constexpr int S = 4; };

// padded staging row: kKC elements + 16 B -> ds_read_b128 fragment reads are conflict-free
template <bool F32> constexpr int stage_stride() { return kKC * Operand<F32>::S + 16; }

// element offset of (b, query q, target row y, row-chunk x) at level l (rmd.h layout)
__device__ __forceinline__ size_t lvl_index(const PyrGeom& g, int l, int b, int y, int xc, int q, int N) {
    return (size_t)g.off[l] + ((((size_t)b * g.ty[l] + y) * g.tx[l] + xc) * N + q) * g.tw[l];
}

// ---------------------------------------------------------------------------------------------
// prep: (B, C, N) f32 -> (B, N, Cp) operand type, zero-padded channels.  64 px x 64 ch per block.
template <typename T>
__global__ void __launch_bounds__(kThreads)
prep_operand(const float* __restrict__ f, T* __restrict__ o, int C, int N, int Cp, float scale) {
    __shared__ float tile[64][65];
    const int b = blockIdx.z, p0 = blockIdx.x * 64, c0 = blockIdx.y * 64, t = threadIdx.x;
    const float* fb = f + (size_t)b * C * N;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int c = c0 + (t >> 6) + 4 * i, p = p0 + (t & 63);
        tile[(t >> 6) + 4 * i][t & 63] = (c < C && p < N) ? fb[(size_t)c * N + p] * scale : 0.f;
    }
    __syncthreads();
    const int p = p0 + (t >> 2);
    if (p >= N) return;
    const int cc = (t & 3) * 16;
    T vals[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) vals[j] = (T)tile[cc + j][t >> 2];
    uint4* dst = reinterpret_cast<uint4*>(o + ((size_t)b * N + p) * Cp + c0 + cc);
    const uint4* src = reinterpret_cast<const uint4*>(vals);
#pragma unroll
    for (int j = 0; j < (int)(16 * sizeof(T) / 16); ++j) dst[j] = src[j];
}

// prep (w8 GEMM path, both operands in one launch): grid (128-element tiles, B, 2).  z = 0: fmap2 ->
// A operand (B, N, 256) bf16 * scale over raster pixels; z = 1: fmap1 -> B operand over the query
// slots of the tiles layout (rmd.h), in MFMA B-fragment order
//   o[b][qt][s][lane][8]  (lane = j + 32h: channels 16s + 8h .. +7 of slot 32 qt + j),
// so each of a wave's 16 B-fragment loads per 32-query tile is one contiguous 1 KiB read.  Read
// phase: a thread loads 8 channels x 4 pixels (a slot quad is 4 consecutive pixels of one row:
// float4 per channel row), converts, and writes the 4 pixels' 16-B channel octets into a bf16 LDS
// tile.  Write phase: one 16-B fragment per lane-store, the tile's output is one contiguous 64 KiB
// block for either operand.  Slots of no pixel take a clamped pixel's features.
constexpr int kPrepPx = 128, kPrepStride = 256 * 2 + 16;     // LDS row: 256 bf16 + 16 B pad

__global__ void __launch_bounds__(512)
prep_pair(const float* __restrict__ f1, const float* __restrict__ f2, __bf16* __restrict__ opA,
          __bf16* __restrict__ opB, int C, int H, int W, int S, int nqt, float scale) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int b = blockIdx.y, which = blockIdx.z;
    const int N = H * W;
    const float* f = which ? f1 : f2;
    const float s = which ? 1.0f : scale;
    const int t = threadIdx.x;
    const int p0 = blockIdx.x * kPrepPx;
    if (p0 >= (which ? S : N)) return;               // block-uniform
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int item = it * 512 + t;               // (channel octet cg, element quad q), q fastest
        const int q = item & 31, cg = item >> 5;
        // the quad's first pixel (y1, x1) and whether all 4 are in the map and 16-B aligned
        int y1, x1;
        if (which) {
            tiles_pixel(p0 + 4 * q, H, W, y1, x1);
        } else {
            y1 = 0;
            x1 = p0 + 4 * q;                         // raster: row 0 of a 1 x N map
        }
        const int lim = which ? W : N;
        const bool full = (which ? y1 < H : true) && x1 + 3 < lim && (lim & 3) == 0;
        const int yc = which ? min(y1, H - 1) : 0;
        const float* src = f + ((size_t)b * C) * N + (size_t)yc * (which ? W : 0);
        float v[8][4];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = cg * 8 + e;
            const float* row = src + (size_t)c * N;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (c < C) {
                if (full) {
                    x = *reinterpret_cast<const float4*>(row + x1);
                } else {
                    x.x = row[min(x1 + 0, lim - 1)];
                    x.y = row[min(x1 + 1, lim - 1)];
                    x.z = row[min(x1 + 2, lim - 1)];
                    x.w = row[min(x1 + 3, lim - 1)];
                }
            }
            v[e][0] = x.x * s;
            v[e][1] = x.y * s;
            v[e][2] = x.z * s;
            v[e][3] = x.w * s;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e][i];
            *reinterpret_cast<bf16x8*>(lds + (size_t)(4 * q + i) * kPrepStride + cg * 16) = o;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int k = it * 512 + t;                  // 16-B output chunk of the tile's 64 KiB block
        int px, c0;
        if (which) {                                 // fragment order per 32-pixel tile: k = (tile, s, lane)
            const int L = k & 63, st = (k >> 6) & 15;
            px = (k >> 10) * 32 + (L & 31);
            c0 = 16 * st + 8 * (L >> 5);
        } else {                                     // pixel-major: k = px * 32 + octet
            px = k >> 5;
            c0 = (k & 31) * 8;
        }
        const bf16x8 o = *reinterpret_cast<const bf16x8*>(lds + (size_t)px * kPrepStride + c0 * 2);
        if (which) {
            const int qt = blockIdx.x * 4 + (k >> 10);
            if (qt < nqt) *reinterpret_cast<bf16x8*>(opB + (((size_t)b * nqt + qt) * 1024 + (k & 1023)) * 8) = o;
        } else if (p0 + px < N) {
            *reinterpret_cast<bf16x8*>(opA + ((size_t)b * N + p0) * 256 + (size_t)k * 8) = o;
        }
    }
}

template <typename TOut> __device__ __forceinline__ TOut cvt_out(float v);
template <> __device__ __forceinline__ float cvt_out<float>(float v) { return v; }
template <> __device__ __forceinline__ __half cvt_out<__half>(float v) { return __float2half_rn(v); }

template <typename TOut, int NE>
__device__ __forceinline__ void put(TOut* p, const float* v) {
    TOut tmp[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) tmp[i] = cvt_out<TOut>(v[i]);
    constexpr int NB = NE * sizeof(TOut);
    if constexpr (NB == 16) *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(tmp);
    else if constexpr (NB == 8) *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(tmp);
    else if constexpr (NB == 4) *reinterpret_cast<unsigned*>(p) = *reinterpret_cast<const unsigned*>(tmp);
    else *p = tmp[0];
}

// ---------------------------------------------------------------------------------------------
// General tiled kernel.  Workgroup = 4 waves = 16x16 targets x 64 queries; wave w owns the 8x8
// target sub-block (rows 8*(w>>1).., cols 8*(w&1)..) for all 64 queries (2x2 MFMA 32x32 tiles).
template <bool F32, typename TOut>
__global__ void __launch_bounds__(kThreads)
corr_pyramid_tiled(const typename Operand<F32>::T* __restrict__ opA,   // fmap2 (B, N, Cp)
                   const typename Operand<F32>::T* __restrict__ opB,   // fmap1 (B, N, Cp)
                   int Cp, float scale, PyrGeom g, TOut* __restrict__ pyr) {
    using T = typename Operand<F32>::T;
    constexpr int S = Operand<F32>::S;
    constexpr int SS = stage_stride<F32>();
    constexpr int PPR = kKC * S / 16;                       // 16-B pieces per staged row

    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* sA = smem;
    unsigned char* sB = smem + kNT * SS;

    const int H = g.height, W = g.width, N = H * W;
    const int q0 = blockIdx.x * kBQ;
    const int ncb = (W + 15) >> 4;
    const int rb = blockIdx.y / ncb, cb = blockIdx.y - rb * ncb;
    const int b = blockIdx.z;
    const int ty0 = rb * 16, tx0 = cb * 16;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;

    const T* gA = opA + (size_t)b * N * Cp;
    const T* gB = opB + (size_t)b * N * Cp;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    // LDS row of this lane's A fragment for target tile tr (4 target rows x 8 target cols)
    int arow[2];
#pragma unroll
    for (int tr = 0; tr < 2; ++tr) arow[tr] = (8 * (w >> 1) + 4 * tr + (r >> 3)) * 16 + 8 * (w & 1) + (r & 7);

    for (int kc = 0; kc < Cp; kc += kKC) {
#pragma unroll 4
        for (int i = 0; i < kNT * PPR / kThreads; ++i) {
            const int id = tid + kThreads * i, row = id / PPR, pc = id - row * PPR;
            const int ty = ty0 + (row >> 4), tx = tx0 + (row & 15);
            uint4 v = make_uint4(0, 0, 0, 0);
            if (ty < H && tx < W)
                v = *reinterpret_cast<const uint4*>(gA + (size_t)(ty * W + tx) * Cp + kc + pc * (16 / S));
            *reinterpret_cast<uint4*>(sA + row * SS + pc * 16) = v;
        }
#pragma unroll
        for (int i = 0; i < kBQ * PPR / kThreads; ++i) {
            const int id = tid + kThreads * i, row = id / PPR, pc = id - row * PPR;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (q0 + row < N)
                v = *reinterpret_cast<const uint4*>(gB + (size_t)(q0 + row) * Cp + kc + pc * (16 / S));
            *reinterpret_cast<uint4*>(sB + row * SS + pc * 16) = v;
        }
        __syncthreads();

        if constexpr (!F32) {
#pragma unroll
            for (int s = 0; s < kKC / 16; ++s) {
                const int kb = (16 * s + 8 * h) * 2;
                bf16x8 a[2], q[2];
#pragma unroll
                for (int tr = 0; tr < 2; ++tr) a[tr] = *reinterpret_cast<const bf16x8*>(sA + arow[tr] * SS + kb);
#pragma unroll
                for (int tq = 0; tq < 2; ++tq) q[tq] = *reinterpret_cast<const bf16x8*>(sB + (32 * tq + r) * SS + kb);
#pragma unroll
                for (int tr = 0; tr < 2; ++tr)
#pragma unroll
                    for (int tq = 0; tq < 2; ++tq)
                        acc[tr][tq] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tr], q[tq], acc[tr][tq], 0, 0, 0);
            }
        } else {
            // exact f32 MFMA; k-slot h of every step walks k = 32h + 4m + u (same map for A and B)
#pragma unroll 2
            for (int m = 0; m < 8; ++m) {
                const int kb = (32 * h + 4 * m) * 4;
                f32x4 a[2], q[2];
#pragma unroll
                for (int tr = 0; tr < 2; ++tr) a[tr] = *reinterpret_cast<const f32x4*>(sA + arow[tr] * SS + kb);
#pragma unroll
                for (int tq = 0; tq < 2; ++tq) q[tq] = *reinterpret_cast<const f32x4*>(sB + (32 * tq + r) * SS + kb);
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int tr = 0; tr < 2; ++tr)
#pragma unroll
                        for (int tq = 0; tq < 2; ++tq)
                            acc[tr][tq] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tr][u], q[tq][u], acc[tr][tq], 0, 0, 0);
            }
        }
        __syncthreads();
    }

    // ---- epilogue: scale, pool in-lane, store each level's row pieces from registers ------------
    const int levels = g.levels;
#pragma unroll
    for (int tq = 0; tq < 2; ++tq) {
        const int q = q0 + 32 * tq + r;
        if (q >= N) continue;
        float o[8][4];                                            // rows 0..7, cols 4h..4h+3
#pragma unroll
        for (int tr = 0; tr < 2; ++tr)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[4 * tr + (e >> 2)][e & 3] = acc[tr][tq][e] * scale;
        // level 0: wave block rows 16rb + 8(w>>1) + row, chunk 2cb + (w&1), elements 4h..4h+3
        {
            const int xc = 2 * cb + (w & 1);
            if (xc < g.tx[0]) {
#pragma unroll
                for (int row = 0; row < 8; ++row) {
                    const int y = 16 * rb + 8 * (w >> 1) + row;
                    if (y < g.ty[0]) put<TOut, 4>(pyr + lvl_index(g, 0, b, y, xc, q, N) + 4 * h, o[row]);
                }
            }
        }
        if (levels < 2) continue;
        float l1[4][2];
#pragma unroll
        for (int yy = 0; yy < 4; ++yy)
#pragma unroll
            for (int xx = 0; xx < 2; ++xx)
                l1[yy][xx] = 0.25f * ((o[2 * yy][2 * xx] + o[2 * yy][2 * xx + 1]) +
                                      (o[2 * yy + 1][2 * xx] + o[2 * yy + 1][2 * xx + 1]));
        if (cb < g.tx[1]) {
#pragma unroll
            for (int yy = 0; yy < 4; ++yy) {
                const int y = 8 * rb + 4 * (w >> 1) + yy;
                if (y < g.ty[1]) put<TOut, 2>(pyr + lvl_index(g, 1, b, y, cb, q, N) + 4 * (w & 1) + 2 * h, l1[yy]);
            }
        }
        if (levels < 3) continue;
        float l2[2];
#pragma unroll
        for (int yy = 0; yy < 2; ++yy)
            l2[yy] = 0.25f * ((l1[2 * yy][0] + l1[2 * yy][1]) + (l1[2 * yy + 1][0] + l1[2 * yy + 1][1]));
        if (cb < g.tx[2]) {
#pragma unroll
            for (int yy = 0; yy < 2; ++yy) {
                const int y = 4 * rb + 2 * (w >> 1) + yy;
                if (y < g.ty[2]) put<TOut, 1>(pyr + lvl_index(g, 2, b, y, cb, q, N) + 2 * (w & 1) + h, &l2[yy]);
            }
        }
        if (levels < 4) continue;
        float s3 = l2[0] + l2[1];
        s3 += __shfl_xor(s3, 32);
        s3 *= 0.25f;
        const int y3 = 2 * rb + (w >> 1);
        if (h == 0 && cb < g.tx[3] && y3 < g.ty[3]) put<TOut, 1>(pyr + lvl_index(g, 3, b, y3, cb, q, N) + (w & 1), &s3);
    }
}

// LDS swizzle of the A block (256 target rows x 32 16-B chunks): chunk' = chunk ^ swz(row).
// A ds_read_b128 fragment read serves the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (and
// +32) in one LDS cycle each iff their 16 addresses fall in distinct 16-B bank slots.  The lanes
// of a fragment read rows base + 16*(j>>3) + (j&7) (j = lane & 31) at one chunk, so the slot must
// separate j&7 AND the parity of j>>3: swz = (row & 7) | ((row >> 4) & 1) << 3.  (row & 15 alone
// maps j and j+8 to one slot: a 2-way conflict on every fragment read.)
__device__ __forceinline__ int a_swz(int row) { return (row & 7) | ((row >> 1) & 8); }

// ---------------------------------------------------------------------------------------------
// Target-stationary kernel (bf16 operands, fp16 pyramid, C = 256): the performance path.
//
// One workgroup = 4 waves (one per SIMD) owns a 16x16 block of target pixels: its A operand
// (256 targets x 256 bf16 = 128 KiB) is loaded into LDS once, 16-B chunks XOR-swizzled by row so the
// 16 rows a ds_read_b128 lane group reads hit distinct banks.  Each wave sweeps 32-query tiles:
// 8 MFMA 32x32x16 tiles per k-step (all 256 targets x 32 queries), then pools in-lane and stores
// every level straight from registers.  v_permlane32_swap pairs the two half-waves' 8-byte row
// halves into full 16-byte row chunks, so one store instruction writes two contiguous 512-byte runs.
// TH = 16-row halves per wave: TH = 2 -> 4 waves (one per SIMD) each own all 16 target rows;
// TH = 1 -> 8 waves (two per SIMD) each own 8 rows, pairs of waves share a query tile.
template <int TH> struct STraits {
    static constexpr int kWaves = TH == 2 ? 4 : 8;
    static constexpr int kThreads = 64 * kWaves;
    static constexpr int kTiles = 4 * TH;                 // MFMA 32x32 tiles per wave
    static constexpr int kRows = 8 * TH;                  // level-0 target rows per wave
    static constexpr int kStores = TH == 2 ? 23 : 12;     // stores per lane per 32-query tile
};

__device__ __forceinline__ unsigned pack_half2(float a, float b) {
    const __half2 h = __floats2half2_rn(a, b);
    return *reinterpret_cast<const unsigned*>(&h);
}

__device__ __forceinline__ void swap32(unsigned& x, unsigned& y) {
    auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    x = r[0];
    y = r[1];
}

// per-wave store geometry: element offsets of the wave's first row/chunk on every level, row and
// chunk strides, valid rows/chunks; a store address is base + uniform constant + per-lane offset
struct SCtx {
    int N;
    size_t base[4];     // level offset + row/chunk origin of this wave's rows (elements)
    size_t rs[4];       // row stride (elements)
    size_t cs[4];       // chunk stride = N * chunk width (elements)
    int rows[4];        // valid rows of this wave per level
    int chunks[4];      // valid chunks of this block per level (<= 2, 1, 1, 1)
};

// B-fragment loads in inline asm, retired by ONE hand-placed `s_waitcnt vmcnt(kStores)`: between a
// tile's loads and that wait the wave issues exactly kStores compiler stores (the epilogue, every
// store unconditional) and no other vector-memory op (no compiler-visible global loads in the
// loop, no spills: checked in the .s by tests/test_asm_audit.py), so the wait retires the loads
// while the previous stores stay in flight.  hipcc does not count asm loads, so it never inserts
// its own draining vmcnt(0).
__device__ __forceinline__ void s_load_b_asm(bf16x8 (&bq)[16], const __bf16* src) {
#define RMD_GLD(S) asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(bq[S]) : "v"(src), "i"((S) * 32) : "memory")
    RMD_GLD(0); RMD_GLD(1); RMD_GLD(2); RMD_GLD(3); RMD_GLD(4); RMD_GLD(5); RMD_GLD(6); RMD_GLD(7);
    RMD_GLD(8); RMD_GLD(9); RMD_GLD(10); RMD_GLD(11); RMD_GLD(12); RMD_GLD(13); RMD_GLD(14); RMD_GLD(15);
#undef RMD_GLD
}

template <int N>
__device__ __forceinline__ void s_wait_b(bf16x8 (&bq)[16]) {
    asm volatile("s_waitcnt vmcnt(%16)"
                 : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]), "+v"(bq[4]), "+v"(bq[5]), "+v"(bq[6]),
                   "+v"(bq[7]), "+v"(bq[8]), "+v"(bq[9]), "+v"(bq[10]), "+v"(bq[11]), "+v"(bq[12]), "+v"(bq[13]),
                   "+v"(bq[14]), "+v"(bq[15])
                 : "i"(N)
                 : "memory");
}

template <int NT>
__device__ __forceinline__ void s_lda(bf16x8 (&a)[NT], const unsigned char* smem, const int (&arow)[NT], int s, int h) {
    constexpr int Cp = 256;
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
        const int row = arow[ti];
        a[ti] = *reinterpret_cast<const bf16x8*>(smem + (size_t)row * Cp * 2 + (((2 * s + h) ^ a_swz(row)) << 4));
    }
}

// 16 k-steps x NT MFMA tiles; the A fragments of step s+1 are read from LDS while step s's MFMAs run
template <int NT>
__device__ __forceinline__ void s_mma(f32x16 (&acc)[NT], const bf16x8 (&bq)[16], const unsigned char* smem,
                                      const int (&arow)[NT], int h) {
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[ti][e] = 0.f;
    bf16x8 a0[NT], a1[NT];
    s_lda<NT>(a0, smem, arow, 0, h);
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
        s_lda<NT>(a1, smem, arow, s + 1, h);
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) acc[ti] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ti], bq[s], acc[ti], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 2 < 16) s_lda<NT>(a0, smem, arow, s + 2, h);
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) acc[ti] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[ti], bq[s + 1], acc[ti], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Every store is unconditional: an invalid one (query past N, row or chunk outside a level, a
// level beyond g.levels) is redirected to this lane's 16-B trash slot, so each tile issues exactly
// kStores stores (see s_load_b_asm).  ABL is a diagnostic ablation (RMD_ABLATE env): 1 = every
// store to trash (no HBM write traffic).
// trash: this lane's slot in store-slot 0; slot k (a distinct 1 KiB line set per store of the
// tile) keeps ABL = 1 stores from being merged by the compiler (the store count must stay exact)
template <int ABL>
__device__ __forceinline__ __half* sel(bool ok, __half* p, __half* trash, int k) {
    if constexpr (ABL == 1) return trash + k * 64 * 8;
    else return ok ? p : trash;
}

template <int TH, int ABL>
__device__ __forceinline__ void s_epilogue(const f32x16 (&acc)[4 * TH], const SCtx& c, int q, int h,
                                           __half* __restrict__ pyr, __half* __restrict__ trash) {
    constexpr int R0 = 8 * TH, R1 = 4 * TH, R2 = 2 * TH;
    const bool qv = q < c.N;
    // per-lane parts of the addresses: query offset and the half-wave's row (h)
    __half* p0 = pyr + c.base[0] + (size_t)q * 8 + h * c.rs[0];
    __half* p1 = pyr + c.base[1] + (size_t)q * 8 + h * c.rs[1];
    // V(row, cg 0..1, k 0..3) = level-0 value at the wave's target row, col 8cg + 4h + k (the
    // 1/sqrt(C) scale is folded into the operands by prep_operand)
#define V(row, cg, k) (acc[2 * ((row) >> 2) + (cg)][((row) & 3) * 4 + (k)])
    // level 0: rows 2m + h after the swap; chunk tc
#pragma unroll
    for (int tc = 0; tc < 2; ++tc) {
#pragma unroll
        for (int m = 0; m < R0 / 2; ++m) {
            const int r0 = 2 * m;
            unsigned x0 = pack_half2(V(r0, tc, 0), V(r0, tc, 1));
            unsigned x1 = pack_half2(V(r0, tc, 2), V(r0, tc, 3));
            unsigned y0 = pack_half2(V(r0 + 1, tc, 0), V(r0 + 1, tc, 1));
            unsigned y1 = pack_half2(V(r0 + 1, tc, 2), V(r0 + 1, tc, 3));
            swap32(x0, y0);
            swap32(x1, y1);
            const bool ok = qv && r0 + h < c.rows[0] && tc < c.chunks[0];
            *reinterpret_cast<uint4*>(sel<ABL>(ok, p0 + r0 * c.rs[0] + tc * c.cs[0], trash, tc * (R0 / 2) + m)) =
                make_uint4(x0, x1, y0, y1);
        }
    }
    // level 1: lane h holds cols {2h, 2h+1} (cg 0) and {4+2h, 5+2h} (cg 1) of R1 rows
    float l1[R1][2][2];
#pragma unroll
    for (int yy = 0; yy < R1; ++yy)
#pragma unroll
        for (int cg = 0; cg < 2; ++cg)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                l1[yy][cg][u] = 0.25f * ((V(2 * yy, cg, 2 * u) + V(2 * yy, cg, 2 * u + 1)) +
                                         (V(2 * yy + 1, cg, 2 * u) + V(2 * yy + 1, cg, 2 * u + 1)));
#undef V
#pragma unroll
    for (int m = 0; m < R1 / 2; ++m) {
        unsigned x0 = pack_half2(l1[2 * m][0][0], l1[2 * m][0][1]);
        unsigned x1 = pack_half2(l1[2 * m][1][0], l1[2 * m][1][1]);
        unsigned y0 = pack_half2(l1[2 * m + 1][0][0], l1[2 * m + 1][0][1]);
        unsigned y1 = pack_half2(l1[2 * m + 1][1][0], l1[2 * m + 1][1][1]);
        swap32(x0, y0);
        swap32(x1, y1);
        const bool ok = qv && 2 * m + h < c.rows[1] && c.chunks[1] > 0;
        *reinterpret_cast<uint4*>(sel<ABL>(ok, p1 + 2 * m * c.rs[1], trash, R0 + m)) = make_uint4(x0, y0, x1, y1);
    }
    // level 2: lane h holds cols {h, 2+h} of R2 rows; it stores rows (R2/2)h .. (R2/2)h + R2/2 - 1
    float l2[R2][2];
#pragma unroll
    for (int yy = 0; yy < R2; ++yy)
#pragma unroll
        for (int cg = 0; cg < 2; ++cg)
            l2[yy][cg] = 0.25f * ((l1[2 * yy][cg][0] + l1[2 * yy][cg][1]) + (l1[2 * yy + 1][cg][0] + l1[2 * yy + 1][cg][1]));
    {
        unsigned mine[R2], other[R2];
#pragma unroll
        for (int yy = 0; yy < R2; ++yy) {
            mine[yy] = pack_half2(l2[yy][0], l2[yy][1]);          // (col h, col 2+h)
            other[yy] = __shfl_xor(mine[yy], 32);
        }
        __half* p2 = pyr + c.base[2] + (size_t)q * 4 + (R2 / 2) * h * c.rs[2];
#pragma unroll
        for (int k = 0; k < R2 / 2; ++k) {
            // row (R2/2)h + k, selected with compile-time indices (a runtime index would go to scratch)
            const unsigned mk = h ? mine[R2 / 2 + k] : mine[k];
            const unsigned ok_ = h ? other[R2 / 2 + k] : other[k];
            const unsigned e0 = h ? ok_ : mk;      // cols 0 and 2 (held by h = 0)
            const unsigned e1 = h ? mk : ok_;      // cols 1 and 3 (held by h = 1)
            const bool ok = qv && (R2 / 2) * h + k < c.rows[2] && c.chunks[2] > 0;
            *reinterpret_cast<uint2*>(sel<ABL>(ok, p2 + k * c.rs[2], trash, R0 + R1 / 2 + k)) =
                make_uint2((e0 & 0xffffu) | (e1 << 16), (e0 >> 16) | (e1 & 0xffff0000u));
        }
    }
    // level 3: TH rows of 2 cols; lane h stores row h (TH = 2) or both halves row 0 (TH = 1,
    // identical values to the same address)
    {
        float t3[TH][2];
#pragma unroll
        for (int yy = 0; yy < TH; ++yy)
#pragma unroll
            for (int cg = 0; cg < 2; ++cg) {
                const float s_ = l2[2 * yy][cg] + l2[2 * yy + 1][cg];
                t3[yy][cg] = 0.25f * (s_ + __shfl_xor(s_, 32));
            }
        const int yrow = TH == 2 ? h : 0;
        unsigned v;
        if constexpr (TH == 2) v = h ? pack_half2(t3[1][0], t3[1][1]) : pack_half2(t3[0][0], t3[0][1]);
        else v = pack_half2(t3[0][0], t3[0][1]);
        const bool ok = qv && yrow < c.rows[3] && c.chunks[3] > 0;
        *reinterpret_cast<unsigned*>(sel<ABL>(ok, pyr + c.base[3] + (size_t)q * 2 + yrow * c.rs[3], trash, R0 + R1 / 2 + R2 / 2)) = v;
    }
}

// ABL (diagnostic, RMD_ABLATE env): 0 = normal, 1 = every store to trash, 2 = no MFMA
template <int TH, int ABL>
__global__ void __launch_bounds__(STraits<TH>::kThreads, 1)
corr_pyramid_stationary(const __bf16* __restrict__ opA, const __bf16* __restrict__ opB, PyrGeom g, int qsplit,
                        __half* __restrict__ pyr, __half* __restrict__ trash_base) {
    using Tr = STraits<TH>;
    constexpr int Cp = 256, CPR = Cp / 8, NT = Tr::kTiles;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int H = g.height, W = g.width, N = H * W;
    const int ncb = (W + 15) >> 4;
    const int nblk = ((H + 15) >> 4) * ncb;
    // XCD-aware bijective remap: consecutive logical blocks (same batch) share an XCD's L2
    const int nwg = gridDim.x;
    const int orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int tb = lid % nblk;
    const int rest = lid / nblk;
    const int split = rest % qsplit;
    const int b = rest / qsplit;
    const int rb = tb / ncb, cb = tb - rb * ncb;
    const int ty0 = rb * 16, tx0 = cb * 16;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);    // wave-uniform: scalar loop control
    const int th = TH == 2 ? 0 : (w & 1);                       // which 8-row half (TH = 1)
    const int qslot = TH == 2 ? w : (w >> 1);                   // query-tile slot
    constexpr int kSlots = TH == 2 ? Tr::kWaves : Tr::kWaves / 2;
    const int j = lane & 31, h = lane >> 5;
    __half* trash = trash_base + lane * 8;            // 16 B per lane (stores of all waves may collide)

    // ---- A block -> LDS (zero rows for targets outside the image) ------------------------------
    const __bf16* gA = opA + (size_t)b * N * Cp;
    for (int id = tid; id < 256 * CPR; id += Tr::kThreads) {
        const int row = id / CPR, c = id - row * CPR;
        const int ty = ty0 + (row >> 4), tx = tx0 + (row & 15);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (ty < H && tx < W) v = *reinterpret_cast<const uint4*>(gA + (size_t)(ty * W + tx) * Cp + c * 8);
        *reinterpret_cast<uint4*>(smem + (size_t)row * Cp * 2 + ((c ^ a_swz(row)) << 4)) = v;
    }
    __syncthreads();

    // LDS row of this lane's A fragment for tile ti (4 target rows x 8 target cols)
    int arow[NT];
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) arow[ti] = (8 * th + 4 * (ti >> 1) + (j >> 3)) * 16 + 8 * (ti & 1) + (j & 7);

    SCtx c;
    c.N = N;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const int cw = g.tw[l], span = (16 >> l) / (3 - TH), nch = l == 0 ? 2 : 1;   // rows of this wave
        const int y0 = rb * (16 >> l) + th * span, xc0 = cb * nch;
        const bool lv = l < g.levels;
        c.cs[l] = (size_t)N * cw;
        c.rs[l] = lv ? (size_t)g.tx[l] * N * cw : 0;
        c.base[l] = lv ? (size_t)g.off[l] + (((size_t)b * g.ty[l] + y0) * g.tx[l] + xc0) * N * cw : 0;
        c.rows[l] = lv ? max(0, min(span, g.ty[l] - y0)) : 0;
        c.chunks[l] = lv ? max(0, min(nch, g.tx[l] - xc0)) : 0;
    }

    const __bf16* gB = opB + (size_t)b * N * Cp;
    const int nqt = (N + 31) >> 5;
    const int stride = kSlots * qsplit;
    int qt = split * kSlots + qslot;
    if (qt >= nqt) return;
    // software pipeline: tile t+1's B fragments load right after tile t's MFMAs (their registers
    // are free then) and land while tile t's epilogue runs; one B buffer, one explicit wait
    bf16x8 bq[16];
    f32x16 acc[NT];
    const int last = nqt - 1;
    const size_t hoff = 8 * h;
    s_load_b_asm(bq, gB + (size_t)min(qt * 32 + j, N - 1) * Cp + hoff);
    s_wait_b<0>(bq);
    while (true) {
        const int qn = qt + stride;
        if constexpr (ABL != 2) s_mma<NT>(acc, bq, smem, arow, h);
        else for (int ti = 0; ti < NT; ++ti) for (int e = 0; e < 16; ++e) acc[ti][e] = bq[0][0] * 0.f;
        s_load_b_asm(bq, gB + (size_t)min(min(qn, last) * 32 + j, N - 1) * Cp + hoff);
        s_epilogue<TH, ABL>(acc, c, qt * 32 + j, h, pyr, trash);
        s_wait_b<Tr::kStores>(bq);
        if (qn >= nqt) break;
        qt = qn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// w8 GEMM (bf16 operands, fp16 pyramid in the tiles layout of rmd.h, C = 256): the performance path.
//
// One workgroup (8 waves, two per SIMD) owns a 16x16 block of level-0 target pixels; its A operand
// (256 targets x 256 channels bf16) stays in LDS while the waves sweep their own 32-query tiles
// (query slots 32 qt .. 32 qt + 31 of the tiles layout: a 2 x 16 patch of query pixels).  Per tile
// a wave runs 16 k-steps x 8 MFMA 32x32x16 tiles into 128 accumulator VGPRs, then the epilogue pools
// in-lane and stores every level straight from registers:
//  * in the 32x32 accumulator layout lane (j, h) holds, for query slot j, target rows 4i..4i+3 x
//    columns 8cg + 4h .. +3 of MFMA tile (i, cg): a 2 x 4 level-0 chunk of the tiles layout is one
//    lane's own 8 values (one 16-B store, lanes h = 0/1 writing neighbouring quads: each store
//    instruction writes two contiguous 512-B runs); level-1 2 x 4 chunks and level-2 1 x 4 chunks
//    need one v_permlane32_swap per row pair, level 3 one lane exchange;
//  * stores are raw buffer stores through one descriptor per level covering the block's valid chunk
//    rows: the per-lane 32-bit offset = slot * chunk bytes + quad * chunk stride (a 1 GiB bias for a
//    quad past the level), rows past the level fall outside num_records and are dropped by the
//    hardware range check — no predication, no redirect.  Slots of no pixel (x >= W) compute and
//    store a clamped query's values into their own slot, so every 128-B line is written whole.
namespace pipe {

constexpr unsigned kBig = 0x40000000u;    // offset bias that lands beyond every level's range

struct Lvl {
    __amdgpu_buffer_rsrc_t rsrc;
    unsigned rs;      // chunk-row stride (bytes)
    unsigned cs;      // chunk stride (bytes): next quad / chunk of the same chunk row
    unsigned hd;      // paired block (corr_pyramid_w8): added to the offsets of the block's second row
                      // half, which holds the NEXT column block's rows: chunks per block * cs - half rows * rs
    int nq;           // valid chunks of this block's chunk rows (level 0: 0..4, 1: 0..2, 2-3: 0..1)
};

struct Ctx {
    Lvl l[4];
};

__device__ __forceinline__ unsigned pk(float a, float b) {
    const __half2 v = __floats2half2_rn(a, b);
    return *reinterpret_cast<const unsigned*>(&v);
}

__device__ __forceinline__ void swp(unsigned& x, unsigned& y) {
    auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    x = r[0];
    y = r[1];
}

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(2))) int i32x2;

// lane-dependent parts of the store offsets of query slot q (bytes)
struct LaneOff {
    unsigned o0[2];   // level 0, column group tc: quad 2 tc + h
    unsigned o1;      // level 1: quad h
    unsigned o2;      // level 2: chunk row h of each stored pair
    unsigned o3;      // level 3: chunk row h
};

__device__ __forceinline__ LaneOff lane_offsets(const Ctx& c, int q, int h) {
    LaneOff r;
    const unsigned uq = (unsigned)q;
#pragma unroll
    for (int tc = 0; tc < 2; ++tc)
        r.o0[tc] = 2 * tc + h < c.l[0].nq ? uq * 16u + (unsigned)(2 * tc + h) * c.l[0].cs : kBig;
    r.o1 = h < c.l[1].nq ? uq * 16u + (unsigned)h * c.l[1].cs : kBig;
    r.o2 = c.l[2].nq > 0 ? uq * 8u + (unsigned)h * c.l[2].rs : kBig;
    r.o3 = c.l[3].nq > 0 ? uq * 4u + (unsigned)h * (c.l[3].rs + c.l[3].hd) : kBig;
    return r;
}

// per-tile running sums of the epilogue (unscaled: level-l sums are 4^l x the average)
struct EpiState {
    float s1[8][2][2];    // level-1 row yy (0..7), col group cg, pair u
    float s2[4][2];       // level-2 row, col group
};

#define V(acc, row, cg, k) (acc[2 * ((row) >> 2) + (cg)][((row) & 3) * 4 + (k)])

// Epilogue piece s (0..15) of one tile, from accumulator set `acc`: level-0 chunk row m = s/2 of
// column group tc = s%2, the level-1 sums of those rows, and every 4th / 8th / 16th piece the level-1
// / level-2 / level-3 stores — so the pieces can ride along the k-steps of the next tile.
// A/B knob (tools/build_variant.sh; the product build uses the default): RMD_W8_AUXH = cache-policy
// bits of the level 1-3 stores (-1: the same as level 0's AUX)
#ifndef RMD_W8_AUXH
#define RMD_W8_AUXH -1
#endif
template <int AUX>
constexpr int kAuxUpper = RMD_W8_AUXH < 0 ? AUX : RMD_W8_AUXH;

template <int S, int AUX>
__device__ __forceinline__ void epi_piece(const f32x16 (&acc)[8], const Ctx& c, const LaneOff& lo, EpiState& st) {
    constexpr int m = S >> 1, tc = S & 1;
    // level 0: chunk rows 2m, 2m+1 x cols 8 tc + 4h .. +3 — this lane's own values
    {
        const i32x4 d = {(int)pk(V(acc, 2 * m, tc, 0), V(acc, 2 * m, tc, 1)),
                         (int)pk(V(acc, 2 * m, tc, 2), V(acc, 2 * m, tc, 3)),
                         (int)pk(V(acc, 2 * m + 1, tc, 0), V(acc, 2 * m + 1, tc, 1)),
                         (int)pk(V(acc, 2 * m + 1, tc, 2), V(acc, 2 * m + 1, tc, 3))};
        __builtin_amdgcn_raw_buffer_store_b128(d, c.l[0].rsrc,
                                               (int)(lo.o0[tc] + (unsigned)m * c.l[0].rs + (m >= 4 ? c.l[0].hd : 0u)),
                                               0, AUX);
    }
    // level-1 sums of level-1 row m, col group tc: cols {2h, 2h+1} (tc 0) / {4+2h, 5+2h} (tc 1)
#pragma unroll
    for (int u = 0; u < 2; ++u)
        st.s1[m][tc][u] = (V(acc, 2 * m, tc, 2 * u) + V(acc, 2 * m, tc, 2 * u + 1)) +
                          (V(acc, 2 * m + 1, tc, 2 * u) + V(acc, 2 * m + 1, tc, 2 * u + 1));
    if constexpr ((S & 3) == 3) {
        // level-1 chunk row p (rows 2p, 2p+1) complete: lane h stores quad h (cols 4h .. 4h+3).  Per
        // row, x = cols {2h, 2h+1}, y = cols {4+2h, 5+2h}; the swap leaves lanes h = 0 with cols 0-3
        // and lanes h = 1 with cols 4-7 as (x, y)
        constexpr int p = S >> 2;
        unsigned x0 = pk(0.25f * st.s1[2 * p][0][0], 0.25f * st.s1[2 * p][0][1]);
        unsigned y0 = pk(0.25f * st.s1[2 * p][1][0], 0.25f * st.s1[2 * p][1][1]);
        unsigned x1 = pk(0.25f * st.s1[2 * p + 1][0][0], 0.25f * st.s1[2 * p + 1][0][1]);
        unsigned y1 = pk(0.25f * st.s1[2 * p + 1][1][0], 0.25f * st.s1[2 * p + 1][1][1]);
        swp(x0, y0);
        swp(x1, y1);
        const i32x4 d = {(int)x0, (int)y0, (int)x1, (int)y1};
        __builtin_amdgcn_raw_buffer_store_b128(d, c.l[1].rsrc,
                                               (int)(lo.o1 + (unsigned)p * c.l[1].rs + (p >= 2 ? c.l[1].hd : 0u)), 0, kAuxUpper<AUX>);
        // level-2 sums of level-2 row p: lane h holds cols {h, 2+h}
#pragma unroll
        for (int cg = 0; cg < 2; ++cg)
            st.s2[p][cg] = (st.s1[2 * p][cg][0] + st.s1[2 * p][cg][1]) + (st.s1[2 * p + 1][cg][0] + st.s1[2 * p + 1][cg][1]);
    }
    if constexpr ((S & 7) == 7) {
        // level-2 rows 2k, 2k+1 complete (k = S >> 3): lanes h -> row 2k+h, 4 cols (8 B)
        constexpr int k = S >> 3;
        unsigned x = pk(0.0625f * st.s2[2 * k][0], 0.0625f * st.s2[2 * k][1]);          // row 2k:   cols h, 2+h
        unsigned y = pk(0.0625f * st.s2[2 * k + 1][0], 0.0625f * st.s2[2 * k + 1][1]);  // row 2k+1: cols h, 2+h
        swp(x, y);          // lane h now holds row 2k+h: x = cols {0,2}, y = cols {1,3}
        const i32x2 d = {(int)__builtin_amdgcn_perm(y, x, 0x05040100u), (int)__builtin_amdgcn_perm(y, x, 0x07060302u)};
        __builtin_amdgcn_raw_buffer_store_b64(d, c.l[2].rsrc,
                                              (int)(lo.o2 + (unsigned)(2 * k) * c.l[2].rs + (k >= 1 ? c.l[2].hd : 0u)), 0, kAuxUpper<AUX>);
    }
    if constexpr (S == 15) {
        // level 3: rows 0, 1 (level-2 rows 0-1 / 2-3), cols 0, 1 (level-2 cols {0,1} / {2,3});
        // own partial of col cg is level-2 col 2cg+h; the swap adds the other half's
        float a0[2], a1[2];
#pragma unroll
        for (int cg = 0; cg < 2; ++cg) {
            a0[cg] = st.s2[0][cg] + st.s2[1][cg];
            a1[cg] = st.s2[2][cg] + st.s2[3][cg];
        }
        unsigned x0 = __float_as_uint(a0[0]), y0 = __float_as_uint(a1[0]);
        unsigned x1 = __float_as_uint(a0[1]), y1 = __float_as_uint(a1[1]);
        swp(x0, y0);        // lane h: x0 + y0 = full row-h sum of col 0
        swp(x1, y1);
        const float inv = 1.0f / 64.0f;
        const unsigned v = pk(inv * (__uint_as_float(x0) + __uint_as_float(y0)),
                              inv * (__uint_as_float(x1) + __uint_as_float(y1)));
        __builtin_amdgcn_raw_buffer_store_b32((int)v, c.l[3].rsrc, (int)lo.o3, 0, kAuxUpper<AUX>);
    }
}
#undef V

}  // namespace pipe

namespace w8 {

// ---- padded, swizzle-free A layout -------------------------------------------------------------
// LDS row of block target (y, x) = (x>>3)*128 + y*8 + (x&7), rows 528 B apart (256 bf16 + 16 B pad).
// The 32 targets of MFMA tile ti (4 rows x 8 cols) are then the consecutive LDS rows
// (ti&1)*128 + (ti>>1)*32 + j, so lane (j, h)'s fragment of tile ti at k-step s sits at
//   base[ti&1] + (ti>>1)*32*528 + 32*s,   base[e] = (e*128 + j)*528 + 16h:
// two address VGPRs for the whole tile loop, everything else an instruction immediate (<= 51168).
// Banks: 528 B = 33 x 16 B, so a ds_read_b128 lane group's 16 rows land in 16-B slots (row + chunk)
// mod 16 = j mod 16 over lanes {0-3,12-15,20-27} and {4-11,16-19,28-31}: conflict-free, no XOR.
constexpr unsigned kPadRow = 528;

__device__ __forceinline__ int pad_row(int y, int x) { return ((x >> 3) << 7) + (y << 3) + (x & 7); }

// ---- B-fragment register ring ------------------------------------------------------------------
// k-step s of every tile lives in slot s % 8 and is loaded 7 k-steps (56 MFMAs) ahead — the previous
// tile's k-steps 9-15 load this tile's 0-6 — instead of all 16 (64 VGPRs) being held for the whole
// tile; the 32 VGPRs freed double-buffer the A fragments: k-step s+1's 8 fragments are read at the
// top of k-step s.  One scheduling region per k-step keeps both sets of loads where they are issued.
constexpr int kEpiStores = 24;  // buffer stores of one ping-pong epilogue (23 in the .s), for vmcnt_pad_n
constexpr int kRing = 8;

template <int S>
__device__ __forceinline__ void read_a8(bf16x8 (&a)[8], const unsigned char* smem, unsigned b0, unsigned b1) {
#pragma unroll
    for (int ti = 0; ti < 8; ++ti)
        a[ti] = *reinterpret_cast<const bf16x8*>(smem + ((ti & 1) ? b1 : b0) + (unsigned)((ti >> 1) * 32 * kPadRow + 32 * S));
}

template <int S>
__device__ __forceinline__ void ksteps_ring(f32x16 (&acc)[8], bf16x8 (&acur)[8], bf16x8 (&anext)[8],
                                            bf16x8 (&ring)[kRing], const unsigned char* smem, unsigned b0,
                                            unsigned b1, const __bf16* cur, const __bf16* nxt) {
    if constexpr (S < 16) {
        if constexpr (S + 1 < 16) read_a8<S + 1>(anext, smem, b0, b1);
        {
            constexpr int T = S + kRing - 1;
            ring[T % kRing] = *reinterpret_cast<const bf16x8*>((T < 16 ? cur : nxt) + 512 * (T & 15));
        }
        const f32x16 zero = {};
#pragma unroll
        for (int ti = 0; ti < 8; ++ti)
            acc[ti] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[ti], ring[S % kRing], S == 0 ? zero : acc[ti], 0, 0, 0);
        // order inside the region: the 8 LDS reads of k-step S+1 and the ring load first, then the MFMAs
        if constexpr (S + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        __builtin_amdgcn_sched_barrier(0);
        ksteps_ring<S + 1>(acc, anext, acur, ring, smem, b0, b1, cur, nxt);
    }
}

template <int S, int AUX>
__device__ __forceinline__ void epilogue(const f32x16 (&acc)[8], const pipe::Ctx& c, const pipe::LaneOff& lo,
                                         pipe::EpiState& st) {
    if constexpr (S < 16) {
        pipe::epi_piece<S, AUX>(acc, c, lo, st);
        epilogue<S + 1, AUX>(acc, c, lo, st);
    }
}

// Balanced schedule (host: w8_balance).
//  * pair: the last block row has at most 8 valid target rows and W % 32 == 0, so two horizontally
//    adjacent last-row blocks share one workgroup: rows 0-7 of its virtual 16x16 block are block
//    cb's rows, rows 8-15 block cb+1's (A staging and the stores' second-half delta Lvl::hd follow),
//    and no workgroup spends half its MFMAs on rows past the map (cfg2: 55 = 3 x 16 + 7).
//  * helpers: with fewer primary workgroups (one per block x batch) than CUs, every primary stops
//    after qfull query tiles and one helper per primary, dispatched after all primaries (so it lands
//    on a CU with no primary), re-stages that block's A and runs tiles [qfull, nqt).
struct Bal {
    int pair;        // last block row paired
    int nprim;       // primary workgroups (blocks x batch x qsplit)
    int qfull;       // query tiles of a primary when helpers exist (== nqt otherwise)
    int helpers;     // 1: one helper per primary
};

}  // namespace w8

// Ping-pong phases: the two waves of each SIMD (w and w + 4) alternate an MFMA phase and an epilogue
// phase, separated by workgroup barriers, so one wave's pooling VALU and stores run while its partner
// owns the matrix pipe (free-running partners drift into lock step: PMC of the free-running kernel
// showed VALU co-issued with MFMA in a third of its VALU cycles; 0.221 vs 0.242 ms,
// profiles/gemm_ab_r02_pp.json).  AUX = cache-policy bits of the pyramid stores (2 = non-temporal:
// 0.213-0.216 vs 0.305-0.309 ms plain, profiles/gemm_ab_r02_cpol.json).
template <int AUX>
__global__ void __launch_bounds__(512, 1)
corr_pyramid_w8(const __bf16* __restrict__ opA, const __bf16* __restrict__ opB, PyrGeom g, int qsplit,
                __half* __restrict__ pyr, w8::Bal bal) {
    constexpr int Cp = 256, CPR = Cp / 8, WAVES = 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int H = g.height, W = g.width, N = H * W;
    const int ncb = (W + 15) >> 4;
    const int nrb = (H + 15) >> 4;
    const int nqt = g.slots >> 5;                 // query tiles (tiles layout: slots % 32 == 0)
    // blocks per image: full blocks, then (pair) the last row's blocks two per workgroup
    const int nfull = bal.pair ? (nrb - 1) * ncb : nrb * ncb;
    const int nblk = nfull + (bal.pair ? ncb / 2 : 0);
    const int orig = blockIdx.x;
    int lid, q_lo = 0, q_hi = nqt;
    if (orig < bal.nprim) {
        // primaries: XCD-aware remap over the primary range (XCD k runs the k-th eighth)
        const int nwg = bal.nprim;
        const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
        lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
        if (bal.helpers) q_hi = bal.qfull;
    } else {
        // helpers: the same logical id as their primary, placed by blockIdx.x - nprim; nprim is a
        // multiple of 8 when helpers exist, so a helper lands on its primary's XCD (its batch's L2)
        const int hid = orig - bal.nprim;
        const int nwg = bal.nprim;
        const int xcd = hid & 7, qq = nwg >> 3, rr = nwg & 7;
        lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (hid >> 3);
        q_lo = bal.qfull;
    }
    const int ib = lid % nblk;
    const int rest = lid / nblk;
    const int split = rest % qsplit;
    const int b = rest / qsplit;
    const bool paired = ib >= nfull;
    const int tb = paired ? (nrb - 1) * ncb + 2 * (ib - nfull) : ib;
    const int rb = tb / ncb, cb = tb - rb * ncb;
    const int ty0 = rb * 16, tx0 = cb * 16;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 31, h = lane >> 5;

    const __bf16* gA = opA + (size_t)b * N * Cp;
    // 16 pieces per thread, all loads in flight before the first LDS store (a load-store loop pays one
    // HBM round trip per piece before the first MFMA)
    constexpr int kPieces = 256 * CPR / (64 * WAVES);
    uint4 av[kPieces];
#pragma unroll
    for (int i = 0; i < kPieces; ++i) {
        const int id = tid + i * 64 * WAVES;
        const int row = id / CPR, c = id - row * CPR;
        // virtual row y >= 8 of a paired block = row y - 8 of the next column block
        const bool second = paired && (row >> 4) >= 8;
        const int ty = ty0 + (row >> 4) - (second ? 8 : 0), tx = tx0 + (row & 15) + (second ? 16 : 0);
        av[i] = make_uint4(0, 0, 0, 0);
        if (ty < H && tx < W) av[i] = *reinterpret_cast<const uint4*>(gA + (size_t)(ty * W + tx) * Cp + c * 8);
    }
#pragma unroll
    for (int i = 0; i < kPieces; ++i) {
        const int id = tid + i * 64 * WAVES;
        const int row = id / CPR, c = id - row * CPR;
        *reinterpret_cast<uint4*>(smem + (size_t)w8::pad_row(row >> 4, row & 15) * w8::kPadRow + c * 16) = av[i];
    }
    __syncthreads();

    const unsigned pb0 = (unsigned)j * w8::kPadRow + 16u * h, pb1 = pb0 + 128u * w8::kPadRow;

    // store context per level: chunk rows cr0 .. of this block (th = 2, 2, 1, 1 target rows each),
    // chunks cc0 .. (tw = 4, 4, 4, 2 columns)
    pipe::Ctx c;
    const unsigned S = (unsigned)g.slots;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const int crows = l <= 1 ? 8 >> l : 4 >> (l - 2);       // chunk rows per 16-row block: 8, 4, 4, 2
        const int cpb = l == 0 ? 4 : (l == 1 ? 2 : 1);          // chunks per 16-column block
        const int cbytes = l <= 1 ? 16 : (l == 2 ? 8 : 4);      // chunk bytes
        const int cr0 = rb * crows, cc0 = cb * cpb;
        const bool lv = l < g.levels;
        const int rows = lv ? max(0, min(crows, g.ty[l] - cr0)) : 0;
        const unsigned cs = S * (unsigned)cbytes;
        const unsigned rs = lv ? (unsigned)g.tx[l] * cs : 0u;
        const size_t base = lv ? ((size_t)g.off[l] * 2 + (((size_t)b * g.ty[l] + cr0) * g.tx[l] + cc0) * (size_t)cs) : 0;
        const unsigned char* bp = reinterpret_cast<const unsigned char*>(pyr) + base;
        const unsigned lo32 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)bp);
        const unsigned hi32 = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)bp >> 32));
        c.l[l].rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi32 << 32) | lo32), (short)0,
                                                        (int)__builtin_amdgcn_readfirstlane((unsigned)rows * rs), 0x00020000);
        c.l[l].rs = __builtin_amdgcn_readfirstlane(rs);
        c.l[l].cs = __builtin_amdgcn_readfirstlane(cs);
        c.l[l].nq = __builtin_amdgcn_readfirstlane(lv ? max(0, min(cpb, g.tx[l] - cc0)) : 0);
        c.l[l].hd = paired ? __builtin_amdgcn_readfirstlane((unsigned)cpb * cs - (unsigned)(crows / 2) * rs) : 0u;
    }

    // B operand in fragment order (prep_pair): tile qt, k-step s = 1 KiB at ((b nqt + qt) 16 + s) KiB
    const __bf16* gB = opB + ((size_t)b * nqt * 1024 + lane) * 8;
    const int stride = WAVES * qsplit;
    // this workgroup's query tiles: [q_lo, q_hi) (all of them unless helpers split the block);
    // waves 4-7 start one phase late; every wave runs 2 * nmax + 1 barriers
    const int f0 = q_lo + split * WAVES;
    int qt = f0 + w;
    const int nmax = f0 < q_hi ? (q_hi - f0 + stride - 1) / stride : 0;
    const int nw = qt < q_hi ? (q_hi - qt + stride - 1) / stride : 0;
    const bool late = w >= 4;
    unsigned b0 = pb0, b1 = pb1;
    asm volatile("" : "+v"(b0), "+v"(b1));
    bf16x8 ring[w8::kRing];
    if (nw > 0) {
#pragma unroll
        for (int s = 0; s < w8::kRing - 1; ++s) ring[s] = *reinterpret_cast<const bf16x8*>(gB + (size_t)qt * 8192 + 512 * s);
    }
    vmcnt_pad_n<w8::kEpiStores>(pyr);
    if (late) __builtin_amdgcn_s_barrier();
    for (int k = 0; k < nmax; ++k) {
        f32x16 acc[8];
        const int qn = qt + stride;
        if (k < nw) {
            // both phases in one wave-uniform branch: every path that loads ring fragments issues
            // the epilogue stores after them (vmcnt_pad_n, rmd_common.h)
            bf16x8 a0[8], a1[8];
            w8::read_a8<0>(a0, smem, b0, b1);
            w8::ksteps_ring<0>(acc, a0, a1, ring, smem, b0, b1, gB + (size_t)qt * 8192,
                               gB + (size_t)min(qn, nqt - 1) * 8192);
            __builtin_amdgcn_s_barrier();
            const pipe::LaneOff lo = pipe::lane_offsets(c, qt * 32 + j, h);
            pipe::EpiState st;
            w8::epilogue<0, AUX>(acc, c, lo, st);
            __builtin_amdgcn_s_barrier();
            qt = qn;
            continue;
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_barrier();
        qt = qn;
    }
    if (!late) __builtin_amdgcn_s_barrier();
}

// GEMM path for a call: the w8 kernel needs bf16 operands, an fp16 pyramid, C <= 256 and 32-bit
// store offsets (one 16-row band of level 0 < 1 GiB); larger maps (e.g. 4K frames) take the
// stationary kernel (64-bit addressing), everything else the tiled kernel.
enum class Path { W8, STATIONARY, TILED, X3 };

// query slots of the tiles layout for an H x W map (rmd.h)
long long tiles_slots(int H, int W) {
    return (long long)(H / 2) * ((W + 15) / 16) * 32 + ((H & 1) ? (long long)(W + 31) / 32 * 32 : 0);
}

Path gemm_path(const rmd_pyramid_desc& d, int C, int compute) {
    const int Cp = (C + kKC - 1) / kKC * kKC;
    if (compute == RMD_BF16X3) return x3::eligible(d, C) ? Path::X3 : Path::TILED;     // TILED: exact f32
    if (compute != RMD_BF16 || d.storage != RMD_F16 || Cp != 256) return Path::TILED;
    const double slots = (double)tiles_slots(d.height, d.width);
    const double span0 = 16.0 * ((d.width + 7) / 8 * 8) * slots * 2;   // one 16-row band of level 0 (bytes)
    if (span0 >= (double)(1u << 30)) return Path::STATIONARY;
    return Path::W8;
}

// the pyramid layout the GEMM of a call writes
int path_layout(Path p) { return p == Path::W8 ? RMD_LAYOUT_TILES : RMD_LAYOUT_ROWS; }

template <bool F32>
int launch_prepare(const float* f1, const float* f2, int C, float scale, const rmd_pyramid_desc& d,
                   void* workspace, hipStream_t st) {
    using T = typename Operand<F32>::T;
    const int N = d.height * d.width;
    const int Cp = (C + kKC - 1) / kKC * kKC;
    T* opA = reinterpret_cast<T*>(workspace);
    T* opB = opA + (size_t)d.batch * N * Cp;
    dim3 pg((N + 63) / 64, Cp / 64, d.batch);
    // bf16 perf path: the scale (1/sqrt(C) for raft.CorrBlock) is folded into fmap2 before rounding
    // (exact for a power of two, e.g. C = 256 or raft_fs's 1); the f32 parity path scales the f32
    // accumulators in the epilogue
    const float prescale = F32 ? 1.0f : scale;
    if constexpr (!F32) {
        if (gemm_path(d, C, RMD_BF16) == Path::W8) {
            const int S = d.query_slots;
            const int nqt = S / 32;
            const int lds = kPrepPx * kPrepStride;
            const int nx = ((N > S ? N : S) + kPrepPx - 1) / kPrepPx;
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(prep_pair), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            prep_pair<<<dim3(nx, d.batch, 2), 512, lds, st>>>(f1, f2, opA, opB, C, d.height, d.width, S, nqt, prescale);
            return check_launch("rmd_corr_prepare");
        }
    }
    prep_operand<T><<<pg, kThreads, 0, st>>>(f2, opA, C, N, Cp, prescale);
    prep_operand<T><<<pg, kThreads, 0, st>>>(f1, opB, C, N, Cp, 1.0f);
    return check_launch("rmd_corr_prepare");
}

// Balanced schedule of the w8 GEMM (w8::Bal): the last block row is paired when it holds at most 8
// target rows.  Measured at cfg2 (profiles/gemm_ab_r02_bal.json): 0.2280 (off) / 0.2257 (pairing) /
// 0.2271 ms (pairing + one helper workgroup per primary running its tail query tiles on the CUs left
// free), all bitwise identical — evening out the per-CU work does not move the kernel: it is bound by
// the chip-wide pyramid write stream, not by any CU's share.  Pairing stays (the same time for 12.5 %
// fewer MFMAs, 224 instead of 256 workgroups); the helper schedule is kept in the kernel (Bal) but not
// used.
w8::Bal w8_balance(const rmd_pyramid_desc& d, int qs) {
    const int nqt = d.query_slots / 32;
    const int nrb = (d.height + 15) / 16, ncb = (d.width + 15) / 16;
    const int rows_last = d.height - 16 * (nrb - 1);
    w8::Bal bal{0, nrb * ncb * d.batch * qs, nqt, 0};
    if (qs != 1) return bal;
    if (nrb >= 2 && rows_last <= 8 && d.width % 32 == 0) {
        bal.pair = 1;
        bal.nprim = ((nrb - 1) * ncb + ncb / 2) * d.batch;
    }
    return bal;
}

template <bool F32, typename TOut>
int launch_pyramid(int C, float scale, const rmd_pyramid_desc& d, void* pyramid, void* workspace, hipStream_t st) {
    using T = typename Operand<F32>::T;
    const int N = d.height * d.width;
    const int Cp = (C + kKC - 1) / kKC * kKC;
    T* opA = reinterpret_cast<T*>(workspace);
    T* opB = opA + (size_t)d.batch * N * Cp;
    const PyrGeom geom = make_geom(d);
    if constexpr (!F32 && sizeof(TOut) == 2) {
        const Path path = gemm_path(d, C, RMD_BF16);
        const int nblk = ((d.height + 15) / 16) * ((d.width + 15) / 16);
        __half* out = reinterpret_cast<__half*>(pyramid);
        if (path == Path::W8) {
            // non-temporal pyramid stores (AUX = 2); query tiles split over workgroups only when the
            // blocks alone do not fill the chip
            const int nqt = d.query_slots / 32;
            int qs = 1;
            while (nblk * d.batch * qs < 256 && qs * 32 <= nqt) qs *= 2;
            auto kern = corr_pyramid_w8<2>;
            const int lds_w8 = 256 * (int)w8::kPadRow;
            const w8::Bal bal = w8_balance(d, qs);
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds_w8);
            kern<<<bal.nprim * (bal.helpers ? 2 : 1), 512, lds_w8, st>>>(opA, opB, geom, qs, out, bal);
            return check_launch("rmd_corr_pyramid/gemm-w8");
        }
        if (path == Path::STATIONARY) {
            const int nqt = (N + 31) / 32;
            int qsplit = 1;
            while (nblk * d.batch * qsplit < 256 && qsplit * 16 <= nqt) qsplit *= 2;
            const int lds = 256 * Cp * 2;
            const int nwg = nblk * d.batch * qsplit;
            __half* trash = reinterpret_cast<__half*>(opB + (size_t)d.batch * nqt * 32 * Cp);
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(corr_pyramid_stationary<2, 0>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            corr_pyramid_stationary<2, 0><<<nwg, STraits<2>::kThreads, lds, st>>>(opA, opB, geom, qsplit, out, trash);
            return check_launch("rmd_corr_pyramid/gemm-stationary");
        }
    }
    constexpr int lds = (kNT + kBQ) * stage_stride<F32>();
    auto kern = corr_pyramid_tiled<F32, TOut>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    dim3 grid((N + kBQ - 1) / kBQ, ((d.height + 15) / 16) * ((d.width + 15) / 16), d.batch);
    kern<<<grid, kThreads, lds, st>>>(opA, opB, Cp, F32 ? scale : 1.0f, geom, reinterpret_cast<TOut*>(pyramid));
    return check_launch("rmd_corr_pyramid/gemm");
}

int check_args(const rmd_pyramid_desc* d, int channels, int compute) {
    RMD_REQUIRE(d, RMD_ERR_ARG, "rmd_corr_pyramid: null desc");
    RMD_REQUIRE(channels > 0, RMD_ERR_SHAPE, "rmd_corr_pyramid: channels must be > 0");
    RMD_REQUIRE(d->levels >= 1 && d->levels <= RMD_MAX_LEVELS, RMD_ERR_SHAPE, "rmd_corr_pyramid: bad levels");
    RMD_REQUIRE(compute == RMD_F32 || compute == RMD_BF16 || compute == RMD_BF16X3, RMD_ERR_ARG,
                "rmd_corr_pyramid: compute must be F32, BF16 or BF16X3");
    RMD_REQUIRE(d->storage == RMD_F32 || d->storage == RMD_F16 || d->storage == RMD_S24, RMD_ERR_ARG,
                "rmd_corr_pyramid: storage must be F32, F16 or S24");
    RMD_REQUIRE(d->storage != RMD_S24 || gemm_path(*d, channels, compute) == Path::X3, RMD_ERR_ARG,
                "rmd_corr_pyramid: S24 storage is written by the BF16X3 GEMM only (C <= 256; describe with "
                "rmd_pyramid_describe_for)");
    const int want = path_layout(gemm_path(*d, channels, compute));
    RMD_REQUIRE(d->layout == want, RMD_ERR_ARG,
                "rmd_corr_pyramid: the %s GEMM writes layout %d, desc has layout %d (describe with rmd_pyramid_describe_for)",
                want == RMD_LAYOUT_TILES ? "w8" : "selected", want, d->layout);
    return RMD_OK;
}

}  // namespace
}  // namespace rmd

extern "C" int rmd_pyramid_describe_for(int batch, int height, int width, int levels, int storage, int channels,
                                        int compute, rmd_pyramid_desc* d) {
    int rc = rmd_pyramid_describe_layout(batch, height, width, levels, storage, RMD_LAYOUT_ROWS, d);
    if (rc || channels <= 0) return rc;
    // S24 is an output format of the x3 GEMM: any other GEMM of this call stores F32
    if (storage == RMD_S24 && rmd::gemm_path(*d, channels, compute) != rmd::Path::X3)
        return rmd_pyramid_describe_layout(batch, height, width, levels, RMD_F32, RMD_LAYOUT_ROWS, d);
    if (rmd::gemm_path(*d, channels, compute) == rmd::Path::W8)
        rc = rmd_pyramid_describe_layout(batch, height, width, levels, storage, RMD_LAYOUT_TILES, d);
    return rc;
}

extern "C" size_t rmd_corr_pyramid_workspace_bytes(const rmd_pyramid_desc* d, int channels, int compute) {
    if (!d || channels <= 0) return 0;
    if (compute == RMD_BF16X3) {
        if (rmd::x3::eligible(*d, channels)) return rmd::x3::workspace_bytes(*d);
        compute = RMD_F32;
    }
    const size_t Cp = (size_t)(channels + rmd::kKC - 1) / rmd::kKC * rmd::kKC;
    const size_t es = compute == RMD_F32 ? 4 : 2;
    const size_t N = (size_t)d->height * d->width;
    const size_t S = d->query_slots > 0 && (size_t)d->query_slots > N ? (size_t)d->query_slots : N;
    const size_t Npad = (S + 31) / 32 * 32;                         // B operand padded to 32-query tiles
    return (size_t)d->batch * (N + Npad) * Cp * es + 32 * 1024;     // + trash slots (<= 32 x 1 KiB)
}

extern "C" const char* rmd_corr_gemm_kernel(const rmd_pyramid_desc* d, int channels, int compute) {
    if (!d || channels <= 0) return "invalid";
    switch (rmd::gemm_path(*d, channels, compute)) {
        case rmd::Path::W8: return "w8";
        case rmd::Path::STATIONARY: return "stationary";
        case rmd::Path::X3: return "x3";
        default: return "tiled";
    }
}

extern "C" int rmd_corr_prepare(const float* fmap1, const float* fmap2, int channels, float scale,
                                const rmd_pyramid_desc* d, int compute, void* workspace, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && workspace, RMD_ERR_ARG, "rmd_corr_prepare: null pointer");
    int rc = rmd::check_args(d, channels, compute);
    if (rc) return rc;
    hipStream_t st = rmd::as_stream(stream);
    if (compute == RMD_BF16X3) {
        if (rmd::gemm_path(*d, channels, compute) == rmd::Path::X3)
            return rmd::x3::prepare(fmap1, fmap2, channels, scale, *d, workspace, st);
        compute = RMD_F32;
    }
    return compute == RMD_BF16 ? rmd::launch_prepare<false>(fmap1, fmap2, channels, scale, *d, workspace, st)
                               : rmd::launch_prepare<true>(fmap1, fmap2, channels, scale, *d, workspace, st);
}

extern "C" int rmd_corr_pyramid_prepared(int channels, float scale, const rmd_pyramid_desc* d, int compute,
                                         void* pyramid, void* workspace, void* stream) {
    RMD_REQUIRE(pyramid && workspace, RMD_ERR_ARG, "rmd_corr_pyramid_prepared: null pointer");
    int rc = rmd::check_args(d, channels, compute);
    if (rc) return rc;
    hipStream_t st = rmd::as_stream(stream);
    if (compute == RMD_BF16X3) {
        if (rmd::gemm_path(*d, channels, compute) == rmd::Path::X3) return rmd::x3::pyramid(*d, pyramid, workspace, st);
        compute = RMD_F32;
    }
    if (compute == RMD_BF16)
        return d->storage == RMD_F16 ? rmd::launch_pyramid<false, __half>(channels, scale, *d, pyramid, workspace, st)
                                     : rmd::launch_pyramid<false, float>(channels, scale, *d, pyramid, workspace, st);
    return d->storage == RMD_F16 ? rmd::launch_pyramid<true, __half>(channels, scale, *d, pyramid, workspace, st)
                                 : rmd::launch_pyramid<true, float>(channels, scale, *d, pyramid, workspace, st);
}

extern "C" int rmd_corr_pyramid(const float* fmap1, const float* fmap2, int channels, float scale,
                                const rmd_pyramid_desc* d, int compute, void* pyramid, void* workspace, void* stream) {
    int rc = rmd_corr_prepare(fmap1, fmap2, channels, scale, d, compute, workspace, stream);
    if (rc) return rc;
    return rmd_corr_pyramid_prepared(channels, scale, d, compute, pyramid, workspace, stream);
}
