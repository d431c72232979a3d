// corr_grad.hip — the two GEMMs of the RAFT correlation backward as split-bf16 (x3) MFMA GEMMs.
//
// Backward of raft.CorrBlock.__init__ (qzed/raft-meets-dicl src/models/impls/raft.py:31-47: corr =
// fmap1^T fmap2 / sqrt(C), then avg_pool2d per level).  With the lookup backward's dense
// query-minor gradient G (B, T, N) over the T pooled targets of all levels (corr_backward.hip) and
// the pooled, scaled target features P (B, C, T), autograd of the matmul is
//   dfmap1 = P . G           (B, C, N)   K = T'       layout 3: G blocked along k (targets)
//   dP     = fmap1 . G^T     (B, C, T')  K = N        layout 2: G blocked along n (targets)
// B operand layouts (element (k, n), ldb = row stride):
//   0: k * ldb + n (K x Nc, n contiguous)       1: n * ldb + k (Nc x K, k contiguous)
//   2: ((n / 8) * ldb + k) * 8 + n % 8          3: ((k / 8) * ldb + n) * 8 + k % 8
// (2 / 3 are the 8-target chunked order of the pyramid gradient G, corr_backward.hip)
// (dP is then un-pooled onto dfmap2 by rmd_corr_unpool_targets).  Both run here in fp32 accuracy
// as three bf16 MFMA products per k-step, x = hi + lo, hi = bf16(x), lo = bf16(x - hi):
//   acc += A_lo.B_hi + A_hi.B_lo + A_hi.B_hi        (the dropped lo.lo term is ~2^-16 relative)
// — the same split as the forward x3 GEMM (corr_pyramid_x3.hip) — instead of hipBLASLt's exact-f32
// MFMA path (v_mfma_f32_32x32x2_f32 runs at 1/16 of the bf16 rate).
//
// Geometry: one workgroup (8 waves, 2 per SIMD) owns a 256 (M) x 128 (Nc) output tile; wave
// (wm = w & 3, wn = w >> 2) owns 64 x 64 = 2 x 2 tiles of v_mfma_f32_32x32x16_bf16.  K runs in
// 32-deep chunks through two LDS buffers (software pipeline, one barrier per chunk): chunk c+1's fp32
// operands, loaded into registers during chunk c-1, are split into hi / lo and stored to the idle
// buffer while chunk c's MFMAs read the other (one 144-B row per operand row: hi 64 B | lo 64 B | 16 B
// pad = 9 x 16 B, so the 8-lane groups of a ds_read_b128 hit 8 distinct 16-B bank slots).  K is split
// over `splits` workgroups when the tile grid alone does not fill the 256 CUs; the partial tiles go to
// a workspace and a second kernel sums them in a fixed order (deterministic, no atomics).

#include "rmd_common.h"

namespace rmd {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kTM = 256, kKC = 32;
constexpr int kRowB = 144;                                  // hi 64 B | lo 64 B | pad 16 B (9 x 16 B: odd)
constexpr int kLdsA = kTM * kRowB;                          // 36,864 B per buffer
// output tile kTM x TN: TN = 128 (two buffers 110,592 B of LDS) or 256 (147,456 B: A re-read half as often)
template <int TN> constexpr int lds_buf() { return kLdsA + TN * kRowB; }

struct GemmArgs {
    const float* A;
    const float* Bm;
    const unsigned short* Bh;   // BBF: B as bfloat16 bits (layouts 2 / 3), instead of Bm
    float* out;                 // final output (splits == 1) or the split workspace
    long long lda, ldb;         // row strides (elements)
    long long sa, sb, so;       // batch strides (elements) of A, Bm, out
    int M, K, Nc, batch;
    int kper;                   // K per split (multiple of kKC)
    int splits, ntm, ntn;
};

__device__ __forceinline__ void split4(float a, float b, float c, float d, bf16x4& hi, bf16x4& lo) {
    hi[0] = (__bf16)a;
    hi[1] = (__bf16)b;
    hi[2] = (__bf16)c;
    hi[3] = (__bf16)d;
    lo[0] = (__bf16)(a - (float)hi[0]);
    lo[1] = (__bf16)(b - (float)hi[1]);
    lo[2] = (__bf16)(c - (float)hi[2]);
    lo[3] = (__bf16)(d - (float)hi[3]);
}

// the 4 consecutive elements k .. k + 3 at `at` (the address of element k; row valid, k < kend
// checked per element)
template <bool VEC>
__device__ __forceinline__ float4 load4(const float* __restrict__ at, int k, int kend) {
    if (VEC && k + 3 < kend) return *reinterpret_cast<const float4*>(at);
    float4 v;
    v.x = k + 0 < kend ? at[0] : 0.f;
    v.y = k + 1 < kend ? at[1] : 0.f;
    v.z = k + 2 < kend ? at[2] : 0.f;
    v.w = k + 3 < kend ? at[3] : 0.f;
    return v;
}

// VA / VB: 16-B aligned rows (row stride % 4 == 0, aligned base) -> float4 loads; LAYOUT 0-3 as above.
//
// Software pipeline over 32-deep K chunks with two LDS buffers and one barrier per chunk: at the top
// of chunk c the registers holding chunk c+1's fp32 operands are split into hi / lo and stored to the
// other buffer, chunk c+2's loads are issued into the same registers, then the 24 MFMAs of chunk c run
// from the current buffer; the barrier at the bottom publishes chunk c+1 and frees buffer c for c+2.
// A global load thus has a whole chunk of MFMAs (two, for its first use) to land, and the hi / lo split
// of the next chunk runs beside the current chunk's MFMAs (waves 0-3 and 4-7 share each SIMD).
// X3 = false (compute RMD_BF16, the bf16 precision mode): one bf16 product per k-step (hi.hi), the lo
// halves are neither split nor stored
// BBF (bf16 compute, layouts 2 / 3): B is bfloat16 already (rmd_corr_grad_build_ex's G): 8-byte loads of
// 4 elements, stored to LDS as the hi operand without conversion — the same bits the fp32 path's
// (__bf16) rounding produces from the fp32 G, at half the bytes
template <bool VA, bool VB, int LAYOUT, bool X3 = true, int TN = 128, bool BBF = false>
__global__ void __launch_bounds__(512, 1)
grad_gemm_x3(GemmArgs p) {
    static_assert(!BBF || (!X3 && LAYOUT >= 2), "bfloat16 B: bf16 compute, blocked layouts");
    constexpr int kTN = TN, kLdsBuf = lds_buf<TN>();
    constexpr int NJ = TN / 64;                 // 32-column MFMA tiles per wave (a wave owns 64 x TN/2)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nwg = gridDim.x;
    int id = xcd_block(blockIdx.x, nwg);       // consecutive ids (same batch, same A rows) share an XCD
    const int tn = id % p.ntn;
    id /= p.ntn;
    const int tm = id % p.ntm;
    id /= p.ntm;
    const int split = id % p.splits;
    const int b = id / p.splits;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w & 3, wn = w >> 2;
    const int m0 = tm * kTM, n0 = tn * kTN;
    const int kb = split * p.kper, ke = min(p.K, kb + p.kper);
    const float* __restrict__ A = p.A + (size_t)b * p.sa;
    const float* __restrict__ Bm = BBF ? nullptr : p.Bm + (size_t)b * p.sb;
    const unsigned short* __restrict__ Bh = BBF ? p.Bh + (size_t)b * p.sb : nullptr;

    // per thread: A 4 x float4 (rows m0 + 64 it + tid / 8, k 4 (tid % 8) .. +3); B TN / 64 x float4
    float4 ra[4], rb[TN / 64];
    auto gload = [&](int k0) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int row = m0 + it * 64 + (tid >> 3), k = k0 + (tid & 7) * 4;
            ra[it] = row < p.M ? load4<VA>(A + (size_t)row * p.lda + k, k, ke) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if constexpr (LAYOUT == 0 || LAYOUT == 2) {
            // thread (kq, nq): k rows 2kq, 2kq + 1 of columns 4nq .. 4nq + 3 (16 kq per 16 lanes of a
            // wave group: lanes (kq & 15, n) read 2 k rows x 64 contiguous bytes; waves 0-3 / 4-7 take
            // column halves 0-63 / 64-127; layout 2: 4 consecutive n of one 8-block are contiguous too)
            const int kq = (lane & 3) | ((w & 3) << 2);
#pragma unroll
            for (int nn = 0; nn < TN / 128; ++nn) {
                const int n = n0 + (TN / 2) * (w >> 2) + 64 * nn + 4 * (lane >> 2);
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int k = k0 + 2 * kq + r;
                    float4& d = rb[2 * nn + r];
                    d = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (BBF && k < ke) {
                        const unsigned short* src = Bh + ((size_t)(n >> 3) * p.ldb + k) * 8 + (n & 7);
                        uint2 v;
                        if (VB && n + 3 < p.Nc) {
                            v = *reinterpret_cast<const uint2*>(src);
                        } else {
                            const unsigned e0 = n + 0 < p.Nc ? src[0] : 0u, e1 = n + 1 < p.Nc ? src[1] : 0u;
                            const unsigned e2 = n + 2 < p.Nc ? src[2] : 0u, e3 = n + 3 < p.Nc ? src[3] : 0u;
                            v = make_uint2(e0 | (e1 << 16), e2 | (e3 << 16));
                        }
                        d.x = __uint_as_float(v.x);
                        d.y = __uint_as_float(v.y);
                    } else if (k < ke) {
                        const float* src = LAYOUT == 0 ? Bm + (size_t)k * p.ldb + n
                                                       : Bm + ((size_t)(n >> 3) * p.ldb + k) * 8 + (n & 7);
                        if (VB && n + 3 < p.Nc) {
                            d = *reinterpret_cast<const float4*>(src);
                        } else {
                            d.x = n + 0 < p.Nc ? src[0] : 0.f;
                            d.y = n + 1 < p.Nc ? src[1] : 0.f;
                            d.z = n + 2 < p.Nc ? src[2] : 0.f;
                            d.w = n + 3 < p.Nc ? src[3] : 0.f;
                        }
                    }
                }
            }
        } else {
#pragma unroll
            for (int it = 0; it < TN / 64; ++it) {
                const int row = n0 + it * 64 + (tid >> 3), k = k0 + (tid & 7) * 4;
                // layout 3: k .. k + 3 lie in one 8-block (k % 4 == 0), contiguous like layout 1's row
                if constexpr (BBF) {
                    const unsigned short* src = Bh + ((size_t)(k >> 3) * p.ldb + row) * 8 + (k & 7);
                    uint2 v = make_uint2(0u, 0u);
                    if (row < p.Nc) {
                        if (VB && k + 3 < ke) {
                            v = *reinterpret_cast<const uint2*>(src);
                        } else {
                            const unsigned e0 = k + 0 < ke ? src[0] : 0u, e1 = k + 1 < ke ? src[1] : 0u;
                            const unsigned e2 = k + 2 < ke ? src[2] : 0u, e3 = k + 3 < ke ? src[3] : 0u;
                            v = make_uint2(e0 | (e1 << 16), e2 | (e3 << 16));
                        }
                    }
                    rb[it] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), 0.f, 0.f);
                    continue;
                }
                const float* src = LAYOUT == 1 ? Bm + (size_t)row * p.ldb + k
                                               : Bm + ((size_t)(k >> 3) * p.ldb + row) * 8 + (k & 7);
                rb[it] = row < p.Nc ? load4<VB>(src, k, ke) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    auto lstore = [&](unsigned char* buf) {
        unsigned char* sA = buf;
        unsigned char* sB = buf + kLdsA;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            bf16x4 hi, lo;
            split4(ra[it].x, ra[it].y, ra[it].z, ra[it].w, hi, lo);
            unsigned char* d = sA + (it * 64 + (tid >> 3)) * kRowB + (tid & 7) * 8;
            *reinterpret_cast<bf16x4*>(d) = hi;
            if constexpr (X3) *reinterpret_cast<bf16x4*>(d + 64) = lo;
        }
        if constexpr (LAYOUT == 0 || LAYOUT == 2) {
            // transpose: column 4nq + j of the thread's 2 k rows -> LDS row of that column, k offset 2kq
            const int kq = (lane & 3) | ((w & 3) << 2);
#pragma unroll
            for (int nn = 0; nn < TN / 128; ++nn) {
                const int nr = (TN / 2) * (w >> 2) + 64 * nn + 4 * (lane >> 2);
                const float4 r0 = rb[2 * nn], r1 = rb[2 * nn + 1];
                if constexpr (BBF) {
                    // 4 bf16 per k row packed in (x, y): column j is half j & 1 of word j >> 1
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const unsigned w0 = __float_as_uint(j < 2 ? r0.x : r0.y), w1 = __float_as_uint(j < 2 ? r1.x : r1.y);
                        const unsigned h0 = (w0 >> (16 * (j & 1))) & 0xffffu, h1 = (w1 >> (16 * (j & 1))) & 0xffffu;
                        *reinterpret_cast<unsigned*>(sB + (nr + j) * kRowB + kq * 4) = h0 | (h1 << 16);
                    }
                    continue;
                }
                const float c0[2] = {r0.x, r1.x}, c1[2] = {r0.y, r1.y};
                const float c2[2] = {r0.z, r1.z}, c3[2] = {r0.w, r1.w};
                const float* cols[4] = {c0, c1, c2, c3};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    __bf16 h0 = (__bf16)cols[j][0], h1 = (__bf16)cols[j][1];
                    __bf16 l0 = (__bf16)(cols[j][0] - (float)h0), l1 = (__bf16)(cols[j][1] - (float)h1);
                    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
                    unsigned char* d = sB + (nr + j) * kRowB + kq * 4;
                    *reinterpret_cast<bf16x2*>(d) = bf16x2{h0, h1};
                    if constexpr (X3) *reinterpret_cast<bf16x2*>(d + 64) = bf16x2{l0, l1};
                }
            }
        } else {
#pragma unroll
            for (int it = 0; it < TN / 64; ++it) {
                if constexpr (BBF) {
                    unsigned char* d = sB + (it * 64 + (tid >> 3)) * kRowB + (tid & 7) * 8;
                    *reinterpret_cast<uint2*>(d) = make_uint2(__float_as_uint(rb[it].x), __float_as_uint(rb[it].y));
                    continue;
                }
                bf16x4 hi, lo;
                split4(rb[it].x, rb[it].y, rb[it].z, rb[it].w, hi, lo);
                unsigned char* d = sB + (it * 64 + (tid >> 3)) * kRowB + (tid & 7) * 8;
                *reinterpret_cast<bf16x4*>(d) = hi;
                if constexpr (X3) *reinterpret_cast<bf16x4*>(d + 64) = lo;
            }
        }
    };

    f32x16 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};

    const int j32 = lane & 31, h = lane >> 5;
    const unsigned aoff = (unsigned)((wm * 64 + j32) * kRowB + h * 16);
    const unsigned boff = (unsigned)(kLdsA + (wn * (TN / 2) + j32) * kRowB + h * 16);
    const int nchunk = (ke - kb + kKC - 1) / kKC;

    // prologue: chunk 0 -> buffer 0, chunk 1 in flight in registers
    gload(kb);
    lstore(smem);
    if (nchunk > 1) gload(kb + kKC);
    __syncthreads();
    for (int c = 0; c < nchunk; ++c) {
        unsigned char* cur = smem + (c & 1) * kLdsBuf;
        if (c + 1 < nchunk) {
            lstore(smem + ((c + 1) & 1) * kLdsBuf);             // chunk c+1: registers -> other buffer
            if (c + 2 < nchunk) gload(kb + (c + 2) * kKC);      // chunk c+2 in flight during this chunk
        }
#pragma unroll
        for (int s = 0; s < kKC / 16; ++s) {
            bf16x8 ah[2], al[2], bh[NJ], bl[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const unsigned char* pa = cur + aoff + i * 32 * kRowB + s * 32;
                ah[i] = *reinterpret_cast<const bf16x8*>(pa);
                if constexpr (X3) al[i] = *reinterpret_cast<const bf16x8*>(pa + 64);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const unsigned char* pb = cur + boff + j * 32 * kRowB + s * 32;
                bh[j] = *reinterpret_cast<const bf16x8*>(pb);
                if constexpr (X3) bl[j] = *reinterpret_cast<const bf16x8*>(pb + 64);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    f32x16 t = acc[i][j];
                    if constexpr (X3) {
                        t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], t, 0, 0, 0);
                        t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], t, 0, 0, 0);
                    }
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], t, 0, 0, 0);
                }
        }
        __syncthreads();                                       // chunk c+1 published; buffer c free
    }

    // C tile (32 x 32): lane (j32, h) holds rows 8 (v >> 2) + 4 h + (v & 3) of column j32
    float* __restrict__ o = p.out + ((size_t)split * p.batch + b) * p.so;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int col = n0 + wn * (TN / 2) + j * 32 + j32;
            if (col >= p.Nc) continue;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int row = m0 + wm * 64 + i * 32 + 8 * (v >> 2) + 4 * h + (v & 3);
                if (row < p.M) o[(size_t)row * p.Nc + col] = acc[i][j][v];
            }
        }
}

// out[e] = sum_s ws[s][e] in split order (deterministic)
__global__ void __launch_bounds__(256)
grad_gemm_reduce(const float* __restrict__ ws, long long n, int splits, float* __restrict__ out) {
    const long long i4 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
    if ((n & 3) == 0 && i4 + 3 < n) {
        float4 s = *reinterpret_cast<const float4*>(ws + i4);
        for (int k = 1; k < splits; ++k) {
            const float4 v = *reinterpret_cast<const float4*>(ws + (size_t)k * n + i4);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        *reinterpret_cast<float4*>(out + i4) = s;
    } else {
        // scalar tail (n % 4 != 0, or the last partial group): this thread's 4 elements only
        const long long iend = i4 + 4 < n ? i4 + 4 : n;
        for (long long i = i4; i < iend; ++i) {
            float s = ws[i];
            for (int k = 1; k < splits; ++k) s += ws[(size_t)k * n + i];
            out[i] = s;
        }
    }
}

struct Plan {
    int ntm, ntn, splits, kper, tn;
};

// output-tile width: 256 columns (A operand re-read half as often through L2) once the matrix is wide
// enough, else 128
#ifndef RMD_GG_TN
#define RMD_GG_TN 256
#endif
inline int tile_n(int Nc) { return RMD_GG_TN == 256 && Nc >= 1024 ? 256 : 128; }

// split count: the s minimising (workgroup rounds over 256 CUs) x (K chunks per split) plus the
// workspace traffic of s > 1 in the same unit — each split writes an M x TN partial tile (kTM / kKC = 8
// chunks' worth of operand reads) and the reduce reads s of them and writes one, at 1.5x a chunk's
// cost per byte (profiles/grad_gemm_splits_r05.json: at cfg2 b8 this picks 1 and 2 splits where the
// round-count-only rule picked 8 and 6, 1.12 vs 1.35 ms for the two GEMMs); a larger s must win by 3 %.
// RMD_GG_MAXSPLIT caps s, RMD_GG_OLDPLAN=1 restores the round-4 rule (A/B builds).
#ifndef RMD_GG_MAXSPLIT
#define RMD_GG_MAXSPLIT 8
#endif
#ifndef RMD_GG_OLDPLAN
#define RMD_GG_OLDPLAN 0
#endif
Plan plan(int batch, int M, int K, int Nc) {
    Plan pl{};
    pl.tn = tile_n(Nc);
    pl.ntm = (M + kTM - 1) / kTM;
    pl.ntn = (Nc + pl.tn - 1) / pl.tn;
    const long long tiles = (long long)pl.ntm * pl.ntn * batch;
    const int nch = (K + kKC - 1) / kKC;
    double best = 1e30;
    pl.splits = 1;
    for (int s = 1; s <= RMD_GG_MAXSPLIT && s <= nch; ++s) {
        const long long rounds = (tiles * s + 255) / 256;
        const int per = (nch + s - 1) / s;
        if (RMD_GG_OLDPLAN) {
            const double cost = (double)rounds * per + (s > 1 ? 0.15 * s * (double)tiles / 256.0 : 0.0);
            if (cost < best - 1e-9) {
                best = cost;
                pl.splits = s;
            }
            continue;
        }
        const double ws = s > 1 ? 1.5 * (kTM / kKC) * (2.0 * s + 1.0) * (double)tiles / 256.0 : 0.0;
        const double cost = (double)rounds * per + ws;
        if (cost < best * 0.97) {
            best = cost;
            pl.splits = s;
        }
    }
    const int per = (nch + pl.splits - 1) / pl.splits;
    pl.kper = per * kKC;
    pl.splits = (nch + per - 1) / per;         // no empty split
    return pl;
}

template <bool VA, bool VB, int LAYOUT, int TN>
void launch_gemm_tn(const GemmArgs& a, int nwg, bool x3, hipStream_t st) {
    auto k = x3 ? grad_gemm_x3<VA, VB, LAYOUT, true, TN> : grad_gemm_x3<VA, VB, LAYOUT, false, TN>;
    if constexpr (LAYOUT >= 2) {
        if (a.Bh) k = grad_gemm_x3<VA, VB, LAYOUT, false, TN, true>;
    }
    // the >64 KB LDS opt-in is per device: set it before every launch (cheap host call), so a process
    // that launches on a second GPU gets it too
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * lds_buf<TN>());
    k<<<nwg, 512, 2 * lds_buf<TN>(), st>>>(a);
}

template <bool VA, bool VB, int LAYOUT>
void launch_gemm(const GemmArgs& a, int nwg, bool x3, int tn, hipStream_t st) {
    if (tn == 256) launch_gemm_tn<VA, VB, LAYOUT, 256>(a, nwg, x3, st);
    else launch_gemm_tn<VA, VB, LAYOUT, 128>(a, nwg, x3, st);
}

}  // namespace
}  // namespace rmd

extern "C" size_t rmd_corr_grad_gemm_workspace_bytes(int batch, int m, int k, int nc) {
    if (batch <= 0 || m <= 0 || k <= 0 || nc <= 0) return 0;
    const rmd::Plan pl = rmd::plan(batch, m, k, nc);
    return pl.splits > 1 ? (size_t)pl.splits * batch * m * nc * sizeof(float) : 0;
}

namespace rmd {
namespace {
int grad_gemm_impl(const float* a, long long lda, const float* bm, const unsigned short* bh, long long ldb, int batch,
                   int m, int k, int nc, int layout, int compute, float* out, void* workspace, void* stream) {
    RMD_REQUIRE(a && (bm || bh) && out, RMD_ERR_ARG, "rmd_corr_grad_gemm: null pointer");
    RMD_REQUIRE(compute == RMD_BF16X3 || compute == RMD_BF16, RMD_ERR_ARG,
                "rmd_corr_grad_gemm: compute must be RMD_BF16X3 or RMD_BF16");
    const bool x3 = compute == RMD_BF16X3;
    RMD_REQUIRE(batch > 0 && m > 0 && k > 0 && nc > 0, RMD_ERR_SHAPE, "rmd_corr_grad_gemm: empty shape");
    RMD_REQUIRE(layout >= 0 && layout <= 3, RMD_ERR_ARG, "rmd_corr_grad_gemm: layout must be 0..3");
    RMD_REQUIRE(!bh || (layout >= 2 && !x3), RMD_ERR_ARG, "rmd_corr_grad_gemm_bf16g: layouts 2 / 3 only");
    RMD_REQUIRE(lda >= k && ldb >= (layout == 0 ? nc : layout == 3 ? nc : k), RMD_ERR_SHAPE,
                "rmd_corr_grad_gemm: bad row stride");
    const Plan pl = plan(batch, m, k, nc);
    RMD_REQUIRE(pl.splits == 1 || workspace, RMD_ERR_ARG, "rmd_corr_grad_gemm: workspace required (%d splits)",
                pl.splits);
    hipStream_t st = as_stream(stream);
    GemmArgs g{};
    g.A = a;
    g.Bm = bm;
    g.Bh = bh;
    g.out = pl.splits > 1 ? static_cast<float*>(workspace) : out;
    g.lda = lda;
    g.ldb = ldb;
    g.sa = (long long)m * lda;
    // batch stride of B: rows x ldb (layouts 0 / 1) or 8-blocks x 8 ldb (layouts 2 / 3)
    g.sb = layout == 0 ? (long long)k * ldb
         : layout == 1 ? (long long)nc * ldb
         : layout == 2 ? (long long)((nc + 7) / 8) * 8 * ldb
                       : (long long)((k + 7) / 8) * 8 * ldb;
    g.so = (long long)m * nc;
    g.M = m;
    g.K = k;
    g.Nc = nc;
    g.batch = batch;
    g.kper = pl.kper;
    g.splits = pl.splits;
    g.ntm = pl.ntm;
    g.ntn = pl.ntn;
    const long long nwg = (long long)pl.ntm * pl.ntn * pl.splits * batch;
    RMD_REQUIRE(nwg < (1LL << 31), RMD_ERR_SHAPE, "rmd_corr_grad_gemm: grid too large");
    // float4 paths need 16-B aligned rows: row stride % 4 == 0 AND a 16-B aligned base pointer (a
    // caller may pass an offset view); layouts 2 / 3 need only the base (4 consecutive elements of an
    // 8-block are contiguous; 8-B aligned for a bfloat16 B)
    const bool a16 = ((uintptr_t)a & 15) == 0;
    const bool b16 = bh ? ((uintptr_t)bh & 7) == 0 : ((uintptr_t)bm & 15) == 0;
    const bool va = a16 && (lda & 3) == 0;
    bool vb = b16 && (ldb & 3) == 0;
#define RMD_GG(VA, VB)                                                                      \
    (layout == 0 ? launch_gemm<VA, VB, 0>(g, (int)nwg, x3, pl.tn, st)                       \
     : layout == 1 ? launch_gemm<VA, VB, 1>(g, (int)nwg, x3, pl.tn, st)                     \
     : layout == 2 ? launch_gemm<VA, VB, 2>(g, (int)nwg, x3, pl.tn, st)                     \
                   : launch_gemm<VA, VB, 3>(g, (int)nwg, x3, pl.tn, st))
    if (layout >= 2) vb = b16;                 // 8-blocks: 4 consecutive elements are contiguous, aligned
    if (va && vb) RMD_GG(true, true);
    else if (va) RMD_GG(true, false);
    else if (vb) RMD_GG(false, true);
    else RMD_GG(false, false);
#undef RMD_GG
    int rc = check_launch("rmd_corr_grad_gemm");
    if (rc != RMD_OK || pl.splits == 1) return rc;
    const long long n = (long long)batch * m * nc;
    const long long blocks = (n / 4 + 255) / 256 + 1;
    grad_gemm_reduce<<<(unsigned)blocks, 256, 0, st>>>(static_cast<const float*>(workspace), n, pl.splits, out);
    return check_launch("rmd_corr_grad_gemm reduce");
}
}  // namespace
}  // namespace rmd

extern "C" int rmd_corr_grad_gemm(const float* a, long long lda, const float* bm, long long ldb, int batch, int m,
                                  int k, int nc, int layout, int compute, float* out, void* workspace, void* stream) {
    return rmd::grad_gemm_impl(a, lda, bm, nullptr, ldb, batch, m, k, nc, layout, compute, out, workspace, stream);
}

extern "C" int rmd_corr_grad_gemm_bf16g(const float* a, long long lda, const void* bm, long long ldb, int batch, int m,
                                        int k, int nc, int layout, float* out, void* workspace, void* stream) {
    RMD_REQUIRE(bm, RMD_ERR_ARG, "rmd_corr_grad_gemm_bf16g: null pointer");
    return rmd::grad_gemm_impl(a, lda, nullptr, static_cast<const unsigned short*>(bm), ldb, batch, m, k, nc, layout,
                               RMD_BF16, out, workspace, stream);
}
