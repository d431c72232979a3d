// corr_pyramid.hip — all-pairs correlation GEMM with the pooled pyramid fused into its epilogue.
//
// Replaces raft.CorrBlock.__init__ (qzed/raft-meets-dicl src/models/impls/raft.py:18-47):
//   corr0[b,p,q] = sum_c f1[b,c,p] f2[b,c,q] / sqrt(C);  level l = avg_pool2d(level l-1, 2, 2)
//
// gfx950 design:
//  * one workgroup = 256 threads = 4 waves computes a 16x16 block of target pixels (256 targets,
//    the MFMA "A"/row side) against 64 query pixels (the "B"/column side), K = C in 64-deep LDS
//    chunks.  Wave w owns the 8x8 target sub-block (rows 8*(w>>1).., cols 8*(w&1)..) for all 64
//    queries: 2x2 MFMA 32x32 tiles, one 32-target tile = 4 target rows x 8 target columns.
//  * with targets on the MFMA rows, lane (h = lane>>5, j = lane&31) holds, for query j, an 8x4
//    patch of target pixels (rows 0..7, cols 4h..4h+3 of the wave's 8x8 block), so the 2x2 pools
//    for levels 1 and 2 are in-lane adds and level 3 needs one xor-32 lane exchange.
//  * every level is written from the f32 accumulators (fp16 or fp32 storage) through a
//    bank-swizzled LDS image as contiguous query-minor tile runs (see rmd.h for the layout).
//  * compute = bf16 operands (v_mfma_f32_32x32x16_bf16) or exact f32 (v_mfma_f32_32x32x2_f32).
//    Operands are first transposed to pixel-major, channel-contiguous (B, N, Cp) by a prep kernel
//    so every fragment read is one 16-byte ds_read_b128.

#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 256;
constexpr int kBQ = 64;      // queries per workgroup
constexpr int kNT = 256;     // targets per workgroup (16 x 16 block)
constexpr int kKC = 64;      // K chunk staged in LDS

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <bool F32> struct Operand { using T = __bf16; static constexpr int S = 2; };
template <> struct Operand<true> { using T = float; static constexpr int S = 4; };

// padded staging row: kKC elements + 16 B -> ds_read_b128 fragment reads are conflict-free
template <bool F32> constexpr int stage_stride() { return kKC * Operand<F32>::S + 16; }

template <bool F32, typename TOut> constexpr int lds_bytes() {
    constexpr int st = (kNT + kBQ) * stage_stride<F32>();
    constexpr int ep = (4 * kBQ * 64 + kBQ * 64 + kBQ * 16 + kBQ * 4) * (int)sizeof(TOut);
    return st > ep ? st : ep;
}

// ---------------------------------------------------------------------------------------------
// prep: (B, C, N) f32 -> (B, N, Cp) operand type, zero-padded channels.  64 px x 64 ch per block.
template <typename T>
__global__ void __launch_bounds__(kThreads)
prep_operand(const float* __restrict__ f, T* __restrict__ o, int C, int N, int Cp) {
    __shared__ float tile[64][65];
    const int b = blockIdx.z, p0 = blockIdx.x * 64, c0 = blockIdx.y * 64, t = threadIdx.x;
    const float* fb = f + (size_t)b * C * N;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int c = c0 + (t >> 6) + 4 * i, p = p0 + (t & 63);
        tile[(t >> 6) + 4 * i][t & 63] = (c < C && p < N) ? fb[(size_t)c * N + p] : 0.f;
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

// ---------------------------------------------------------------------------------------------
template <typename TOut> __device__ __forceinline__ TOut cvt_out(float v);
template <> __device__ __forceinline__ float cvt_out<float>(float v) { return v; }
template <> __device__ __forceinline__ __half cvt_out<__half>(float v) { return __float2half_rn(v); }

// write `n` (2 or 4) consecutive output elements at element offset `e` of query q's tile image
// whose 16-byte chunks are XOR-swizzled by the query index (conflict-free ds_write / ds_read)
template <typename TOut, int NE>
__device__ __forceinline__ void img_put(unsigned char* img, int q, int tile_elems, int e,
                                        const float* v) {
    constexpr int S = sizeof(TOut);
    const int cq = tile_elems * S / 16;                   // 16-B chunks per query tile
    const int byte = e * S;
    const int chunk = (byte >> 4) ^ (q & (cq - 1));
    unsigned char* p = img + (size_t)(q * cq + chunk) * 16 + (byte & 15);
    TOut tmp[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) tmp[i] = cvt_out<TOut>(v[i]);
    if constexpr (NE * S == 16) {
        *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(tmp);
    } else if constexpr (NE * S == 8) {
        *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(tmp);
    } else {
        static_assert(NE * S == 4, "unsupported image write");
        *reinterpret_cast<unsigned*>(p) = *reinterpret_cast<const unsigned*>(tmp);
    }
}

// copy nq queries' swizzled tile images (16-B chunks) to a contiguous global run
__device__ __forceinline__ void img_store(const unsigned char* img, unsigned char* dst, int nq,
                                          int cq, int worker, int nworkers) {
    const int total = nq * cq;
    for (int id = worker; id < total; id += nworkers) {
        const int q = id / cq, c = id - q * cq;
        const uint4 v = *reinterpret_cast<const uint4*>(img + (size_t)(q * cq + (c ^ (q & (cq - 1)))) * 16);
        *reinterpret_cast<uint4*>(dst + (size_t)id * 16) = v;
    }
}

template <bool F32, typename TOut>
__global__ void __launch_bounds__(kThreads)
corr_pyramid_kernel(const typename Operand<F32>::T* __restrict__ opA,   // fmap2 (B, N, Cp)
                    const typename Operand<F32>::T* __restrict__ opB,   // fmap1 (B, N, Cp)
                    int Cp, float scale, PyrGeom g, TOut* __restrict__ pyr) {
    using T = typename Operand<F32>::T;
    constexpr int S = Operand<F32>::S;
    constexpr int SS = stage_stride<F32>();
    constexpr int PPR = kKC * S / 16;                       // 16-B pieces per staged row
    constexpr int SO = sizeof(TOut);

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
        // ---- stage the A (targets) and B (queries) chunk into LDS -----------------------------
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

        // ---- MFMA over the chunk ------------------------------------------------------------
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

    // ---- epilogue: scale, pool, write LDS images ----------------------------------------------
    unsigned char* img0 = smem;                                   // [4 waves][64 q][64 el]
    unsigned char* img1 = img0 + 4 * kBQ * 64 * SO;               // [64 q][64 el]   (8x8 tile)
    unsigned char* img2 = img1 + kBQ * 64 * SO;                   // [64 q][16 el]   (4x4 tile)
    unsigned char* img3 = img2 + kBQ * 16 * SO;                   // [64 q][4 el]    (2x2 tile)
    const int levels = g.levels;

#pragma unroll
    for (int tq = 0; tq < 2; ++tq) {
        const int q = 32 * tq + r;
        float o[8][4];                                            // rows 0..7, cols 4h..4h+3
#pragma unroll
        for (int tr = 0; tr < 2; ++tr)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[4 * tr + (e >> 2)][e & 3] = acc[tr][tq][e] * scale;
        unsigned char* im0 = img0 + (size_t)w * kBQ * 64 * SO;
#pragma unroll
        for (int row = 0; row < 8; ++row) img_put<TOut, 4>(im0, q, 64, row * 8 + 4 * h, o[row]);
        if (levels > 1) {
            float l1[4][2];
#pragma unroll
            for (int yy = 0; yy < 4; ++yy)
#pragma unroll
                for (int xx = 0; xx < 2; ++xx)
                    l1[yy][xx] = 0.25f * ((o[2 * yy][2 * xx] + o[2 * yy][2 * xx + 1]) +
                                          (o[2 * yy + 1][2 * xx] + o[2 * yy + 1][2 * xx + 1]));
#pragma unroll
            for (int yy = 0; yy < 4; ++yy)
                img_put<TOut, 2>(img1, q, 64, (4 * (w >> 1) + yy) * 8 + 4 * (w & 1) + 2 * h, l1[yy]);
            if (levels > 2) {
                float l2[2];
#pragma unroll
                for (int yy = 0; yy < 2; ++yy)
                    l2[yy] = 0.25f * ((l1[2 * yy][0] + l1[2 * yy][1]) + (l1[2 * yy + 1][0] + l1[2 * yy + 1][1]));
                TOut* im2 = reinterpret_cast<TOut*>(img2) + q * 16;
#pragma unroll
                for (int yy = 0; yy < 2; ++yy) im2[(2 * (w >> 1) + yy) * 4 + 2 * (w & 1) + h] = cvt_out<TOut>(l2[yy]);
                if (levels > 3) {
                    float s3 = l2[0] + l2[1];
                    s3 += __shfl_xor(s3, 32);
                    if (h == 0) reinterpret_cast<TOut*>(img3)[q * 4 + (w >> 1) * 2 + (w & 1)] = cvt_out<TOut>(0.25f * s3);
                }
            }
        }
    }
    __syncthreads();

    // ---- contiguous query-minor tile runs -> HBM -----------------------------------------------
    const int nq = min(kBQ, N - q0);
    {
        const int trow = 2 * rb + (w >> 1), tcol = 2 * cb + (w & 1);
        if (trow < g.ty[0] && tcol < g.tx[0]) {
            const size_t base = (size_t)g.off[0] + (((size_t)b * g.ty[0] + trow) * g.tx[0] + tcol) * N * 64 + (size_t)q0 * 64;
            img_store(img0 + (size_t)w * kBQ * 64 * SO, reinterpret_cast<unsigned char*>(pyr + base), nq,
                      64 * SO / 16, lane, 64);
        }
    }
    if (levels > 1 && rb < g.ty[1] && cb < g.tx[1]) {
        const size_t base = (size_t)g.off[1] + (((size_t)b * g.ty[1] + rb) * g.tx[1] + cb) * N * 64 + (size_t)q0 * 64;
        img_store(img1, reinterpret_cast<unsigned char*>(pyr + base), nq, 64 * SO / 16, tid, kThreads);
    }
    if (levels > 2 && rb < g.ty[2] && cb < g.tx[2]) {
        const size_t base = (size_t)g.off[2] + (((size_t)b * g.ty[2] + rb) * g.tx[2] + cb) * N * 16 + (size_t)q0 * 16;
        const uint4* src = reinterpret_cast<const uint4*>(img2);
        uint4* dst = reinterpret_cast<uint4*>(pyr + base);
        for (int id = tid; id < nq * 16 * SO / 16; id += kThreads) dst[id] = src[id];
    }
    if (levels > 3 && rb < g.ty[3] && cb < g.tx[3]) {
        const size_t base = (size_t)g.off[3] + (((size_t)b * g.ty[3] + rb) * g.tx[3] + cb) * N * 4 + (size_t)q0 * 4;
        if constexpr (SO == 2) {
            const uint2* src = reinterpret_cast<const uint2*>(img3);
            uint2* dst = reinterpret_cast<uint2*>(pyr + base);
            for (int id = tid; id < nq; id += kThreads) dst[id] = src[id];
        } else {
            const uint4* src = reinterpret_cast<const uint4*>(img3);
            uint4* dst = reinterpret_cast<uint4*>(pyr + base);
            for (int id = tid; id < nq; id += kThreads) dst[id] = src[id];
        }
    }
}

template <bool F32, typename TOut>
int launch_pyramid(const float* f1, const float* f2, int C, const rmd_pyramid_desc& d, void* pyramid,
                   void* workspace, hipStream_t st) {
    using T = typename Operand<F32>::T;
    const int N = d.height * d.width;
    const int Cp = (C + kKC - 1) / kKC * kKC;
    T* opA = reinterpret_cast<T*>(workspace);
    T* opB = opA + (size_t)d.batch * N * Cp;
    dim3 pg((N + 63) / 64, Cp / 64, d.batch);
    prep_operand<T><<<pg, kThreads, 0, st>>>(f2, opA, C, N, Cp);
    prep_operand<T><<<pg, kThreads, 0, st>>>(f1, opB, C, N, Cp);
    int rc = check_launch("rmd_corr_pyramid/prep");
    if (rc) return rc;
    constexpr int lds = lds_bytes<F32, TOut>();
    auto kern = corr_pyramid_kernel<F32, TOut>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    dim3 grid((N + kBQ - 1) / kBQ, ((d.height + 15) / 16) * ((d.width + 15) / 16), d.batch);
    const float scale = 1.0f / sqrtf((float)C);
    kern<<<grid, kThreads, lds, st>>>(opA, opB, Cp, scale, make_geom(d), reinterpret_cast<TOut*>(pyramid));
    return check_launch("rmd_corr_pyramid/gemm");
}

}  // namespace
}  // namespace rmd

extern "C" size_t rmd_corr_pyramid_workspace_bytes(const rmd_pyramid_desc* d, int channels, int compute) {
    if (!d || channels <= 0) return 0;
    const size_t Cp = (size_t)(channels + rmd::kKC - 1) / rmd::kKC * rmd::kKC;
    const size_t es = compute == RMD_F32 ? 4 : 2;
    return 2 * (size_t)d->batch * d->height * d->width * Cp * es;
}

extern "C" int rmd_corr_pyramid(const float* fmap1, const float* fmap2, int channels, const rmd_pyramid_desc* d,
                                int compute, void* pyramid, void* workspace, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && d && pyramid && workspace, RMD_ERR_ARG, "rmd_corr_pyramid: null pointer");
    RMD_REQUIRE(channels > 0, RMD_ERR_SHAPE, "rmd_corr_pyramid: channels must be > 0");
    RMD_REQUIRE(d->levels >= 1 && d->levels <= RMD_MAX_LEVELS, RMD_ERR_SHAPE, "rmd_corr_pyramid: bad levels");
    RMD_REQUIRE(compute == RMD_F32 || compute == RMD_BF16, RMD_ERR_ARG, "rmd_corr_pyramid: compute must be F32 or BF16");
    hipStream_t st = rmd::as_stream(stream);
    if (compute == RMD_BF16) {
        if (d->storage == RMD_F16) return rmd::launch_pyramid<false, __half>(fmap1, fmap2, channels, *d, pyramid, workspace, st);
        if (d->storage == RMD_F32) return rmd::launch_pyramid<false, float>(fmap1, fmap2, channels, *d, pyramid, workspace, st);
    } else {
        if (d->storage == RMD_F16) return rmd::launch_pyramid<true, __half>(fmap1, fmap2, channels, *d, pyramid, workspace, st);
        if (d->storage == RMD_F32) return rmd::launch_pyramid<true, float>(fmap1, fmap2, channels, *d, pyramid, workspace, st);
    }
    rmd::set_error("rmd_corr_pyramid: storage must be F32 or F16");
    return RMD_ERR_ARG;
}
