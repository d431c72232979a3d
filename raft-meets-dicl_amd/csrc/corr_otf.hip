// corr_otf.hip — on-the-fly windowed correlation lookup: no all-pairs volume in HBM.
//
// Replaces raft_fs.CorrBlock (qzed/raft-meets-dicl src/models/impls/raft_fs.py:13-87) — pooled
// fmap2 levels sampled on the (2r+1)^2 window of each query and dotted with fmap1, no 1/sqrt(C) —
// and, with one level and scale 1/sqrt(C), the window dot of corr/dot.py:25-57.  SURVEY.md §8(f)
// rank 1: memory O(B*C*N) instead of O(B*N^2).
//
// Per launch: grid (query blocks of 16 x 2 pixels, levels, batch), 256 threads.  The 32 queries'
// (2r+2)^2 integer patches at level l are bounded by one box (clipped to the level map); if it has
// at most kMaxT targets, S = targets x queries is one dense MFMA product (bf16 32x32x16, or exact
// f32 32x32x2) into LDS, target rows gathered from the pooled pixel-major fmap2 (rmd_corr_otf_prepare)
// and query fragments from the pixel-major fmap1.  Every query then interpolates its window from
// LDS exactly as rmd_corr_lookup does (shared bilinear weights, zero padding per tap, NaN for
// 1-pixel levels, zeroed masked levels).  A box larger than kMaxT (pathological flow spread) falls
// back to per-query patch dots on the VALU.
#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 256;
constexpr int kBX = 16, kBY = 2, kQ = kBX * kBY;     // query block
constexpr int kMaxT = 512;                            // LDS: kQ x kMaxT f32 = 64 KiB
constexpr int kCp = 32;                               // channel padding of the operand rows

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

struct OtfGeom {
    int B, C, Cp, H, W, L;
    int lh[RMD_MAX_LEVELS], lw[RMD_MAX_LEVELS];
    long long toff[RMD_MAX_LEVELS], T;
};

OtfGeom make_otf_geom(int B, int C, int H, int W, int L) {
    OtfGeom g{};
    g.B = B;
    g.C = C;
    g.Cp = (C + kCp - 1) / kCp * kCp;
    g.H = H;
    g.W = W;
    g.L = L;
    long long t = 0;
    for (int l = 0; l < L; ++l) {
        g.lh[l] = H >> l;
        g.lw[l] = W >> l;
        g.toff[l] = t;
        t += (long long)g.lh[l] * g.lw[l];
    }
    g.T = t;
    return g;
}

template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

// rows[b][t][c] = scale * mean over the 2^l x 2^l block of f[b][c][...] (level l of target t), in the
// compute type, channels zero-padded to Cp.  levels = 1, scale = s gives the query operand.
template <typename T>
__global__ void __launch_bounds__(kThreads)
otf_rows_kernel(const float* __restrict__ f, OtfGeom g, float scale, T* __restrict__ rows) {
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    const int CG = g.Cp / 8;
    const long long total = (long long)g.B * g.T * CG;
    if (idx >= total) return;
    const int cg = (int)(idx % CG);
    const long long bt = idx / CG;
    const long long t = bt % g.T;
    const int b = (int)(bt / g.T);
    int l = 0;
#pragma unroll
    for (int k = 1; k < RMD_MAX_LEVELS; ++k)
        if (k < g.L && t >= g.toff[k]) l = k;
    const int tl = (int)(t - g.toff[l]);
    const int y = tl / g.lw[l], x = tl - y * g.lw[l];
    const int s = 1 << l;
    T out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = cg * 8 + e;
        float acc = 0.f;
        if (c < g.C) {
            const float* src = f + ((size_t)b * g.C + c) * g.H * g.W + (size_t)(y * s) * g.W + x * s;
            for (int dy = 0; dy < s; ++dy)
                for (int dx = 0; dx < s; ++dx) acc += src[(size_t)dy * g.W + dx];
            acc *= scale / (float)(s * s);
        }
        out[e] = from_f32<T>(acc);
    }
    T* dst = rows + ((size_t)b * g.T + t) * g.Cp + cg * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) dst[e] = out[e];
}

template <typename T> struct Mfma;
template <> struct Mfma<__bf16> {
    static constexpr int KS = 16;        // k per MFMA
    static __device__ __forceinline__ void step(f32x16& acc, const __bf16* a, const __bf16* b) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(a);
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(b);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    }
    static constexpr int lane_k(int h) { return 8 * h; }
};
template <> struct Mfma<float> {
    static constexpr int KS = 2;
    static __device__ __forceinline__ void step(f32x16& acc, const float* a, const float* b) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(*a, *b, acc, 0, 0, 0);
    }
    static constexpr int lane_k(int h) { return h; }
};

template <typename T, int R>
__global__ void __launch_bounds__(kThreads)
otf_lookup_kernel(const T* __restrict__ qrows, const T* __restrict__ trows, OtfGeom g,
                  const float* __restrict__ coords, unsigned zmask, float* __restrict__ out) {
    constexpr int D = 2 * R + 1, K = 2 * R + 2, KK = K * K;
    extern __shared__ float S[];                       // [kQ][kMaxT] (box) or [kQ][KK] (per query)
    __shared__ int box[4];                             // x0, x1, y0, y1 (min / max)
    const int nbx = (g.W + kBX - 1) / kBX;
    const int qx0 = (blockIdx.x % nbx) * kBX, qy0 = (blockIdx.x / nbx) * kBY;
    const int L = blockIdx.y, b = blockIdx.z;
    const int N = g.H * g.W;
    const int lh = g.lh[L], lw = g.lw[L];
    const int tid = threadIdx.x;
    float* ob = out + ((size_t)b * g.L + L) * D * D * (size_t)N;

    // masked / degenerate level: constant output (raft_fs.py:77-78; 1-pixel levels divide by zero)
    const bool masked = (zmask >> L) & 1u;
    if (masked || lh < 2 || lw < 2) {
        const float v = masked ? 0.f : __builtin_nanf("");
        for (int idx = tid; idx < kQ * D * D; idx += kThreads) {
            const int q = idx % kQ, c = idx / kQ;
            const int y = qy0 + q / kBX, x = qx0 + q % kBX;
            if (y < g.H && x < g.W) ob[(size_t)c * N + y * g.W + x] = v;
        }
        return;
    }

    // per-query patch origin at level L
    auto origin = [&](int q, int& xs, int& ys, float& fx, float& fy) {
        const int y = min(qy0 + q / kBX, g.H - 1), x = min(qx0 + q % kBX, g.W - 1);
        const float inv = 1.0f / (float)(1 << L);
        float cx = coords[((size_t)b * 2 + 0) * N + y * g.W + x] * inv;
        float cy = coords[((size_t)b * 2 + 1) * N + y * g.W + x] * inv;
        cx = fminf(fmaxf(cx, -1.0e6f), 1.0e6f);
        cy = fminf(fmaxf(cy, -1.0e6f), 1.0e6f);
        const float fx0 = floorf(cx), fy0 = floorf(cy);
        fx = cx - fx0;
        fy = cy - fy0;
        xs = (int)fx0 - R;
        ys = (int)fy0 - R;
    };
    if (tid == 0) {
        box[0] = 1 << 30;
        box[1] = -(1 << 30);
        box[2] = 1 << 30;
        box[3] = -(1 << 30);
    }
    __syncthreads();
    if (tid < kQ) {
        int xs, ys;
        float fx, fy;
        origin(tid, xs, ys, fx, fy);
        atomicMin(&box[0], xs);
        atomicMax(&box[1], xs + K - 1);
        atomicMin(&box[2], ys);
        atomicMax(&box[3], ys + K - 1);
    }
    __syncthreads();
    const int bx0 = max(box[0], 0), bx1 = min(box[1], lw - 1);
    const int by0 = max(box[2], 0), by1 = min(box[3], lh - 1);
    const int tw = max(bx1 - bx0 + 1, 0), th = max(by1 - by0 + 1, 0);
    const int tb = tw * th;
    const bool dense = tb <= kMaxT;
    const T* qb = qrows + (size_t)b * N * g.Cp;
    const T* tl = trows + ((size_t)b * g.T + g.toff[L]) * g.Cp;

    if (dense && tb > 0) {
        // S[q][t] for the box's targets: 32-target MFMA tiles spread over the 4 waves
        const int lane = tid & 63, w = tid >> 6, j = lane & 31, h = lane >> 5;
        const int qy = min(qy0 + j / kBX, g.H - 1), qx = min(qx0 + j % kBX, g.W - 1);
        const T* qrow = qb + (size_t)(qy * g.W + qx) * g.Cp + Mfma<T>::lane_k(h);
        const int ntile = (tb + 31) / 32;
        for (int tile = w; tile < ntile; tile += 4) {
            const int t = min(tile * 32 + j, tb - 1);
            const int ty = by0 + t / tw, tx = bx0 + t % tw;
            const T* trow = tl + (size_t)(ty * lw + tx) * g.Cp + Mfma<T>::lane_k(h);
            f32x16 acc = {};
            for (int k = 0; k < g.Cp; k += Mfma<T>::KS) Mfma<T>::step(acc, trow + k, qrow + k);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int tt = tile * 32 + 8 * (e >> 2) + 4 * h + (e & 3);
                if (tt < tb) S[j * kMaxT + tt] = acc[e];
            }
        }
    } else if (!dense) {
        // fallback: each query's own (2r+2)^2 patch, one dot product per thread
        for (int idx = tid; idx < kQ * KK; idx += kThreads) {
            const int q = idx / KK, r = idx - q * KK;
            int xs, ys;
            float fx, fy;
            origin(q, xs, ys, fx, fy);
            const int ty = ys + r / K, tx = xs + r % K;
            float acc = 0.f;
            if (ty >= 0 && ty < lh && tx >= 0 && tx < lw) {
                const int qy = min(qy0 + q / kBX, g.H - 1), qx = min(qx0 + q % kBX, g.W - 1);
                const T* qrow = qb + (size_t)(qy * g.W + qx) * g.Cp;
                const T* trow = tl + (size_t)(ty * lw + tx) * g.Cp;
                for (int c = 0; c < g.C; ++c) acc = fmaf((float)qrow[c], (float)trow[c], acc);
            }
            S[q * KK + r] = acc;
        }
    }
    __syncthreads();

    // interpolation: thread (q, a) produces the D outputs of x-offset a for query q
    for (int idx = tid; idx < kQ * D; idx += kThreads) {
        const int q = idx % kQ, a = idx / kQ;
        const int y = qy0 + q / kBX, x = qx0 + q % kBX;
        if (y >= g.H || x >= g.W) continue;
        int xs, ys;
        float fx, fy;
        origin(q, xs, ys, fx, fy);
        float hx[K];
#pragma unroll
        for (int jj = 0; jj < K; ++jj) {
            const int ty = ys + jj;
            float v[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int tx = xs + a + u;
                float e = 0.f;
                if (ty >= 0 && ty < lh && tx >= 0 && tx < lw)
                    e = dense ? S[q * kMaxT + (ty - by0) * tw + (tx - bx0)] : S[q * KK + jj * K + a + u];
                v[u] = e;
            }
            hx[jj] = fmaf(fx, v[1] - v[0], v[0]);
        }
        float* o = ob + (size_t)(a * D) * N + y * g.W + x;
#pragma unroll
        for (int bb = 0; bb < D; ++bb) o[(size_t)bb * N] = fmaf(fy, hx[bb + 1] - hx[bb], hx[bb]);
    }
}

int check_otf(int batch, int channels, int height, int width, int levels, int compute) {
    RMD_REQUIRE(batch > 0 && channels > 0 && height > 0 && width > 0, RMD_ERR_SHAPE, "rmd_corr_otf: bad sizes");
    RMD_REQUIRE(levels >= 1 && levels <= RMD_MAX_LEVELS, RMD_ERR_SHAPE, "rmd_corr_otf: bad levels");
    RMD_REQUIRE((height >> (levels - 1)) >= 1 && (width >> (levels - 1)) >= 1, RMD_ERR_SHAPE,
                "rmd_corr_otf: level %d of a %dx%d map is empty", levels - 1, height, width);
    RMD_REQUIRE(compute == RMD_F32 || compute == RMD_BF16, RMD_ERR_ARG, "rmd_corr_otf: compute must be F32 or BF16");
    return RMD_OK;
}

}  // namespace
}  // namespace rmd

using namespace rmd;

extern "C" size_t rmd_corr_otf_workspace_bytes(int batch, int channels, int height, int width, int levels,
                                               int compute) {
    if (check_otf(batch, channels, height, width, levels, compute)) return 0;
    const OtfGeom g = make_otf_geom(batch, channels, height, width, levels);
    const size_t es = compute == RMD_F32 ? 4 : 2;
    return (size_t)batch * ((size_t)height * width + g.T) * g.Cp * es;
}

extern "C" int rmd_corr_otf_prepare(const float* fmap1, const float* fmap2, int batch, int channels, int height,
                                    int width, int levels, float scale, int compute, void* workspace, void* stream) {
    RMD_REQUIRE(fmap1 && fmap2 && workspace, RMD_ERR_ARG, "rmd_corr_otf_prepare: null pointer");
    int rc = check_otf(batch, channels, height, width, levels, compute);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    const OtfGeom g = make_otf_geom(batch, channels, height, width, levels);
    const OtfGeom g1 = make_otf_geom(batch, channels, height, width, 1);
    const long long nq = (long long)batch * g1.T * (g.Cp / 8), nt = (long long)batch * g.T * (g.Cp / 8);
    const unsigned gq = (unsigned)((nq + kThreads - 1) / kThreads), gt = (unsigned)((nt + kThreads - 1) / kThreads);
    if (compute == RMD_BF16) {
        __bf16* q = reinterpret_cast<__bf16*>(workspace);
        __bf16* t = q + (size_t)batch * height * width * g.Cp;
        otf_rows_kernel<__bf16><<<gq, kThreads, 0, st>>>(fmap1, g1, scale, q);
        otf_rows_kernel<__bf16><<<gt, kThreads, 0, st>>>(fmap2, g, 1.0f, t);
    } else {
        float* q = reinterpret_cast<float*>(workspace);
        float* t = q + (size_t)batch * height * width * g.Cp;
        otf_rows_kernel<float><<<gq, kThreads, 0, st>>>(fmap1, g1, scale, q);
        otf_rows_kernel<float><<<gt, kThreads, 0, st>>>(fmap2, g, 1.0f, t);
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
    dim3 grid(((width + kBX - 1) / kBX) * ((height + kBY - 1) / kBY), levels, batch);
    const size_t lds = sizeof(float) * kQ * kMaxT;
    const size_t qn = (size_t)batch * height * width * g.Cp;
#define RMD_OTF(T, RR)                                                                                         \
    do {                                                                                                       \
        auto k = otf_lookup_kernel<T, RR>;                                                                     \
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)lds);                                                                   \
        const T* q = reinterpret_cast<const T*>(workspace);                                                    \
        k<<<grid, kThreads, lds, st>>>(q, q + qn, g, coords, zero_level_mask, out);                            \
    } while (0)
#define RMD_OTF_R(T)                                     \
    switch (radius) {                                    \
        case 1: RMD_OTF(T, 1); break;                    \
        case 2: RMD_OTF(T, 2); break;                    \
        case 3: RMD_OTF(T, 3); break;                    \
        case 4: RMD_OTF(T, 4); break;                    \
        case 5: RMD_OTF(T, 5); break;                    \
        case 6: RMD_OTF(T, 6); break;                    \
        case 7: RMD_OTF(T, 7); break;                    \
        default: RMD_OTF(T, 8); break;                   \
    }
    if (compute == RMD_BF16) {
        RMD_OTF_R(__bf16)
    } else {
        RMD_OTF_R(float)
    }
#undef RMD_OTF_R
#undef RMD_OTF
    return check_launch("rmd_corr_otf_lookup");
}
