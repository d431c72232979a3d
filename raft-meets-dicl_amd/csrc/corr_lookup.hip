// corr_lookup.hip — per-GRU-iteration windowed bilinear lookup into the tiled correlation pyramid.
//
// Replaces raft.CorrBlock.__call__ (qzed/raft-meets-dicl src/models/impls/raft.py:49-95).
// For query p and level i the reference grid-samples the (2r+1)^2 window centred at
// (x/2^i, y/2^i) with integer offsets; all taps therefore share one bilinear weight set and the
// window reads exactly the (2r+2)^2 integer patch [x0-r, x0+r+1] x [y0-r, y0+r+1] of p's own
// level-i map.
//
// gfx950 design: one lane per query, 64 consecutive queries per wave so every
// output store (one channel, 64 queries) is a coalesced 256-byte row of the (B, L*(2r+1)^2, H, W)
// result.  Each patch row is fetched as whole tile rows (16 B for fp16 8x8 tiles) — 2 or 3
// vector loads per row instead of 2r+2 scalar loads — and aligned with a log-step barrel shift
// on packed 32-bit words.  Rows/columns outside the level are zero (grid_sample zero padding).

#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 256;

template <int NB> struct Chunk;
template <> struct Chunk<4> { using T = unsigned; };
template <> struct Chunk<8> { using T = uint2; };
template <> struct Chunk<16> { using T = uint4; };

template <int NW>
__device__ __forceinline__ void load_words(unsigned (&dst)[NW], int at, const unsigned char* src) {
    // NW words (4, 8, 16 or 32 bytes) from a 4/8/16-byte aligned address
    constexpr int NB = NW * 4;
    if constexpr (NB <= 16) {
        typename Chunk<NB>::T v = *reinterpret_cast<const typename Chunk<NB>::T*>(src);
        const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
        for (int i = 0; i < NW; ++i) dst[at + i] = u[i];
    } else {
#pragma unroll
        for (int k = 0; k < NB / 16; ++k) {
            uint4 v = reinterpret_cast<const uint4*>(src)[k];
            dst[at + 4 * k + 0] = v.x;
            dst[at + 4 * k + 1] = v.y;
            dst[at + 4 * k + 2] = v.z;
            dst[at + 4 * k + 3] = v.w;
        }
    }
}

template <typename T> __device__ __forceinline__ float word_elem(unsigned w, int i);
template <> __device__ __forceinline__ float word_elem<float>(unsigned w, int) { return __uint_as_float(w); }
template <> __device__ __forceinline__ float word_elem<__half>(unsigned w, int i) {
    const unsigned short s = i ? (unsigned short)(w >> 16) : (unsigned short)(w & 0xffff);
    return __half2float(__ushort_as_half(s));
}

// One patch row (2R+2 values) of level L for this lane.  Columns outside [0, lw) are zero.
template <typename T, int R, int TW>
__device__ __forceinline__ void load_row(const T* __restrict__ lvl_base, long long tile_row_base,
                                         long long tile_stride, int tiles_x, int yin, int xs, int lw,
                                         float (&v)[2 * R + 2]) {
    constexpr int S = sizeof(T);
    constexpr int EPW = 4 / S;                           // elements per 32-bit word
    constexpr int K = 2 * R + 2;                         // patch width
    constexpr int NC = (K + TW - 1 + TW - 1) / TW;       // tile chunks a row can span
    constexpr int CW = TW * S / 4;                       // words per chunk
    constexpr int NW = NC * CW;
    constexpr int KW = (K + EPW - 1) / EPW + 1;          // words kept after the shift
    unsigned wd[NW + 1];
    const int tc0 = (xs >= 0) ? xs / TW : -((TW - 1 - xs) / TW);   // floor(xs / TW)
    const int sh = xs - tc0 * TW;                                   // 0 .. TW-1
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int tc = tc0 + c;
        if (tc >= 0 && tc < tiles_x && c * TW < sh + K) {
            const T* p = lvl_base + tile_row_base + (long long)tc * tile_stride + yin * TW;
            unsigned tmp[CW];
            load_words<CW>(tmp, 0, reinterpret_cast<const unsigned char*>(p));
#pragma unroll
            for (int i = 0; i < CW; ++i) wd[c * CW + i] = tmp[i];
        } else {
#pragma unroll
            for (int i = 0; i < CW; ++i) wd[c * CW + i] = 0u;
        }
    }
    wd[NW] = 0u;
    // barrel shift left by sh elements: whole words first (log steps), then a half-word
    const int wsh = (sh * S) >> 2;
    constexpr int MAXW = (TW - 1) * S / 4;               // largest whole-word shift
#pragma unroll
    for (int step = 1; step <= MAXW; step <<= 1) {
        if (wsh & step) {
#pragma unroll
            for (int i = 0; i < NW + 1; ++i) wd[i] = (i + step < NW + 1) ? wd[i + step] : 0u;
        }
    }
    if constexpr (S == 2) {
        if (sh & 1) {
#pragma unroll
            for (int i = 0; i < KW; ++i) wd[i] = __builtin_amdgcn_alignbyte(wd[i + 1], wd[i], 2);
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const float e = word_elem<T>(wd[j / EPW], j % EPW);
        const int col = xs + j;
        v[j] = (col >= 0 && col < lw) ? e : 0.f;
    }
}

template <typename T, int R, int L>
__device__ __forceinline__ void lookup_level(const T* __restrict__ pyr, const PyrGeom& g, int b, int p, int N,
                                             float x, float y, unsigned zmask, float* __restrict__ outq,
                                             bool active) {
    constexpr int D = 2 * R + 1;
    constexpr int K = 2 * R + 2;
    constexpr int TL = level_tile(L);
    float* o = outq + (size_t)L * D * D * N;
    const int lh = g.lh[L], lw = g.lw[L];
    if ((zmask >> L) & 1u) {
        if (active)
            for (int c = 0; c < D * D; ++c) o[(size_t)c * N] = 0.f;
        return;
    }
    if (lh < 2 || lw < 2) {     // the reference normalises by (size-1) = 0 -> NaN (raft.py:73-74)
        if (active)
            for (int c = 0; c < D * D; ++c) o[(size_t)c * N] = __builtin_nanf("");
        return;
    }
    const float inv = 1.0f / (float)(1 << L);
    float cx = x * inv, cy = y * inv;
    cx = fminf(fmaxf(cx, -1.0e6f), 1.0e6f);
    cy = fminf(fmaxf(cy, -1.0e6f), 1.0e6f);
    const float fx0 = floorf(cx), fy0 = floorf(cy);
    const float fx = cx - fx0, fy = cy - fy0;
    const int x0 = (int)fx0, y0 = (int)fy0;
    const int xs = x0 - R, ys = y0 - R;
    const bool hit = active && xs <= lw - 1 && xs + K - 1 >= 0 && ys <= lh - 1 && ys + K - 1 >= 0;

    const T* lvl = pyr + g.off[L];
    const long long tile_stride = (long long)N * TL * TL;          // next tile column
    const long long bq = (long long)b * g.ty[L];

    float hprev[D];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int yy = ys + j;
        float v[K];
        if (hit && yy >= 0 && yy < lh) {
            const int trow = yy / TL;
            const long long row_base = ((bq + trow) * g.tx[L]) * tile_stride + (long long)p * TL * TL;
            load_row<T, R, TL>(lvl, row_base, tile_stride, g.tx[L], yy - trow * TL, xs, lw, v);
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = 0.f;
        }
        float hcur[D];
#pragma unroll
        for (int a = 0; a < D; ++a) hcur[a] = fmaf(fx, v[a + 1] - v[a], v[a]);
        if (j > 0 && active) {
            const int bb = j - 1;
#pragma unroll
            for (int a = 0; a < D; ++a) o[(size_t)(a * D + bb) * N] = fmaf(fy, hcur[a] - hprev[a], hprev[a]);
        }
#pragma unroll
        for (int a = 0; a < D; ++a) hprev[a] = hcur[a];
    }
}

template <typename T, int R>
__global__ void __launch_bounds__(kThreads)
corr_lookup_kernel(const T* __restrict__ pyr, PyrGeom g, const float* __restrict__ coords, unsigned zmask,
                   float* __restrict__ out) {
    const int N = g.height * g.width;
    const long long gid = (long long)blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y;
    const int p = (int)gid;
    const bool active = p < N;
    const int pc = active ? p : N - 1;
    const float x = coords[((size_t)b * 2 + 0) * N + pc];
    const float y = coords[((size_t)b * 2 + 1) * N + pc];
    constexpr int D = 2 * R + 1;
    float* outq = out + (size_t)b * g.levels * D * D * N + pc;
    lookup_level<T, R, 0>(pyr, g, b, pc, N, x, y, zmask, outq, active);
    if (g.levels > 1) lookup_level<T, R, 1>(pyr, g, b, pc, N, x, y, zmask, outq, active);
    if (g.levels > 2) lookup_level<T, R, 2>(pyr, g, b, pc, N, x, y, zmask, outq, active);
    if (g.levels > 3) lookup_level<T, R, 3>(pyr, g, b, pc, N, x, y, zmask, outq, active);
}

template <typename T>
int launch_lookup(const void* pyr, const rmd_pyramid_desc& d, const float* coords, int radius, unsigned zmask,
                  float* out, hipStream_t st) {
    const int N = d.height * d.width;
    dim3 grid((N + kThreads - 1) / kThreads, d.batch);
    const T* p = reinterpret_cast<const T*>(pyr);
    const PyrGeom g = make_geom(d);
    switch (radius) {
#define RMD_CASE(RR) case RR: corr_lookup_kernel<T, RR><<<grid, kThreads, 0, st>>>(p, g, coords, zmask, out); break;
        RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4) RMD_CASE(5) RMD_CASE(6) RMD_CASE(7) RMD_CASE(8)
#undef RMD_CASE
        default:
            set_error("rmd_corr_lookup: radius %d not in 1..8", radius);
            return RMD_ERR_SHAPE;
    }
    return check_launch("rmd_corr_lookup");
}

}  // namespace
}  // namespace rmd

extern "C" int rmd_corr_lookup(const void* pyramid, const rmd_pyramid_desc* d, const float* coords, int radius,
                               unsigned zero_level_mask, float* out, void* stream) {
    RMD_REQUIRE(pyramid && d && coords && out, RMD_ERR_ARG, "rmd_corr_lookup: null pointer");
    RMD_REQUIRE(d->levels >= 1 && d->levels <= RMD_MAX_LEVELS, RMD_ERR_SHAPE, "rmd_corr_lookup: bad levels");
    hipStream_t st = rmd::as_stream(stream);
    if (d->storage == RMD_F16) return rmd::launch_lookup<__half>(pyramid, *d, coords, radius, zero_level_mask, out, st);
    if (d->storage == RMD_F32) return rmd::launch_lookup<float>(pyramid, *d, coords, radius, zero_level_mask, out, st);
    rmd::set_error("rmd_corr_lookup: storage must be F32 or F16");
    return RMD_ERR_ARG;
}
