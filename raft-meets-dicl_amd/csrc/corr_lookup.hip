// corr_lookup.hip — per-GRU-iteration windowed bilinear lookup into the tiled correlation pyramid.
//
// Replaces raft.CorrBlock.__call__ (qzed/raft-meets-dicl src/models/impls/raft.py:49-95).
// For query p and level i the reference grid-samples the (2r+1)^2 window centred at
// (x/2^i, y/2^i) with integer offsets; all taps therefore share one bilinear weight set and the
// window reads exactly the (2r+2)^2 integer patch [x0-r, x0+r+1] x [y0-r, y0+r+1] of p's own
// level-i map.
//
// gfx950 design: one lane per (query, level, third of the window's output rows), 64
// consecutive queries per wave, so
// every output store (one channel, 64 queries) is a coalesced 256-byte row of the
// (B, L*(2r+1)^2, H, W) result.  Each patch row is fetched as whole row chunks (16 B for fp16 at
// levels 0-1) — 2 or 3 vector loads per row instead of 2r+2 scalar loads — and aligned with a
// log-step barrel shift on packed 32-bit words.  In the query-minor chunk layout (rmd.h) lanes
// with similar flow read the same chunk of adjacent queries, i.e. contiguous memory.  Rows and
// columns outside the level are zero (grid_sample zero padding).

#include "rmd_common.h"

namespace rmd {
namespace {

#ifndef RMD_LOOKUP_THREADS
#define RMD_LOOKUP_THREADS 64      // one wave per workgroup: 25.64 vs 25.89 us (256) in the bench sequence
                                   // (profiles/lookup_threads_r01.json; A/B builds: tools/_gpu_threads.sh)
#endif
constexpr int kThreads = RMD_LOOKUP_THREADS;

typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
template <int NB> struct Chunk;
template <> struct Chunk<4> { using T = unsigned; };
template <> struct Chunk<8> { using T = u32x2; };
template <> struct Chunk<16> { using T = u32x4; };

// NT (A/B knob RMD_LOOKUP_NT): bit 0 = non-temporal output stores, bit 1 = non-temporal pyramid loads
template <int NT, typename V>
__device__ __forceinline__ V ld(const V* p) {
    if constexpr ((NT & 2) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int NW, int NT>
__device__ __forceinline__ void load_words(unsigned (&dst)[NW], int at, const unsigned char* src) {
    // NW words (4, 8, 16 or 32 bytes) from a 4/8/16-byte aligned address
    constexpr int NB = NW * 4;
    if constexpr (NB <= 16) {
        typename Chunk<NB>::T v = ld<NT>(reinterpret_cast<const typename Chunk<NB>::T*>(src));
        const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
        for (int i = 0; i < NW; ++i) dst[at + i] = u[i];
    } else {
#pragma unroll
        for (int k = 0; k < NB / 16; ++k) {
            u32x4 v = ld<NT>(reinterpret_cast<const u32x4*>(src) + k);
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

// Load one patch row (2R+2 values) of a level whose tiles are TW wide.  Branch-free: the tile
// chunks a row can span are fetched from clamped addresses (an unneeded chunk re-reads chunk 0's
// line) and everything outside the level is zeroed with selects, so all loads of a patch issue
// back to back.
template <typename T, int R, int TW, int NT>
__device__ __forceinline__ void load_row(const T* __restrict__ row_ptr, long long tile_stride, int tiles_x, int xs,
                                         int lw, bool row_ok, float (&v)[2 * R + 2]) {
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
    const int tcl = min(max(tc0, 0), tiles_x - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int tc = tc0 + c;
        const bool need = tc >= 0 && tc < tiles_x && c * TW < sh + K;
        const T* p = row_ptr + (long long)(need ? tc : tcl) * tile_stride;
        unsigned tmp[CW];
        load_words<CW, NT>(tmp, 0, reinterpret_cast<const unsigned char*>(p));
#pragma unroll
        for (int i = 0; i < CW; ++i) wd[c * CW + i] = need ? tmp[i] : 0u;
    }
    wd[NW] = 0u;
    // barrel shift left by sh elements: whole words first (log steps), then a half-word
    const int wsh = (sh * S) >> 2;
    constexpr int MAXW = (TW - 1) * S / 4;               // largest whole-word shift
#pragma unroll
    for (int step = 1; step <= MAXW; step <<= 1) {
        const bool on = (wsh & step) != 0;
#pragma unroll
        for (int i = 0; i < NW + 1; ++i) wd[i] = on ? ((i + step < NW + 1) ? wd[i + step] : 0u) : wd[i];
    }
    if constexpr (S == 2) {
        const bool odd = (sh & 1) != 0;
#pragma unroll
        for (int i = 0; i < KW; ++i) wd[i] = odd ? __builtin_amdgcn_alignbyte(wd[i + 1], wd[i], 2) : wd[i];
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const float e = word_elem<T>(wd[j / EPW], j % EPW);
        const int col = xs + j;
        v[j] = (row_ok && col >= 0 && col < lw) ? e : 0.f;
    }
}

// ABL (diagnostic build only, RMD_ABLATE env, fp16/r=4): 0 normal, 1 = outputs to one channel slot
// (no output HBM traffic), 2 = no pyramid loads (zero patch)
// PR (A/B knob RMD_LOOKUP_SPLIT): output rows per lane.  PR == D is one lane per (query, level);
// PR < D splits a window's D output rows over ceil(D/PR) lanes (part = 0, 1, ...), each loading
// PR+1 patch rows: more waves in flight for the same stores, at +1 patch row per extra part.
template <typename T, int R, int L, int ABL = 0, int NT = 0, int PR = 2 * R + 1>
__device__ __forceinline__ void lookup_level(const T* __restrict__ pyr, const PyrGeom& g, int b, int p, int N,
                                             float x, float y, unsigned zmask, float* __restrict__ o,
                                             bool active, int part = 0) {
    constexpr int D = 2 * R + 1;
    constexpr int K = 2 * R + 2;
    constexpr int KR = PR + 1;                                      // patch rows this lane loads
    const int lh = g.lh[L], lw = g.lw[L];
    const int own0 = part * PR;                                     // first output row this part owns
    const int bb0 = min(own0, D - PR);                              // first output row it computes
    if ((zmask >> L) & 1u) {
        if (active)
            for (int c = 0; c < D * D; ++c)
                if (c % D >= own0 && c % D < own0 + PR) o[(size_t)c * N] = 0.f;
        return;
    }
    if (lh < 2 || lw < 2) {     // the reference normalises by (size-1) = 0 -> NaN (raft.py:73-74)
        if (active)
            for (int c = 0; c < D * D; ++c)
                if (c % D >= own0 && c % D < own0 + PR) o[(size_t)c * N] = __builtin_nanf("");
        return;
    }
    const float inv = 1.0f / (float)(1 << L);
    const float rx = x * inv, ry = y * inv;
    const float cx = fminf(fmaxf(rx, -1.0e6f), 1.0e6f), cy = fminf(fmaxf(ry, -1.0e6f), 1.0e6f);
    const float fx0 = floorf(cx), fy0 = floorf(cy);
    // weights from the unclamped coordinate: NaN / +-inf give a NaN weight and so a NaN window, as
    // the reference's grid_sample does (tests/golden corr_b2_c16_12x20_nonfinite); finite
    // coordinates beyond +-1e6 have weight 0 either way and read nothing (window off the map)
    const float fx = rx - floorf(rx), fy = ry - floorf(ry);
    const int xs = (int)fx0 - R, ys = (int)fy0 - R;

    const T* lvl = pyr + g.off[L];
    constexpr int CW = level_chunk(L);                              // row-chunk width (elements)
    const long long chunk_stride = (long long)N * CW;               // next chunk of the same row
    const long long bq = (long long)b * lh;                         // tiles_y[L] == level height
    const int txs = g.tx[L];

    float hprev[D];
#pragma unroll
    for (int jj = 0; jj < KR; ++jj) {
        const int j = bb0 + jj;
        const int yy = ys + j;
        const bool row_ok = yy >= 0 && yy < lh;
        const int yc = min(max(yy, 0), lh - 1);
        const T* row_ptr = lvl + ((bq + yc) * txs) * chunk_stride + (long long)p * CW;
        float v[K];
        if constexpr (ABL >= 2) {
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = fx * (float)k;
        } else {
            load_row<T, R, CW, NT>(row_ptr, chunk_stride, txs, xs, lw, row_ok, v);
        }
        float hcur[D];
#pragma unroll
        for (int a = 0; a < D; ++a) hcur[a] = fmaf(fx, v[a + 1] - v[a], v[a]);
        if (jj > 0 && active && (PR == D || j - 1 >= own0)) {
            const int bb = j - 1;
#pragma unroll
            for (int a = 0; a < D; ++a) {
                float* dst = o + ((ABL & 1) ? 0 : (size_t)(a * D + bb) * N);
                const float val = fmaf(fy, hcur[a] - hprev[a], hprev[a]);
                if constexpr ((NT & 1) != 0) __builtin_nontemporal_store(val, dst);
                else *dst = val;
            }
        }
#pragma unroll
        for (int a = 0; a < D; ++a) hprev[a] = hcur[a];
    }
}

// grid: (query blocks, batch, level + levels * part) — one lane per (query, level, row part)
template <typename T, int R, int ABL = 0, int NT = 0, int PR = 2 * R + 1>
__global__ void __launch_bounds__(kThreads)
corr_lookup_kernel(const T* __restrict__ pyr, PyrGeom g, const float* __restrict__ coords, unsigned zmask,
                   float* __restrict__ out) {
    const int N = g.height * g.width;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y;
    const int L = (int)blockIdx.z % g.levels;
    const int part = (int)blockIdx.z / g.levels;
    const bool active = p < N;
    const int pc = active ? p : N - 1;
    const float x = coords[((size_t)b * 2 + 0) * N + pc];
    const float y = coords[((size_t)b * 2 + 1) * N + pc];
    constexpr int D = 2 * R + 1;
    float* o = out + ((size_t)b * g.levels + L) * D * D * N + pc;
    switch (L) {
        case 0: lookup_level<T, R, 0, ABL, NT, PR>(pyr, g, b, pc, N, x, y, zmask, o, active, part); break;
        case 1: lookup_level<T, R, 1, ABL, NT, PR>(pyr, g, b, pc, N, x, y, zmask, o, active, part); break;
        case 2: lookup_level<T, R, 2, ABL, NT, PR>(pyr, g, b, pc, N, x, y, zmask, o, active, part); break;
        default: lookup_level<T, R, 3, ABL, NT, PR>(pyr, g, b, pc, N, x, y, zmask, o, active, part); break;
    }
}

#ifdef RMD_DIAG
// ---- v4 (diagnostic build, RMD_LOOKUP_V=4): all patch rows in flight, fewer instructions -------
// Hypothesis tested: the product kernel waits for every patch row's loads (vmcnt(0), which on gfx9
// also drains the previous row's 9 stores) before the next row's loads issue, and spends 46 % of its
// wave cycles parked in s_waitcnt (profiles/lookup_pmc_r02.json).  This version
//  * issues the loads of all PR+1 patch rows before any arithmetic or store (one round trip; the
//    stores come after, so no store sits in front of a load's vmcnt);
//  * folds the zero padding into per-lane weights computed once per (query, level) — a patch
//    column is in the map or not for every row alike: wl[a] = (1-fx) in(a), wr[a] = fx in(a+1);
//    row validity enters the two vertical weights of each output row — so each output costs one
//    multiply + one fma per direction and no selects;
//  * stores through a wave-uniform plane pointer + 32-bit lane offset (no 64-bit address math).
// Same arithmetic as the reference up to rounding order.  Result (profiles/lookup_ab_r02.json):
// 27.8 vs 23.8 us — 14 % fewer VALU instructions and one memory round trip per wave do not pay: the
// product kernel moves 141 MB (counters) in 24 us = 5.9 TB/s, i.e. it is HBM-bound at ~94 % of the
// 6.3 TB/s a streaming copy reaches, and more reads in flight per wave only cost occupancy (74 vs
// 57 VGPRs).  Kept for re-measurement; not compiled into librmd.so.
template <typename T, int R, int TW>
__device__ __forceinline__ void fetch_row_words(const T* __restrict__ row_ptr, long long tile_stride, int tiles_x,
                                                int tc0, unsigned (&wd)[((2 * R + 2 + 2 * TW - 2) / TW) * TW * sizeof(T) / 4]) {
    constexpr int S = sizeof(T);
    constexpr int EPW = 4 / S;
    constexpr int K = 2 * R + 2;
    constexpr int NC = (K + TW - 1 + TW - 1) / TW;
    constexpr int CW = TW * S / 4;
    // words shift_row_words can consume: the K kept elements after a shift of up to MAXW words (+1
    // word for the odd half-word step) — the last chunk is loaded only that far, so no load result
    // is dead (a dead load destination forces a vmcnt wait before its register is reused)
    constexpr int MAXW = (TW - 1) * S / 4;
    constexpr int NEED = (K - 1) / EPW + (S == 2 ? 1 : 0) + MAXW + 1;
    constexpr int LW = NEED - (NC - 1) * CW;                               // 1 .. CW words
    constexpr int LWP = LW <= 1 ? 1 : (LW <= 2 ? 2 : (LW <= 4 ? 4 : CW));
    static_assert(LW >= 1 && LW <= CW, "chunk geometry");
#pragma unroll
    for (int c = 0; c < NC - 1; ++c) {
        const int tc = min(max(tc0 + c, 0), tiles_x - 1);
        unsigned tmp[CW];
        load_words<CW, 0>(tmp, 0, reinterpret_cast<const unsigned char*>(row_ptr + (long long)tc * tile_stride));
#pragma unroll
        for (int i = 0; i < CW; ++i) wd[c * CW + i] = tmp[i];
    }
    {
        const int tc = min(max(tc0 + NC - 1, 0), tiles_x - 1);
        unsigned tmp[LWP];
        load_words<LWP, 0>(tmp, 0, reinterpret_cast<const unsigned char*>(row_ptr + (long long)tc * tile_stride));
#pragma unroll
        for (int i = 0; i < CW; ++i) wd[(NC - 1) * CW + i] = i < LWP ? tmp[i < LWP ? i : 0] : 0u;
    }
}

template <typename T, int R, int TW>
__device__ __forceinline__ void shift_row_words(const unsigned (&wd0)[((2 * R + 2 + 2 * TW - 2) / TW) * TW * sizeof(T) / 4],
                                                int sh, float (&v)[2 * R + 2]) {
    constexpr int S = sizeof(T);
    constexpr int EPW = 4 / S;
    constexpr int K = 2 * R + 2;
    constexpr int NW = ((K + 2 * TW - 2) / TW) * TW * S / 4;
    constexpr int KW = (K + EPW - 1) / EPW + 1;
    unsigned wd[NW + 1];
#pragma unroll
    for (int i = 0; i < NW; ++i) wd[i] = wd0[i];
    wd[NW] = 0u;
    const int wsh = (sh * S) >> 2;
    constexpr int MAXW = (TW - 1) * S / 4;
#pragma unroll
    for (int step = 1; step <= MAXW; step <<= 1) {
        const bool on = (wsh & step) != 0;
#pragma unroll
        for (int i = 0; i < NW + 1; ++i) wd[i] = on ? ((i + step < NW + 1) ? wd[i + step] : 0u) : wd[i];
    }
    if constexpr (S == 2) {
        const bool odd = (sh & 1) != 0;
#pragma unroll
        for (int i = 0; i < KW; ++i) wd[i] = odd ? __builtin_amdgcn_alignbyte(wd[i + 1], wd[i], 2) : wd[i];
    }
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = word_elem<T>(wd[j / EPW], j % EPW);
}

template <typename T, int R, int L, int PR>
__device__ __forceinline__ void lookup_level_v4(const T* __restrict__ pyr, const PyrGeom& g, int b, int p, int N,
                                                float x, float y, unsigned zmask, float* __restrict__ slab,
                                                bool active, int part) {
    constexpr int D = 2 * R + 1;
    constexpr int K = 2 * R + 2;
    constexpr int KR = PR + 1;
    constexpr int CW = level_chunk(L);
    constexpr int NW = ((K + 2 * CW - 2) / CW) * CW * (int)sizeof(T) / 4;
    const int lh = g.lh[L], lw = g.lw[L];
    const int own0 = part * PR;
    const int bb0 = min(own0, D - PR);
    if (((zmask >> L) & 1u) || lh < 2 || lw < 2) {
        // masked level -> 0; 1-pixel level -> NaN (the reference normalises by size-1 = 0, raft.py:73-74)
        const float v = ((zmask >> L) & 1u) ? 0.f : __builtin_nanf("");
        if (active)
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int r = 0; r < PR; ++r)
                    if (own0 + r < D) __builtin_nontemporal_store(v, slab + (size_t)(a * D + own0 + r) * N + (unsigned)p);
        return;
    }
    const float inv = 1.0f / (float)(1 << L);
    const float rx = x * inv, ry = y * inv;
    const float cx = fminf(fmaxf(rx, -1.0e6f), 1.0e6f), cy = fminf(fmaxf(ry, -1.0e6f), 1.0e6f);
    const float fx0 = floorf(cx), fy0 = floorf(cy);
    const int xs = (int)fx0 - R, ys = (int)fy0 - R;

    // ---- all patch rows' loads first ----
    const T* lvl = pyr + g.off[L];
    const long long chunk_stride = (long long)N * CW;
    const long long bq = (long long)b * lh;
    const int txs = g.tx[L];
    const int tc0 = (xs >= 0) ? xs / CW : -((CW - 1 - xs) / CW);
    const int sh = xs - tc0 * CW;
    unsigned wd[KR][NW];
#pragma unroll
    for (int jj = 0; jj < KR; ++jj) {
        const int yc = min(max(ys + bb0 + jj, 0), lh - 1);
        fetch_row_words<T, R, CW>(lvl + ((bq + yc) * txs) * chunk_stride + (long long)p * CW, chunk_stride, txs, tc0,
                                  wd[jj]);
    }
    __builtin_amdgcn_sched_barrier(0);      // keep every load of the patch ahead of the arithmetic

    // weights from the unclamped coordinate: NaN / +-inf -> NaN window (tests/golden *_nonfinite)
    const float fx = rx - floorf(rx), fy = ry - floorf(ry);
    float wl[D], wr[D];
    {
        float in[K];
#pragma unroll
        for (int j = 0; j < K; ++j) in[j] = ((unsigned)(xs + j) < (unsigned)lw) ? 1.f : 0.f;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            wl[a] = (1.f - fx) * in[a];
            wr[a] = fx * in[a + 1];
        }
    }

    float hprev[D];
    float okprev = 0.f;
#pragma unroll
    for (int jj = 0; jj < KR; ++jj) {
        const int j = bb0 + jj;
        const float ok = ((unsigned)(ys + j) < (unsigned)lh) ? 1.f : 0.f;
        float v[K];
        shift_row_words<T, R, CW>(wd[jj], sh, v);
        float hcur[D];
#pragma unroll
        for (int a = 0; a < D; ++a) hcur[a] = fmaf(wr[a], v[a + 1], wl[a] * v[a]);
        if (jj > 0 && (PR == D || j - 1 >= own0)) {
            const int bb = j - 1;
            const float w0 = (1.f - fy) * okprev, w1 = fy * ok;
            if (active)
#pragma unroll
                for (int a = 0; a < D; ++a) {
                    float* plane = slab + (size_t)(a * D + bb) * N;                 // wave-uniform
                    __builtin_nontemporal_store(fmaf(w1, hcur[a], w0 * hprev[a]), plane + (unsigned)p);
                }
        }
#pragma unroll
        for (int a = 0; a < D; ++a) hprev[a] = hcur[a];
        okprev = ok;
    }
}

// grid: (query blocks, batch, level + levels * part)
template <typename T, int R, int PR>
__global__ void __launch_bounds__(kThreads)
corr_lookup_v4_kernel(const T* __restrict__ pyr, PyrGeom g, const float* __restrict__ coords, unsigned zmask,
                      float* __restrict__ out) {
    constexpr int D = 2 * R + 1;
    const int N = g.height * g.width;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y;
    const int L = (int)blockIdx.z % g.levels;
    const int part = (int)blockIdx.z / g.levels;
    const bool active = p < N;
    const int pc = active ? p : N - 1;
    const float x = coords[((size_t)b * 2 + 0) * N + pc];
    const float y = coords[((size_t)b * 2 + 1) * N + pc];
    float* slab = out + ((size_t)b * g.levels + L) * D * D * N;
    switch (L) {
        case 0: lookup_level_v4<T, R, 0, PR>(pyr, g, b, pc, N, x, y, zmask, slab, active, part); break;
        case 1: lookup_level_v4<T, R, 1, PR>(pyr, g, b, pc, N, x, y, zmask, slab, active, part); break;
        case 2: lookup_level_v4<T, R, 2, PR>(pyr, g, b, pc, N, x, y, zmask, slab, active, part); break;
        default: lookup_level_v4<T, R, 3, PR>(pyr, g, b, pc, N, x, y, zmask, slab, active, part); break;
    }
}
#endif  // RMD_DIAG

// Row-exchange variant (diagnostic build, RMD_LOOKUP_XCH=1): one workgroup = 3 waves over the same 64
// queries and level.  Wave w owns output rows [w*D/3, (w+1)*D/3) and loads only the patch rows no
// other wave loads: wave 0 rows 0..ob1, wave w > 0 rows ob0+1..ob1.  The one row a wave w > 0 also
// needs (its first output row's upper row, loaded by wave w-1) is handed over as the horizontally
// interpolated row (D floats per lane) through 2*D*64*4 bytes of LDS after one barrier; the wave
// stores all other rows before it.  A window thus loads its 2r+2 patch rows once (10 for r = 4)
// instead of 3*(PR+1) = 12 for the independent 3-way split, at the same 3 waves per (64 queries, level).
template <typename T, int R, int L>
__device__ __forceinline__ void lookup_level_xch(const T* __restrict__ pyr, const PyrGeom& g, int b, int p, int N,
                                                 float x, float y, unsigned zmask, float* __restrict__ o,
                                                 bool active, int w, int lane, float* __restrict__ xch) {
    constexpr int D = 2 * R + 1;
    constexpr int K = 2 * R + 2;
    constexpr int KRM = (D + 2) / 3 + 1;                           // most patch rows one wave loads
    const int ob0 = (w * D) / 3, ob1 = ((w + 1) * D) / 3;          // output rows [ob0, ob1)
    const int lh = g.lh[L], lw = g.lw[L];
    // the early exits depend on the level only: uniform over the workgroup, taken before the barrier
    if ((zmask >> L) & 1u) {
        if (active)
            for (int bb = ob0; bb < ob1; ++bb)
                for (int a = 0; a < D; ++a) __builtin_nontemporal_store(0.f, o + (size_t)(a * D + bb) * N);
        return;
    }
    if (lh < 2 || lw < 2) {     // the reference normalises by (size-1) = 0 -> NaN (raft.py:73-74)
        if (active)
            for (int bb = ob0; bb < ob1; ++bb)
                for (int a = 0; a < D; ++a)
                    __builtin_nontemporal_store(__builtin_nanf(""), o + (size_t)(a * D + bb) * N);
        return;
    }
    const float inv = 1.0f / (float)(1 << L);
    const float rx = x * inv, ry = y * inv;
    const float cx = fminf(fmaxf(rx, -1.0e6f), 1.0e6f), cy = fminf(fmaxf(ry, -1.0e6f), 1.0e6f);
    const float fx0 = floorf(cx), fy0 = floorf(cy);
    // weights from the unclamped coordinate: NaN / +-inf give a NaN weight and so a NaN window, as
    // the reference's grid_sample does (tests/golden corr_b2_c16_12x20_nonfinite); finite
    // coordinates beyond +-1e6 have weight 0 either way and read nothing (window off the map)
    const float fx = rx - floorf(rx), fy = ry - floorf(ry);
    const int xs = (int)fx0 - R, ys = (int)fy0 - R;

    const T* lvl = pyr + g.off[L];
    constexpr int CW = level_chunk(L);
    const long long chunk_stride = (long long)N * CW;
    const long long bq = (long long)b * lh;
    const int txs = g.tx[L];

    const int r0 = w == 0 ? 0 : ob0 + 1;                            // patch rows [r0, ob1]
    float hprev[D], hfirst[D];
#pragma unroll
    for (int jj = 0; jj < KRM; ++jj) {
        const int j = r0 + jj;
        if (j <= ob1) {                                             // wave-uniform
            const int yy = ys + j;
            const bool row_ok = yy >= 0 && yy < lh;
            const int yc = min(max(yy, 0), lh - 1);
            const T* row_ptr = lvl + ((bq + yc) * txs) * chunk_stride + (long long)p * CW;
            float v[K];
            load_row<T, R, CW, 0>(row_ptr, chunk_stride, txs, xs, lw, row_ok, v);
            float hcur[D];
#pragma unroll
            for (int a = 0; a < D; ++a) hcur[a] = fmaf(fx, v[a + 1] - v[a], v[a]);
            if (jj > 0 && active) {
#pragma unroll
                for (int a = 0; a < D; ++a)
                    __builtin_nontemporal_store(fmaf(fy, hcur[a] - hprev[a], hprev[a]),
                                                o + (size_t)(a * D + j - 1) * N);
            }
#pragma unroll
            for (int a = 0; a < D; ++a) {
                if (jj == 0) hfirst[a] = hcur[a];
                hprev[a] = hcur[a];
            }
        }
    }
    if (w < 2) {
#pragma unroll
        for (int a = 0; a < D; ++a) xch[(w * D + a) * 64 + lane] = hprev[a];   // row ob1
    }
    __syncthreads();
    if (w > 0 && active) {
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const float up = xch[((w - 1) * D + a) * 64 + lane];            // row ob0
            __builtin_nontemporal_store(fmaf(fy, hfirst[a] - up, up), o + (size_t)(a * D + ob0) * N);
        }
    }
}

// grid: (query blocks of 64, batch, level); block: 3 waves (row parts of one window)
template <typename T, int R>
__global__ void __launch_bounds__(192)
corr_lookup_xch_kernel(const T* __restrict__ pyr, PyrGeom g, const float* __restrict__ coords, unsigned zmask,
                       float* __restrict__ out) {
    constexpr int D = 2 * R + 1;
    __shared__ float xch[2 * D * 64];
    const int N = g.height * g.width;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int p = blockIdx.x * 64 + lane;
    const int b = blockIdx.y;
    const int L = blockIdx.z;
    const bool active = p < N;
    const int pc = active ? p : N - 1;
    const float x = coords[((size_t)b * 2 + 0) * N + pc];
    const float y = coords[((size_t)b * 2 + 1) * N + pc];
    float* o = out + ((size_t)b * g.levels + L) * D * D * N + pc;
    switch (L) {
        case 0: lookup_level_xch<T, R, 0>(pyr, g, b, pc, N, x, y, zmask, o, active, w, lane, xch); break;
        case 1: lookup_level_xch<T, R, 1>(pyr, g, b, pc, N, x, y, zmask, o, active, w, lane, xch); break;
        case 2: lookup_level_xch<T, R, 2>(pyr, g, b, pc, N, x, y, zmask, o, active, w, lane, xch); break;
        default: lookup_level_xch<T, R, 3>(pyr, g, b, pc, N, x, y, zmask, o, active, w, lane, xch); break;
    }
}

template <typename T>
int launch_lookup(const void* pyr, const rmd_pyramid_desc& d, const float* coords, int radius, unsigned zmask,
                  float* out, hipStream_t st) {
    const int N = d.height * d.width;
    dim3 grid((N + kThreads - 1) / kThreads, d.batch, d.levels);
    const T* p = reinterpret_cast<const T*>(pyr);
    const PyrGeom g = make_geom(d);
#ifdef RMD_DIAG
    // A/B variants (tools/lookup_ab.py, librmd_diag.so only):
    //  RMD_ABLATE (fp16, r = 4): 1 = outputs to one channel slot, 2 = no pyramid loads (results wrong)
    //  RMD_LOOKUP_NT: 0 plain, 1 (product) nt output stores, 2 nt pyramid loads, 3 both.  cfg2
    //    (profiles/lookup_ab_r01.json): 27.1 / 24.4 / 36.6 / 36.8 us — the 73 MB output is written
    //    once and must not evict the pyramid lines that neighbouring queries' row chunks re-read.
    //  RMD_LOOKUP_SPLIT (r = 4): output rows per lane, 9 (no split) / 5 / 3 (product) / 2 / 1 —
    //    27.1 / 25.9 / 25.4 / 25.5 / 27.5 us in the bench sequence (profiles/lookup_split_r01.json).
    {
        const int abl = env_knob("RMD_ABLATE", 0);
        const int nt = env_knob("RMD_LOOKUP_NT", 1);
        const int pr = env_knob("RMD_LOOKUP_SPLIT", 3);
        if constexpr (sizeof(T) == 2) {
            // ablations of the product kernel (3-way split, nt stores): 1 = no output traffic, 2 = no
            // pyramid loads, 3 = neither (profiles/lookup_ablate_r02.json)
            const dim3 g3(grid.x, grid.y, grid.z * 3);
            if (radius == 4 && abl == 1) { corr_lookup_kernel<T, 4, 1, 1, 3><<<g3, kThreads, 0, st>>>(p, g, coords, zmask, out); return check_launch("rmd_corr_lookup"); }
            if (radius == 4 && abl == 2) { corr_lookup_kernel<T, 4, 2, 1, 3><<<g3, kThreads, 0, st>>>(p, g, coords, zmask, out); return check_launch("rmd_corr_lookup"); }
            if (radius == 4 && abl == 3) { corr_lookup_kernel<T, 4, 3, 1, 3><<<g3, kThreads, 0, st>>>(p, g, coords, zmask, out); return check_launch("rmd_corr_lookup"); }
        }
        if (radius == 4 && nt == 1 && pr != 3) {
            const dim3 gs(grid.x, grid.y, grid.z * ((9 + pr - 1) / pr));
            if (pr == 5) corr_lookup_kernel<T, 4, 0, 1, 5><<<gs, kThreads, 0, st>>>(p, g, coords, zmask, out);
            else if (pr == 2) corr_lookup_kernel<T, 4, 0, 1, 2><<<gs, kThreads, 0, st>>>(p, g, coords, zmask, out);
            else if (pr == 1) corr_lookup_kernel<T, 4, 0, 1, 1><<<gs, kThreads, 0, st>>>(p, g, coords, zmask, out);
            else corr_lookup_kernel<T, 4, 0, 1><<<grid, kThreads, 0, st>>>(p, g, coords, zmask, out);
            return check_launch("rmd_corr_lookup");
        }
        if (radius == 4 && nt != 1) {
            if (nt == 0) corr_lookup_kernel<T, 4, 0, 0><<<grid, kThreads, 0, st>>>(p, g, coords, zmask, out);
            else if (nt == 2) corr_lookup_kernel<T, 4, 0, 2><<<grid, kThreads, 0, st>>>(p, g, coords, zmask, out);
            else corr_lookup_kernel<T, 4, 0, 3><<<grid, kThreads, 0, st>>>(p, g, coords, zmask, out);
            return check_launch("rmd_corr_lookup");
        }
    }
#endif
#ifdef RMD_DIAG
    // RMD_LOOKUP_XCH=1: the row-exchange kernel (each patch row loaded once, 10 instead of 12 rows
    // per r = 4 window).  cfg2 A/B (profiles/lookup_xch_r02.json): 24.56 vs 24.00 us (bf16), 32.1 vs
    // 32.2 (fp32) — the split's duplicated rows are L2 hits, and the barrier costs more than they do.
    if (env_knob("RMD_LOOKUP_XCH", 0) != 0) {
        const dim3 gx((N + 63) / 64, d.batch, d.levels);
        switch (radius) {
#define RMD_CASE(RR) case RR: corr_lookup_xch_kernel<T, RR><<<gx, 192, 0, st>>>(p, g, coords, zmask, out); break;
            RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4) RMD_CASE(5) RMD_CASE(6) RMD_CASE(7) RMD_CASE(8)
#undef RMD_CASE
            default:
                set_error("rmd_corr_lookup: radius %d not in 1..8", radius);
                return RMD_ERR_SHAPE;
        }
        return check_launch("rmd_corr_lookup");
    }
#endif
    const dim3 g3(grid.x, grid.y, grid.z * 3);
#ifdef RMD_DIAG
    // RMD_LOOKUP_V=4: all patch rows in flight + weight-folded padding (see lookup_level_v4)
    if (env_knob("RMD_LOOKUP_V", 2) == 4) {
        switch (radius) {
#define RMD_CASE(RR) case RR: \
            corr_lookup_v4_kernel<T, RR, (2 * RR + 3) / 3><<<g3, kThreads, 0, st>>>(p, g, coords, zmask, out); \
            break;
            RMD_CASE(1) RMD_CASE(2) RMD_CASE(3) RMD_CASE(4) RMD_CASE(5) RMD_CASE(6) RMD_CASE(7) RMD_CASE(8)
#undef RMD_CASE
            default:
                set_error("rmd_corr_lookup: radius %d not in 1..8", radius);
                return RMD_ERR_SHAPE;
        }
        return check_launch("rmd_corr_lookup");
    }
#endif
    // Product path: non-temporal output stores, and every radius splits a window's 2r+1 output rows
    // over 3 lanes (PR = floor((2r+3)/3) rows each, ceil((2r+1)/PR) = 3 for r = 1..8): with one lane
    // per (query, level) the cfg2 grid is 3.5 waves per SIMD that load, then store, in lock step; 3
    // parts give the memory system 10.5 waves whose read and write phases overlap.
    switch (radius) {
#define RMD_CASE(RR) case RR: \
        corr_lookup_kernel<T, RR, 0, 1, (2 * RR + 3) / 3><<<g3, kThreads, 0, st>>>(p, g, coords, zmask, out); \
        break;
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
