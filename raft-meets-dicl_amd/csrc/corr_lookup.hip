// corr_lookup.hip — per-GRU-iteration windowed bilinear lookup into the tiled correlation pyramid.
//
// Replaces raft.CorrBlock.__call__ (qzed/raft-meets-dicl src/models/impls/raft.py:49-95).
// For query p and level i the reference grid-samples the (2r+1)^2 window centred at
// (x/2^i, y/2^i) with integer offsets; all taps therefore share one bilinear weight set and the
// window reads exactly the (2r+2)^2 integer patch [x0-r, x0+r+1] x [y0-r, y0+r+1] of p's own
// level-i map.
//
// gfx950 design: one lane per (query slot, level, third of the window's output rows),
// 64 consecutive query slots per wave, so every output store (one channel, 64 queries) is a coalesced
// 256-byte write of the (B, L*(2r+1)^2, H, W) result and every pyramid load instruction reads 64
// consecutive slots' chunks of one chunk position (contiguous memory).  A patch row is fetched as
// whole chunks (16 B at fp16 levels 0-1) — 2-4 vector loads per row instead of 2r+2 scalar loads —
// and aligned with a log-step barrel shift on packed 32-bit words.  Rows and columns outside the
// level are zero (grid_sample zero padding).  Two pyramid layouts (include/rmd.h):
//  * rows  — 1 x cw chunks, slots in raster order (f32 / x3 / tiled / stationary pyramids);
//  * tiles — 2 x 4 chunks on levels 0-1 and 2 x 4 query patches per 128-B line (w8 pyramids): a
//    lane loads 2-3 chunk rows of 3-4 quads and picks each patch row's half-chunks by the parity of
//    its first patch row.

#include <type_traits>

#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 64;       // one wave per workgroup: 25.64 vs 25.89 us (256) in the bench
                                   // sequence (profiles/lookup_threads_r01.json)

typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
template <int NB> struct Chunk;
template <> struct Chunk<4> { using T = unsigned; };
template <> struct Chunk<8> { using T = u32x2; };
template <> struct Chunk<16> { using T = u32x4; };

template <int NW>
__device__ __forceinline__ void load_words(unsigned (&dst)[NW], const unsigned char* src) {
    // NW words (4, 8, 16 or 32 bytes) from a 4/8/16-byte aligned address
    constexpr int NB = NW * 4;
    if constexpr (NB <= 16) {
        typename Chunk<NB>::T v = *reinterpret_cast<const typename Chunk<NB>::T*>(src);
        const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
        for (int i = 0; i < NW; ++i) dst[i] = u[i];
    } else {
#pragma unroll
        for (int k = 0; k < NB / 16; ++k) {
            const u32x4 v = reinterpret_cast<const u32x4*>(src)[k];
            dst[4 * k + 0] = v.x;
            dst[4 * k + 1] = v.y;
            dst[4 * k + 2] = v.z;
            dst[4 * k + 3] = v.w;
        }
    }
}

template <typename T> __device__ __forceinline__ float word_elem(unsigned w, int i);
template <> __device__ __forceinline__ float word_elem<float>(unsigned w, int) { return __uint_as_float(w); }
template <> __device__ __forceinline__ float word_elem<__half>(unsigned w, int i) {
    const unsigned short s = i ? (unsigned short)(w >> 16) : (unsigned short)(w & 0xffff);
    return __half2float(__ushort_as_half(s));
}

__device__ __forceinline__ int floor_div(int a, int d) { return a >= 0 ? a / d : -((d - 1 - a) / d); }

// Shift NW words (+1 zero word) left by sh elements of T (sh < TW): whole words in log steps, then a
// half-word for fp16, and extract the K patch values with zero padding outside [0, lw) / bad rows.
template <typename T, int K, int TW, int NW, bool MASK = true>
__device__ __forceinline__ void shift_extract(unsigned (&wd)[NW + 1], int sh, int xs, int lw, bool row_ok,
                                              float (&v)[K]) {
    constexpr int S = sizeof(T);
    constexpr int EPW = 4 / S;                           // elements per 32-bit word
    constexpr int KW = (K + EPW - 1) / EPW + 1;          // words kept after the shift
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
    if constexpr (MASK) {
        // zero padding as word masks on the aligned words (element j valid iff 0 <= xs + j < lw and the
        // row is): row-invariant, so the compiler computes them once per level, in VGPRs — not one
        // SGPR-pair compare per element and row
#pragma unroll
        for (int i = 0; i < (K + EPW - 1) / EPW; ++i) {
            unsigned m;
            if constexpr (EPW == 2)
                m = ((unsigned)(xs + 2 * i) < (unsigned)lw ? 0xFFFFu : 0u) |
                    ((unsigned)(xs + 2 * i + 1) < (unsigned)lw ? 0xFFFF0000u : 0u);
            else
                m = (unsigned)(xs + i) < (unsigned)lw ? ~0u : 0u;
            wd[i] &= row_ok ? m : 0u;
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = word_elem<T>(wd[j / EPW], j % EPW);
}

// ---- buffer loads (BUF): image b's slab of a level as one buffer resource -----------------------
// A chunk that is not needed, or lies outside the level (row or chunk index out of range), is loaded
// from offset kOOB >= the slab size: the hardware returns zeros without touching memory, so no select
// zeroes loaded words and no clamped address re-reads a line.  The host enables BUF when every
// per-image level slab is below 2^31 bytes.
constexpr unsigned kOOB = 0x80000000u;

// A/B ablation builds only (tools/build_variant.sh): bit 0 drops the output stores, bit 1 the pyramid
// loads, by sending them to kOOB (same instruction stream, no memory traffic).  0 in the product.
#ifndef RMD_LOOKUP_ABL
#define RMD_LOOKUP_ABL 0
#endif
#if RMD_LOOKUP_ABL & 4
__device__ unsigned g_abl_off = 0x80000000u;
#endif
// A/B knob: cache-policy bits of the pyramid loads (gfx950 CPol: 1 sc0, 2 nt, 16 sc1); 0 in the product
#ifndef RMD_LOOKUP_LAUX
#define RMD_LOOKUP_LAUX 0
#endif
constexpr int kLoadAux = RMD_LOOKUP_LAUX;

// RMD_S24 storage element (include/rmd.h): bytes 1..3 of an fp32 word, little endian
struct s24_t {
    unsigned char b[3];
};
template <typename T> constexpr bool kIsS24 = false;
template <> constexpr bool kIsS24<s24_t> = true;

template <typename T>
__device__ __forceinline__ const T* level_base(const T* pyr, const PyrGeom& g, int L, int b) {
    return pyr + g.off[L] + (long long)b * ((long long)g.ty[L] * g.tx[L] * g.slots * g.th[L] * g.tw[L]);
}

template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t level_rsrc(const T* pyr, const PyrGeom& g, int L, int b) {
    const long long per = (long long)g.ty[L] * g.tx[L] * g.slots * g.th[L] * g.tw[L];     // elements per image
    const T* base = level_base(pyr, g, L, b);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)base);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)base >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane((unsigned)(per * sizeof(T))),
                                             0x00020000);
}

template <int NW>
__device__ __forceinline__ void buf_words(unsigned (&dst)[NW], __amdgpu_buffer_rsrc_t rs, unsigned off) {
    if constexpr ((RMD_LOOKUP_ABL & 2) != 0) off = kOOB;
#if RMD_LOOKUP_ABL & 4
    off |= g_abl_off;                 // ABL builds: every load to kOOB through a mutable global (not foldable)
#endif
    if constexpr (NW == 4) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, kLoadAux);
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[i] = (unsigned)v[i];
    } else if constexpr (NW == 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, kLoadAux);
        dst[0] = (unsigned)v[0];
        dst[1] = (unsigned)v[1];
    } else if constexpr (NW == 1) {
        dst[0] = (unsigned)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, kLoadAux);
    } else {
#pragma unroll
        for (int k = 0; k < NW / 4; ++k) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u * k), 0, kLoadAux);
#pragma unroll
            for (int i = 0; i < 4; ++i) dst[4 * k + i] = (unsigned)v[i];
        }
    }
}

// One S24 chunk of CW = 8 or 4 elements (3 CW bytes at byte offset off of the slab, 4-aligned: level
// offsets, slot strides and chunk strides are multiples of 12 bytes) -> CW fp32 words: 12-byte loads,
// each 3 words widened with v_perm.
template <int CW>
__device__ __forceinline__ void buf_s24(unsigned (&dst)[CW], __amdgpu_buffer_rsrc_t rs, unsigned off) {
    static_assert(CW == 8 || CW == 4, "S24 chunks are 1 x 8 or 1 x 4");
    if constexpr ((RMD_LOOKUP_ABL & 2) != 0) off = kOOB;
    {
        // (16 + 8-byte loads of the 8-aligned level-0/1 chunks measured the same, profiles/s24_ab_r05.json)
        unsigned w[3 * CW / 4];
#pragma unroll
        for (int k = 0; k < CW / 4; ++k) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(off + 12u * k), 0, kLoadAux);
            w[3 * k] = (unsigned)v[0];
            w[3 * k + 1] = (unsigned)v[1];
            w[3 * k + 2] = (unsigned)v[2];
        }
#pragma unroll
        for (int k = 0; k < CW / 4; ++k) {
            const unsigned w0 = w[3 * k], w1 = w[3 * k + 1], w2 = w[3 * k + 2];
            dst[4 * k + 0] = w0 << 8;
            dst[4 * k + 1] = __builtin_amdgcn_perm(w1, w0, 0x0504030Cu);
            dst[4 * k + 2] = __builtin_amdgcn_perm(w2, w1, 0x0403020Cu);
            dst[4 * k + 3] = w2 & 0xffffff00u;
        }
    }
}

// Load one patch row (2R+2 values) of a row-layout level whose chunks are TW wide.  Branch-free: the
// chunks a row can span are fetched from clamped addresses (an unneeded chunk re-reads chunk 0's
// line) and everything outside the level is zeroed with selects, so all loads of a patch issue
// back to back.
template <typename T, int R, int TW>
__device__ __forceinline__ void load_row(const T* __restrict__ row_ptr, long long chunk_stride, int tiles_x, int xs,
                                         int lw, bool row_ok, float (&v)[2 * R + 2]) {
    constexpr int S = sizeof(T);
    constexpr int K = 2 * R + 2;                         // patch width
    constexpr int NC = (K + TW - 1 + TW - 1) / TW;       // chunks a row can span
    constexpr int CW = TW * S / 4;                       // words per chunk
    constexpr int NW = NC * CW;
    unsigned wd[NW + 1];
    const int tc0 = floor_div(xs, TW);
    const int sh = xs - tc0 * TW;                        // 0 .. TW-1
    const int tcl = min(max(tc0, 0), tiles_x - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int tc = tc0 + c;
        const bool need = tc >= 0 && tc < tiles_x && c * TW < sh + K;
        unsigned tmp[CW];
        load_words<CW>(tmp, reinterpret_cast<const unsigned char*>(row_ptr + (long long)(need ? tc : tcl) * chunk_stride));
#pragma unroll
        for (int i = 0; i < CW; ++i) wd[c * CW + i] = need ? tmp[i] : 0u;
    }
    wd[NW] = 0u;
    shift_extract<T, K, TW, NW>(wd, sh, xs, lw, row_ok, v);
}

// BUF: the (b, level) block of output planes as one buffer; plane offsets go in the instruction's
// scalar offset and an inactive lane's kOOB offset drops its stores (no branch, no 64-bit addresses)
struct OutBuf {
    __amdgpu_buffer_rsrc_t rs;
    unsigned voff;     // p * 4, or kOOB for an inactive lane
};

__device__ __forceinline__ OutBuf out_buf(float* o_block, int N, int D, int p, bool active) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)o_block);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)o_block >> 32));
    OutBuf r;
    r.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo), (short)0,
                                             (int)((unsigned)D * D * N * 4u), 0x00020000);
    r.voff = (active && (RMD_LOOKUP_ABL & 1) == 0) ? (unsigned)p * 4u : kOOB;
    return r;
}

template <int D>
__device__ __forceinline__ void emit_row_buf(const OutBuf& ob, int N, int bb, float fy, const float (&hprev)[D],
                                             const float (&hcur)[D]) {
#pragma unroll
    for (int a = 0; a < D; ++a)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(fmaf(fy, hcur[a] - hprev[a], hprev[a])), ob.rs, (int)ob.voff,
                                              (int)__builtin_amdgcn_readfirstlane((unsigned)((a * D + bb) * N) * 4u), 2);
}

// Write the part's output rows: vertical interpolation of consecutive horizontally interpolated rows
template <int D>
__device__ __forceinline__ void emit_row(float* __restrict__ o, int N, int bb, float fy, const float (&hprev)[D],
                                         const float (&hcur)[D]) {
#pragma unroll
    for (int a = 0; a < D; ++a)
        __builtin_nontemporal_store(fmaf(fy, hcur[a] - hprev[a], hprev[a]), o + (size_t)(a * D + bb) * N);
}

// Per-level window geometry; false when the level is masked (zeros) or a 1-pixel level (NaN), in
// which case the part's outputs are already written.
template <int R>
__device__ __forceinline__ bool level_setup(const PyrGeom& g, int L, float x, float y, unsigned zmask,
                                            float* __restrict__ o, int N, bool active, int own0, int PR,
                                            float& fx, float& fy, int& xs, int& ys) {
    constexpr int D = 2 * R + 1;
    const int lh = g.lh[L], lw = g.lw[L];
    if (((zmask >> L) & 1u) || lh < 2 || lw < 2) {
        // masked level -> 0; 1-pixel level -> NaN (the reference normalises by size-1 = 0, raft.py:73-74)
        const float val = ((zmask >> L) & 1u) ? 0.f : __builtin_nanf("");
        if (active)
            for (int c = 0; c < D * D; ++c)
                if (c % D >= own0 && c % D < own0 + PR) o[(size_t)c * N] = val;
        return false;
    }
    const float inv = 1.0f / (float)(1 << L);
    const float rx = x * inv, ry = y * inv;
    const float cx = fminf(fmaxf(rx, -1.0e6f), 1.0e6f), cy = fminf(fmaxf(ry, -1.0e6f), 1.0e6f);
    // weights from the unclamped coordinate: NaN / +-inf give a NaN weight and so a NaN window, as
    // the reference's grid_sample does (tests/golden corr_b2_c16_12x20_nonfinite); finite
    // coordinates beyond +-1e6 have weight 0 either way and read nothing (window off the map)
    fx = rx - floorf(rx);
    fy = ry - floorf(ry);
    xs = (int)floorf(cx) - R;
    ys = (int)floorf(cy) - R;
    return true;
}

// PR: output rows per lane.  A window's D = 2R+1 output rows are split over ceil(D/PR) lanes (part =
// 0, 1, ...), each loading PR+1 patch rows: more waves in flight for the same stores.  Row layout,
// or a tiles-layout level with 1-row chunks (levels 2-3).
//
// BUF (per-image level slabs < 2^31 B): buffer loads, zeros for chunks off the level from kOOB, and
// per-element padding masks only in waves where some lane's window reaches past the level's right
// edge (MASK; a chunk there holds padding columns).  Rows off the level are whole chunks off the level.
// S24 chunks are widened to fp32 words as they arrive and then shifted like an f32 level.
template <typename T, int R, int L, int PR, bool MASK>
__device__ __forceinline__ void rows_body_buf(__amdgpu_buffer_rsrc_t rs, const PyrGeom& g, int slot, int N,
                                              float fx, float fy, int xs, int ys, const OutBuf& ob, int own0, int bb0) {
    constexpr bool S24 = kIsS24<T>;
    using TE = typename std::conditional<S24, float, T>::type;     // element type of the loaded words
    constexpr int D = 2 * R + 1, K = 2 * R + 2, KR = PR + 1;
    constexpr int CW = S24 && L == 3 ? 4 : level_chunk(L);          // 8, 8, 4, 2 elements (S24: 8, 8, 4, 4)
    constexpr int CB = CW * (int)sizeof(T);                         // chunk bytes
    constexpr int CWW = S24 ? CW : CB / 4;                          // chunk words (S24: widened)
    constexpr int NC = (K + CW - 1 + CW - 1) / CW;                  // chunks a row can span
    const int lh = g.lh[L], lw = g.lw[L], txs = g.tx[L];
    const unsigned cs = (unsigned)g.slots * CB, rsb = (unsigned)txs * cs;
    const int tc0 = floor_div(xs, CW);
    const int sh = xs - tc0 * CW;
    const unsigned off0 = (unsigned)tc0 * cs + (unsigned)slot * CB;  // wraps for tc0 < 0: used only when valid
    float hprev[D];
#pragma unroll
    for (int jj = 0; jj < KR; ++jj) {
        const int j = bb0 + jj;
        const int yy = ys + j;
        const bool rv = yy >= 0 && yy < lh;
        const unsigned roff = off0 + (unsigned)yy * rsb;
        unsigned wd[NC * CWW + 1];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int tc = tc0 + c;
            const bool valid = rv && tc >= 0 && tc < txs && c * CW < sh + K;
            unsigned tmp[CWW];
            if constexpr (S24)
                buf_s24<CW>(tmp, rs, valid ? roff + (unsigned)c * cs : kOOB);
            else
                buf_words<CWW>(tmp, rs, valid ? roff + (unsigned)c * cs : kOOB);
#pragma unroll
            for (int i = 0; i < CWW; ++i) wd[c * CWW + i] = tmp[i];
        }
        wd[NC * CWW] = 0u;
        float v[K];
        shift_extract<TE, K, CW, NC * CWW, MASK>(wd, sh, xs, lw, true, v);
        float hcur[D];
#pragma unroll
        for (int a = 0; a < D; ++a) hcur[a] = fmaf(fx, v[a + 1] - v[a], v[a]);
        if (jj > 0 && (PR == D || j - 1 >= own0)) emit_row_buf<D>(ob, N, j - 1, fy, hprev, hcur);
#pragma unroll
        for (int a = 0; a < D; ++a) hprev[a] = hcur[a];
    }
}

template <typename T, int R, int L, int PR, bool BUF>
__device__ __forceinline__ void lookup_level_rows(const T* __restrict__ pyr, const PyrGeom& g, int b, int slot, int N,
                                                  float x, float y, unsigned zmask, float* __restrict__ o,
                                                  const OutBuf& ob, bool active, int part) {
    constexpr int D = 2 * R + 1;
    constexpr int K = 2 * R + 2;
    constexpr int KR = PR + 1;                                      // patch rows this lane loads
    const int own0 = part * PR;                                     // first output row this part owns
    const int bb0 = min(own0, D - PR);                              // first output row it computes
    float fx, fy;
    int xs, ys;
    if (!level_setup<R>(g, L, x, y, zmask, o, N, active, own0, PR, fx, fy, xs, ys)) return;
    const int lh = g.lh[L], lw = g.lw[L];
    if constexpr (BUF) {
        const __amdgpu_buffer_rsrc_t rs = level_rsrc(pyr, g, L, b);
        if (__any(xs + K > lw))
            rows_body_buf<T, R, L, PR, true>(rs, g, slot, N, fx, fy, xs, ys, ob, own0, bb0);
        else
            rows_body_buf<T, R, L, PR, false>(rs, g, slot, N, fx, fy, xs, ys, ob, own0, bb0);
        return;
    } else {
        static_assert(!kIsS24<T>, "S24 pyramids are read through buffer loads only");
        const T* lvl = pyr + g.off[L];
        constexpr int CW = level_chunk(L);                              // 8, 8, 4, 2 (tiles layout: only L >= 2)
        const long long chunk_stride = (long long)g.slots * CW;         // next chunk of the same row
        const long long bq = (long long)b * g.ty[L];
        const int txs = g.tx[L];

        float hprev[D];
#pragma unroll
        for (int jj = 0; jj < KR; ++jj) {
            const int j = bb0 + jj;
            const int yy = ys + j;
            const bool row_ok = yy >= 0 && yy < lh;
            const int yc = min(max(yy, 0), lh - 1);
            const T* row_ptr = lvl + ((bq + yc) * txs) * chunk_stride + (long long)slot * CW;
            float v[K];
            load_row<T, R, CW>(row_ptr, chunk_stride, txs, xs, lw, row_ok, v);
            float hcur[D];
#pragma unroll
            for (int a = 0; a < D; ++a) hcur[a] = fmaf(fx, v[a + 1] - v[a], v[a]);
            if (jj > 0 && active && (PR == D || j - 1 >= own0)) emit_row<D>(o, N, j - 1, fy, hprev, hcur);
#pragma unroll
            for (int a = 0; a < D; ++a) hprev[a] = hcur[a];
        }
    }
}

// Tiles-layout level 0/1: 2 x 4 fp16 chunks (16 B: row 0 in words 0-1, row 1 in words 2-3).  BUF: each
// of the part's KR patch rows loads its own 8-B half of NQ chunks; chunks that are not needed or lie off
// the level (and the padding half of an odd last row) load zeros from kOOB, and padding columns are
// masked per word only in waves where some lane's window reaches the level's edge (MASK).  !BUF (slabs
// of 2 GiB and more): whole chunks of NCR chunk rows from clamped addresses (an L2 hit); patch row jj
// sits in chunk row (jj + par) >> 1, half (jj + par) & 1 with par = ya & 1, selected per lane.
template <int R, int L, int PR, bool BUF, bool MASK>
__device__ __forceinline__ void tiles_body(const __half* __restrict__ pyr, const PyrGeom& g, int b, int slot, int N,
                                           float fx, float fy, int xs, int ys, float* __restrict__ o, const OutBuf& ob,
                                           bool active, int own0, int bb0) {
    constexpr int D = 2 * R + 1;
    constexpr int K = 2 * R + 2;
    constexpr int KR = PR + 1;
    constexpr int NCR = KR / 2 + 1;                                 // chunk rows a part can span
    constexpr int NQ = (K + 3 + 3) / 4;                             // quads a patch row can span
    const int lh = g.lh[L], lw = g.lw[L];
    const int ya = ys + bb0;
    const int cr0 = floor_div(ya, 2);
    const int par = ya - 2 * cr0;
    const int q0 = floor_div(xs, 4);
    const int sh = xs - 4 * q0;                                     // 0 .. 3
    const int tys = g.ty[L], txs = g.tx[L];

    // BUF: per patch row, NQ 8-B loads straight from the row's half of each chunk (no parity select;
    // 64 VGPRs vs 72 for whole-chunk loads + selects, 1-2 % faster, profiles/lookup_ab_r04.json)
    unsigned hw[KR][2 * NQ];
    if constexpr (BUF) {
        const __amdgpu_buffer_rsrc_t rs = level_rsrc(pyr, g, L, b);
        const unsigned cs = (unsigned)g.slots * 16u;
#pragma unroll
        for (int jj = 0; jj < KR; ++jj) {
            const int yy = ya + jj;
            const int crow = floor_div(yy, 2);
            const bool rneed = crow >= 0 && crow < tys && yy < lh;      // the odd last row's padding half: zeros
            const unsigned rbase = (unsigned)(crow * txs + q0) * cs + (unsigned)slot * 16u + 8u * (unsigned)(yy - 2 * crow);
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                const int q = q0 + c;
                const bool need = rneed && q >= 0 && q < txs && c * 4 < sh + K;
                unsigned t2[2];
                buf_words<2>(t2, rs, need ? rbase + (unsigned)c * cs : kOOB);
                hw[jj][2 * c] = t2[0];
                hw[jj][2 * c + 1] = t2[1];
            }
        }
    }
    unsigned wd[NCR][NQ][4];
    if constexpr (!BUF) {
        const int crl = min(max(cr0, 0), tys - 1), ql = min(max(q0, 0), txs - 1);
        const long long cs = (long long)g.slots * 8;                // next quad (elements)
        const __half* base = pyr + g.off[L] + (long long)slot * 8;
        const long long bq = (long long)b * tys;
#pragma unroll
        for (int cr = 0; cr < NCR; ++cr) {
            const int crow = cr0 + cr;
            const bool rneed = crow >= 0 && crow < tys && 2 * cr <= par + KR - 1;
            const long long rp = (bq + (rneed ? crow : crl)) * txs;
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                const int q = q0 + c;
                const bool need = rneed && q >= 0 && q < txs && c * 4 < sh + K;
                const u32x4 v = *reinterpret_cast<const u32x4*>(base + (rp + (need ? q : ql)) * cs);
                wd[cr][c][0] = need ? v.x : 0u;
                wd[cr][c][1] = need ? v.y : 0u;
                wd[cr][c][2] = need ? v.z : 0u;
                wd[cr][c][3] = need ? v.w : 0u;
            }
        }
    }

    float hprev[D];
#pragma unroll
    for (int jj = 0; jj < KR; ++jj) {
        const int yy = ya + jj;
        const bool row_ok = yy >= 0 && yy < lh;
        unsigned rw[2 * NQ + 1];
        // parity 0: chunk row jj >> 1, half jj & 1; parity 1: chunk row (jj + 1) >> 1, half (jj + 1) & 1
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            if constexpr (BUF) {
                rw[2 * c] = hw[jj][2 * c];
                rw[2 * c + 1] = hw[jj][2 * c + 1];
                continue;
            }
            const int r0 = jj >> 1, h0 = (jj & 1) * 2;
            const int r1 = (jj + 1) >> 1, h1 = ((jj + 1) & 1) * 2;
            const unsigned a0 = wd[r0][c][h0], a1 = wd[r0][c][h0 + 1];
            const unsigned b0 = r1 < NCR ? wd[r1 < NCR ? r1 : 0][c][h1] : 0u;
            const unsigned b1 = r1 < NCR ? wd[r1 < NCR ? r1 : 0][c][h1 + 1] : 0u;
            rw[2 * c] = par ? b0 : a0;
            rw[2 * c + 1] = par ? b1 : a1;
        }
        rw[2 * NQ] = 0u;
        float v[K];
        shift_extract<__half, K, 4, 2 * NQ, MASK>(rw, sh, xs, lw, row_ok, v);
        float hcur[D];
#pragma unroll
        for (int a = 0; a < D; ++a) hcur[a] = fmaf(fx, v[a + 1] - v[a], v[a]);
        const int j = bb0 + jj;
        if (jj > 0 && (PR == D || j - 1 >= own0)) {
            if constexpr (BUF) emit_row_buf<D>(ob, N, j - 1, fy, hprev, hcur);
            else if (active) emit_row<D>(o, N, j - 1, fy, hprev, hcur);
        }
#pragma unroll
        for (int a = 0; a < D; ++a) hprev[a] = hcur[a];
    }
}

template <int R, int L, int PR, bool BUF>
__device__ __forceinline__ void lookup_level_tiles(const __half* __restrict__ pyr, const PyrGeom& g, int b, int slot,
                                                   int N, float x, float y, unsigned zmask, float* __restrict__ o,
                                                   const OutBuf& ob, bool active, int part) {
    constexpr int D = 2 * R + 1, K = 2 * R + 2, KR = PR + 1;
    const int own0 = part * PR;
    const int bb0 = min(own0, D - PR);
    float fx, fy;
    int xs, ys;
    if (!level_setup<R>(g, L, x, y, zmask, o, N, active, own0, PR, fx, fy, xs, ys)) return;
    if constexpr (BUF) {
        if (__any(xs + K > g.lw[L] || ys + bb0 + KR > g.lh[L]))
            tiles_body<R, L, PR, true, true>(pyr, g, b, slot, N, fx, fy, xs, ys, o, ob, active, own0, bb0);
        else
            tiles_body<R, L, PR, true, false>(pyr, g, b, slot, N, fx, fy, xs, ys, o, ob, active, own0, bb0);
    } else {
        tiles_body<R, L, PR, false, true>(pyr, g, b, slot, N, fx, fy, xs, ys, o, ob, active, own0, bb0);
    }
}

// grid: (slot blocks of 64, batch, level + levels * part) — one lane per (query slot, level, row part).
// (Row parts adjacent in dispatch order, one XCD apart, and level 0 last measured no gain,
// profiles/lookup_order_ab_r05.json.)
#ifndef RMD_LOOKUP_WPE8
#define RMD_LOOKUP_WPE8 0
#endif
#if RMD_LOOKUP_WPE8
#define RMD_LOOKUP_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
#else
#define RMD_LOOKUP_ATTR
#endif
template <typename T, int R, int PR, int LAY, bool BUF>
__global__ void __launch_bounds__(kThreads) RMD_LOOKUP_ATTR
corr_lookup_kernel(const T* __restrict__ pyr, PyrGeom g, const float* __restrict__ coords, unsigned zmask,
                   float* __restrict__ out) {
    const int N = g.height * g.width;
    const int s = blockIdx.x * kThreads + threadIdx.x;
    const int L = (int)blockIdx.z % g.levels;
    const int part = (int)blockIdx.z / g.levels;
    const int b = blockIdx.y;
    bool active;
    int p, slot;
    if constexpr (LAY == RMD_LAYOUT_TILES) {
        slot = min(s, g.slots - 1);
        int y1, x1;
        tiles_pixel(slot, g.height, g.width, y1, x1);
        active = s < g.slots && y1 < g.height && x1 < g.width;
        p = active ? y1 * g.width + x1 : 0;
    } else {
        active = s < N;
        p = active ? s : N - 1;
        slot = p;
    }
    const float x = coords[((size_t)b * 2 + 0) * N + p];
    const float y = coords[((size_t)b * 2 + 1) * N + p];
    constexpr int D = 2 * R + 1;
    float* ob_block = out + ((size_t)b * g.levels + L) * D * D * N;
    float* o = ob_block + p;
    OutBuf ob;
    if constexpr (BUF) ob = out_buf(ob_block, N, D, p, active);
    if constexpr (LAY == RMD_LAYOUT_TILES) {
        switch (L) {
            case 0: lookup_level_tiles<R, 0, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
            case 1: lookup_level_tiles<R, 1, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
            case 2: lookup_level_rows<T, R, 2, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
            default: lookup_level_rows<T, R, 3, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
        }
    } else {
        switch (L) {
            case 0: lookup_level_rows<T, R, 0, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
            case 1: lookup_level_rows<T, R, 1, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
            case 2: lookup_level_rows<T, R, 2, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
            default: lookup_level_rows<T, R, 3, PR, BUF>(pyr, g, b, slot, N, x, y, zmask, o, ob, active, part); break;
        }
    }
}

// Every radius splits a window's 2r+1 output rows over 3 lanes (PR = floor((2r+3)/3) rows each,
// ceil((2r+1)/PR) = 3 for r = 1..8): with one lane per (query, level) the cfg2 grid is 3.5 waves per
// SIMD that load, then store, in lock step; 3 parts give the memory system 10.5 waves whose read and
// write phases overlap (cfg2: 27.1 / 25.9 / 25.4 / 25.5 / 27.5 us for 9 / 5 / 3 / 2 / 1 rows per lane,
// profiles/lookup_split_r01.json).  Output stores are non-temporal (24.4 vs 27.1 us plain; the 73 MB
// output must not evict the pyramid lines neighbouring queries re-read, profiles/lookup_ab_r01.json).
template <typename T, int LAY>
int launch_lookup(const void* pyr, const rmd_pyramid_desc& d, const float* coords, int radius, unsigned zmask,
                  float* out, hipStream_t st) {
    const PyrGeom g = make_geom(d);
    const dim3 grid((g.slots + kThreads - 1) / kThreads, d.batch, d.levels * 3);
    const T* p = reinterpret_cast<const T*>(pyr);
    // buffer loads need every per-image level slab below 2^31 bytes (kOOB must lie past it); the
    // pointer path stays for larger pyramids (-DRMD_LOOKUP_BUF=0 forces it for A/B builds)
#ifndef RMD_LOOKUP_BUF
#define RMD_LOOKUP_BUF 1
#endif
    bool buf = RMD_LOOKUP_BUF != 0;
    for (int l = 0; l < d.levels; ++l)
        buf = buf && (double)d.tiles_y[l] * d.tiles_x[l] * d.query_slots * d.tile_h[l] * d.tile_w[l] * sizeof(T) <
                         2147483648.0;
    buf = buf && (double)(2 * radius + 1) * (2 * radius + 1) * d.height * d.width * 4.0 < 2147483648.0;   // output block
    if (kIsS24<T> && !buf) {
        set_error("rmd_corr_lookup: S24 pyramids need per-image level slabs < 2 GiB");
        return RMD_ERR_SHAPE;
    }
    switch (radius) {
#define RMD_CASE(RR) case RR: \
        if (buf) corr_lookup_kernel<T, RR, (2 * RR + 3) / 3, LAY, true><<<grid, kThreads, 0, st>>>(p, g, coords, zmask, out); \
        else if constexpr (!kIsS24<T>) corr_lookup_kernel<T, RR, (2 * RR + 3) / 3, LAY, false><<<grid, kThreads, 0, st>>>(p, g, coords, zmask, out); \
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
    RMD_REQUIRE(d->query_slots >= d->height * d->width, RMD_ERR_SHAPE, "rmd_corr_lookup: bad query_slots");
    hipStream_t st = rmd::as_stream(stream);
    if (d->layout == RMD_LAYOUT_TILES) {
        RMD_REQUIRE(d->storage == RMD_F16, RMD_ERR_ARG, "rmd_corr_lookup: the tiles layout is fp16 only");
        return rmd::launch_lookup<__half, RMD_LAYOUT_TILES>(pyramid, *d, coords, radius, zero_level_mask, out, st);
    }
    RMD_REQUIRE(d->layout == RMD_LAYOUT_ROWS, RMD_ERR_ARG, "rmd_corr_lookup: bad layout %d", d->layout);
    if (d->storage == RMD_F16)
        return rmd::launch_lookup<__half, RMD_LAYOUT_ROWS>(pyramid, *d, coords, radius, zero_level_mask, out, st);
    if (d->storage == RMD_F32)
        return rmd::launch_lookup<float, RMD_LAYOUT_ROWS>(pyramid, *d, coords, radius, zero_level_mask, out, st);
    if (d->storage == RMD_S24)
        return rmd::launch_lookup<rmd::s24_t, RMD_LAYOUT_ROWS>(pyramid, *d, coords, radius, zero_level_mask, out, st);
    rmd::set_error("rmd_corr_lookup: storage must be F32, F16 or S24");
    return RMD_ERR_ARG;
}
