// rmd_common.h — shared host/device helpers for the gfx950 cost-volume kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "rmd.h"

namespace rmd {

// ---- error reporting (C-ABI: negative code + per-thread message) -------------------------------
void set_error(const char* fmt, ...);
void clear_error();

#define RMD_REQUIRE(cond, code, ...)        \
    do {                                    \
        if (!(cond)) {                      \
            ::rmd::set_error(__VA_ARGS__);  \
            return (code);                  \
        }                                   \
    } while (0)

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return RMD_ERR_LAUNCH;
    }
    clear_error();
    return RMD_OK;
}

// ---- pyramid geometry (POD copy of rmd_pyramid_desc, passed by value to kernels) --------------
struct PyrGeom {
    int batch, height, width, levels;
    int lh[RMD_MAX_LEVELS], lw[RMD_MAX_LEVELS];
    int th[RMD_MAX_LEVELS], tw[RMD_MAX_LEVELS];
    int ty[RMD_MAX_LEVELS], tx[RMD_MAX_LEVELS];
    long long off[RMD_MAX_LEVELS];
    int layout;       // RMD_LAYOUT_ROWS / RMD_LAYOUT_TILES
    int slots;        // query slots per chunk position (H*W in the row layout)
};

inline PyrGeom make_geom(const rmd_pyramid_desc& d) {
    PyrGeom g{};
    g.batch = d.batch;
    g.height = d.height;
    g.width = d.width;
    g.levels = d.levels;
    for (int l = 0; l < RMD_MAX_LEVELS; ++l) {
        g.lh[l] = d.level_h[l];
        g.lw[l] = d.level_w[l];
        g.th[l] = d.tile_h[l];
        g.tw[l] = d.tile_w[l];
        g.ty[l] = d.tiles_y[l];
        g.tx[l] = d.tiles_x[l];
        g.off[l] = d.level_offset[l];
    }
    g.layout = d.layout;
    g.slots = d.query_slots;
    return g;
}

// Query slots of the tiles layout (rmd.h RMD_LAYOUT_TILES): 2 x 16 query tiles of 32 slots whose
// 8-slot groups are 2 x 4 query patches, row pairs in order, an odd last row in raster order.
__host__ __device__ __forceinline__ int tiles_slot(int y1, int x1, int H, int W) {
    const int qx = (W + 15) >> 4, hp = H >> 1;
    if (y1 < 2 * hp)
        return (((y1 >> 1) * qx + (x1 >> 4)) << 5) + (((x1 & 15) >> 2) << 3) + ((y1 & 1) << 2) + (x1 & 3);
    return hp * qx * 32 + x1;
}

// pixel of slot s (x1 >= W or y1 >= H: a padding slot)
__host__ __device__ __forceinline__ void tiles_pixel(int s, int H, int W, int& y1, int& x1) {
    const int qx = (W + 15) >> 4, hp = H >> 1, base = hp * qx * 32;
    if (s < base) {
        const int t = s >> 5, j = s & 31;
        y1 = 2 * (t / qx) + ((j >> 2) & 1);
        x1 = 16 * (t % qx) + ((j >> 3) << 2) + (j & 3);
    } else {
        y1 = (H & 1) ? H - 1 : H;
        x1 = s - base;
    }
}

// row-chunk width of level l: 8, 8, 4, 2 elements — the 16 target columns of a GEMM workgroup
// map to whole chunks on every level
__host__ __device__ constexpr int level_chunk(int l) { return l <= 1 ? 8 : (l == 2 ? 4 : 2); }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// XCD-aware block order: the dispatcher deals workgroups of a 1-D grid round-robin over the 8 XCDs
// (block i -> XCD i mod 8); remap so that XCD k runs the k-th contiguous eighth of the logical
// block range, keeping what consecutive logical blocks share (one batch image's feature maps) in
// that XCD's own L2.
__device__ __forceinline__ int xcd_block(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// vmcnt on gfx950 (as on every gfx9-family CU) is ONE in-order counter for vector loads AND stores.
// The GEMM tile loops load the next tile's first B fragments (a register ring) before the current
// tile's epilogue stores; the compiler's wait before a ring register's first use must then leave the
// stores issued after that load outstanding.  But at the loop header it merges the back-edge state
// with the preheader's — where nothing follows the prologue loads — and keeps the smaller distance:
// vmcnt(ring) instead of vmcnt(ring + stores), so every tile's first MFMAs also wait for the write
// acknowledgements of the previous epilogue.  NPAD stores into a zero-range buffer (dropped by the
// range check: no memory traffic) after the prologue loads give the preheader path the same distance.
template <int NPAD>
__device__ __forceinline__ void vmcnt_pad_n(void* base) {
    const __amdgpu_buffer_rsrc_t nul = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0, 0x00020000);
#pragma unroll
    for (int i = 0; i < NPAD; ++i) __builtin_amdgcn_raw_buffer_store_b32(0, nul, 64 * i, 0, 0);   // 64-B apart: not merged
}

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(__half v) { return __half2float(v); }

}  // namespace rmd
