/*
 * rmd.h — C ABI of the MI355X (gfx950) cost-volume backend for qzed/raft-meets-dicl.
 *
 * Plain pointers, sizes and a HIP stream handle; no torch types.  Every entry point enqueues
 * work on `stream` (a hipStream_t passed as void*; NULL = the default stream) and returns
 * immediately: launchers never allocate, free or synchronise, so a caller may capture them into
 * a hipGraph.  Outputs and workspaces are caller-allocated device memory.
 *
 * Return codes: RMD_OK (0) or a negative RMD_ERR_* code; rmd_last_error() returns a
 * human-readable message for the last failing call on the calling thread.
 *
 * Each entry point names the reference function it replaces (qzed/raft-meets-dicl v2,
 * file:line).  The reference has no native code: these are the boundary its Python modules bind
 * through (ctypes stub in INTEGRATION.md; host mirror in raft-meets-dicl_amd/rmd/).
 *
 * Tensor conventions (all device pointers, contiguous, row-major):
 *   fmap   (B, C, H, W)  float32      feature maps at 1/8 resolution (raft.py:381 `.float()`)
 *   coords (B, 2, H, W)  float32      ch0 = x, ch1 = y, level-0 pixel units (grid.py:4-12)
 *   out    (B, L*(2r+1)^2, H, W) float32, channel = level*(2r+1)^2 + a*(2r+1) + b with x-offset
 *          a-r and y-offset b-r (meshgrid(dx, dy, indexing='ij'), raft.py:57-59).
 */
#ifndef RMD_H
#define RMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMD_OK 0
#define RMD_ERR_ARG (-1)          /* null pointer / bad enum */
#define RMD_ERR_SHAPE (-2)        /* unsupported or inconsistent sizes */
#define RMD_ERR_LAUNCH (-3)       /* kernel launch failed (hipGetLastError) */

/* element / compute types */
#define RMD_F32 0
#define RMD_F16 1
#define RMD_BF16 2

#define RMD_MAX_LEVELS 4

/*
 * Layout of a correlation pyramid in HBM (one allocation, `total_elements` elements of
 * `storage` type).  Level l has floor-halved sizes level_h[l] x level_w[l] (raft.py:38-47) and is
 * cut into tile_h[l] x tile_w[l] target tiles (8x8, 8x8, 4x4, 2x2).  Tiles are query-minor:
 *
 *   element(b, p, y, x) at level l =
 *     level_offset[l] + ((((b*tiles_y[l] + y/tile_h[l])*tiles_x[l] + x/tile_w[l]) * (H*W) + p)
 *                        * tile_h[l]*tile_w[l]) + (y%tile_h[l])*tile_w[l] + x%tile_w[l]
 *
 * where p = y1*W + x1 is the query pixel.  One lookup window (2r+2)^2 then touches ~4.5 tiles of
 * 128 B (fp16) per level instead of 2r+2 cache-line rows, and the correlation GEMM's epilogue
 * writes every level as contiguous runs.  Padding elements inside edge tiles
 * hold unspecified values and are never read.
 */
typedef struct rmd_pyramid_desc {
    int batch, height, width;          /* query grid == level-0 target grid                  */
    int levels;                        /* 1 .. RMD_MAX_LEVELS                                */
    int storage;                       /* RMD_F32 or RMD_F16                                 */
    int level_h[RMD_MAX_LEVELS], level_w[RMD_MAX_LEVELS];
    int tile_h[RMD_MAX_LEVELS], tile_w[RMD_MAX_LEVELS];
    int tiles_y[RMD_MAX_LEVELS], tiles_x[RMD_MAX_LEVELS];
    long long level_offset[RMD_MAX_LEVELS];    /* in elements */
    long long total_elements;
} rmd_pyramid_desc;

/* Fill `desc` for a (batch, height, width) query grid.  Host-only, no device work. */
int rmd_pyramid_describe(int batch, int height, int width, int levels, int storage,
                         rmd_pyramid_desc* desc);

/* Bytes of device workspace rmd_corr_pyramid needs for `compute` (operand staging). */
size_t rmd_corr_pyramid_workspace_bytes(const rmd_pyramid_desc* desc, int channels, int compute);

/*
 * All-pairs correlation + pooled pyramid.  Replaces raft.CorrBlock.__init__
 * (src/models/impls/raft.py:18-47): corr0 = fmap1^T fmap2 / sqrt(C) over each batch, then
 * levels-1 successive 2x2 average pools over the target dims, floor sizes.
 *   compute = RMD_F32  : exact f32 MFMA (v_mfma_f32_32x32x2_f32), the parity mode
 *   compute = RMD_BF16 : bf16 MFMA operands, f32 accumulation (performance mode)
 * All levels are produced by the GEMM epilogue from the f32 accumulators and stored as
 * desc->storage.
 */
int rmd_corr_pyramid(const float* fmap1, const float* fmap2, int channels,
                     const rmd_pyramid_desc* desc, int compute, void* pyramid, void* workspace,
                     void* stream);

/*
 * Windowed bilinear pyramid lookup.  Replaces raft.CorrBlock.__call__ (raft.py:49-95):
 * level i is sampled at (x/2^i + a - r, y/2^i + b - r), bilinear, align_corners=True, zero
 * padding per tap.  Bit i of `zero_level_mask` zeroes level i (mask_costs entry i+3,
 * raft.py:86-87).  A level with height or width 1 yields NaN (the reference divides by zero at
 * raft.py:73-74).  radius 1..8.
 */
int rmd_corr_lookup(const void* pyramid, const rmd_pyramid_desc* desc, const float* coords,
                    int radius, unsigned zero_level_mask, float* out, void* stream);

/* Message for the last failing call on this thread ("" if none). */
const char* rmd_last_error(void);

/* Library version string, e.g. "rmd 0.1 gfx950". */
const char* rmd_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RMD_H */
