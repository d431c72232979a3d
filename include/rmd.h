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
#define RMD_BF16X3 3   /* compute only: fp32-accurate split bf16, hi.hi + hi.lo + lo.hi per k-step */
#define RMD_S24 4      /* storage only: an fp32 value rounded to its top 24 bits (sign, exponent, 15 mantissa
                          bits; round half away from zero, NaN stays NaN), stored as 3 little-endian bytes
                          (bytes 1..3 of the float); row layout only, written by the x3 GEMM */

#define RMD_MAX_LEVELS 4

/*
 * Layout of a correlation pyramid in HBM (one allocation, `total_elements` elements of
 * `storage` type).  Level l has floor-halved sizes level_h[l] x level_w[l] (raft.py:38-47).  The
 * target map of each level is cut into chunks of tile_h[l] x tile_w[l] elements and chunks are
 * QUERY-MINOR: every chunk position holds the chunk of all `query_slots` queries back to back,
 *
 *   element(b, p, y, x) at level l =
 *     level_offset[l] + ((((b*tiles_y[l] + y/tile_h[l])*tiles_x[l] + x/tile_w[l]) * query_slots
 *                         + slot(p)) * tile_h[l]*tile_w[l]) + (y%tile_h[l])*tile_w[l] + x%tile_w[l]
 *
 * with tiles_y[l] = ceil(level_h[l] / tile_h[l]), tiles_x[l] = ceil(level_w[l] / tile_w[l]) and
 * p = y1*W + x1 the query pixel.  Two layouts (`layout`):
 *
 *  RMD_LAYOUT_ROWS  (every GEMM except w8): chunks 1 x (8, 8, 4, 2) (RMD_S24 storage: 1 x (8, 8, 4, 4),
 *    so every S24 chunk is a multiple of 4 bytes), slot(p) = p, query_slots = H*W.
 *  RMD_LAYOUT_TILES (the w8 GEMM: bf16 compute, fp16 storage): chunks 2x4, 2x4, 1x4, 1x2 and query
 *    slots in 2 x 16 query tiles whose 8-slot groups are 2 x 4 query patches:
 *      y1 < 2*floor(H/2): slot = ((y1/2)*QX + x1/16)*32 + ((x1%16)/4)*8 + (y1%2)*4 + x1%4, QX = ceil(W/16)
 *      y1 = H-1, H odd  : slot = floor(H/2)*QX*32 + x1            (the last row in raster order)
 *    query_slots = floor(H/2)*QX*32 (+ ceil(W/32)*32 for odd H); slots of no pixel (x1 >= W) hold
 *    unspecified values.  A 128-B line of a level-0/1 chunk position then holds a 2 x 4 target patch
 *    of a 2 x 4 query patch, so the windows of neighbouring queries share lines in both directions
 *    (cfg2 lookup reads 55 MB modelled vs 66 MB in the row layout, tools/lookup_line_model.py).
 *
 * In both layouts consecutive slots' chunks are adjacent, so a wave of 64 consecutive slots reads
 * (lookup) and writes (GEMM epilogue) 64 x 16 B of contiguous memory per chunk position (DESIGN.md
 * §3).  Padding rows/columns of a level's last chunks hold unspecified values and are never read.
 */
#define RMD_LAYOUT_ROWS 0
#define RMD_LAYOUT_TILES 1

typedef struct rmd_pyramid_desc {
    int batch, height, width;          /* query grid == level-0 target grid                  */
    int levels;                        /* 1 .. RMD_MAX_LEVELS                                */
    int storage;                       /* RMD_F32, RMD_F16 or RMD_S24 (3 bytes per element)   */
    int level_h[RMD_MAX_LEVELS], level_w[RMD_MAX_LEVELS];
    int tile_h[RMD_MAX_LEVELS], tile_w[RMD_MAX_LEVELS];
    int tiles_y[RMD_MAX_LEVELS], tiles_x[RMD_MAX_LEVELS];
    long long level_offset[RMD_MAX_LEVELS];    /* in elements */
    long long total_elements;
    int layout;                        /* RMD_LAYOUT_ROWS or RMD_LAYOUT_TILES                */
    int query_slots;                   /* query positions per chunk position (>= H*W)        */
} rmd_pyramid_desc;

/* Fill `desc` for a (batch, height, width) query grid in the row layout.  Host-only, no device work. */
int rmd_pyramid_describe(int batch, int height, int width, int levels, int storage,
                         rmd_pyramid_desc* desc);

/* Same for an explicit layout (RMD_LAYOUT_TILES needs storage RMD_F16). */
int rmd_pyramid_describe_layout(int batch, int height, int width, int levels, int storage, int layout,
                                rmd_pyramid_desc* desc);

/* Describe the pyramid rmd_corr_pyramid writes for (channels, compute): the tiles layout when the
 * call runs the w8 GEMM (see rmd_corr_gemm_kernel), the row layout otherwise.  rmd_corr_pyramid
 * rejects a desc whose layout its GEMM does not write. */
int rmd_pyramid_describe_for(int batch, int height, int width, int levels, int storage, int channels,
                             int compute, rmd_pyramid_desc* desc);

/* Bytes of device workspace rmd_corr_pyramid needs for `compute` (operand staging). */
size_t rmd_corr_pyramid_workspace_bytes(const rmd_pyramid_desc* desc, int channels, int compute);

/*
 * All-pairs correlation + pooled pyramid.  Replaces raft.CorrBlock.__init__
 * (src/models/impls/raft.py:18-47): corr0 = scale * fmap1^T fmap2 over each batch, then
 * levels-1 successive 2x2 average pools over the target dims, floor sizes.  scale = 1/sqrt(C) is
 * raft.CorrBlock (raft.py:33); scale = 1 gives raft_fs.CorrBlock's unnormalised products
 * (src/models/impls/raft_fs.py:13-87, whose pooled-feature dot equals the pooled volume).
 *   compute = RMD_F32    : exact f32 MFMA (v_mfma_f32_32x32x2_f32)
 *   compute = RMD_BF16X3 : fp32-accurate split bf16 MFMA, x = hi + lo, three bf16 products per
 *                          k-step (~2^-16 relative per product; f32 storage, C <= 256; other cases
 *                          run the exact f32 kernel) — the default parity mode
 *   compute = RMD_BF16   : bf16 MFMA operands, f32 accumulation (performance mode)
 * All levels are produced by the GEMM epilogue from the f32 accumulators and stored as
 * desc->storage.
 */
int rmd_corr_pyramid(const float* fmap1, const float* fmap2, int channels, float scale,
                     const rmd_pyramid_desc* desc, int compute, void* pyramid, void* workspace,
                     void* stream);

/* Name of the GEMM kernel rmd_corr_pyramid runs for these arguments: "w8" (bf16 operands, fp16
 * pyramid, C <= 256: the performance path), "stationary" (the same with 64-bit store addressing, for
 * maps whose level-0 row span passes 1 GiB, e.g. 4K frames), "x3" (RMD_BF16X3 with an f32 pyramid),
 * "tiled" (exact f32 MFMA or any other combination), or "invalid".  Host-only; for tests and introspection. */
const char* rmd_corr_gemm_kernel(const rmd_pyramid_desc* desc, int channels, int compute);

/* The two halves of rmd_corr_pyramid, for callers that time or overlap them separately:
 * rmd_corr_prepare transposes/converts both feature maps into the workspace (pixel-major,
 * channel-contiguous operands); rmd_corr_pyramid_prepared runs the GEMM + pyramid epilogue on them. */
int rmd_corr_prepare(const float* fmap1, const float* fmap2, int channels, float scale,
                     const rmd_pyramid_desc* desc, int compute, void* workspace, void* stream);
int rmd_corr_pyramid_prepared(int channels, float scale, const rmd_pyramid_desc* desc, int compute,
                              void* pyramid, void* workspace, void* stream);

/*
 * Windowed bilinear pyramid lookup.  Replaces raft.CorrBlock.__call__ (raft.py:49-95):
 * level i is sampled at (x/2^i + a - r, y/2^i + b - r), bilinear, align_corners=True, zero
 * padding per tap.  Bit i of `zero_level_mask` zeroes level i (mask_costs entry i+3,
 * raft.py:86-87).  A level with height or width 1 yields NaN (the reference divides by zero at
 * raft.py:73-74).  radius 1..8.
 */
int rmd_corr_lookup(const void* pyramid, const rmd_pyramid_desc* desc, const float* coords,
                    int radius, unsigned zero_level_mask, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * On-the-fly windowed correlation (no all-pairs volume).  Replaces raft_fs.CorrBlock
 * (src/models/impls/raft_fs.py:13-87; scale = 1) and, with levels = 1 and scale = 1/sqrt(C), the
 * window dot of corr/dot.py:25-57.  rmd_corr_otf_prepare writes the pixel-major query rows
 * (fmap1 * scale) and the avg-pooled target rows of every level into `workspace`
 * (rmd_corr_otf_workspace_bytes; compute RMD_BF16X3 = fp32-accurate split-bf16 MFMA, lo.hi + hi.lo +
 * hi.hi over operands stored as (hi, lo) bf16 pairs; RMD_F32 = exact f32 MFMA; RMD_BF16 = bf16 MFMA);
 * rmd_corr_otf_lookup then produces rmd_corr_lookup's output for `coords` from them each iteration.
 */
size_t rmd_corr_otf_workspace_bytes(int batch, int channels, int height, int width, int levels, int compute);
int rmd_corr_otf_prepare(const float* fmap1, const float* fmap2, int batch, int channels, int height, int width,
                         int levels, float scale, int compute, void* workspace, void* stream);
int rmd_corr_otf_lookup(const void* workspace, int batch, int channels, int height, int width, int levels,
                        int compute, const float* coords, int radius, unsigned zero_level_mask, float* out,
                        void* stream);

/*
 * Backward of the on-the-fly lookup (training at resolutions where the volume does not fit; autograd of
 * raft_fs.py:25-87 — grid_sample backward, the matmul with fmap1 and the avg-pool chain — without any
 * O(N^2) buffer).  After each lookup's forward, its backward records the lookup's per-query patch
 * weights: rmd_corr_otf_record turns grad_out (B, L*(2r+1)^2, H, W) and the lookup's coords into a
 * record of rmd_corr_otf_record_bytes() (per level and query: the window origin and the (2r+2)^2
 * bilinear patch weights of grad_out).  rmd_corr_otf_backward then computes, from all records of one
 * rmd_corr_otf_prepare (fmap1, fmap2, scale as given there, its workspace unchanged):
 *   grad_fmap1 = scale * sum_l G_l P_l,   grad_fmap2 = sum_l avgpool_l^T(G_l^T (scale * fmap1))
 * with G_l the sum of the records' level-l patch weights and P_l the level-l pooled fmap2; both
 * outputs are overwritten (B, C, H, W) float32.  C <= 256.  compute as in rmd_corr_otf_prepare
 * (RMD_F32 and RMD_BF16X3: split-bf16 products, fp32 accumulation; RMD_BF16: bf16 products).
 * Masked and 1-pixel levels and non-finite coordinates record no contribution.  `records` is a host
 * array of `nrecords` device pointers.  Deterministic: records are summed in a fixed order, and the
 * pooled gradient adds per-workgroup fp32 tile sums as 64-bit fixed point (integer atomics, associative,
 * so bitwise order-independent for any dynamic range) at a power-of-two scale chosen per call from the
 * largest recorded |weight| and |scale * fmap1| so that no sum can overflow; non-finite contributions
 * propagate through a float side buffer.  A record carries a 256-B header after its weights.
 */
size_t rmd_corr_otf_record_bytes(int batch, int height, int width, int levels, int radius);
int rmd_corr_otf_record(const float* grad_out, const float* coords, int batch, int height, int width, int levels,
                        int radius, unsigned zero_level_mask, void* record, void* stream);
size_t rmd_corr_otf_backward_workspace_bytes(int batch, int channels, int height, int width, int levels, int compute);
int rmd_corr_otf_backward(const float* fmap1, const float* fmap2, const void* otf_workspace, int batch, int channels,
                          int height, int width, int levels, float scale, int compute, int radius, int nrecords,
                          const void* const* records, float* grad_fmap1, float* grad_fmap2, void* workspace,
                          void* stream);

/* ---------------------------------------------------------------------------------------------
 * Backward of the RAFT correlation (training; autograd of raft.py:18-95).  Coordinates are
 * detached in the reference (raft.py:402), so only the feature maps receive gradients.
 *
 * Gradient of the pyramid, dense float32 "G", in the forward pyramid's chunked query-minor order
 * with 8-target chunks: target row (l, y) is cut into nch(l) = ceil(W_l/8) chunks, chunk
 * ch(l, y, x) = coff(l) + y*nch(l) + x/8 with coff(l) = sum_{l'<l} H_l'*nch(l'), TC chunks per image,
 * and element (b, target (l, y, x), query p) at ((b*TC + ch)*N + p)*8 + x%8.  Seen as a matrix over
 * the padded targets t' = 8*ch + x%8 (T' = 8*TC = rmd_corr_grad_targets(); pad targets x >= W_l stay
 * zero) G is (T' x N) stored in 8-row blocks.  With P = rmd_corr_pool_targets(fmap2, scale =
 * 1/sqrt(C)) as (B, C, T') in the same target order:
 *   grad_fmap1 (B, C, N) = P G     (rmd_corr_grad_gemm layout 3, lda = T', ldb = N)
 *   dP (B, C, T') = fmap1 G^T      (rmd_corr_grad_gemm layout 2, lda = N, ldb = N)
 *   grad_fmap2 = rmd_corr_unpool_targets(dP, scale = 1/sqrt(C)).
 * A wave of 64 consecutive queries whose (smooth) flow moves their windows one column per query
 * touches 3 128-B lines per 8 lanes at every tap (8 lines in a plain (B, T, N) order).
 */

/* Padded targets per image of G (T' = 8 * chunks over all levels), or -1 on bad sizes.  Host-only. */
long long rmd_corr_grad_targets(int height, int width, int levels);

/* grad_levels (G, caller-zeroed once per forward) += d(lookup)/d(pyramid)^T grad_out, where
 * grad_out is (B, L*(2r+1)^2, H, W) like rmd_corr_lookup's output.  Replaces the
 * grid_sampler_2d_backward of raft.py:80.  Zeroed levels (mask) and 1-pixel (NaN) levels add
 * nothing.  Deterministic (no atomics). */
int rmd_corr_lookup_backward(const float* grad_out, const rmd_pyramid_desc* desc, const float* coords,
                             int radius, unsigned zero_level_mask, float* grad_levels, void* stream);

/* G of ALL nlookups lookups of one forward in one pass: grad_levels = (accumulate ? G : 0)
 * + sum over i in order of lookup i's contribution (grad_outs[i], coords[i], zero_level_masks[i] —
 * each as in rmd_corr_lookup_backward; masks may be NULL), writing every element of G (no zero fill
 * needed).  Same arithmetic and summation order as the sequence of rmd_corr_lookup_backward calls
 * i = 0, 1, ... into a zeroed G.  grad_outs / coords / zero_level_masks are HOST arrays of device
 * pointers / values.  Replaces the per-lookup grid_sampler_2d_backward of raft.py:80 plus the
 * accumulation of those gradients into the correlation volume that autograd performs. */
int rmd_corr_grad_build(const float* const* grad_outs, const float* const* coords,
                        const unsigned* zero_level_masks, int nlookups, const rmd_pyramid_desc* desc, int radius,
                        int accumulate, float* grad_levels, void* stream);

/* rmd_corr_grad_build with bf16_out != 0: G stored as bfloat16 (round to nearest even of the fp32 sums,
 * the same element order, 2 bytes each) — what rmd_corr_grad_gemm_bf16g reads in the bf16 precision
 * mode, whose fp32-G GEMM rounds G to bfloat16 on load anyway (bit-identical results, half the G
 * traffic).  bf16_out requires accumulate == 0 and nlookups <= 16. */
int rmd_corr_grad_build_ex(const float* const* grad_outs, const float* const* coords,
                           const unsigned* zero_level_masks, int nlookups, const rmd_pyramid_desc* desc, int radius,
                           int accumulate, int bf16_out, void* grad_levels, void* stream);

/* pooled (B, C, T') = avg_pool_{2^l}(fmap2) * scale for every level, in G's padded target order (pad
 * targets 0) (raft.py:35-47 applied to the feature map, which commutes with the product). */
int rmd_corr_pool_targets(const float* fmap2, int batch, int channels, int height, int width, int levels,
                          float scale, float* pooled, void* stream);

/* grad_fmap2 (B, C, H, W) = scale * sum_l avg_pool_{2^l}^T(grad_pooled level l)  (avg_pool2d_backward);
 * grad_pooled is (B, C, T') in G's padded target order. */
int rmd_corr_unpool_targets(const float* grad_pooled, int batch, int channels, int height, int width, int levels,
                            float scale, float* grad_fmap2, void* stream);

/* The two GEMMs of the backward (autograd of the matmul at raft.py:31-33), batched over `batch`;
 * compute RMD_BF16X3: fp32-accurate from three split-bf16 MFMA products (hi.hi + hi.lo + lo.hi, the fp32
 * precision modes); RMD_BF16: one bf16 product per k-step, fp32 accumulation (the bf16 mode):
 *   out[b] (m x nc, row-major) = a[b] (m x k, row stride lda) . B[b]
 *   layout 0: B element (k, n) at bm[k*ldb + n]                 (k x nc, ldb >= nc)
 *   layout 1: B element (k, n) at bm[n*ldb + k]                 (nc x k, ldb >= k)
 *   layout 2: B element (k, n) at bm[((n/8)*ldb + k)*8 + n%8]   (ldb >= k)  -> dP = fmap1 G^T
 *   layout 3: B element (k, n) at bm[((k/8)*ldb + n)*8 + k%8]   (ldb >= nc) -> grad_fmap1 = P G
 * Batch strides are m*lda for a and k*ldb, nc*ldb, ceil(nc/8)*8*ldb, ceil(k/8)*8*ldb for bm
 * (layouts 0-3); out is contiguous.  K may be
 * split over workgroups: then `workspace` must hold rmd_corr_grad_gemm_workspace_bytes() bytes
 * (0 = none needed) and a second pass sums the partial tiles in a fixed order (deterministic). */
size_t rmd_corr_grad_gemm_workspace_bytes(int batch, int m, int k, int nc);
int rmd_corr_grad_gemm(const float* a, long long lda, const float* bm, long long ldb, int batch, int m, int k, int nc,
                       int layout, int compute, float* out, void* workspace, void* stream);

/* rmd_corr_grad_gemm with compute RMD_BF16 and a bfloat16 B (layouts 2 / 3: G from
 * rmd_corr_grad_build_ex with bf16_out): the fp32-B GEMM rounds B to bfloat16 on load, so the result
 * is bit-identical to rmd_corr_grad_gemm(..., RMD_BF16, ...) on the fp32 G; B's base 8-byte aligned
 * for vector loads.  Same workspace as rmd_corr_grad_gemm_workspace_bytes. */
int rmd_corr_grad_gemm_bf16g(const float* a, long long lda, const void* bm, long long ldb, int batch, int m, int k,
                             int nc, int layout, float* out, void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------------
 * DICL cost volumes.  Shapes: fmap1 (B, C, h, w); fmap2 (B, C, hl, wl); coords (B, 2, h, w);
 * stack (B, d, d, 2C [+2], h, w) float32 contiguous with d = 2r+1, dim 1 the x-offset a-r and
 * dim 2 the y-offset b-r — exactly the MatchingNet input (blocks/dicl.py:111-118).  h*w must be a
 * multiple of 4 (MatchingNet already needs even h and w).
 */

/*
 * Displacement stack with bilinear sampling.  Replaces the grid_sample/expand/cat of
 * corr.dicl.CorrelationModule.forward (src/models/common/corr/dicl.py:26-54; dicl_1x1.py:51-79),
 * of dicl_emb.py:51-89 (extra_delta = 1 appends the (a-r, b-r) channels) and the per-level gather
 * of raft_dicl_ml.CorrelationModule.forward (src/models/impls/raft_dicl_ml.py:294-315):
 *   stack[b,a,bb,0:C]  = fmap1
 *   stack[b,a,bb,C:2C] = bilinear(fmap2, ((x/2^level + a-r) * (wl-1)/(norm_w-1),
 *                                        (y/2^level + bb-r) * (hl-1)/(norm_h-1)))
 * zero padding per tap.  corr/dicl.py: level 0, norm = (h, w) = (hl, wl); raft_dicl_ml level i:
 * norm = fmap1's (h, w) (the reference normalises with the full-resolution size, :300-305).
 */
int rmd_dicl_stack(const float* fmap1, const float* fmap2, const float* coords, int batch, int channels,
                   int height, int width, int level_height, int level_width, int radius, int level,
                   int norm_height, int norm_width, int extra_delta, float* out, void* stream);

/* Gradients of rmd_dicl_stack: grad_fmap1 = sum over displacements of the first C channels
 * (deterministic); grad_fmap2 = bilinear scatter of channels C..2C-1 (float atomics, as ATen's
 * grid_sampler_2d_backward).  Coordinates carry no gradient (they are detached, raft.py:402). */
int rmd_dicl_stack_backward(const float* grad_stack, const float* coords, int batch, int channels,
                            int height, int width, int level_height, int level_width, int radius,
                            int level, int norm_height, int norm_width, int extra_delta,
                            float* grad_fmap1, float* grad_fmap2, void* stream);

/* Bytes of device workspace rmd_dicl_stack_int(_backward) needs (occlusion mask, 1 B/pixel). */
size_t rmd_dicl_stack_int_workspace_bytes(int batch, int height, int width);

/*
 * DICL baseline integer matching volume with occlusion mask.  Replaces
 * FlowLevel.compute_cost's volume build (src/models/impls/dicl.py:212-238): for di = i-ru (x),
 * dj = j-rv (y), both halves are copied where (x+di, y+dj) is inside and zero elsewhere, then the
 * whole 2C vector is zeroed where sum_c of its f2 half == 0.  out (B, 2ru+1, 2rv+1, 2C, h, w).
 */
int rmd_dicl_stack_int(const float* fmap1, const float* fmap2, int batch, int channels, int height, int width,
                       int ru, int rv, float* out, void* workspace, void* stream);

/* Gradients of rmd_dicl_stack_int (the mask is detached, dicl.py:236): deterministic gathers. */
int rmd_dicl_stack_int_backward(const float* grad_mvol, const float* fmap2, int batch, int channels,
                                int height, int width, int ru, int rv, float* grad_fmap1,
                                float* grad_fmap2, void* workspace, void* stream);

/*
 * Backward warping.  Replaces common.warp.warp_backwards (src/models/common/warp.py:5-33):
 *   out[b,c,y,x] = mask * bilinear(img2[b,c], x + flow[b,0,y,x], y + flow[b,1,y,x])   (zero padding,
 *   align_corners=True), mask = (in-bounds bilinear weight > 1 - eps) (grid_sample of ones, :28-30).
 * img2, out (B, C, h, w); flow (B, 2, h, w); mask (B, h, w) uint8 or NULL (the reference's bool mask is
 * this plane broadcast over C).  The flow carries no gradient (dicl.py:178 detaches it).
 */
int rmd_warp_backwards(const float* img2, const float* flow, int batch, int channels, int height, int width,
                       float eps, float* out, unsigned char* mask, void* stream);

/* d img2 (B, C, h, w) = bilinear^T(mask * grad_out); zeroes grad_img2 first (float atomics, like ATen). */
int rmd_warp_backwards_backward(const float* grad_out, const float* flow, int batch, int channels, int height,
                                int width, float eps, float* grad_img2, void* stream);

/* Bytes of device workspace rmd_dicl_stack_int_warped(_backward) needs (warped map + flags). */
size_t rmd_dicl_stack_int_warped_workspace_bytes(int batch, int channels, int height, int width);

/*
 * FlowLevel with a coarse flow (src/models/impls/dicl.py:171-238): feat2 is warped back by `flow`
 * (warp_backwards, eps 1e-5) and the masked integer volume of rmd_dicl_stack_int is built on it.  The
 * warp runs inside the occlusion-flag pass, so the volume costs the same launches as without warping.
 */
int rmd_dicl_stack_int_warped(const float* fmap1, const float* fmap2, const float* flow, int batch, int channels,
                              int height, int width, int ru, int rv, float* out, void* workspace, void* stream);

/* Gradients of rmd_dicl_stack_int_warped w.r.t. fmap1 and fmap2 (flow and masks detached). */
int rmd_dicl_stack_int_warped_backward(const float* grad_mvol, const float* fmap2, const float* flow, int batch,
                                       int channels, int height, int width, int ru, int rv, float* grad_fmap1,
                                       float* grad_fmap2, void* workspace, void* stream);

/*
 * Displacement-aware projection: out[b,o,p] = sum_i W[o,i] x[b,i,p] (1x1 conv, no bias) with
 * W = conv1.weight[:,:,0,0] (D x D).  Replaces DisplacementAwareProjection.forward
 * (src/models/common/blocks/dicl.py:143-150), the per-level DAPs of raft.py:146-168 and the
 * 324x324 'full' DAP of raft_dicl_ml.py:268-273,339-341.  transpose = 1 applies W^T (the input
 * gradient).  x, out: (B, D, pixels) float32.  Computed as a split-bf16 MFMA GEMM (W and x split
 * into hi + lo bf16, W_lo.x_hi + W_hi.x_lo + W_hi.x_hi accumulated in fp32: ~1.5e-5 of float64)
 * for D <= 1024; larger D falls back to an exact-fp32 VALU kernel.
 */
int rmd_dap(const float* x, const float* weight, int batch, int disp, int pixels, int transpose, float* out,
            void* stream);

/* Weight gradient of rmd_dap (autograd of the 1x1 conv weight, blocks/dicl.py:137,147):
 *   grad_weight[o][i] = sum_b sum_p grad_out[b, o, p] x[b, i, p]      (D x D, overwritten)
 * split-bf16 MFMA (lo.hi + hi.lo + hi.hi, fp32 accumulation), the batch x pixel sum split over
 * workgroups into `workspace` (rmd_dap_weight_grad_workspace_bytes) and summed in a fixed order
 * (deterministic). */
size_t rmd_dap_weight_grad_workspace_bytes(int batch, int disp, int pixels);
int rmd_dap_weight_grad(const float* grad_out, const float* x, int batch, int disp, int pixels, float* grad_weight,
                        void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Per-iteration flow heads on either side of the lookup.
 */

/*
 * Convex 8x upsampling.  Replaces the tail of Up8Network.forward (src/models/impls/raft.py:319-331)
 * after its two convolutions: mask (B, 576, h, w) logits with channel = k*64 + i*8 + j (neighbour
 * k = 3*ky + kx, sub-pixel (i, j)), flow (B, 2, h, w) ->
 *   out[b, c, 8y+i, 8x+j] = sum_k softmax_k(mask[b, k*64+i*8+j, y, x] / temperature) * 8*flow[b, c, y+ky-1, x+kx-1]
 * (zero outside the map; F.unfold(8*flow, 3, padding=1)).  out (B, 2, 8h, 8w) float32.
 */
int rmd_up8(const float* mask, const float* flow, int batch, int height, int width, float temperature,
            float* out, void* stream);

/* Bytes of device workspace rmd_up8_backward needs (per-pixel neighbour sums, 72 B/pixel). */
size_t rmd_up8_workspace_bytes(int batch, int height, int width);

/* Gradients of rmd_up8 w.r.t. mask (B, 576, h, w) and flow (B, 2, h, w); deterministic (no atomics). */
int rmd_up8_backward(const float* mask, const float* flow, const float* grad_out, int batch, int height, int width,
                     float temperature, float* grad_mask, float* grad_flow, void* workspace, void* stream);

/*
 * Soft-argmax flow regression.  Replaces raft.SoftArgMaxFlowRegression.forward (raft.py:112-135;
 * levels = L, level l scaled by 2^l) and the single-level SoftArgMaxFlowRegression of
 * corr/dicl.py:64-85, corr/dot.py:69-90, dicl_1x1.py:89-110, dicl_emb.py:107-134 (levels = 1):
 *   p_k = softmax_k(cost[b, l*(2r+1)^2 + k, :] / temperature),  k = a*(2r+1) + bb,
 *   flows[l, b, 0] = 2^l * sum_k p_k (a - r),  flows[l, b, 1] = 2^l * sum_k p_k (bb - r).
 * cost (B, cost_channels, pixels) float32 with cost_channels >= L*(2r+1)^2 (extra trailing channels
 * are ignored: dicl_emb regresses on the first (2r+1)^2 of its embedding); flows (L, B, 2, pixels).
 * radius 1..4.  The *WithDap variants run rmd_dap on each level first (raft.py:139-181).
 */
int rmd_softargmax(const float* cost, int batch, int cost_channels, int pixels, int levels, int radius,
                   float temperature, float* flows, void* stream);

/* d cost for channels [0, L*(2r+1)^2) of each batch row (others untouched) from grad_flows (L, B, 2, pixels). */
int rmd_softargmax_backward(const float* cost, const float* grad_flows, int batch, int cost_channels, int pixels,
                            int levels, int radius, float temperature, float* grad_cost, void* stream);

/*
 * Input format (src/models/input.py).  rmd_input_images replaces Input.__getitem__'s clip and range
 * map (input.py:215-221), ModuloPadding.apply (input.py:79-138) and TorchAdapter's permute to NCHW
 * (input.py:280-281) for one image tensor of a pair:
 *   out[b, k, y, x] = (range_max - range_min) * clip(img[b, sy, sx, k], clip_min, clip_max) + range_min
 * with (sy, sx) = (y - pad_top, x - pad_left) mapped into the image by the pad mode, or the constant
 * 0 / 1 for RMD_PAD_ZEROS / RMD_PAD_ONES outside it.  img (B, H, W, C) float32 NHWC, out (B, C, H', W').
 * Modes: numpy 'edge' == torch 'replicate' (EDGE), numpy/torch 'reflect' (REFLECT), numpy 'symmetric',
 * numpy 'wrap' == torch 'circular' (WRAP).  The statistic modes (maximum, mean, median, minimum) are
 * not provided (no config uses them; every cfg pads with zeros).
 * rmd_input_flow replaces the flow / valid side (input.py:120-122, 301-313): flow (B, H, W, 2) float32,
 * valid (B, H, W) bytes -> flow_out (B, 2, H', W') with NaN -> 0 and values clipped to +-flow_inf,
 * valid_out (B, H', W') bytes; padding is zero flow / invalid.
 */
#define RMD_PAD_ZEROS 0
#define RMD_PAD_ONES 1
#define RMD_PAD_EDGE 2
#define RMD_PAD_REFLECT 3
#define RMD_PAD_SYMMETRIC 4
#define RMD_PAD_WRAP 5

int rmd_input_images(const float* img, int batch, int height, int width, int channels, float clip_min,
                     float clip_max, float range_min, float range_max, int padded_height, int padded_width,
                     int pad_top, int pad_left, int mode, float* out, void* stream);

int rmd_input_flow(const float* flow, const unsigned char* valid, int batch, int height, int width,
                   int padded_height, int padded_width, int pad_top, int pad_left, float flow_inf, float* flow_out,
                   unsigned char* valid_out, void* stream);

/* Message for the last failing call on this thread ("" if none). */
const char* rmd_last_error(void);

/* Library version string, e.g. "rmd 0.2 gfx950 abi 2". */
const char* rmd_version(void);

/* ABI revision of the exported signatures.  A binding checks it against the RMD_ABI_VERSION of the
 * header it was written for and refuses a mismatch (rmd/_lib.py does).  History:
 *   1  rounds 1-4
 *   2  rmd_corr_grad_gemm gained `compute` (RMD_BF16X3 / RMD_BF16) before `out` (round 5) */
#define RMD_ABI_VERSION 2
int rmd_abi_version(void);

/* Fingerprint of the sources this library was built from (16 hex digits of the sha256 of
 * raft-meets-dicl_amd/csrc/{*.cpp,*.h,*.hip} in name order followed by this header; the Makefile
 * computes it).  Not part of the reference interface: it lets a binding or a test tell a library
 * rebuilt from the tree it sits in from a stale one.  Additive, so the ABI revision stays 2. */
const char* rmd_source_hash(void);

#ifdef __cplusplus
}
#endif

#endif /* RMD_H */
