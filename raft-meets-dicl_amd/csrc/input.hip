// input.hip — the evaluation/training input format on the GPU: clip + range map + modulo padding +
// NHWC -> NCHW of a frame pair, and the padded flow / validity targets.
//
// Replaces (qzed/raft-meets-dicl v2, src/models/input.py):
//  * Input.__getitem__ clip and range map           input.py:215-221
//  * ModuloPadding.apply (numpy / torch pad modes)   input.py:79-138
//  * TorchAdapter.__getitem__ permute to NCHW, flow   input.py:245-313 (nan_to_num, clip to +-1e10)
// -> rmd_input_images, rmd_input_flow
//
// Both are byte movers (one read + one write per element): one lane per output pixel of a
// (b, padded row) strip, so every channel plane store is a coalesced 256-B wave row and the
// 12-B (RGB) / 8-B (flow) source pixels of a wave are one contiguous run.

#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 256;

// source index along one axis for an output coordinate o in the padded extent: pad0 elements
// before the data of length n.  Returns -1 for a constant-mode (zeros / ones) pad position.
__device__ __forceinline__ int src_index(int o, int pad0, int n, int mode) {
    int i = o - pad0;
    if (i >= 0 && i < n) return i;
    switch (mode) {
        case RMD_PAD_EDGE:                  // numpy 'edge' == torch 'replicate'
            return i < 0 ? 0 : n - 1;
        case RMD_PAD_REFLECT: {             // numpy 'reflect' == torch 'reflect' (edge not repeated)
            if (n == 1) return 0;
            const int period = 2 * (n - 1);
            int m = i % period;
            if (m < 0) m += period;
            return m < n ? m : period - m;
        }
        case RMD_PAD_SYMMETRIC: {           // numpy 'symmetric' (edge repeated)
            const int period = 2 * n;
            int m = i % period;
            if (m < 0) m += period;
            return m < n ? m : period - 1 - m;
        }
        case RMD_PAD_WRAP: {                // numpy 'wrap' == torch 'circular'
            int m = i % n;
            return m < 0 ? m + n : m;
        }
        default:
            return -1;
    }
}

// grid: (ceil(W'/256), H', B)
__global__ void __launch_bounds__(kThreads)
input_images_kernel(const float* __restrict__ img, int h, int w, int c, int hp, int wp, int ph0, int pw0, int mode,
                    float cmin, float cmax, float scale, float offset, float fill, float* __restrict__ out) {
    const int x = blockIdx.x * kThreads + threadIdx.x;
    const int y = blockIdx.y, b = blockIdx.z;
    if (x >= wp) return;
    const int sy = src_index(y, ph0, h, mode), sx = src_index(x, pw0, w, mode);
    const size_t plane = (size_t)hp * wp;
    float* o = out + (size_t)b * c * plane + (size_t)y * wp + x;
    if (sy < 0 || sx < 0) {
        for (int k = 0; k < c; ++k) o[(size_t)k * plane] = fill;
        return;
    }
    const float* s = img + (((size_t)b * h + sy) * w + sx) * c;
    for (int k = 0; k < c; ++k) {
        // (max - min) * clip(v, lo, hi) + min, as input.py:220-221 (np.clip, then one multiply-add)
        const float sv = s[k];
        const float v = sv < cmin ? cmin : (sv > cmax ? cmax : sv);     // NaN passes through, as np.clip
        o[(size_t)k * plane] = __fadd_rn(__fmul_rn(scale, v), offset);     // two roundings, as numpy
    }
}

// grid: (ceil(W'/256), H', B).  flow NHWC (B,h,w,2) -> (B,2,h',w'); valid (B,h,w) bytes -> (B,h',w')
__global__ void __launch_bounds__(kThreads)
input_flow_kernel(const float* __restrict__ flow, const unsigned char* __restrict__ valid, int h, int w, int hp,
                  int wp, int ph0, int pw0, float flow_inf, float* __restrict__ fout, unsigned char* __restrict__ vout) {
    const int x = blockIdx.x * kThreads + threadIdx.x;
    const int y = blockIdx.y, b = blockIdx.z;
    if (x >= wp) return;
    const int sy = y - ph0, sx = x - pw0;
    const bool in = sy >= 0 && sy < h && sx >= 0 && sx < w;
    const size_t plane = (size_t)hp * wp, q = (size_t)y * wp + x;
    float u = 0.f, v = 0.f;
    unsigned char ok = 0;
    if (in) {
        const size_t si = ((size_t)b * h + sy) * w + sx;
        u = flow[2 * si];
        v = flow[2 * si + 1];
        ok = valid[si] != 0;
        // np.nan_to_num(nan=0, posinf=+inf_value, neginf=-inf_value), then np.clip to +-inf_value
        u = isnan(u) ? 0.f : fminf(fmaxf(u, -flow_inf), flow_inf);
        v = isnan(v) ? 0.f : fminf(fmaxf(v, -flow_inf), flow_inf);
    }
    fout[(size_t)b * 2 * plane + q] = u;
    fout[(size_t)b * 2 * plane + plane + q] = v;
    vout[(size_t)b * plane + q] = ok;
}

}  // namespace
}  // namespace rmd

using namespace rmd;

extern "C" int rmd_input_images(const float* img, int batch, int height, int width, int channels, float clip_min,
                                float clip_max, float range_min, float range_max, int padded_height,
                                int padded_width, int pad_top, int pad_left, int mode, float* out, void* stream) {
    RMD_REQUIRE(img && out, RMD_ERR_ARG, "rmd_input_images: null pointer");
    RMD_REQUIRE(batch > 0 && batch <= 65535 && height > 0 && width > 0 && channels > 0, RMD_ERR_SHAPE,
                "rmd_input_images: bad sizes");
    RMD_REQUIRE(padded_height >= height && padded_width >= width && padded_height <= 65535 && pad_top >= 0 &&
                pad_left >= 0 && pad_top <= padded_height - height && pad_left <= padded_width - width,
                RMD_ERR_SHAPE, "rmd_input_images: bad padding");
    RMD_REQUIRE(mode >= RMD_PAD_ZEROS && mode <= RMD_PAD_WRAP, RMD_ERR_ARG, "rmd_input_images: bad pad mode %d", mode);
    const float scale = range_max - range_min;
    const float fill = mode == RMD_PAD_ONES ? 1.0f : 0.0f;
    dim3 grid((padded_width + kThreads - 1) / kThreads, padded_height, batch);
    input_images_kernel<<<grid, kThreads, 0, as_stream(stream)>>>(img, height, width, channels, padded_height,
                                                                  padded_width, pad_top, pad_left, mode, clip_min,
                                                                  clip_max, scale, range_min, fill, out);
    return check_launch("rmd_input_images");
}

extern "C" int rmd_input_flow(const float* flow, const unsigned char* valid, int batch, int height, int width,
                              int padded_height, int padded_width, int pad_top, int pad_left, float flow_inf,
                              float* flow_out, unsigned char* valid_out, void* stream) {
    RMD_REQUIRE(flow && valid && flow_out && valid_out, RMD_ERR_ARG, "rmd_input_flow: null pointer");
    RMD_REQUIRE(batch > 0 && batch <= 65535 && height > 0 && width > 0, RMD_ERR_SHAPE, "rmd_input_flow: bad sizes");
    RMD_REQUIRE(padded_height >= height && padded_width >= width && padded_height <= 65535 && pad_top >= 0 &&
                pad_left >= 0 && pad_top <= padded_height - height && pad_left <= padded_width - width,
                RMD_ERR_SHAPE, "rmd_input_flow: bad padding");
    dim3 grid((padded_width + kThreads - 1) / kThreads, padded_height, batch);
    input_flow_kernel<<<grid, kThreads, 0, as_stream(stream)>>>(flow, valid, height, width, padded_height,
                                                                padded_width, pad_top, pad_left, flow_inf, flow_out,
                                                                valid_out);
    return check_launch("rmd_input_flow");
}
