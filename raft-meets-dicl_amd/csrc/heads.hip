// heads.hip — per-GRU-iteration flow heads that sit on both sides of the cost-volume lookup.
//
// * Convex 8x upsampling, the tail of Up8Network.forward (qzed/raft-meets-dicl
//   src/models/impls/raft.py:313-331): softmax over the 9 neighbour logits of each of the 64
//   sub-pixels, weighted sum of the 3x3 neighbourhood of 8*flow (F.unfold, zero padding).
// * Soft-argmax flow regression (raft.py:98-181, corr/dicl.py:64-110, corr/dot.py:69-120 and the
//   identical classes of dicl_1x1.py / dicl_emb.py): softmax over the (2r+1)^2 costs of a level,
//   expectation of the displacement (dx, dy) * 2^level.
//
// Both are HBM-bound elementwise reductions: 2.3 KB of mask logits per low-res
// pixel for Up8, 324 B of costs per pixel-level for soft-argmax.  Layouts are the reference's
// channel-major tensors; a wave covers 64 consecutive pixels so every per-channel load is one
// coalesced 256 B row, and the Up8 output row segment of a pixel (8 floats) is written as two
// float4 stores, i.e. 64 lanes write 2 KB of one output row contiguously.

#include "rmd_common.h"

namespace rmd {
namespace {

constexpr int kThreads = 256;

// ---- Up8 convex upsampling -----------------------------------------------------------------------

// u[c][k] = 8 * flow[c, y+ky-1, x+kx-1] (zero outside), k = 3*ky + kx (F.unfold order, raft.py:324)
__device__ __forceinline__ void up8_neighbours(const float* __restrict__ flow, int b, int y, int x, int h, int w,
                                               float (&u)[2][9]) {
    const size_t n = (size_t)h * w;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int yy = y + ky - 1, xx = x + kx - 1;
            const bool in = yy >= 0 && yy < h && xx >= 0 && xx < w;
            const size_t at = in ? (size_t)yy * w + xx : 0;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const float v = flow[((size_t)b * 2 + c) * n + at];
                u[c][3 * ky + kx] = in ? 8.0f * v : 0.0f;
            }
        }
    }
}

// softmax over the 9 neighbours of (logit / temperature), as torch.softmax(mask / T, dim=2); returns
// the index of the (first) largest logit, around which the backward pass centres its differences
__device__ __forceinline__ int softmax9(float (&m)[9], float temperature) {
    float mx = -INFINITY;
    int am = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        m[k] = m[k] / temperature;
        if (m[k] > mx) {
            mx = m[k];
            am = k;
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        m[k] = expf(m[k] - mx);
        s += m[k];
    }
    const float inv = 1.0f / s;
#pragma unroll
    for (int k = 0; k < 9; ++k) m[k] *= inv;
    return am;
}

// grid (ceil(N/256), 8 sub-rows, B): one lane per (low-res pixel, sub-row i), all 8 sub-columns
__global__ void __launch_bounds__(kThreads) up8_kernel(const float* __restrict__ mask, const float* __restrict__ flow,
                                                       int h, int w, float temperature, float* __restrict__ out) {
    const int n = h * w;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int i = blockIdx.y, b = blockIdx.z;
    if (p >= n) return;
    const int y = p / w, x = p - y * w;
    float u[2][9];
    up8_neighbours(flow, b, y, x, h, w, u);
    const float* mb = mask + (size_t)b * 576 * n + (size_t)(i * 8) * n + p;
    float r0[8], r1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float m[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = __builtin_nontemporal_load(mb + ((size_t)k * 64 + j) * n);
        softmax9(m, temperature);
        float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            a0 = fmaf(m[k], u[0][k], a0);
            a1 = fmaf(m[k], u[1][k], a1);
        }
        r0[j] = a0;
        r1[j] = a1;
    }
    const size_t W8 = (size_t)8 * w;
    const size_t row = (size_t)(8 * y + i) * W8 + 8 * x;
    // the upsampled flow is written once per iteration: non-temporal stores keep it out of the way
    // of the mask/flow lines neighbouring lanes re-read
    typedef __attribute__((ext_vector_type(4))) float v4;
    v4* o0 = reinterpret_cast<v4*>(out + ((size_t)b * 2 + 0) * 64 * n + row);
    v4* o1 = reinterpret_cast<v4*>(out + ((size_t)b * 2 + 1) * 64 * n + row);
    __builtin_nontemporal_store(v4{r0[0], r0[1], r0[2], r0[3]}, o0);
    __builtin_nontemporal_store(v4{r0[4], r0[5], r0[6], r0[7]}, o0 + 1);
    __builtin_nontemporal_store(v4{r1[0], r1[1], r1[2], r1[3]}, o1);
    __builtin_nontemporal_store(v4{r1[4], r1[5], r1[6], r1[7]}, o1 + 1);
}

// Backward, pass 1.  Block (64 pixels, 8 sub-rows), grid (ceil(N/64), B).  Writes d mask and the
// per-pixel neighbour sums q[b][c][k][p] = sum_{i,j} softmax_k(i,j) * grad_out[c](i,j) (summed over
// the block's sub-rows in LDS, deterministic) for pass 2.
constexpr int kUpPix = 64;

__global__ void __launch_bounds__(kUpPix * 8) up8_backward_mask_kernel(
    const float* __restrict__ mask, const float* __restrict__ flow, const float* __restrict__ grad_out, int h, int w,
    float temperature, float* __restrict__ grad_mask, float* __restrict__ q) {
    __shared__ float red[8][18][kUpPix];
    const int n = h * w;
    const int lane = threadIdx.x, i = threadIdx.y, b = blockIdx.y;
    const int p = blockIdx.x * kUpPix + lane;
    const bool active = p < n;
    float acc[2][9];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[c][k] = 0.0f;
    if (active) {
        const int y = p / w, x = p - y * w;
        float u[2][9];
        up8_neighbours(flow, b, y, x, h, w, u);
        const size_t W8 = (size_t)8 * w;
        const size_t row = (size_t)(8 * y + i) * W8 + 8 * x;
        float g[2][8];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float4* gp = reinterpret_cast<const float4*>(grad_out + ((size_t)b * 2 + c) * 64 * n + row);
            const float4 g0 = gp[0], g1 = gp[1];
            g[c][0] = g0.x; g[c][1] = g0.y; g[c][2] = g0.z; g[c][3] = g0.w;
            g[c][4] = g1.x; g[c][5] = g1.y; g[c][6] = g1.z; g[c][7] = g1.w;
        }
        const size_t base = (size_t)b * 576 * n + (size_t)(i * 8) * n + p;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float m[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) m[k] = mask[base + ((size_t)k * 64 + j) * n];
            const int am = softmax9(m, temperature);
            // d logit_k = p_k (g_k - sum_j p_j g_j) / T, with the bracket evaluated as
            // (g_k - g_am) - sum_j p_j (g_j - g_am): no cancellation when one neighbour dominates
            float gk[9], gam = 0.0f;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                gk[k] = fmaf(g[0][j], u[0][k], g[1][j] * u[1][k]);
                gam = am == k ? gk[k] : gam;
                acc[0][k] = fmaf(m[k], g[0][j], acc[0][k]);
                acc[1][k] = fmaf(m[k], g[1][j], acc[1][k]);
            }
            float corr = 0.0f;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                gk[k] -= gam;
                corr = fmaf(m[k], gk[k], corr);
            }
#pragma unroll
            for (int k = 0; k < 9; ++k)
                grad_mask[base + ((size_t)k * 64 + j) * n] = m[k] * (gk[k] - corr) / temperature;
        }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int k = 0; k < 9; ++k) red[i][c * 9 + k][lane] = acc[c][k];
    __syncthreads();
    // 18 sums x 64 pixels over the 8 sub-rows; 512 threads, fixed order
    for (int t = i * kUpPix + lane; t < 18 * kUpPix; t += 8 * kUpPix) {
        const int ck = t / kUpPix, l = t - ck * kUpPix;
        float s = 0.0f;
#pragma unroll
        for (int r = 0; r < 8; ++r) s += red[r][ck][l];
        const int pp = blockIdx.x * kUpPix + l;
        if (pp < n) q[((size_t)b * 18 + ck) * n + pp] = s;
    }
}

// Backward, pass 2: d flow[b,c,Y,X] = 8 * sum_k q[b,c,k](Y+1-ky, X+1-kx) — the transpose of F.unfold.
__global__ void __launch_bounds__(kThreads) up8_backward_flow_kernel(const float* __restrict__ q, int h, int w,
                                                                     float* __restrict__ grad_flow) {
    const int n = h * w;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int c = blockIdx.y, b = blockIdx.z;
    if (p >= n) return;
    const int Y = p / w, X = p - Y * w;
    const float* qb = q + ((size_t)b * 18 + c * 9) * n;
    float s = 0.0f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int y = Y + 1 - ky, x = X + 1 - kx;
            if (y >= 0 && y < h && x >= 0 && x < w) s += qb[(size_t)(3 * ky + kx) * n + (size_t)y * w + x];
        }
    }
    grad_flow[((size_t)b * 2 + c) * n + p] = 8.0f * s;
}

// ---- soft-argmax regression ----------------------------------------------------------------------

// Displacement k = a*(2r+1) + bb has (dx, dy) = (a - r, bb - r): meshgrid(dx, dy, indexing='ij'), raft.py:106-109.
// One lane per (pixel, level); grid (ceil(N/256), B, L).  Costs are read from channel
// level*(2r+1)^2 + k of a (B, cost_channels, N) tensor (cost_channels >= L*(2r+1)^2: dicl_emb
// regresses on the first (2r+1)^2 channels of a wider embedding).  For r <= 4 the costs stay in
// registers between the max and exp passes; larger windows re-read them (L1/L2 hits).
template <int R>
__device__ __forceinline__ int softargmax_probs(const float* __restrict__ c, size_t n, float temperature,
                                                float (&v)[(2 * R + 1) * (2 * R + 1)], float& inv_sum) {
    constexpr int D = (2 * R + 1) * (2 * R + 1);
    float mx = -INFINITY;
    int am = 0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        v[k] = c[k * n] / temperature;
        if (v[k] > mx) {
            mx = v[k];
            am = k;
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        v[k] = expf(v[k] - mx);
        s += v[k];
    }
    inv_sum = 1.0f / s;
    return am;
}

template <int R>
__global__ void __launch_bounds__(kThreads) softargmax_kernel(const float* __restrict__ cost, int cost_channels, int n,
                                                              float temperature, float* __restrict__ flows) {
    constexpr int D2 = 2 * R + 1, D = D2 * D2;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y, l = blockIdx.z;
    if (p >= n) return;
    const float* c = cost + ((size_t)b * cost_channels + (size_t)l * D) * n + p;
    float v[D], inv;
    softargmax_probs<R>(c, n, temperature, v, inv);
    float fx = 0.0f, fy = 0.0f;
#pragma unroll
    for (int a = 0; a < D2; ++a) {
#pragma unroll
        for (int bb = 0; bb < D2; ++bb) {
            const float pk = v[a * D2 + bb] * inv;
            fx = fmaf(pk, (float)(a - R), fx);
            fy = fmaf(pk, (float)(bb - R), fy);
        }
    }
    const float s = (float)(1 << l);
    float* o = flows + (((size_t)l * gridDim.y + b) * 2) * n + p;
    o[0] = fx * s;
    o[n] = fy * s;
}

// d cost_k = p_k * s * (gx (dx_k - E[dx]) + gy (dy_k - E[dy])) / T.  The centred displacements are
// evaluated around the argmax m as (dx_k - dx_m) - sum_j p_j (dx_j - dx_m), which keeps full relative
// accuracy when the softmax is peaked (computing E[dx] first would cancel against dx_m).
template <int R>
__global__ void __launch_bounds__(kThreads) softargmax_backward_kernel(const float* __restrict__ cost,
                                                                       int cost_channels, int n, float temperature,
                                                                       const float* __restrict__ grad_flows,
                                                                       float* __restrict__ grad_cost) {
    constexpr int D2 = 2 * R + 1, D = D2 * D2;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    const int b = blockIdx.y, l = blockIdx.z;
    if (p >= n) return;
    const size_t off = ((size_t)b * cost_channels + (size_t)l * D) * n + p;
    float v[D], inv;
    const int am = softargmax_probs<R>(cost + off, n, temperature, v, inv);
    const int ma = am / D2, mb = am - ma * D2;
    const float s = (float)(1 << l);
    const float* g = grad_flows + (((size_t)l * gridDim.y + b) * 2) * n + p;
    const float gx = g[0] * s / temperature, gy = g[n] * s / temperature;
    float rx = 0.0f, ry = 0.0f;
#pragma unroll
    for (int a = 0; a < D2; ++a)
#pragma unroll
        for (int bb = 0; bb < D2; ++bb) {
            v[a * D2 + bb] *= inv;
            rx = fmaf(v[a * D2 + bb], (float)(a - ma), rx);
            ry = fmaf(v[a * D2 + bb], (float)(bb - mb), ry);
        }
    float* gc = grad_cost + off;
#pragma unroll
    for (int a = 0; a < D2; ++a)
#pragma unroll
        for (int bb = 0; bb < D2; ++bb) {
            const float cx = (float)(a - ma) - rx, cy = (float)(bb - mb) - ry;
            gc[(size_t)(a * D2 + bb) * n] = v[a * D2 + bb] * fmaf(gx, cx, gy * cy);
        }
}

}  // namespace
}  // namespace rmd

using namespace rmd;

extern "C" int rmd_up8(const float* mask, const float* flow, int batch, int height, int width, float temperature,
                       float* out, void* stream) {
    RMD_REQUIRE(mask && flow && out, RMD_ERR_ARG, "rmd_up8: null pointer");
    RMD_REQUIRE(batch >= 1 && height >= 1 && width >= 1 && batch <= 65535, RMD_ERR_SHAPE,
                "rmd_up8: bad sizes (batch=%d height=%d width=%d)", batch, height, width);
    RMD_REQUIRE((long long)batch * 576 * height * width < (1ll << 40), RMD_ERR_SHAPE, "rmd_up8: too large");
    RMD_REQUIRE(temperature > 0.0f, RMD_ERR_ARG, "rmd_up8: temperature must be > 0");
    const int n = height * width;
    dim3 grid((n + kThreads - 1) / kThreads, 8, batch);
    up8_kernel<<<grid, kThreads, 0, as_stream(stream)>>>(mask, flow, height, width, temperature, out);
    return check_launch("rmd_up8");
}

extern "C" size_t rmd_up8_workspace_bytes(int batch, int height, int width) {
    if (batch < 1 || height < 1 || width < 1) return 0;
    return (size_t)batch * 18 * height * width * sizeof(float);
}

extern "C" int rmd_up8_backward(const float* mask, const float* flow, const float* grad_out, int batch, int height,
                                int width, float temperature, float* grad_mask, float* grad_flow, void* workspace,
                                void* stream) {
    RMD_REQUIRE(mask && flow && grad_out && grad_mask && grad_flow && workspace, RMD_ERR_ARG,
                "rmd_up8_backward: null pointer");
    RMD_REQUIRE(batch >= 1 && height >= 1 && width >= 1 && batch <= 65535, RMD_ERR_SHAPE,
                "rmd_up8_backward: bad sizes (batch=%d height=%d width=%d)", batch, height, width);
    RMD_REQUIRE(temperature > 0.0f, RMD_ERR_ARG, "rmd_up8_backward: temperature must be > 0");
    const int n = height * width;
    hipStream_t st = as_stream(stream);
    float* q = static_cast<float*>(workspace);
    up8_backward_mask_kernel<<<dim3((n + kUpPix - 1) / kUpPix, batch), dim3(kUpPix, 8), 0, st>>>(
        mask, flow, grad_out, height, width, temperature, grad_mask, q);
    int rc = check_launch("rmd_up8_backward(mask)");
    if (rc) return rc;
    up8_backward_flow_kernel<<<dim3((n + kThreads - 1) / kThreads, 2, batch), kThreads, 0, st>>>(q, height, width,
                                                                                                 grad_flow);
    return check_launch("rmd_up8_backward(flow)");
}

#define RMD_SAM_CASES(X) X(1) X(2) X(3) X(4)

extern "C" int rmd_softargmax(const float* cost, int batch, int cost_channels, int pixels, int levels, int radius,
                              float temperature, float* flows, void* stream) {
    RMD_REQUIRE(cost && flows, RMD_ERR_ARG, "rmd_softargmax: null pointer");
    RMD_REQUIRE(radius >= 1 && radius <= 4, RMD_ERR_SHAPE, "rmd_softargmax: radius %d not in 1..4", radius);
    RMD_REQUIRE(batch >= 1 && batch <= 65535 && pixels >= 1 && levels >= 1 && levels <= 16, RMD_ERR_SHAPE,
                "rmd_softargmax: bad sizes (batch=%d pixels=%d levels=%d)", batch, pixels, levels);
    RMD_REQUIRE(cost_channels >= levels * (2 * radius + 1) * (2 * radius + 1), RMD_ERR_SHAPE,
                "rmd_softargmax: %d cost channels < levels * (2r+1)^2", cost_channels);
    RMD_REQUIRE(temperature > 0.0f, RMD_ERR_ARG, "rmd_softargmax: temperature must be > 0");
    dim3 grid((pixels + kThreads - 1) / kThreads, batch, levels);
    hipStream_t st = as_stream(stream);
    switch (radius) {
#define RMD_SAM(RR) \
    case RR: softargmax_kernel<RR><<<grid, kThreads, 0, st>>>(cost, cost_channels, pixels, temperature, flows); break;
        RMD_SAM_CASES(RMD_SAM)
#undef RMD_SAM
    }
    return check_launch("rmd_softargmax");
}

extern "C" int rmd_softargmax_backward(const float* cost, const float* grad_flows, int batch, int cost_channels,
                                       int pixels, int levels, int radius, float temperature, float* grad_cost,
                                       void* stream) {
    RMD_REQUIRE(cost && grad_flows && grad_cost, RMD_ERR_ARG, "rmd_softargmax_backward: null pointer");
    RMD_REQUIRE(radius >= 1 && radius <= 4, RMD_ERR_SHAPE, "rmd_softargmax_backward: radius %d not in 1..4", radius);
    RMD_REQUIRE(batch >= 1 && batch <= 65535 && pixels >= 1 && levels >= 1 && levels <= 16, RMD_ERR_SHAPE,
                "rmd_softargmax_backward: bad sizes (batch=%d pixels=%d levels=%d)", batch, pixels, levels);
    RMD_REQUIRE(cost_channels >= levels * (2 * radius + 1) * (2 * radius + 1), RMD_ERR_SHAPE,
                "rmd_softargmax_backward: %d cost channels < levels * (2r+1)^2", cost_channels);
    RMD_REQUIRE(temperature > 0.0f, RMD_ERR_ARG, "rmd_softargmax_backward: temperature must be > 0");
    dim3 grid((pixels + kThreads - 1) / kThreads, batch, levels);
    hipStream_t st = as_stream(stream);
    switch (radius) {
#define RMD_SAM(RR)                                                                                               \
    case RR:                                                                                                      \
        softargmax_backward_kernel<RR><<<grid, kThreads, 0, st>>>(cost, cost_channels, pixels, temperature,      \
                                                                  grad_flows, grad_cost);                         \
        break;
        RMD_SAM_CASES(RMD_SAM)
#undef RMD_SAM
    }
    return check_launch("rmd_softargmax_backward");
}
