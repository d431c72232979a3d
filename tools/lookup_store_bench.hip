// lookup_store_bench.hip — diagnostic (not product code): HBM write rate of the lookup's output stream
// alone at cfg2 (B=8, 55x128 queries, 4 levels, r=4: 324 fp32 planes of N=7040 per image, 73.0 MB) under
// candidate store patterns, no loads, no compute:
//   tiles_wave : the product — one-wave workgroups over 64 tiles-layout query slots (two 2x16 query tiles:
//                every b32 store instruction writes two 128-B runs, pixel rows y and y+1), grid (110, B, 12),
//                each wave one (level, row part): 3 output rows x 9 columns = 27 planes
//   raster_wave: the same with slots in raster order (one 256-B run per instruction)
//   pair_b128  : 256-thread workgroups over one query row pair (2 x 128 pixels = 1 KiB contiguous per
//                plane): each wave writes a quarter of the 27 planes, one b128 store per lane = 1 KiB per
//                instruction (what an LDS transpose of the tiles-order results allows)
//   pair_b32   : the same workgroups, b32 stores: 4 waves x 256 B cover one plane's 1 KiB
//   pair_b128_w: one-wave workgroups each writing the 27 planes of one row pair as 1-KiB b128 stores
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_ab/lookup_store_bench tools/lookup_store_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int B = 8, H = 55, W = 128, N = H * W, L = 4, D = 9, PL = L * D * D;
constexpr int QX = W / 16, HP = H / 2, SLOTS = HP * QX * 32 + W;   // 7040 (odd H: last row raster)
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void tiles_pixel(int s, int& y1, int& x1) {
    const int base = HP * QX * 32;
    if (s < base) {
        const int t = s >> 5, j = s & 31;
        y1 = 2 * (t / QX) + ((j >> 2) & 1);
        x1 = 16 * (t % QX) + ((j >> 3) << 2) + (j & 3);
    } else {
        y1 = H - 1;
        x1 = s - base;
    }
}

template <bool TILES>
__global__ void __launch_bounds__(64) wave_store(float* __restrict__ out) {
    const int s = blockIdx.x * 64 + threadIdx.x, b = blockIdx.y, lv = blockIdx.z % L, part = blockIdx.z / L;
    if (s >= SLOTS) return;
    int p;
    if constexpr (TILES) {
        int y1, x1;
        tiles_pixel(s, y1, x1);
        p = y1 * W + x1;
    } else {
        p = s;
    }
    float* o = out + ((size_t)b * PL + lv * D * D) * N + p;
    const float v = (float)s;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int a = 0; a < D; ++a) __builtin_nontemporal_store(v + a, o + (size_t)(a * D + part * 3 + j) * N);
}

// blockIdx.x = row pair (the odd last row: pair HP, 128 pixels)
template <bool B128>
__global__ void __launch_bounds__(256) pair_store(float* __restrict__ out) {
    const int rp = blockIdx.x, b = blockIdx.y, lv = blockIdx.z % L, part = blockIdx.z / L;
    const int npx = rp < HP ? 2 * W : W;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* o = out + ((size_t)b * PL + lv * D * D) * N + (size_t)rp * 2 * W;
    const float v = (float)threadIdx.x;
    if constexpr (B128) {
        // plane k of the part's 27 goes to wave k % 4
        for (int k = wv; k < 27; k += 4) {
            const int j = k / D, a = k % D;
            float* op = o + (size_t)(a * D + part * 3 + j) * N;
            if (4 * lane < npx) __builtin_nontemporal_store(f32x4{v, v, v, v + k}, reinterpret_cast<f32x4*>(op + 4 * lane));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int a = 0; a < D; ++a) {
                float* op = o + (size_t)(a * D + part * 3 + j) * N;
                if ((int)threadIdx.x < npx) __builtin_nontemporal_store(v + a, op + threadIdx.x);
            }
    }
}

__global__ void __launch_bounds__(64) pair_store_wave(float* __restrict__ out) {
    const int rp = blockIdx.x, b = blockIdx.y, lv = blockIdx.z % L, part = blockIdx.z / L;
    const int npx = rp < HP ? 2 * W : W;
    const int lane = threadIdx.x;
    float* o = out + ((size_t)b * PL + lv * D * D) * N + (size_t)rp * 2 * W;
    const float v = (float)lane;
    for (int k = 0; k < 27; ++k) {
        const int j = k / D, a = k % D;
        float* op = o + (size_t)(a * D + part * 3 + j) * N;
        if (4 * lane < npx) __builtin_nontemporal_store(f32x4{v, v, v, v + k}, reinterpret_cast<f32x4*>(op + 4 * lane));
    }
}

int main() {
    const size_t bytes = (size_t)B * PL * N * 4;
    float* p;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        std::vector<float> ts;
        for (int it = 0; it < 40; ++it) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it >= 5) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"pattern\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"MB\": %.1f, \"TBps\": %.3f}\n", name,
               ts[ts.size() / 2] * 1e3, ts[0] * 1e3, bytes / 1e6, bytes / (ts[ts.size() / 2] * 1e-3) / 1e12);
        fflush(stdout);
    };
    const dim3 gw((SLOTS + 63) / 64, B, 3 * L), gp(HP + 1, B, 3 * L);
    for (int rep = 0; rep < 2; ++rep) {
        run("tiles_wave", [&] { wave_store<true><<<gw, 64>>>(p); });
        run("raster_wave", [&] { wave_store<false><<<gw, 64>>>(p); });
        run("pair_b128", [&] { pair_store<true><<<gp, 256>>>(p); });
        run("pair_b32", [&] { pair_store<false><<<gp, 256>>>(p); });
        run("pair_b128_w", [&] { pair_store_wave<<<gp, 64>>>(p); });
    }
    CK(hipFree(p));
    return 0;
}
