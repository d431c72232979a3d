// store_pattern_bench.hip — diagnostic (not product code): HBM write rate of candidate level-0 pyramid
// store patterns under the w8 GEMM's schedule (256 workgroups of 8 waves, one 16x16 target block each,
// image b on XCD b, waves sweeping 32-query tiles; cfg2: B=8, 55x128, 7040 query slots), no compute:
//   tiles2x4 : the product tiles layout — per chunk row pair m and column group tc one 16-B store per
//              lane at quad 4cb + 2tc + h (two contiguous 512-B runs per instruction)
//   tiles4x4 : 4x4 chunks (32 B per slot): per row block i and column group tc two 16-B stores per lane
//              (halves of its own 4x4 accumulator block), slot stride 32 B
//   rows1x8  : the round-2 row layout (1x8 chunks, two 512-B runs per instruction after the lane swap)
//   tiles2x8 : 2x8 chunks (32 B per slot): per chunk row m and column chunk tc one 16-B store per lane,
//              half-wave h writing bytes 16h..16h+15 of each slot's chunk — one contiguous 1-KiB run per
//              instruction (round 4 candidate)
// (a sequential-store reference is tools/hbm_store_bench.hip's seq: 6.3 TB/s)
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_ab/store_pattern_bench tools/store_pattern_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int B = 8, H = 55, W = 128, S = 7040, NQT = S / 32;
constexpr int RB = (H + 15) / 16, CB = W / 16;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(512, 1) level0_store(unsigned char* __restrict__ pyr) {
    const int b = blockIdx.x & 7, blk = blockIdx.x >> 3;
    const int rb = blk / CB, cb = blk % CB;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    for (int qt = wv; qt < NQT; qt += 8) {
        const unsigned q = (unsigned)(qt * 32 + j);
        const u32x4 d = {q, q + 1u, q + 2u, q + 3u};
        if constexpr (MODE == 0) {            // tiles 2x4: TY = 28 chunk rows, TX = 32 quads
            for (int m = 0; m < 8; ++m) {
                const int cr = rb * 8 + m;
                if (cr >= 28) break;
#pragma unroll
                for (int tc = 0; tc < 2; ++tc) {
                    const size_t pos = ((size_t)b * 28 + cr) * 32 + 4 * cb + 2 * tc + h;
                    __builtin_nontemporal_store(d, reinterpret_cast<u32x4*>(pyr + (pos * S + q) * 16));
                }
            }
        } else if constexpr (MODE == 1) {     // tiles 4x4: TY = 14 chunk rows of 4, TX = 32 quads, 32 B per slot
            for (int i = 0; i < 4; ++i) {
                const int cr = rb * 4 + i;
                if (cr >= 14) break;
#pragma unroll
                for (int tc = 0; tc < 2; ++tc) {
                    const size_t pos = ((size_t)b * 14 + cr) * 32 + 4 * cb + 2 * tc + h;
#pragma unroll
                    for (int half = 0; half < 2; ++half)
                        __builtin_nontemporal_store(d, reinterpret_cast<u32x4*>(pyr + (pos * S + q) * 32 + 16 * half));
                }
            }
        } else if constexpr (MODE == 3) {     // tiles 2x8: TY = 28 chunk rows, TX = 16 chunks of 8 columns
            for (int m = 0; m < 8; ++m) {
                const int cr = rb * 8 + m;
                if (cr >= 28) break;
#pragma unroll
                for (int tc = 0; tc < 2; ++tc) {
                    const size_t pos = ((size_t)b * 28 + cr) * 16 + 2 * cb + tc;
                    __builtin_nontemporal_store(d, reinterpret_cast<u32x4*>(pyr + (pos * S + q) * 32 + 16 * h));
                }
            }
        } else if constexpr (MODE == 2) {     // rows 1x8: 55 rows, 16 chunks; lane h writes row 2m + h
            for (int m = 0; m < 8; ++m) {
                const int y = rb * 16 + 2 * m + h;
#pragma unroll
                for (int tc = 0; tc < 2; ++tc) {
                    if (y < H) {
                        const size_t pos = ((size_t)b * H + y) * 16 + 2 * cb + tc;
                        __builtin_nontemporal_store(d, reinterpret_cast<u32x4*>(pyr + (pos * S + q) * 16));
                    }
                }
            }
        }
    }
}

int main() {
    const size_t bytes = (size_t)B * 28 * 32 * S * 16 + (1u << 20);
    unsigned char* p;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = B * RB * CB;
    auto run = [&](const char* name, void (*k)(unsigned char*), double nbytes) {
        std::vector<float> ts;
        for (int it = 0; it < 25; ++it) {
            CK(hipEventRecord(e0));
            k<<<grid, 512>>>(p);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it >= 5) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"pattern\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"MB\": %.1f, \"TBps\": %.3f}\n", name,
               ts[ts.size() / 2], ts[0], nbytes / 1e6, nbytes / (ts[ts.size() / 2] * 1e-3) / 1e12);
        fflush(stdout);
    };
    const double b2x4 = (double)B * 28 * 32 * S * 16, b4x4 = (double)B * 14 * 32 * S * 32, brow = (double)B * 55 * 16 * S * 16;
    for (int rep = 0; rep < 2; ++rep) {
        run("tiles2x4", level0_store<0>, b2x4);
        run("tiles4x4", level0_store<1>, b4x4);
        run("rows1x8", level0_store<2>, brow);
        run("tiles2x8", level0_store<3>, b2x4);
    }
    CK(hipFree(p));
    return 0;
}
