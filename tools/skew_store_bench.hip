// skew_store_bench.hip — diagnostic (not product code): what a per-query column skew of the level-0
// pyramid chunks would cost the correlation GEMM's store stream.
//
// Writes the cfg2 level-0 fp16 pyramid (B=8, 55x128 targets, N=7040 queries, 8-column chunks) with
// the w8 GEMM's schedule — 256 workgroups of 8 waves, one 16x16 target block each, image b on XCD b,
// waves sweeping 32-query tiles, per tile per lane 16 rows x 16 columns of one query — no compute:
//   mode 0  current layout: chunk k = columns [8k, 8k+8); per row pair 2 full 16-B stores per lane
//           (two contiguous 512-B runs per instruction)
//   mode 1  skewed layout: query q's chunk k' holds columns [8(k'-1) + s, 8(k'-1) + s + 8), s = q & 7
//           (17 chunks per row).  A block's 16 columns become one full chunk + a head piece (s halves,
//           end of chunk 2cb) + a tail piece (8-s halves, start of chunk 2cb+2); the head and tail
//           chunks are shared with the neighbouring column blocks, i.e. every other 128-B line is
//           completed by two workgroups.  Pieces are split into aligned b64/b32/b16 stores (7 per row).
//   mode 2  skewed layout, full chunks only (head/tail stores dropped): the line-address pattern
//           without the partial writes (lower bound for mode 1)
// Non-temporal stores throughout, like the product epilogue.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_bin/skew_store_bench tools/skew_store_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int B = 8, H = 55, W = 128, N = H * W, NQT = (N + 31) / 32;
constexpr int RB = (H + 15) / 16, CB = W / 16;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <typename V>
__device__ __forceinline__ void st(unsigned char* base, size_t off, V v) {
    __builtin_nontemporal_store(v, reinterpret_cast<V*>(base + off));
}

template <int MODE>
__global__ void __launch_bounds__(512, 1) level0_store(unsigned char* __restrict__ pyr) {
    const int b = blockIdx.x & 7, blk = blockIdx.x >> 3;           // image b on XCD b
    const int rb = blk / CB, cb = blk % CB;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    constexpr int NCH = MODE == 0 ? 16 : 17;                         // chunks per row
    const size_t cs = (size_t)N * 16;                                // chunk stride (bytes)
    for (int qt = wv; qt < NQT; qt += 8) {
        const int q = min(qt * 32 + j, N - 1);
        const unsigned s = (unsigned)q & 7u;
        // this lane's 16 columns of a row as 8 dwords (fake data: query and column ids)
        unsigned v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (unsigned)q * 65537u + (unsigned)i;
#pragma unroll 2
        for (int m = 0; m < 8; ++m) {
            const int y = rb * 16 + 2 * m + h;
            if (y >= H) continue;
            const size_t row = ((size_t)b * H + y) * NCH;
            if constexpr (MODE == 0) {
#pragma unroll
                for (int tc = 0; tc < 2; ++tc) {
                    const u32x4 d = {v[4 * tc], v[4 * tc + 1], v[4 * tc + 2], v[4 * tc + 3]};
                    st(pyr, ((row + 2 * cb + tc) * N + q) * 16, d);
                }
            } else {
                // rotate the 16 halves left by s: r[0..3] = columns s..s+7 (mid chunk), r[4..7] =
                // columns s+8..15, 0..s-1 (tail piece then head piece)
                unsigned r[8];
                const unsigned wsh = s >> 1;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    unsigned a = v[0], c = v[0];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        a = ((i + wsh) & 7u) == (unsigned)k ? v[k] : a;
                        c = ((i + wsh + 1) & 7u) == (unsigned)k ? v[k] : c;
                    }
                    r[i] = (s & 1u) ? __builtin_amdgcn_alignbyte(c, a, 2) : a;
                }
                const size_t hb = ((row + 2 * cb + 0) * N + q) * 16;     // head chunk
                const size_t mb = ((row + 2 * cb + 1) * N + q) * 16;     // mid chunk
                const size_t tb = ((row + 2 * cb + 2) * N + q) * 16;     // tail chunk
                const u32x4 mid = {r[0], r[1], r[2], r[3]};
                st(pyr, mb, mid);
                if constexpr (MODE == 1) {
                    const unsigned T = 8u - s;                            // tail halves (positions 0..T-1)
                    // tail: b64 [0,4) if T >= 4; b32 at p1 if 2 more; b16 at p2 if 1 more
                    if (T >= 4u) st(pyr, tb, (u32x2){r[4], r[5]});
                    const unsigned p1 = T >= 4u ? 4u : 0u;
                    if (T - p1 >= 2u && T != 8u) st(pyr, tb + 2 * p1, p1 ? r[6] : r[4]);
                    const unsigned p2 = p1 + ((T - p1 >= 2u) ? 2u : 0u);
                    if ((T & 1u) != 0u) {
                        const unsigned wv2 = p2 >> 1;                     // dword of the wrap holding position p2
                        const unsigned dv = wv2 == 0 ? r[4] : (wv2 == 1 ? r[5] : (wv2 == 2 ? r[6] : r[7]));
                        st(pyr, tb + 2 * p2, (unsigned short)(dv & 0xffffu));
                    }
                    // head: positions [8-s, 8) hold wrap positions [8-s, 8): b64 [4,8) if s >= 4 (for
                    // s == 0 this slot writes the tail's [4,8)); b32 ending at e1; b16 before it
                    if (s >= 4u || s == 0u) st(pyr, (s == 0u ? tb : hb) + 8, (u32x2){r[6], r[7]});
                    const unsigned e1 = s >= 4u ? 4u : 8u, r1 = s >= 4u ? s - 4u : s;
                    if (r1 >= 2u) st(pyr, hb + 2 * (e1 - 2u), e1 == 4u ? r[5] : r[7]);
                    if ((s & 1u) != 0u) {
                        const unsigned p3 = e1 - (r1 >= 2u ? 2u : 0u) - 1u;   // odd position
                        const unsigned wv3 = p3 >> 1;
                        const unsigned dv = wv3 == 0 ? r[4] : (wv3 == 1 ? r[5] : (wv3 == 2 ? r[6] : r[7]));
                        st(pyr, hb + 2 * p3, (unsigned short)(dv >> 16));
                    }
                }
            }
        }
    }
}

int main() {
    const size_t bytes17 = (size_t)B * H * 17 * N * 16;
    unsigned char* p;
    CK(hipMalloc(&p, bytes17 + 64));
    CK(hipMemset(p, 0, bytes17));
    const double algo = (double)B * H * W * N * 2;                  // level-0 bytes written
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = B * RB * CB;
    auto run = [&](const char* name, void (*k)(unsigned char*)) {
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
        printf("{\"pattern\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"TBps_algorithmic\": %.3f}\n", name,
               ts[ts.size() / 2], ts[0], algo / (ts[ts.size() / 2] * 1e-3) / 1e12);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("level0_current", level0_store<0>);
        run("level0_skew_partial", level0_store<1>);
        run("level0_skew_fullonly", level0_store<2>);
    }
    CK(hipFree(p));
    return 0;
}
