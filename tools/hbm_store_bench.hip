// hbm_store_bench.hip — diagnostic: HBM write efficiency of the correlation-GEMM epilogue's store
// pattern vs. alternatives (not product code).  Writes the cfg2 fp16 pyramid footprint (B=8,
// 55x128 queries, 4 levels) with no compute, timing each pattern with HIP events.
//   seq      : grid-stride sequential 16-B-per-lane stores (upper bound)
//   gemm     : the GEMM epilogue's per-wave pattern (23 stores per 32-query tile, 4 waves/WG,
//              wave w takes tiles w, w+4, ...), plain stores
//   gemm_nt  : same with non-temporal stores
//   gemm_sync: same, the 4 waves of a workgroup barrier-synchronised every tile
//   gemm64   : each wave writes 64 consecutive queries per tile (1 KiB contiguous per row chunk per
//              store instruction), half the tiles
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_bin/hbm_store_bench tools/hbm_store_bench.hip
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int B = 8, H = 55, W = 128, N = H * W;

struct Geo {
    long long off[4];
    int lh[4], lw[4], cw[4], tx[4];
};

__global__ void seq_store(uint4* p, long long n16) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        p[i] = make_uint4((unsigned)i, 1, 2, 3);
}


// each wave writes a private contiguous region, U x 1 KiB per step (16 B per lane per store)
template <int U, bool NT>
__global__ void __launch_bounds__(256) wave_region_store(uint4* p, long long n16) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const long long waves = (long long)gridDim.x * 4;
    const long long wid = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long long per = n16 / waves;                  // 16-B units per wave
    u4* q = reinterpret_cast<u4*>(p) + wid * per;
    const u4 v = {(unsigned)lane, 1u, 2u, 3u};
    for (long long i = 0; i + 64 * U <= per; i += 64 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v, q + i + u * 64 + lane);
            else q[i + u * 64 + lane] = v;
        }
    }
}

template <bool NT>
__global__ void seq_store2(uint4* p, long long n16) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const long long stride = (long long)gridDim.x * blockDim.x;
    const u4 v = {1u, 1u, 2u, 3u};
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u4*>(p) + i);
        else reinterpret_cast<u4*>(p)[i] = v;
    }
}


// blocked layout: one record of 340 targets x 32 queries (fp16) per (block, 32-query tile); the
// WAVES waves of a workgroup write records qt = w, w+WAVES, ... of their block, store by store:
// 16 + 4 x 1 KiB, 2 x 512 B (8 B/lane), 1 x 256 B (4 B/lane)
template <int WAVES, bool NT, bool QTMAJOR = false>
__global__ void __launch_bounds__(512) blocked_store(unsigned char* pyr, int nblk_total, int nqt) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int blk = blockIdx.x;
    if (w >= WAVES) return;
    const u4 v = {(unsigned)lane, 1u, 2u, 3u};
    for (int qt = w; qt < nqt; qt += WAVES) {
        unsigned char* rec = QTMAJOR ? pyr + ((size_t)qt * nblk_total + blk) * 21760 : pyr + ((size_t)blk * nqt + qt) * 21760;
        for (int k = 0; k < 20; ++k) {
            u4* p = reinterpret_cast<u4*>(rec + k * 1024) + lane;
            if (NT) __builtin_nontemporal_store(v, p); else *p = v;
        }
        for (int k = 0; k < 2; ++k) *reinterpret_cast<uint2*>(rec + 20480 + k * 512 + lane * 8) = make_uint2(1, 2);
        *reinterpret_cast<unsigned*>(rec + 21504 + lane * 4) = 5u;
    }
}

template <int MODE, int QT>
__global__ void __launch_bounds__(256) gemm_store(__half* pyr, Geo g) {
    const int ncb = (W + 15) / 16, nblk = ((H + 15) / 16) * ncb;
    const int b = blockIdx.x / nblk, tb = blockIdx.x % nblk;
    const int rb = tb / ncb, cb = tb % ncb;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = lane % QT, h = lane / QT;                // QT = 32: two rows per store; 64: one row
    const int nqt = (N + QT - 1) / QT;
    const uint4 v = make_uint4(lane, w, b, 7);
    for (int qt = w; qt < ((nqt + 3) / 4) * 4; qt += 4) {
        if (MODE == 2) __syncthreads();
        if (qt >= nqt) continue;
        const int q = min(qt * QT + j, N - 1);
        for (int l = 0; l < 4; ++l) {
            const int span = 16 >> l, nch = l == 0 ? 2 : 1;
            const int rows = min(span, g.lh[l] - rb * span);
            const int cw = g.cw[l];
            const int rpi = 64 / QT;                          // rows per store instruction
            for (int r0 = 0; r0 < span; r0 += rpi)
                for (int tc = 0; tc < nch; ++tc) {
                    const int row = r0 + h;
                    const int xc = cb * nch + tc;
                    if (row >= rows || xc >= g.tx[l]) continue;
                    const int y = rb * span + row;
                    __half* p = pyr + g.off[l] + (((long long)b * g.lh[l] + y) * g.tx[l] + xc) * N * cw + (long long)q * cw;
                    const int bytes = cw * 2;
                    if (bytes == 16) {
                        if (MODE == 1) { typedef unsigned u4 __attribute__((ext_vector_type(4))); const u4 vv = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(vv, reinterpret_cast<u4*>(p)); }
                        else *reinterpret_cast<uint4*>(p) = v;
                    } else if (bytes == 8) {
                        *reinterpret_cast<uint2*>(p) = make_uint2(v.x, v.y);
                    } else {
                        *reinterpret_cast<unsigned*>(p) = v.x;
                    }
                }
        }
    }
}

int main() {
    Geo g;
    long long off = 0;
    const int cws[4] = {8, 8, 4, 2};
    for (int l = 0; l < 4; ++l) {
        g.lh[l] = H >> l;
        g.lw[l] = W >> l;
        g.cw[l] = cws[l];
        g.tx[l] = (g.lw[l] + cws[l] - 1) / cws[l];
        g.off[l] = off;
        off += (long long)B * g.lh[l] * g.tx[l] * N * cws[l];
    }
    const size_t bytes = off * 2;
    __half* pyr;
    CK(hipMalloc(&pyr, bytes + (size_t)300 * 1024 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nblk = ((H + 15) / 16) * ((W + 15) / 16);
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int i = 0; i < 10; ++i) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"pattern\": \"%s\", \"median_ms\": %.4f, \"TBps\": %.3f}\n", name, ts[5], bytes / (ts[5] * 1e-3) / 1e12);
        fflush(stdout);
    };
    timeit("memset", [&] { CK(hipMemsetAsync(pyr, 0, bytes)); });
    timeit("seq_256wg", [&] { seq_store2<false><<<256, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("seq_1024wg", [&] { seq_store2<false><<<1024, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("seq_16384wg", [&] { seq_store2<false><<<16384, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("seq_nt_4096wg", [&] { seq_store2<true><<<4096, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("region_u1_256wg", [&] { wave_region_store<1, false><<<256, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("region_u4_256wg", [&] { wave_region_store<4, false><<<256, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("region_u4_nt_256wg", [&] { wave_region_store<4, true><<<256, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("region_u4_1024wg", [&] { wave_region_store<4, false><<<1024, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("region_u4_nt_1024wg", [&] { wave_region_store<4, true><<<1024, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("region_u8_nt_512wg", [&] { wave_region_store<8, true><<<512, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    {
        const int nqt = (N + 31) / 32, nb = B * nblk;
        timeit("blocked_w8", [&] { blocked_store<8, false><<<nb, 512>>>(reinterpret_cast<unsigned char*>(pyr), nb, nqt); });
        timeit("blocked_w8_nt", [&] { blocked_store<8, true><<<nb, 512>>>(reinterpret_cast<unsigned char*>(pyr), nb, nqt); });
        timeit("blocked_w4", [&] { blocked_store<4, false><<<nb, 512>>>(reinterpret_cast<unsigned char*>(pyr), nb, nqt); });
        timeit("blocked_w8_qtmajor", [&] { blocked_store<8, false, true><<<nb, 512>>>(reinterpret_cast<unsigned char*>(pyr), nb, nqt); });
        timeit("blocked_w8_qtmajor_nt", [&] { blocked_store<8, true, true><<<nb, 512>>>(reinterpret_cast<unsigned char*>(pyr), nb, nqt); });
        timeit("blocked_w8_again", [&] { blocked_store<8, false><<<nb, 512>>>(reinterpret_cast<unsigned char*>(pyr), nb, nqt); });
    }
    timeit("seq", [&] { seq_store<<<4096, 256>>>(reinterpret_cast<uint4*>(pyr), (long long)(bytes / 16)); });
    timeit("gemm", [&] { gemm_store<0, 32><<<B * nblk, 256>>>(pyr, g); });
    timeit("gemm_nt", [&] { gemm_store<1, 32><<<B * nblk, 256>>>(pyr, g); });
    timeit("gemm_sync", [&] { gemm_store<2, 32><<<B * nblk, 256>>>(pyr, g); });
    timeit("gemm64", [&] { gemm_store<0, 64><<<B * nblk, 256>>>(pyr, g); });
    timeit("gemm64_nt", [&] { gemm_store<1, 64><<<B * nblk, 256>>>(pyr, g); });
    CK(hipFree(pyr));
    return 0;
}
