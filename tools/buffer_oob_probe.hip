// Does the raw-buffer range check include the scalar offset (soffset)?  One wave loads and stores
// through a descriptor of 256 bytes over a 4 KiB buffer of known values; prints what came back and
// which bytes past the range were written.  hipcc --offload-arch=gfx950 -O2 buffer_oob_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(float* buf, float* res) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)buf);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)buf >> 32));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo), (short)0, 256, 0x00020000);
    const int l = threadIdx.x;
    // res[0..]: in range via voffset; voffset past the end; soffset past the end; both inside but sum past
    res[0 * 64 + l] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * (l & 15), 0, 0));
    res[1 * 64 + l] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 256 + 4 * (l & 15), 0, 0));
    res[2 * 64 + l] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * (l & 15), 256, 0));
    res[3 * 64 + l] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 128 + 4 * (l & 15), 192, 0));
    // stores: soffset past the end (bytes 512..575), and voffset past the end (bytes 1024..1087)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(-1.f), r, 4 * (l & 15), 512, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(-2.f), r, 1024 + 4 * (l & 15), 0, 0);
}

int main() {
    float h[1024], *d, *res, hr[256];
    for (int i = 0; i < 1024; ++i) h[i] = (float)(i + 1);
    hipMalloc(&d, sizeof h);
    hipMalloc(&res, sizeof hr);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(d, res);
    hipMemcpy(hr, res, sizeof hr, hipMemcpyDeviceToHost);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("{\"in_range\": %g, \"voffset_past\": %g, \"soffset_past\": %g, \"sum_past\": %g, "
           "\"store_soffset_past_written\": %d, \"store_voffset_past_written\": %d}\n",
           hr[1], hr[64 + 1], hr[128 + 1], hr[192 + 1], h[128 + 1] == -1.f, h[256 + 1] == -2.f);
    return 0;
}
