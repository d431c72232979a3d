// perm_probe.hip — diagnostic: the lane semantics of v_permlane16_swap / v_permlane32_swap on gfx950.
// Prints, for x = lane id and y = 100 + lane id, the two results of each builtin for lanes 0, 15, 16, 31,
// 32, 47, 48, 63.  build: hipcc --offload-arch=gfx950 -O3 -o tools/_ab/perm_probe tools/perm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned* o) {
    const unsigned l = threadIdx.x;
    unsigned x = l, y = 100 + l;
    auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    o[l] = r[0];
    o[64 + l] = r[1];
    auto s = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    o[128 + l] = s[0];
    o[192 + l] = s[1];
}

int main() {
    unsigned* d;
    unsigned h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    probe<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const int ls[] = {0, 15, 16, 31, 32, 47, 48, 63};
    for (int k = 0; k < 4; ++k) {
        printf("%s:", k == 0 ? "p16 vdst" : k == 1 ? "p16 src " : k == 2 ? "p32 vdst" : "p32 src ");
        for (int i : ls) printf(" %d->%u", i, h[64 * k + i]);
        printf("\n");
    }
    return 0;
}
