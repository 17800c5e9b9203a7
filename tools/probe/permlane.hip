// probe: semantics of v_permlane32_swap / v_permlane16_swap on gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* o) {
    unsigned x = threadIdx.x, y = 100 + threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    auto s = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    o[threadIdx.x] = r[0]; o[64 + threadIdx.x] = r[1];
    o[128 + threadIdx.x] = s[0]; o[192 + threadIdx.x] = s[1];
}
int main() {
    unsigned* d; unsigned h[256];
    hipMalloc(&d, 1024);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    const char* nm[4] = {"p32 vdst", "p32 vsrc", "p16 vdst", "p16 vsrc"};
    for (int a = 0; a < 4; a++) {
        printf("%s:", nm[a]);
        for (int i = 0; i < 64; i++) printf(" %u", h[a * 64 + i]);
        printf("\n");
    }
    return 0;
}
