// permlane_probe: semantics of gfx950 v_permlane16_swap / v_permlane32_swap
// (diagnostic).  Prints, per lane, the two results for a = lane, b = 100 + lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o)
{
    const unsigned a = threadIdx.x, b = 100 + threadIdx.x;
    auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    auto s = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    o[4 * threadIdx.x + 0] = r[0];
    o[4 * threadIdx.x + 1] = r[1];
    o[4 * threadIdx.x + 2] = s[0];
    o[4 * threadIdx.x + 3] = s[1];
}
int main()
{
    unsigned *d, h[256];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l += 8)
        printf("lane %2d: p16 (%u, %u)  p32 (%u, %u)\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
    return 0;
}
