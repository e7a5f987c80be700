// hbm_probe: streaming-read ceilings on this MI355X for the access shapes the
// CRC kernels use.  Measured roofline denominators, not product code.
//   coalesced : lane l reads 16 B at 16*l + 1024*i (1 KiB per wave-instruction)
//   lane64    : lane l reads its own 64 B piece (4 x 16 B) at 64*l, step 4 KiB
//   lane128   : lane l reads 128 B (8 x 16 B) at 128*l, step 8 KiB
// POL (cache policy of the loads): 0 plain global_load, 1 __builtin_nontemporal_load,
//   2.. buffer_load with aux = POL - 2 (aux 2 = nt, 1 = sc0, 3 = sc0 nt)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *g4p;

template <int PIECE, int POL = 0>  // bytes per lane per step (16 = coalesced)
__global__ __launch_bounds__(1024) void rd(const char *buf, size_t n, unsigned *out)
{
    const size_t step = 64 * PIECE;
    const size_t wave = (size_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * 16;
    const int lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (size_t s = wave; s * step < n; s += nw) {
        g4p q = (g4p)(buf + s * step + (size_t)lane * PIECE);
#pragma unroll
        for (int i = 0; i < PIECE / 16; ++i) {
            u32x4 v;
            if (POL == 0) {
                v = q[i];
            } else if (POL == 1) {
                v = __builtin_nontemporal_load(q + i);
            } else {
                /* per-wave descriptor at the wave's step base (wave-uniform) */
                const char *wb = buf + s * step;
                const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)wb);
                const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)wb >> 32));
                const char *ub = (const char *)(((uintptr_t)hi << 32) | lo);
                __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)ub, 0, (int)step, 0x00020000);
                v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * PIECE + 16 * i, 0, POL - 2);
            }
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int P, int POL = 0>
float run(const char *d, size_t n, unsigned *o, int grid, int reps)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((rd<P, POL>), dim3(grid), dim3(1024), 0, 0, d, n, o);
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL((rd<P, POL>), dim3(grid), dim3(1024), 0, 0, d, n, o);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv)
{
    size_t n = (size_t)4 << 30;
    char *d; unsigned *o;
    if (hipMalloc(&d, n) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(d, 1, n);
    hipDeviceSynchronize();
    int cu = 0; hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int mult : {1, 2, 4}) {
        int grid = cu * mult;
        float c = run<16>(d, n, o, grid, 10), l64 = run<64>(d, n, o, grid, 10), l128 = run<128>(d, n, o, grid, 10);
        printf("{\"grid\": %d, \"coalesced_GBs\": %.1f, \"lane64_GBs\": %.1f, \"lane128_GBs\": %.1f}\n", grid,
               n / c / 1e6, n / l64 / 1e6, n / l128 / 1e6);
    }
    /* cache policies, lane64 shape (the team kernels' piece loads) and coalesced */
    const float p[] = {run<64, 0>(d, n, o, cu, 10), run<64, 1>(d, n, o, cu, 10), run<64, 2>(d, n, o, cu, 10),
                       run<64, 3>(d, n, o, cu, 10), run<64, 4>(d, n, o, cu, 10), run<64, 5>(d, n, o, cu, 10),
                       run<16, 1>(d, n, o, cu, 10), run<16, 4>(d, n, o, cu, 10)};
    printf("{\"grid\": %d, \"lane64_plain\": %.1f, \"lane64_nontemporal\": %.1f, \"lane64_buf_aux0\": %.1f, "
           "\"lane64_buf_sc0\": %.1f, \"lane64_buf_nt\": %.1f, \"lane64_buf_sc0nt\": %.1f, "
           "\"coalesced_nontemporal\": %.1f, \"coalesced_buf_nt\": %.1f}\n", cu,
           n / p[0] / 1e6, n / p[1] / 1e6, n / p[2] / 1e6, n / p[3] / 1e6, n / p[4] / 1e6, n / p[5] / 1e6,
           n / p[6] / 1e6, n / p[7] / 1e6);
    return 0;
}
