// lds_chain_probe: throughput of dependent slice-by-4 lookup chains (v_perm +
// 4 x ds_read_b32 from 32-replica bank-private tables) with C independent
// chains per lane, 16 waves/CU, no global memory.  Reports lookups/clk/CU
// equivalent as GB/s of "CRC bytes" (1 lookup = 1 byte).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__device__ __forceinline__ unsigned lds32(const char *L, unsigned a) { return *(const unsigned *)(L + a); }
__device__ __forceinline__ unsigned m4(const char *L, unsigned x, unsigned c_lo, unsigned c_hi)
{
    unsigned a0 = __builtin_amdgcn_perm(x, c_lo, 0x0C020400u), a1 = __builtin_amdgcn_perm(x, c_lo, 0x0C020500u);
    unsigned a2 = __builtin_amdgcn_perm(x, c_hi, 0x0C020600u), a3 = __builtin_amdgcn_perm(x, c_hi, 0x0C020700u);
    return lds32(L, a0) ^ lds32(L, a1 + 128) ^ lds32(L, a2) ^ lds32(L, a3 + 128);
}

template <int C>
__global__ __launch_bounds__(1024) void chain(int iters, unsigned *out)
{
    __shared__ __attribute__((aligned(16))) char L[131072];
    for (int i = threadIdx.x; i < 32768; i += 1024) ((unsigned *)L)[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const unsigned c_lo = (lane & 31) << 2, c_hi = c_lo | 0x10000u;
    unsigned acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = threadIdx.x * 7 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = m4(L, acc[c] ^ (unsigned)i, c_lo, c_hi);
    }
    unsigned r = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) r ^= acc[c];
    out[blockIdx.x * 1024 + threadIdx.x] = r;
}

template <int C>
void run(int cu, unsigned *o)
{
    const int iters = 4096 / C;   // same total lookups per lane for every C
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    hipLaunchKernelGGL(chain<C>, dim3(cu), dim3(1024), 0, 0, iters, o);
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(chain<C>, dim3(cu), dim3(1024), 0, 0, iters, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    double bytes = (double)cu * 1024 * 4096 * 4;  // 4 lookups (= 4 CRC bytes) per m4
    printf("{\"chains\": %d, \"ms\": %.4f, \"GBs_equiv\": %.1f}\n", C, t[2], bytes / t[2] / 1e6);
}

int main()
{
    int cu = 0; (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *o; (void)hipMalloc(&o, cu * 1024 * 4);
    run<1>(cu, o); run<2>(cu, o); run<4>(cu, o); run<8>(cu, o);
    return 0;
}
