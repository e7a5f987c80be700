// unaligned_probe: does global_load_dwordx4 at 1/2/4/8/12-byte misalignment
// return the right bytes on gfx950, and at what bandwidth?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *g4p;
typedef const __attribute__((address_space(1))) unsigned char *g8p;

__global__ __launch_bounds__(1024) void x4(const char *buf, size_t n, int off, unsigned *out)
{
    const size_t wave = (size_t)blockIdx.x * 16 + (threadIdx.x >> 6), nw = (size_t)gridDim.x * 16;
    const int lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (size_t s = wave; (s + 1) * 4096 + 64 < n; s += nw) {
        g4p q = (g4p)(buf + off + s * 4096 + (size_t)lane * 64);
#pragma unroll
        for (int i = 0; i < 4; ++i) { u32x4 v = q[i]; acc += v.x * 3 + v.y * 5 + v.z * 7 + v.w * 11; }
    }
    atomicAdd(out, acc);
}
__global__ __launch_bounds__(1024) void bytes(const char *buf, size_t n, int off, unsigned *out)
{
    const size_t wave = (size_t)blockIdx.x * 16 + (threadIdx.x >> 6), nw = (size_t)gridDim.x * 16;
    const int lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (size_t s = wave; (s + 1) * 4096 + 64 < n; s += nw) {
        g8p q = (g8p)(buf + off + s * 4096 + (size_t)lane * 64);
        for (int i = 0; i < 4; ++i) {
            unsigned w[4];
            for (int k = 0; k < 4; ++k)
                w[k] = q[16 * i + 4 * k] | (q[16 * i + 4 * k + 1] << 8) | (q[16 * i + 4 * k + 2] << 16) | ((unsigned)q[16 * i + 4 * k + 3] << 24);
            acc += w[0] * 3 + w[1] * 5 + w[2] * 7 + w[3] * 11;
        }
    }
    atomicAdd(out, acc);
}
int main()
{
    size_t n = (size_t)1 << 30;
    char *d; unsigned *o;
    (void)hipMalloc(&d, n); (void)hipMalloc(&o, 64);
    std::vector<unsigned char> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (unsigned char)(i * 2654435761u >> 13);
    (void)hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice);
    int cu = 0; (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int off : {0, 4, 8, 12, 1, 2, 3}) {
        unsigned a = 0, b = 0;
        (void)hipMemset(o, 0, 8);
        hipLaunchKernelGGL(x4, dim3(cu), dim3(1024), 0, 0, d, n, off, o);
        hipLaunchKernelGGL(bytes, dim3(cu), dim3(1024), 0, 0, d, n, off, o + 1);
        if (hipDeviceSynchronize() != hipSuccess) { printf("{\"off\": %d, \"error\": true}\n", off); return 1; }
        (void)hipMemcpy(&a, o, 4, hipMemcpyDeviceToHost); (void)hipMemcpy(&b, o + 1, 4, hipMemcpyDeviceToHost);
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        std::vector<float> t;
        for (int r = 0; r < 7; ++r) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(x4, dim3(cu), dim3(1024), 0, 0, d, n, off, o);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("{\"off\": %d, \"match\": %s, \"x4_GBs\": %.1f}\n", off, a == b ? "true" : "false", n / t[3] / 1e6);
    }
    return 0;
}
