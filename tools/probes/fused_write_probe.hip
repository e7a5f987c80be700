// The in-place writer's floor with the stores inside the read stream: a
// streaming read of a 4 GiB image (stream_read_kernel's shape: 16 waves per
// CU, a wave step = 4 KiB as 4 rows of 64 lanes x 16 B, the next step's loads
// in flight) that also writes ten million 4-byte fields (config-4 spacing,
// gaps 200-660 B, 8-aligned + 4) as it passes them:
//   read     no writes (the read floor)
//   w4       each field's 4 bytes (what commit_kernel does now)
//   w64_reg  the 64-byte aligned block around each field, written from the
//            registers that just read it: the four lanes holding the block
//            store their 16 B, the field patched in
//   w64_rmw  the field's lane reloads the 64-byte block (plain loads) and
//            stores it back patched
// The image is timing-only garbage; fields never share a 64-byte block.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/fwp tools/probes/fused_write_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *g4p;

constexpr uint64_t BLK = 4096;

__device__ __forceinline__ uint64_t or64(uint64_t m)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
        m |= __shfl_xor(m, d);
    return m;
}

template <int MODE>
__global__ __launch_bounds__(1024) void fw(uint8_t *buf, uint64_t n, const uint64_t *field, const uint32_t *bstart,
                                           uint32_t *out)
{
    const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * 16;
    const int lane = threadIdx.x & 63;
    const uint64_t nb = n / BLK;
    uint32_t acc = 0;
    u32x4 a[4], b[4];
    uint64_t s = wave;
    uint64_t fa = 0, fb = 0; /* this step's / the next step's field (lane j: field j), 0 = none */
    if (s < nb) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            a[i] = __builtin_nontemporal_load((g4p)(buf + s * BLK + 1024 * i + 16 * lane));
        if (MODE > 0) {
            const uint32_t f0 = bstart[s], f1 = bstart[s + 1];
            fa = (uint32_t)lane < f1 - f0 ? field[f0 + lane] : 0;
        }
    }
    while (s < nb) {
        const uint64_t t = s + nw;
        if (t < nb) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                b[i] = __builtin_nontemporal_load((g4p)(buf + t * BLK + 1024 * i + 16 * lane));
            if (MODE > 0) {
                const uint32_t f0 = bstart[t], f1 = bstart[t + 1];
                fb = (uint32_t)lane < f1 - f0 ? field[f0 + lane] : 0;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
        if constexpr (MODE > 0) {
            const bool mine = fa != 0;
            const uint64_t f = fa;
            const uint32_t v = acc | 1u;
            if constexpr (MODE == 1) {
                if (mine)
                    *reinterpret_cast<uint32_t *>(buf + f) = v;
            } else if constexpr (MODE == 2) {
                const uint64_t blocks = or64(mine ? 1ull << ((f - s * BLK) >> 6) : 0ull);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t blk = (uint32_t)(1024 * i + 16 * lane) >> 6;
                    if ((blocks >> blk) & 1ull) {
                        u32x4 w = a[i];
                        w.y ^= v; // stands in for patching the field
                        *reinterpret_cast<u32x4 *>(buf + s * BLK + 1024 * i + 16 * lane) = w;
                    }
                }
            } else {
                if (mine) {
                    u32x4 *p = reinterpret_cast<u32x4 *>(buf + (f & ~63ull));
                    u32x4 w[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        w[k] = p[k];
                    w[(f >> 4) & 3].w = v;
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        p[k] = w[k];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            a[i] = b[i];
        fa = fb;
        s = t;
    }
    if (acc == 0x9E3779B9u)
        out[0] = acc;
}

template <int MODE>
static float run(uint8_t *buf, uint64_t n, const uint64_t *field, const uint32_t *bstart, uint32_t *out, int grid,
                 hipEvent_t e0, hipEvent_t e1, int reps)
{
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(fw<MODE>, dim3(grid), dim3(1024), 0, 0, buf, n, field, bstart, out);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main()
{
    const uint64_t n = 4ull << 30;
    const uint64_t nb = n / BLK;
    std::vector<uint64_t> h;
    std::vector<uint32_t> bs(nb + 1, 0);
    std::mt19937_64 rng(4);
    for (uint64_t at = 256; at + 1024 < n; at += 200 + 8 * (rng() % 58))
        h.push_back(at + 4);
    for (uint64_t i = 0, k = 0; i <= nb; ++i) {
        while (k < h.size() && h[k] < i * BLK)
            ++k;
        bs[i] = (uint32_t)k;
    }
    for (uint64_t i = 0; i < nb; ++i)
        if (bs[i + 1] - bs[i] > 64)
            return 3;
    uint8_t *buf;
    uint64_t *field;
    uint32_t *bstart, *out;
    if (hipMalloc(&buf, n) != hipSuccess || hipMalloc(&field, h.size() * 8) != hipSuccess ||
        hipMalloc(&bstart, bs.size() * 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess)
        return 1;
    hipMemset(buf, 0x5a, n);
    hipMemcpy(field, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(bstart, bs.data(), bs.size() * 4, hipMemcpyHostToDevice);
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    using F = float (*)(uint8_t *, uint64_t, const uint64_t *, const uint32_t *, uint32_t *, int, hipEvent_t,
                        hipEvent_t, int);
    const F fns[] = {run<0>, run<1>, run<2>, run<3>};
    const char *names[] = {"read", "w4", "w64_reg", "w64_rmw"};
    constexpr int NM = 4;
    std::vector<float> t[NM];
    for (int w = 0; w < 30; ++w)
        fns[0](buf, n, field, bstart, out, ncu, e0, e1, 1);
    for (int round = 0; round < 5; ++round)
        for (int m = 0; m < NM; ++m)
            t[m].push_back(fns[m](buf, n, field, bstart, out, ncu, e0, e1, 10));
    printf("{\"fields\": %zu, \"image_bytes\": %llu}\n", h.size(), (unsigned long long)n);
    for (int m = 0; m < NM; ++m) {
        std::sort(t[m].begin(), t[m].end());
        printf("{\"mode\": \"%s\", \"ms\": %.4f, \"ms_min\": %.4f}\n", names[m], t[m][t[m].size() / 2], t[m][0]);
    }
    return 0;
}
