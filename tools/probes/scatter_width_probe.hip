// Scattered field writes into a 4 GiB image: does the write granule set the
// in-place writer's floor?  Ten million 4-byte fields (the config-4 CRC
// fields: one per commit, gaps of 200-660 B, 8-byte aligned) are stored
//   mode W = 4:       the 4-byte field alone (what the writer does now)
//   mode W = 8..128:  the whole W-aligned block holding the field, as 16-byte
//                     stores (W = 8: one 8-byte store), bytes rewritten from
//                     the block's own copy loaded first ("rmw") or constants
//                     ("blind", the write cost alone)
// One thread a field, fields in address order across the grid (as the
// commit kernel's waves meet them).  Interleaved over rounds; prints one JSON
// line per mode (ms, median).  Timing only: the image is garbage.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/swp tools/probes/scatter_width_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int W, bool RMW>
__global__ __launch_bounds__(256) void scatter(uint8_t *img, const uint64_t *field, uint32_t n)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t f = field[i];
    const uint32_t v = 0x9E3779B9u ^ i;
    if constexpr (W == 4) {
        *reinterpret_cast<uint32_t *>(img + f) = v;
    } else if constexpr (W == 8) {
        uint64_t *p = reinterpret_cast<uint64_t *>(img + (f & ~7ull));
        uint64_t w = RMW ? *p : 0x0123456789abcdefull;
        w ^= (uint64_t)v << ((f & 4) * 8);
        *p = w;
    } else {
        u32x4 *p = reinterpret_cast<u32x4 *>(img + (f & ~(uint64_t)(W - 1)));
        u32x4 b[W / 16];
#pragma unroll
        for (int k = 0; k < W / 16; ++k)
            b[k] = RMW ? p[k] : u32x4{1u, 2u, 3u, (uint32_t)k};
        const uint32_t q = (uint32_t)(f & (W - 1)) >> 2;
        b[q >> 2][q & 3] = v;
#pragma unroll
        for (int k = 0; k < W / 16; ++k)
            p[k] = b[k];
    }
}

template <int W, bool RMW>
static float run(uint8_t *img, const uint64_t *field, uint32_t n, hipEvent_t e0, hipEvent_t e1, int reps)
{
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((scatter<W, RMW>), dim3((n + 255) / 256), dim3(256), 0, 0, img, field, n);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main()
{
    const uint64_t size = 4ull << 30;
    std::vector<uint64_t> h;
    std::mt19937_64 rng(4);
    for (uint64_t at = 256; at + 1024 < size; at += 200 + 8 * (rng() % 58))
        h.push_back(at + 4); // a 4-byte field in the second half of an 8-byte word
    const uint32_t n = (uint32_t)h.size();
    uint8_t *img;
    uint64_t *field;
    if (hipMalloc(&img, size) != hipSuccess || hipMalloc(&field, n * 8ull) != hipSuccess)
        return 1;
    hipMemset(img, 0x5a, size);
    hipMemcpy(field, h.data(), n * 8ull, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    using F = float (*)(uint8_t *, const uint64_t *, uint32_t, hipEvent_t, hipEvent_t, int);
    const F fns[] = {run<4, false>,  run<8, false>,  run<8, true>,  run<16, false>, run<16, true>,
                     run<32, false>, run<32, true>,  run<64, false>, run<64, true>, run<128, false>,
                     run<128, true>};
    const char *names[] = {"w4",       "w8_blind",  "w8_rmw",   "w16_blind", "w16_rmw", "w32_blind",
                           "w32_rmw",  "w64_blind", "w64_rmw",  "w128_blind", "w128_rmw"};
    constexpr int NM = sizeof(fns) / sizeof(fns[0]);
    std::vector<float> t[NM];
    for (int w = 0; w < 20; ++w)
        fns[0](img, field, n, e0, e1, 1);
    for (int round = 0; round < 5; ++round)
        for (int m = 0; m < NM; ++m)
            t[m].push_back(fns[m](img, field, n, e0, e1, 10));
    printf("{\"fields\": %u, \"image_bytes\": %llu}\n", n, (unsigned long long)size);
    for (int m = 0; m < NM; ++m) {
        std::sort(t[m].begin(), t[m].end());
        printf("{\"mode\": \"%s\", \"ms\": %.4f, \"ms_min\": %.4f}\n", names[m], t[m][t[m].size() / 2], t[m][0]);
    }
    return 0;
}
