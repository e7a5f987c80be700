// coop_probe: read rates of cooperative load shapes over zsbench-like records
// (312-byte spans every 320 bytes, piece grid end-aligned: each record read as
// 5 x 64 B from 8 bytes before the span, files shifting the grid by 48 B every
// 2 MiB).  K lanes share each 16-byte-per-lane row of a record chunk of K x 16 B:
//   K = 4 : quad-cooperative (burst_kernel: one instruction = 16 records x 64 B)
//   K = 8 : octo (8 records x 128 B)     K = 16: row (4 records x 256 B)
// Loads only (XOR-reduced), 512-thread workgroups, 8 waves per CU as the burst
// kernel runs.  Measured ceilings for the short-record path; not product code.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *g4p;

constexpr size_t FILE_BYTES = 2097328, HDR = 40, PAIR = 320, PAIRS = 6554;

__device__ __forceinline__ size_t rec_start(size_t r)
{
    const size_t f = r / PAIRS, k = r % PAIRS;
    return f * FILE_BYTES + HDR + k * PAIR - 8; /* grid start: 8 B before the span */
}

/* K lanes per record chunk; a wave round covers 64 records (their 320 B each). */
template <int K, int POL>
__global__ __launch_bounds__(512) void coop(const char *buf, size_t nrec, unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 8 + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * 8;
    constexpr int RPI = 64 / K;         /* records per instruction */
    constexpr int CH = K * 16;          /* bytes per record per instruction */
    constexpr int NI = (320 + CH - 1) / CH; /* instructions per record group */
    unsigned acc = 0;
    for (size_t base = wave * 64; base < nrec; base += nw * 64) {
        u32x4 v[64 / RPI * NI];
#pragma unroll
        for (int gI = 0; gI < 64 / RPI; ++gI) {      /* record groups of this round */
#pragma unroll
            for (int p = 0; p < NI; ++p) {
                const size_t r = base + gI * RPI + lane / K;
                const size_t rr = r < nrec ? r : nrec - 1;
                size_t off = rec_start(rr) + (size_t)p * CH + 16 * (lane % K);
                const size_t lim = rec_start(rr) + 320 - 16;
                off = off > lim ? lim : off;
                const g4p q = (g4p)(buf + off);
                v[gI * NI + p] = POL ? __builtin_nontemporal_load(q) : *q;
            }
        }
#pragma unroll
        for (int i = 0; i < 64 / RPI * NI; ++i)
            acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

template <typename F>
float timeit(F kern, int grid, const char *d, size_t n, unsigned *o)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, d, n, o);
    std::vector<float> t;
    for (int r = 0; r < 10; ++r) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, d, n, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main()
{
    const size_t nfiles = 1526, nrec = nfiles * PAIRS;
    const size_t n = nfiles * FILE_BYTES;
    char *d;
    unsigned *o;
    if (hipMalloc(&d, n + 4096) != hipSuccess || hipMalloc(&o, 64) != hipSuccess)
        return 1;
    (void)hipMemset(d, 1, n + 4096);
    (void)hipDeviceSynchronize();
    int cu = 0;
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    const double bytes = (double)nrec * 320;
    struct { const char *name; float ms; } r[] = {
        {"quad plain", timeit(coop<4, 0>, cu, d, nrec, o)},
        {"octo plain", timeit(coop<8, 0>, cu, d, nrec, o)},
        {"row plain", timeit(coop<16, 0>, cu, d, nrec, o)},
        {"quad nt", timeit(coop<4, 1>, cu, d, nrec, o)},
        {"octo nt", timeit(coop<8, 1>, cu, d, nrec, o)},
        {"row nt", timeit(coop<16, 1>, cu, d, nrec, o)},
        {"quad plain x2", timeit(coop<4, 0>, 2 * cu, d, nrec, o)},
        {"octo plain x2", timeit(coop<8, 0>, 2 * cu, d, nrec, o)},
    };
    for (auto &x : r)
        printf("{\"case\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f}\n", x.name, x.ms, bytes / x.ms / 1e6);
    return 0;
}
