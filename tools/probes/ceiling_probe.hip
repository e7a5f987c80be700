// ceiling_probe: HBM streaming-read ceilings on this MI355X, every load kept
// in flight by a software pipeline (the round-1 hbm_probe waited on each
// iteration's loads, so its "coalesced" row under-states the chip).  Measured
// roofline denominators for bench.py's measured_read_peak and for the team
// kernels' access shapes; not product code.
//
//   coal<D,POL,WG>  : each wave sweeps blocks of D x 1 KiB (lane l: 16 B at
//                     16*l + 1024*i), next block in flight while one is XORed
//   team<S,POL,WG>  : config-3 shape -- 16-lane teams, lane j reads its 64 B
//                     piece of a 1 KiB team step (four 16-B loads), S steps of
//                     its 64 KiB chunk in flight; chunks strided over teams
//   glds<D,POL,WG>  : global_load_lds_dwordx4 of D x 1 KiB per wave into an
//                     LDS ring (two halves), consumed with ds_read_b128
// POL: 0 plain, 1 non-temporal (__builtin_nontemporal_load / glds aux nt)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *g4p;

template <int POL>
__device__ __forceinline__ u32x4 ld(g4p p)
{
    if (POL == 1)
        return __builtin_nontemporal_load(p);
    return *p;
}

template <int D, int POL, int WG>
__global__ __launch_bounds__(WG) void coal(const char *buf, size_t n, unsigned *out)
{
    constexpr int W = WG / 64;
    const size_t blk = (size_t)D * 1024;
    const size_t wave = (size_t)blockIdx.x * W + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * W;
    const int lane = threadIdx.x & 63;
    const size_t nb = n / blk;
    unsigned acc = 0;
    u32x4 a[D];
    size_t s = wave;
    if (s < nb) {
#pragma unroll
        for (int i = 0; i < D; ++i)
            a[i] = ld<POL>((g4p)(buf + s * blk + 1024 * i + 16 * lane));
    }
    while (s < nb) {
        const size_t t = s + nw;
        u32x4 b[D];
        if (t < nb) {
#pragma unroll
            for (int i = 0; i < D; ++i)
                b[i] = ld<POL>((g4p)(buf + t * blk + 1024 * i + 16 * lane));
        }
#pragma unroll
        for (int i = 0; i < D; ++i)
            acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
        for (int i = 0; i < D; ++i)
            a[i] = b[i];
        s = t;
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

/* 16-lane teams over 64 KiB chunks, S steps (1 KiB each) in flight per team. */
template <int S, int POL, int WG>
__global__ __launch_bounds__(WG) void team(const char *buf, size_t n, unsigned *out)
{
    constexpr int W = WG / 64;
    constexpr size_t CH = 65536, STEPS = CH / 1024;
    const int lane = threadIdx.x & 63, j = lane & 15;
    const size_t tm = ((size_t)blockIdx.x * W + (threadIdx.x >> 6)) * 4 + (lane >> 4);
    const size_t nt = (size_t)gridDim.x * W * 4;
    const size_t nch = n / CH;
    unsigned acc = 0;
    const size_t total = ((nch + nt - 1 - tm) / nt) * STEPS; /* this team's steps */
    u32x4 r[S][4];
    auto addr = [&](size_t k) {
        const size_t c = tm + (k / STEPS) * nt;
        return buf + c * CH + (k % STEPS) * 1024 + 64 * j;
    };
#pragma unroll
    for (int q = 0; q < S; ++q)
        if ((size_t)q < total)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                r[q][i] = ld<POL>((g4p)(addr(q) + 16 * i));
    for (size_t k = 0; k < total; k += S) {
#pragma unroll
        for (int q = 0; q < S; ++q) {
            if (k + q >= total)
                break;
            u32x4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                v[i] = r[q][i];
            if (k + q + S < total) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    r[q][i] = ld<POL>((g4p)(addr(k + q + S) + 16 * i));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

/* 16-lane teams, coalesced form: instruction i of a 1 KiB team step reads
 * 16 B at 256*i + 16*m (lane m of the team): four 256-byte segments per
 * wave-instruction, every line consumed by one instruction (what a quad
 * transpose turns into 64-byte pieces). */
template <int S, int POL, int WG>
__global__ __launch_bounds__(WG) void teamq(const char *buf, size_t n, unsigned *out)
{
    constexpr int W = WG / 64;
    constexpr size_t CH = 65536, STEPS = CH / 1024;
    const int lane = threadIdx.x & 63, j = lane & 15;
    const size_t tm = ((size_t)blockIdx.x * W + (threadIdx.x >> 6)) * 4 + (lane >> 4);
    const size_t nt = (size_t)gridDim.x * W * 4;
    const size_t nch = n / CH;
    unsigned acc = 0;
    const size_t total = ((nch + nt - 1 - tm) / nt) * STEPS;
    u32x4 r[S][4];
    auto addr = [&](size_t k) {
        const size_t c = tm + (k / STEPS) * nt;
        return buf + c * CH + (k % STEPS) * 1024 + 16 * j;
    };
#pragma unroll
    for (int q = 0; q < S; ++q)
        if ((size_t)q < total)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                r[q][i] = ld<POL>((g4p)(addr(q) + 256 * i));
    for (size_t k = 0; k < total; k += S) {
#pragma unroll
        for (int q = 0; q < S; ++q) {
            if (k + q >= total)
                break;
            u32x4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                v[i] = r[q][i];
            if (k + q + S < total) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    r[q][i] = ld<POL>((g4p)(addr(k + q + S) + 256 * i));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

/* LDS-DMA: per wave a ring of 2 x D KiB; block t's D loads land while block
 * t-1 is read back. */
template <int D, int POL, int WG>
__global__ __launch_bounds__(WG) void glds(const char *buf, size_t n, unsigned *out)
{
    constexpr int W = WG / 64;
    __shared__ __attribute__((aligned(16))) char L[W * 2 * D * 1024];
    const size_t blk = (size_t)D * 1024;
    const int wv = threadIdx.x >> 6;
    const size_t wave = (size_t)blockIdx.x * W + wv;
    const size_t nw = (size_t)gridDim.x * W;
    const int lane = threadIdx.x & 63;
    const size_t nb = n / blk;
    char *ring = L + wv * 2 * D * 1024;
    unsigned acc = 0;
    int h = 0;
    size_t s = wave;
    if (s < nb) {
#pragma unroll
        for (int i = 0; i < D; ++i)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(buf + s * blk + 1024 * i + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(ring + 1024 * i), 16, 0,
                                             POL ? 2 : 0);
    }
    while (s < nb) {
        const size_t t = s + nw;
        char *nxt = ring + (h ^ 1) * D * 1024;
        if (t < nb) {
#pragma unroll
            for (int i = 0; i < D; ++i)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(buf + t * blk + 1024 * i + 16 * lane),
                                                 (__attribute__((address_space(3))) void *)(nxt + 1024 * i), 16, 0,
                                                 POL ? 2 : 0);
            /* the D loads of block s were issued before these D */
            __builtin_amdgcn_s_waitcnt(0x0F70 | (D & 15) | ((D >> 4) << 14)); /* vmcnt(D) */
        } else {
            __builtin_amdgcn_s_waitcnt(0x0F70); /* vmcnt(0) */
        }
        const char *cur = ring + h * D * 1024;
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const u32x4 v = *(const u32x4 *)(cur + 1024 * i + 16 * lane);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        h ^= 1;
        s = t;
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

template <typename K>
float timeit(K kern, int grid, int wg, const char *d, size_t n, unsigned *o, int reps)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), 0, 0, d, n, o);
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), 0, 0, d, n, o);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

static size_t g_n;
static const char *g_d;
static unsigned *g_o;
static int g_cu;

#define RUN(NAME, KERN, WGV)                                                                         \
    for (int mult : {1, 2, 4}) {                                                                     \
        const int grid = g_cu * mult * (1024 / (WGV));                                              \
        const float ms = timeit(KERN, grid, WGV, g_d, g_n, g_o, 10);                                 \
        printf("{\"case\": \"%s\", \"wg\": %d, \"grid\": %d, \"ms\": %.4f, \"GBs\": %.1f}\n", NAME, WGV, \
               grid, ms, g_n / ms / 1e6);                                                            \
        fflush(stdout);                                                                              \
    }

int main()
{
    g_n = (size_t)4 << 30;
    char *d;
    if (hipMalloc(&d, g_n) != hipSuccess || hipMalloc(&g_o, 64) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(d, 1, g_n);
    hipDeviceSynchronize();
    g_d = d;
    hipDeviceGetAttribute(&g_cu, hipDeviceAttributeMultiprocessorCount, 0);
    RUN("coal D1 nt", (coal<1, 1, 1024>), 1024);
    RUN("coal D2 nt", (coal<2, 1, 1024>), 1024);
    RUN("coal D4 nt", (coal<4, 1, 1024>), 1024);
    RUN("coal D8 nt", (coal<8, 1, 1024>), 1024);
    RUN("teamq S1 nt", (teamq<1, 1, 1024>), 1024);
    RUN("teamq S2 nt", (teamq<2, 1, 1024>), 1024);
    RUN("teamq S3 nt", (teamq<3, 1, 1024>), 1024);
    RUN("teamq S2 nt wg512", (teamq<2, 1, 512>), 512);
    RUN("teamq S4 nt wg512", (teamq<4, 1, 512>), 512);
    RUN("teamq S1 plain", (teamq<1, 0, 1024>), 1024);
    RUN("teamq S2 plain", (teamq<2, 0, 1024>), 1024);
    RUN("team S1 plain", (team<1, 0, 1024>), 1024);
    return 0;
}
