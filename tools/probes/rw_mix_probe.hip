// rw_mix_probe: config 2's memory floor without the hash.  Config 2 reads
// 4 GiB of 64-byte records per launch and writes 4 B per record (256 MiB of
// results, 1/16 of the bytes read).  This probe reads the same 4 GiB with
// multi64_kernel's load shape (eight coalesced non-temporal 1 KiB loads per
// 8 KiB chunk per wave, the next chunk in flight) and writes one dword per 64
// bytes read, in several shapes, to find what the read+write mix itself costs
// on this memory system.  Not product code.
//   read      : no stores (the read floor)
//   write     : the 256 MiB of results alone (coalesced 256-byte stores)
//   mix<G,P>  : a wave takes G consecutive chunks, keeps their results in
//               registers and writes them as one contiguous G x 512 B block
//               after the G chunks' reads (G = 1: two 256 B stores after every
//               chunk, the shipped shape).  P: store policy 0 plain, 1 sc1,
//               2 nt.
//   split<S>  : waves w % S == 0 only write (a write stream of their own at
//               the same rate), the others only read: reads and writes apart
//               in the CUs but not in time.
//   phase<Q>  : the launch in Q launches of 4 GiB / Q reads each, the results
//               of each written by the next launch's first waves (read and
//               write phases apart in time, per launch)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *g4p;

constexpr int WG = 1024, WAVES = WG / 64;
constexpr size_t CHUNK = 8192; /* 128 records of 64 B */

template <int P>
__device__ __forceinline__ void st(uint32_t *p, uint32_t v)
{
    if (P == 1)
        asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if (P == 2)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

__device__ __forceinline__ void ld(const char *b, size_t chunk, uint32_t voff, uint32_t (&w)[32])
{
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u32x4 v = __builtin_nontemporal_load((g4p)(b + chunk * CHUNK + voff + 1024u * i));
        w[4 * i] = v.x;
        w[4 * i + 1] = v.y;
        w[4 * i + 2] = v.z;
        w[4 * i + 3] = v.w;
    }
}

/* two per-lane "results" from a chunk's registers (cheap, not a CRC) */
__device__ __forceinline__ void fold(const uint32_t (&w)[32], uint32_t &r0, uint32_t &r1)
{
    uint32_t a = 0, b = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        a ^= w[k];
        b ^= w[16 + k];
    }
    r0 = a;
    r1 = b;
}

/* chunks [c0, c1) of the buffer; G consecutive chunks per wave step */
template <int G, int P, bool STORE>
__global__ __launch_bounds__(WG) void mix(const char *buf, size_t c0, size_t c1, uint32_t *out)
{
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const uint32_t voff = 64u * c + 16u * g;
    const size_t wave = (size_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * WAVES;
    const size_t groups = (c1 - c0) / G;
    uint32_t wa[32], wb[32];
    for (size_t q = wave; q < groups; q += nw) {
        const size_t base = c0 + q * G;
        uint32_t r[2 * G];
        ld(buf, base, voff, wa);
#pragma unroll
        for (int j = 0; j < G; j += 2) {
            if (j + 1 < G)
                ld(buf, base + j + 1, voff, wb);
            fold(wa, r[2 * j], r[2 * j + 1]);
            if (j + 2 < G)
                ld(buf, base + j + 2, voff, wa);
            if (j + 1 < G)
                fold(wb, r[2 * j + 2], r[2 * j + 3]);
        }
        if (STORE) {
#pragma unroll
            for (int j = 0; j < 2 * G; ++j)
                st<P>(out + base * 128 + 64 * j + lane, r[j]);
        } else {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 2 * G; ++j)
                x ^= r[j];
            if (x == 0x9E3779B9u)
                out[lane] = x;
        }
    }
}

/* results only: 256 B per wave instruction */
__global__ __launch_bounds__(WG) void wr(uint32_t *out, size_t words)
{
    const size_t wave = (size_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * WAVES;
    const int lane = threadIdx.x & 63;
    for (size_t s = wave; s * 64 < words; s += nw)
        out[s * 64 + lane] = (uint32_t)s;
}

/* waves w % S == 0 write (their share of the results), the rest read */
template <int S, bool W = true>
__global__ __launch_bounds__(WG) void split(const char *buf, size_t chunks, uint32_t *out)
{
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const uint32_t voff = 64u * c + 16u * g;
    const size_t wave = (size_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * WAVES;
    const size_t nwr = nw / S, nrd = nw - nwr;
    if (wave % S == 0) {
        if (!W)
            return;
        const size_t ww = wave / S;
        for (size_t s = ww; s < chunks * 2; s += nwr)
            out[s * 64 + lane] = (uint32_t)s;
        return;
    }
    const size_t rw = wave - wave / S - 1;
    uint32_t w[32], x = 0;
    for (size_t k = rw; k < chunks; k += nrd) {
        ld(buf, k, voff, w);
        uint32_t a, b;
        fold(w, a, b);
        x ^= a ^ b;
    }
    if (x == 0x9E3779B9u)
        out[lane] = x;
}


/* In-kernel phases: phase k's reads are chunks [k nw G, (k + 1) nw G) (wave w
 * its G consecutive ones), results held in registers; a grid barrier (every
 * workgroup resident: one 1,024-thread workgroup per CU) after the phase's
 * reads; then every wave writes its G x 512 B.  B2: a second barrier after
 * the writes, so no read of phase k + 1 overlaps them.  The barrier spins on
 * a device-scope counter that only grows (base = launches so far x barriers
 * per launch x workgroups); a spin gives up after ~50 ms (no hang). */
__device__ __forceinline__ void grid_bar(unsigned long long *ctr, unsigned long long target)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull)
                break;
        }
    }
    __syncthreads();
}

template <int G, bool B2, bool BAR = true>
__global__ __launch_bounds__(WG) void phased(const char *buf, size_t chunks, uint32_t *out, unsigned long long *ctr,
                                             unsigned long long base)
{
    __shared__ uint32_t SL[WAVES * 2 * G * 64]; /* the phase's results, per wave */
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const uint32_t voff = 64u * c + 16u * g;
    const size_t wave = (size_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * WAVES;
    const size_t per = nw * G, nph = chunks / per;
    uint32_t *S = SL + (threadIdx.x >> 6) * 2 * G * 64;
    unsigned long long tgt = base;
    uint32_t wa[32], wb[32];
    for (size_t k = 0; k < nph; ++k) {
        const size_t c0 = k * per + wave * G;
        ld(buf, c0, voff, wa);
#pragma unroll 1
        for (int j = 0; j < G; j += 2) {
            ld(buf, c0 + j + 1, voff, wb);
            __builtin_amdgcn_sched_barrier(0);
            uint32_t r0, r1;
            fold(wa, r0, r1);
            S[128 * j + lane] = r0;
            S[128 * j + 64 + lane] = r1;
            if (j + 2 < G)
                ld(buf, c0 + j + 2, voff, wa);
            __builtin_amdgcn_sched_barrier(0);
            fold(wb, r0, r1);
            S[128 * j + 128 + lane] = r0;
            S[128 * j + 192 + lane] = r1;
        }
        tgt += gridDim.x;
        if (BAR)
            grid_bar(ctr, tgt);
#pragma unroll 4
        for (int j = 0; j < 2 * G; ++j)
            st<1>(out + c0 * 128 + 64 * j + lane, S[64 * j + lane]);
        if (B2) {
            tgt += gridDim.x;
            grid_bar(ctr, tgt);
        } else {
            __syncthreads();
        }
    }
}


/* scratch -> out, 256 B per wave instruction */
__global__ __launch_bounds__(WG) void cp(const uint32_t *src, uint32_t *dst, size_t words)
{
    const size_t wave = (size_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * WAVES;
    const int lane = threadIdx.x & 63;
    for (size_t s = wave; s * 64 < words; s += nw)
        dst[s * 64 + lane] = src[s * 64 + lane];
}

/* mix<2, 0, true> over chunks [c0, c1), results to scratch at (chunk - c0) */
__global__ __launch_bounds__(WG) void mix_to(const char *buf, size_t c0, size_t c1, uint32_t *scr)
{
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const uint32_t voff = 64u * c + 16u * g;
    const size_t wave = (size_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * WAVES;
    uint32_t wa[32], wb[32];
    for (size_t q = wave; 2 * q < c1 - c0; q += nw) {
        const size_t k = c0 + 2 * q;
        uint32_t r0, r1, r2, r3;
        ld(buf, k, voff, wa);
        ld(buf, k + 1, voff, wb);
        fold(wa, r0, r1);
        fold(wb, r2, r3);
        uint32_t *o = scr + (k - c0) * 128 + lane;
        o[0] = r0;
        o[64] = r1;
        o[128] = r2;
        o[192] = r3;
    }
}

template <typename F>
float timeit(F f, int reps = 10)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i)
        f();
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    hipEventDestroy(a);
    hipEventDestroy(b);
    return t[t.size() / 2];
}

int main(int argc, char **argv)
{
    const size_t n = (size_t)4 << 30, chunks = n / CHUNK, words = n / 16;
    char *d;
    uint32_t *o;
    if (hipMalloc(&d, n) != hipSuccess || hipMalloc(&o, words * 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(d, 1, n);
    hipMemset(o, 0, words * 4);
    hipDeviceSynchronize();
    int cu = 0;
    hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cu;
    if (argc > 1) { /* one case, N launches, for the PMC passes (rocprofv3 --pmc) */
        const std::string c = argv[1];
        const int reps = argc > 2 ? atoi(argv[2]) : 5;
        for (int r = 0; r < reps; ++r) {
            if (c == "read")
                hipLaunchKernelGGL((mix<2, 0, false>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o);
            else if (c == "mix_g1_sc1")
                hipLaunchKernelGGL((mix<1, 1, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o);
            else if (c == "mix_g1_plain")
                hipLaunchKernelGGL((mix<1, 0, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o);
            else if (c == "phase_4")
                for (int k = 0; k < 4; ++k) {
                    hipLaunchKernelGGL((mix<2, 0, false>), dim3(grid), dim3(WG), 0, 0, d, chunks / 4 * k,
                                       chunks / 4 * (k + 1), o);
                    hipLaunchKernelGGL(wr, dim3(grid), dim3(WG), 0, 0, o + chunks / 4 * 128 * k, chunks / 4 * 128);
                }
            else {
                printf("unknown case %s\n", c.c_str());
                return 2;
            }
        }
        (void)hipDeviceSynchronize();
        printf("{\"case\": \"%s\", \"launches\": %d}\n", c.c_str(), reps);
        return 0;
    }
    auto line = [&](const char *name, float ms) {
        printf("{\"case\": \"%s\", \"ms\": %.4f, \"read_GBs\": %.1f, \"total_GBs\": %.1f}\n", name, ms, n / ms / 1e6,
               (n + words * 4) / ms / 1e6);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        line("read", timeit([&] { hipLaunchKernelGGL((mix<2, 0, false>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("write", timeit([&] { hipLaunchKernelGGL(wr, dim3(grid), dim3(WG), 0, 0, o, words); }));
        line("mix_g1_plain", timeit([&] { hipLaunchKernelGGL((mix<1, 0, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("mix_g1_sc1", timeit([&] { hipLaunchKernelGGL((mix<1, 1, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("mix_g2_sc1", timeit([&] { hipLaunchKernelGGL((mix<2, 1, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("mix_g8_plain", timeit([&] { hipLaunchKernelGGL((mix<8, 0, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("mix_g8_sc1", timeit([&] { hipLaunchKernelGGL((mix<8, 1, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("mix_g8_nt", timeit([&] { hipLaunchKernelGGL((mix<8, 2, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("mix_g16_sc1", timeit([&] { hipLaunchKernelGGL((mix<16, 1, true>), dim3(grid), dim3(WG), 0, 0, d, 0, chunks, o); }));
        line("split_16", timeit([&] { hipLaunchKernelGGL((split<16>), dim3(grid), dim3(WG), 0, 0, d, chunks, o); }));
        line("split_16_readers_only", timeit([&] { hipLaunchKernelGGL((split<16, false>), dim3(grid), dim3(WG), 0, 0, d, chunks, o); }));
        line("split_8", timeit([&] { hipLaunchKernelGGL((split<8>), dim3(grid), dim3(WG), 0, 0, d, chunks, o); }));

        {
            unsigned long long *ctr;
            unsigned long long bases = 0;
            (void)hipMalloc(&ctr, 8);
            (void)hipMemset(ctr, 0, 8);
            const size_t nw = (size_t)grid * WAVES;
            line("phased_g16", timeit([&] {
                     hipLaunchKernelGGL((phased<16, false>), dim3(grid), dim3(WG), 0, 0, d, chunks, o, ctr, bases);
                     bases += (chunks / (nw * 16)) * grid;
                 }));
            line("phased_g16_b2", timeit([&] {
                     hipLaunchKernelGGL((phased<16, true>), dim3(grid), dim3(WG), 0, 0, d, chunks, o, ctr, bases);
                     bases += 2 * (chunks / (nw * 16)) * grid;
                 }));
            line("phased_g8", timeit([&] {
                     hipLaunchKernelGGL((phased<8, false>), dim3(grid), dim3(WG), 0, 0, d, chunks, o, ctr, bases);
                     bases += (chunks / (nw * 8)) * grid;
                 }));
            line("phased_g4", timeit([&] {
                     hipLaunchKernelGGL((phased<4, false>), dim3(grid), dim3(WG), 0, 0, d, chunks, o, ctr, bases);
                     bases += (chunks / (nw * 4)) * grid;
                 }));
            line("staged_g16_nobarrier", timeit([&] {
                     hipLaunchKernelGGL((phased<16, false, false>), dim3(grid), dim3(WG), 0, 0, d, chunks, o, ctr, 0ull);
                 }));
            unsigned long long got = 0;
            (void)hipMemcpy(&got, ctr, 8, hipMemcpyDeviceToHost);
            printf("{\"case\": \"barrier_check\", \"ctr\": %llu, \"expected\": %llu}\n", got, bases);
            (void)hipFree(ctr);
        }
        for (int Q : {4, 16}) {
            char name[32];
            snprintf(name, sizeof name, "phase_scratch_%d", Q);
            const size_t per = chunks / Q;
            uint32_t *scr;
            (void)hipMalloc(&scr, per * 128 * 4);
            line(name, timeit([&] {
                     for (int k = 0; k < Q; ++k) {
                         hipLaunchKernelGGL(mix_to, dim3(grid), dim3(WG), 0, 0, d, per * k, per * (k + 1), scr);
                         hipLaunchKernelGGL(cp, dim3(grid), dim3(WG), 0, 0, scr, o + per * 128 * k, per * 128);
                     }
                 }));
            snprintf(name, sizeof name, "mix_to_direct_%d", Q);
            line(name, timeit([&] {
                     for (int k = 0; k < Q; ++k)
                         hipLaunchKernelGGL(mix_to, dim3(grid), dim3(WG), 0, 0, d, per * k, per * (k + 1), o + per * 128 * k);
                 }));
            (void)hipFree(scr);
        }
        for (int Q : {4, 16, 64}) {
            char name[32];
            snprintf(name, sizeof name, "phase_%d", Q);
            line(name, timeit([&] {
                     const size_t per = chunks / Q;
                     for (int k = 0; k < Q; ++k) {
                         hipLaunchKernelGGL((mix<2, 0, false>), dim3(grid), dim3(WG), 0, 0, d, per * k, per * (k + 1), o);
                         hipLaunchKernelGGL(wr, dim3(grid), dim3(WG), 0, 0, o + per * 128 * k, per * 128);
                     }
                 }));
        }
    }
    return 0;
}
