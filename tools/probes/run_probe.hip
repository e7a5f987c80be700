// run_probe: where config 4's run rounds (burst_kernel run_issue/run_hash)
// lose time.  10 M back-to-back 320-byte grids (3.2 GB); a wave takes 64 of
// them (20 KiB) per round as 20 coalesced 1 KiB loads.  Load-only and
// load+hash forms at 8 waves per CU with the next round in flight (the
// product's shape) and at 16 waves per CU with one round per wave, with the
// per-record descriptor loads and result stores of a commit batch (plain,
// non-temporal, one or two per record).  The hash is the run rounds' chain work (five
// chains x 16 words of slice-by-4 from 32-replica LDS tables); results are
// XOR-folded.  Measurement tooling, not product code.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *g4p;

constexpr size_t NREC = 10000000, GRID = 320;

__device__ __forceinline__ unsigned lds32(const char *L, unsigned a) { return *(const unsigned *)(L + a); }
__device__ __forceinline__ unsigned m4(const char *L, unsigned x, unsigned c_lo, unsigned c_hi)
{
    const unsigned a0 = __builtin_amdgcn_perm(x, c_lo, 0x0C020400u);
    const unsigned a1 = __builtin_amdgcn_perm(x, c_lo, 0x0C020500u);
    const unsigned a2 = __builtin_amdgcn_perm(x, c_hi, 0x0C020600u);
    const unsigned a3 = __builtin_amdgcn_perm(x, c_hi, 0x0C020700u);
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(lds32(L, a0), lds32(L, a1 + 128), lds32(L, a2), 0x96),
                                       lds32(L, a3 + 128), 0u, 0x96);
}

template <bool NT = true>
__device__ __forceinline__ void issue(const char *buf, size_t round, unsigned voff, unsigned (&w)[5][16])
{
    const char *V = buf + round * 64 * GRID;
#pragma unroll
    for (int p = 0; p < 5; ++p)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const g4p a = (g4p)(V + 4096 * p + 1024 * t + voff);
            const u32x4 v = NT ? __builtin_nontemporal_load(a) : *a;
            w[p][4 * t] = v.x;
            w[p][4 * t + 1] = v.y;
            w[p][4 * t + 2] = v.z;
            w[p][4 * t + 3] = v.w;
        }
}

template <int HASH>
__device__ __forceinline__ unsigned consume(const char *L, unsigned (&w)[5][16], unsigned c_lo, unsigned c_hi)
{
    if (!HASH) {
        unsigned a = 0;
#pragma unroll
        for (int p = 0; p < 5; ++p)
#pragma unroll
            for (int k = 0; k < 16; ++k)
                a ^= w[p][k];
        return a;
    }
    unsigned y[5];
#pragma unroll
    for (int p = 0; p < 5; ++p)
        y[p] = w[p][0];
#pragma unroll
    for (int k = 1; k < 16; ++k)
#pragma unroll
        for (int p = 0; p < 5; ++p)
            y[p] = m4(L, y[p], c_lo, c_hi) ^ w[p][k];
    return y[0] ^ y[1] ^ y[2] ^ y[3] ^ y[4];
}

__device__ void fill(char *L)
{
    for (int i = threadIdx.x; i < 32768; i += blockDim.x)
        ((unsigned *)L)[i] = i * 2654435761u;
    __syncthreads();
}

/* DB = 1: next round in flight (two buffers); DB = 0: one round per wave.
 * X & 1: per-record descriptor loads (off, len: 16 B per lane, issued with
 * the round's data); X & 2: two coalesced result stores per record (the
 * product's out / status) */
template <int WG, int DB, int HASH, int X = 0>
__global__ __launch_bounds__(WG) void run_probe(const char *buf, unsigned *out)
{
    typedef const __attribute__((address_space(1))) unsigned long long *g64p;
    typedef __attribute__((address_space(1))) unsigned *gw32p;
    const g64p desc = (g64p)(buf + NREC * GRID);
    __shared__ __attribute__((aligned(16))) char L[131072];
    if (HASH)
        fill(L);
    const int lane = threadIdx.x & 63;
    const unsigned voff = 64u * (lane & 15) + 16u * (lane >> 4);
    const unsigned c_lo = (unsigned)(lane & 31) << 2, c_hi = c_lo | 0x10000u;
    size_t nw = (size_t)gridDim.x * (WG / 64);
    size_t r = (size_t)blockIdx.x * (WG / 64) + (threadIdx.x >> 6);
    size_t rend = NREC / 64;
    if (X & 64) { /* blocked: wave w takes rounds [w R, (w + 1) R), one after another */
        const size_t R = (NREC / 64 + nw - 1) / nw;
        r = r * R;
        rend = r + R < NREC / 64 ? r + R : NREC / 64;
        nw = 1;
    }
    unsigned acc = 0;
    unsigned a[5][16], b[5][16];
    if (DB) {
        if (r < rend)
            issue(buf, r, voff, a);
        while (r < rend) {
            const size_t s = r + nw;
            if (s < rend)
                issue(buf, s, voff, b);
            acc ^= consume<HASH>(L, a, c_lo, c_hi);
            r = s;
            if (r >= rend)
                break;
            const size_t t = r + nw;
            if (t < rend)
                issue(buf, t, voff, a);
            acc ^= consume<HASH>(L, b, c_lo, c_hi);
            r = t;
        }
    } else if (X & 16) {
        /* results stored one round late: issued after the next round's loads,
         * so waiting for those loads never waits for the stores */
        unsigned ph = 0;
        size_t pr = ~(size_t)0;
        for (; r < rend; r += nw) {
            issue(buf, r, voff, a);
            if (pr != ~(size_t)0) {
                ((gw32p)out)[16 + pr * 64 + lane] = ph;
                ((gw32p)out)[16 + NREC + pr * 64 + lane] = ph >> 1;
            }
            ph = consume<HASH>(L, a, c_lo, c_hi);
            pr = r;
        }
        if (pr != ~(size_t)0) {
            ((gw32p)out)[16 + pr * 64 + lane] = ph;
            ((gw32p)out)[16 + NREC + pr * 64 + lane] = ph >> 1;
        }
    } else {
        for (; r < rend; r += nw) {
            unsigned long long o = 0, l = 0;
            if (X & 1) {
                o = desc[r * 64 + lane];
                l = desc[NREC + r * 64 + lane];
            }
            issue<!(X & 8192)>(buf, r, voff, a);
            const unsigned h = consume<HASH>(L, a, c_lo, c_hi) ^ (unsigned)o ^ (unsigned)l;
            if (X & 1024) { /* the whole 128 B L2 line holding the record's CRC field */
                typedef __attribute__((address_space(1))) u32x4 *gw4p;
                char *R = (char *)buf + (r * 64 + lane) * GRID;
                char *C = (char *)((uintptr_t)(R + 316) & ~(uintptr_t)127);
                const u32x4 v = {h, h >> 1, h >> 2, h >> 3};
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    *(gw4p)(C + 16 * k) = v;
            } else if (X & (128 | 256 | 512)) { /* in place, at the record's own commit word */
                typedef __attribute__((address_space(1))) u32x4 *gw4p;
                char *R = (char *)buf + (r * 64 + lane) * GRID;
                const u32x4 v = {h, h >> 1, h >> 2, h >> 3};
                if (X & 128) /* one 4-byte CRC field: a partial 32 B sector */
                    *(gw32p)(R + 316) = h;
                else if (X & 256) { /* the whole 32 B sector holding it */
                    *(gw4p)(R + 288) = v;
                    *(gw4p)(R + 304) = v;
                } else { /* the whole 64 B line holding it */
                    *(gw4p)(R + 256) = v;
                    *(gw4p)(R + 272) = v;
                    *(gw4p)(R + 288) = v;
                    *(gw4p)(R + 304) = v;
                }
            } else if (X & 32) { /* stores to a 16 KiB region: L2-resident, no HBM writes */
                ((gw32p)out)[16 + (r & 63) * 64 + lane] = h;
            } else if (X & 4) { /* non-temporal result stores */
                __builtin_nontemporal_store(h, (gw32p)out + 16 + r * 64 + lane);
                __builtin_nontemporal_store(h >> 1, (gw32p)out + 16 + NREC + r * 64 + lane);
            } else if (X & 8) { /* one store per record */
                ((gw32p)out)[16 + r * 64 + lane] = h;
            } else if (X & 2) {
                ((gw32p)out)[16 + r * 64 + lane] = h;
                ((gw32p)out)[16 + NREC + r * 64 + lane] = h >> 1;
            } else {
                acc ^= h;
            }
        }
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

/* the writer's stores alone: 10 M in-place stores into the records' CRC
 * fields (W = 4: the 4-byte field; 128: the whole 128 B line holding it), no
 * reads -- what a separate scatter launch after a read-only pass would cost */
template <int W>
__global__ __launch_bounds__(1024) void scatter_probe(const char *buf, unsigned *o)
{
    typedef __attribute__((address_space(1))) u32x4 *gw4p;
    typedef __attribute__((address_space(1))) unsigned *gw32p;
    const size_t nt = (size_t)gridDim.x * blockDim.x;
    for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < NREC; r += nt) {
        char *R = (char *)buf + r * GRID;
        const unsigned h = (unsigned)r * 2654435761u;
        if (W == 4) {
            *(gw32p)(R + 316) = h;
        } else {
            char *C = (char *)((uintptr_t)(R + 316) & ~(uintptr_t)127);
            const u32x4 v = {h, h >> 1, h >> 2, h >> 3};
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *(gw4p)(C + 16 * k) = v;
        }
    }
}

template <typename F>
float timeit(F kern, int grid, int wg, const char *d, unsigned *o)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 5; ++i)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), 0, 0, d, o);
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), 0, 0, d, o);
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
    char *d;
    unsigned *o;
    const size_t n = NREC * GRID;
    if (hipMalloc(&d, n + 16 * NREC + 65536) != hipSuccess || hipMalloc(&o, 64 + 8 * NREC + 64) != hipSuccess)
        return 1;
    (void)hipMemset(d, 3, n + 16 * NREC + 65536);
    (void)hipDeviceSynchronize();
    int cu = 0;
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    struct {
        const char *name;
        float ms;
    } r[] = {
        {"load 8w db", timeit(run_probe<512, 1, 0>, cu, 512, d, o)},
        {"load 16w sb", timeit(run_probe<1024, 0, 0>, cu, 1024, d, o)},
        {"load 8w sb", timeit(run_probe<512, 0, 0>, cu, 512, d, o)},
        {"hash 8w db", timeit(run_probe<512, 1, 1>, cu, 512, d, o)},
        {"hash 16w sb", timeit(run_probe<1024, 0, 1>, cu, 1024, d, o)},
        {"hash 8w sb", timeit(run_probe<512, 0, 1>, cu, 512, d, o)},
        {"hash 8w db x2grid", timeit(run_probe<512, 1, 1>, 2 * cu, 512, d, o)},
        {"hash 8w sb +desc", timeit(run_probe<512, 0, 1, 1>, cu, 512, d, o)},
        {"hash 8w sb +stores", timeit(run_probe<512, 0, 1, 2>, cu, 512, d, o)},
        {"hash 8w sb +desc+stores", timeit(run_probe<512, 0, 1, 3>, cu, 512, d, o)},
        {"hash 8w sb +nt stores", timeit(run_probe<512, 0, 1, 4>, cu, 512, d, o)},
        {"hash 8w sb +1 store", timeit(run_probe<512, 0, 1, 8>, cu, 512, d, o)},
        {"load 8w sb +stores", timeit(run_probe<512, 0, 0, 2>, cu, 512, d, o)},
        {"load 8w sb +nt stores", timeit(run_probe<512, 0, 0, 4>, cu, 512, d, o)},
        {"hash 8w sb +late stores", timeit(run_probe<512, 0, 1, 16>, cu, 512, d, o)},
        {"hash 16w sb +late stores", timeit(run_probe<1024, 0, 1, 16>, cu, 1024, d, o)},
        {"hash 8w sb (again)", timeit(run_probe<512, 0, 1>, cu, 512, d, o)},
        {"hash 8w sb +L2 stores", timeit(run_probe<512, 0, 1, 32>, cu, 512, d, o)},
        {"hash 8w sb blocked", timeit(run_probe<512, 0, 1, 64>, cu, 512, d, o)},
        {"hash 8w sb blocked +stores", timeit(run_probe<512, 0, 1, 66>, cu, 512, d, o)},
        {"hash 8w sb +inplace 4B", timeit(run_probe<512, 0, 1, 128>, cu, 512, d, o)},
        {"hash 8w sb +inplace 32B sector", timeit(run_probe<512, 0, 1, 256>, cu, 512, d, o)},
        {"hash 8w sb +inplace 64B line", timeit(run_probe<512, 0, 1, 512>, cu, 512, d, o)},
        {"hash 8w sb +inplace 128B line", timeit(run_probe<512, 0, 1, 1024>, cu, 512, d, o)},
        {"hash 8w sb plain loads", timeit(run_probe<512, 0, 1, 8192>, cu, 512, d, o)},
        {"hash 8w sb plain loads +inplace 4B", timeit(run_probe<512, 0, 1, 8192 | 128>, cu, 512, d, o)},
        {"hash 8w sb plain loads +inplace 128B line", timeit(run_probe<512, 0, 1, 8192 | 1024>, cu, 512, d, o)},
        {"scatter only: 4 B CRC fields", timeit(scatter_probe<4>, 4 * cu, 1024, d, o)},
        {"scatter only: 128 B lines", timeit(scatter_probe<128>, 4 * cu, 1024, d, o)},
        {"hash 8w sb (end)", timeit(run_probe<512, 0, 1>, cu, 512, d, o)},
    };
    for (auto &x : r)
        printf("{\"case\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f}\n", x.name, x.ms, (double)n / x.ms / 1e6);
    return 0;
}
