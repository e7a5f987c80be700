/*
 * zs_oracle.c -- CPU restatement of zeroskip's CRC32C (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the *checker*.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product (zeroskip_amd/,
 * libzscrc.so) never links or calls it.
 *
 * It restates, without copying, the algorithms of the reference
 * /root/reference/src/crc32c.c:
 *   - oracle_crc32c_sw : slice-by-4 over little-endian 32-bit words, byte tail
 *                        (crc32c.c:613-645, tables crc32c_lookup :459-596).
 *   - oracle_crc32c_hw : SSE4.2 crc32 instruction, align-to-8 head, 3-way
 *                        interleave over 3x8192 then 3x256 byte blocks merged
 *                        with "shift by zeros" operator tables, 8-byte words,
 *                        byte tail (crc32c.c:370-453, crc32c_shift :363-367,
 *                        zero-operator tables crc32c_long/short :85-360).
 *   - oracle_crc32c    : dispatch as crc32c.c:675-684 (sw unless init saw SSE4.2).
 *   - map / iovec / cstring / buf wrappers (crc32c.c:686-711).
 * Every table is *generated* here from the Castagnoli polynomial instead of
 * being transcribed, and an independent bit-at-a-time definition
 * (oracle_crc32c_bitwise) is kept alongside to cross-check all of them.
 *
 * Parity pinning: the reference's crc32c.c cannot be compiled here as-is
 * (it includes the autoconf-generated <config.h>, which this image cannot
 * produce), so this restatement is pinned by the reference's own known answer
 * (tests/unit-crc32c.c:36, crc32c("lorem ipsum") = 0xdfb4e6c9, also chained)
 * and by the published CRC-32C check vectors (see tests/golden/).
 */
#define _GNU_SOURCE /* pthread_setaffinity_np (the bench leg's pinned threads) */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#if defined(__x86_64__)
#include <emmintrin.h>
#endif
#include <sys/uio.h>
#include <pthread.h>
#include <time.h>

#define POLY 0x82F63B78u /* reflected Castagnoli polynomial */

/* ---------------------------------------------------------------- tables */
static uint32_t g_sb4[4][256];     /* slice-by-4: g_sb4[k][b] = byte b then k zero bytes */
static uint32_t g_zlong[4][256];   /* shift register by 8192 zero bytes (crc32c.c LONG)  */
static uint32_t g_zshort[4][256];  /* shift register by 256 zero bytes (crc32c.c SHORT)  */
static int g_ready;
static int g_have_sse42;           /* mirrors have_sse42, crc32c.c:665 */

/* One zero bit through the reflected register. */
static inline uint32_t step_bit(uint32_t r) { return (r >> 1) ^ ((r & 1u) ? POLY : 0u); }

/* GF(2) product of two reflected residues (bit 31 == x^0). */
static uint32_t gf2_mul(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 31; i >= 0; --i) {
        if (a & (1u << i))
            p ^= b;
        b = step_bit(b);
    }
    return p;
}

/* x^(8*n) mod P, reflected. */
static uint32_t xpow8n(uint64_t n)
{
    uint32_t result = 0x80000000u; /* x^0 */
    uint32_t sq = 0x00800000u;     /* x^8 */
    while (n) {
        if (n & 1)
            result = gf2_mul(result, sq);
        sq = gf2_mul(sq, sq);
        n >>= 1;
    }
    return result;
}

/* Register after n zero bytes. */
uint32_t oracle_shift(uint32_t reg, uint64_t nbytes) { return gf2_mul(xpow8n(nbytes), reg); }

static void build_zero_table(uint32_t t[4][256], uint64_t nbytes)
{
    uint32_t m = xpow8n(nbytes);
    for (int j = 0; j < 4; ++j)
        for (int b = 0; b < 256; ++b)
            t[j][b] = gf2_mul(m, (uint32_t)b << (8 * j));
}

static void oracle_init_tables(void)
{
    if (g_ready)
        return;
    for (int b = 0; b < 256; ++b) {
        uint32_t r = (uint32_t)b;
        for (int i = 0; i < 8; ++i)
            r = step_bit(r);
        g_sb4[0][b] = r;
    }
    for (int k = 1; k < 4; ++k)
        for (int b = 0; b < 256; ++b)
            g_sb4[k][b] = g_sb4[0][g_sb4[k - 1][b] & 0xff] ^ (g_sb4[k - 1][b] >> 8);
    build_zero_table(g_zlong, 8192);
    build_zero_table(g_zshort, 256);
#if defined(__x86_64__) || defined(__i386__)
    __builtin_cpu_init();
    g_have_sse42 = __builtin_cpu_supports("sse4.2");
#endif
    g_ready = 1;
}

void oracle_get_sb4(uint32_t out[4][256])
{
    oracle_init_tables();
    memcpy(out, g_sb4, sizeof(g_sb4));
}

/* ---------------------------------------------------------------- bitwise */
uint32_t oracle_crc32c_bitwise(uint32_t crc, const void *buf, size_t len)
{
    const uint8_t *p = buf;
    uint32_t r = ~crc;
    while (len--) {
        r ^= *p++;
        for (int i = 0; i < 8; ++i)
            r = step_bit(r);
    }
    return ~r;
}

/* ------------------------------------------------------ sw: crc32c.c:613-645 */
uint32_t oracle_crc32c_sw(uint32_t crc, const void *buf, size_t len)
{
    oracle_init_tables();
    const uint8_t *p = buf;
    uint32_t r = crc ^ 0xffffffffu;
    while (len >= 4) {
        uint32_t w;
        memcpy(&w, p, 4); /* the reference reads an unaligned uint32_t* here */
        w ^= r;
        r = g_sb4[0][w >> 24] ^ g_sb4[1][(w >> 16) & 0xff] ^
            g_sb4[2][(w >> 8) & 0xff] ^ g_sb4[3][w & 0xff];
        p += 4;
        len -= 4;
    }
    while (len--)
        r = (r >> 8) ^ g_sb4[0][(r ^ *p++) & 0xff];
    return r ^ 0xffffffffu;
}

/* ------------------------------------------------------ hw: crc32c.c:370-453 */
static inline uint32_t zero_shift(const uint32_t t[4][256], uint32_t r)
{
    return t[0][r & 0xff] ^ t[1][(r >> 8) & 0xff] ^ t[2][(r >> 16) & 0xff] ^ t[3][r >> 24];
}

#if defined(__x86_64__)
__attribute__((target("sse4.2")))
static uint32_t crc32c_hw_impl(uint32_t crc, const void *buf, size_t len)
{
    const uint8_t *next = buf;
    uint64_t c0 = crc ^ 0xffffffffu, c1, c2;
    enum { LONGB = 8192, SHORTB = 256 };

    while (len && ((uintptr_t)next & 7)) {
        c0 = __builtin_ia32_crc32qi((uint32_t)c0, *next++);
        --len;
    }
    while (len >= 3 * LONGB) {
        const uint8_t *end = next + LONGB;
        c1 = c2 = 0;
        do {
            uint64_t a, b, c;
            memcpy(&a, next, 8);
            memcpy(&b, next + LONGB, 8);
            memcpy(&c, next + 2 * LONGB, 8);
            c0 = __builtin_ia32_crc32di(c0, a);
            c1 = __builtin_ia32_crc32di(c1, b);
            c2 = __builtin_ia32_crc32di(c2, c);
            next += 8;
        } while (next < end);
        c0 = zero_shift(g_zlong, (uint32_t)c0) ^ c1;
        c0 = zero_shift(g_zlong, (uint32_t)c0) ^ c2;
        next += 2 * LONGB;
        len -= 3 * LONGB;
    }
    while (len >= 3 * SHORTB) {
        const uint8_t *end = next + SHORTB;
        c1 = c2 = 0;
        do {
            uint64_t a, b, c;
            memcpy(&a, next, 8);
            memcpy(&b, next + SHORTB, 8);
            memcpy(&c, next + 2 * SHORTB, 8);
            c0 = __builtin_ia32_crc32di(c0, a);
            c1 = __builtin_ia32_crc32di(c1, b);
            c2 = __builtin_ia32_crc32di(c2, c);
            next += 8;
        } while (next < end);
        c0 = zero_shift(g_zshort, (uint32_t)c0) ^ c1;
        c0 = zero_shift(g_zshort, (uint32_t)c0) ^ c2;
        next += 2 * SHORTB;
        len -= 3 * SHORTB;
    }
    while (len >= 8) {
        uint64_t a;
        memcpy(&a, next, 8);
        c0 = __builtin_ia32_crc32di(c0, a);
        next += 8;
        len -= 8;
    }
    while (len--)
        c0 = __builtin_ia32_crc32qi((uint32_t)c0, *next++);
    return (uint32_t)c0 ^ 0xffffffffu;
}
#endif

int oracle_have_sse42(void)
{
    oracle_init_tables();
    return g_have_sse42;
}

uint32_t oracle_crc32c_hw(uint32_t crc, const void *buf, size_t len)
{
    oracle_init_tables();
#if defined(__x86_64__)
    if (g_have_sse42)
        return crc32c_hw_impl(crc, buf, len);
#endif
    return oracle_crc32c_sw(crc, buf, len); /* same function, no SSE4.2 on this host */
}

/* ------------------------------------------------- dispatch: crc32c.c:668-684 */
static int g_init_called;
void oracle_crc32c_init(void)
{
    oracle_init_tables();
    g_init_called = g_have_sse42;
}

uint32_t oracle_crc32c(uint32_t crc, const void *buf, size_t len)
{
    return g_init_called ? oracle_crc32c_hw(crc, buf, len) : oracle_crc32c_sw(crc, buf, len);
}

/* ------------------------------------------------- wrappers: crc32c.c:686-711 */
uint32_t oracle_crc32c_map(const char *base, unsigned len)
{
    return oracle_crc32c(0, base, (size_t)len);
}

uint32_t oracle_crc32c_iovec(const struct iovec *iov, int iovcnt)
{
    uint32_t crc = oracle_crc32c(0, 0, 0);
    for (int n = 0; n < iovcnt; ++n)
        if (iov[n].iov_len)
            crc = oracle_crc32c(crc, iov[n].iov_base, iov[n].iov_len);
    return crc;
}

uint32_t oracle_crc32c_buf(const char *buf) { return oracle_crc32c_map(buf, (unsigned)strlen(buf)); }

/* crc(A||B) from crc(A), crc(B), |B| (used by tests for chaining checks). */
uint32_t oracle_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    oracle_init_tables();
    return oracle_shift(crc_a, len_b) ^ crc_b;
}

/* ------------------------------------------------------------------ batches */
/* out[i] = crc32c(seed_i, base + off_i, len_i).  off/len/seed may be NULL,
 * in which case record i sits at i*stride with length fixed_len and seed 0.
 * impl: 0 = sw, 1 = hw, 2 = bitwise.  Used as checker and as the bench
 * cpu_baseline ("port") leg. */
struct batch_job {
    const uint8_t *base;
    const uint64_t *off, *len;
    const uint32_t *seed;
    uint32_t *out;
    uint64_t lo, hi, stride, fixed_len;
    int impl;
};

static void *batch_worker(void *arg)
{
    struct batch_job *j = arg;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint8_t *p = j->base + (j->off ? j->off[i] : i * j->stride);
        uint64_t n = j->len ? j->len[i] : j->fixed_len;
        uint32_t s = j->seed ? j->seed[i] : 0;
        j->out[i] = j->impl == 1 ? oracle_crc32c_hw(s, p, n)
                  : j->impl == 2 ? oracle_crc32c_bitwise(s, p, n)
                                 : oracle_crc32c_sw(s, p, n);
    }
    return NULL;
}

int oracle_batch(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                 const uint32_t *seed, uint32_t *out, uint64_t n, uint64_t stride,
                 uint64_t fixed_len, int impl, int nthreads)
{
    oracle_init_tables();
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    struct batch_job jobs[256];
    uint64_t per = (n + nthreads - 1) / nthreads;
    int started = 0;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (struct batch_job){base, off, len, seed, out, t * per,
                                     (t + 1) * per < n ? (t + 1) * per : n, stride, fixed_len, impl};
        if (jobs[t].lo >= jobs[t].hi)
            break;
        if (t == 0)
            continue;
        if (pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0)
            return -1;
        started = t;
    }
    if (jobs[0].lo < jobs[0].hi)
        batch_worker(&jobs[0]);
    for (int t = 1; t <= started; ++t)
        pthread_join(th[t], NULL);
    return 0;
}

/* Seconds on CLOCK_MONOTONIC (bench timing helper). */
double oracle_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* --------------------------------------------- the bench's all-core timing leg
 * oracle_batch splits a batch by record count and starts its threads on every
 * call: a sample holding one long span runs on one thread, and a small sample
 * pays the thread starts each call.  This leg times the same batch as
 * bench.py's cpu_baseline measures it: the records are laid end to end as one
 * byte stream, each of nthreads persistent threads (optionally pinned to
 * cpus[t]) owns an equal byte range of it, a record cut by a range boundary
 * is hashed in pieces (the first from its seed, the others from 0) and the
 * pieces joined by the zero shift (crc32c_shift, crc32c.c:363-367; combine
 * as oracle_combine).  Passes repeat, a barrier between them, until `budget`
 * seconds have gone; out[] holds the last pass's CRCs.  mode 0 = crc32c
 * (impl as oracle_batch), 3 = read only (64-bit sums of the same bytes: the
 * host memory's rate over this sample, the bound an all-core CRC cannot pass). */

struct rate_piece {
    uint64_t rec, skip, len;
    uint32_t crc;
};

#define RATE_MAX_CHUNKS 4096

struct rate_pool {
    const uint8_t *base;
    const uint64_t *off, *len, *pos; /* pos: prefix sums of the lengths (n + 1) */
    const uint32_t *seed;
    uint32_t *out;
    uint64_t n, stride, fixed_len, total;
    int impl, nthreads;
    const int *cpus;
    pthread_barrier_t bar;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int go;
    volatile int stop;
    double t0, budget;
    uint64_t passes;
    /* the bytes are dealt in chunks from a counter (a thread slowed by
     * another tenant on its core takes fewer: a static share per thread made
     * every pass wait for the slowest one, profiles/r05/cpu_threads64.jsonl) */
    uint64_t chunk, nchunks;
    uint64_t next_chunk;
    struct rate_piece piece[RATE_MAX_CHUNKS][2];
    int npiece[RATE_MAX_CHUNKS];
    volatile uint64_t sink[256 * 8];
};

struct rate_arg {
    struct rate_pool *pool;
    int t;
};

static inline uint64_t rp_pos(const struct rate_pool *P, uint64_t i)
{
    return P->pos ? P->pos[i] : i * P->fixed_len;
}

static inline uint64_t rp_len(const struct rate_pool *P, uint64_t i)
{
    return P->len ? P->len[i] : P->fixed_len;
}

/* first record of byte range start b: the smallest i with pos_i + max(len_i, 1)
 * > b (a zero-length record at b belongs to the range that starts there) */
static uint64_t rp_first(const struct rate_pool *P, uint64_t b)
{
    uint64_t lo = 0, hi = P->n;
    while (lo < hi) {
        const uint64_t m = lo + (hi - lo) / 2;
        const uint64_t l = rp_len(P, m);
        if (rp_pos(P, m) + (l ? l : 1) > b)
            hi = m;
        else
            lo = m + 1;
    }
    return lo;
}

/* 64-bit lane sums of n bytes (the tail under 64 bytes ignored): four
 * independent 128-bit chains, so the loads bound it, not the adds */
static uint64_t read_sum(const uint8_t *p, uint64_t n)
{
#if defined(__x86_64__)
    __m128i a0 = _mm_setzero_si128(), a1 = a0, a2 = a0, a3 = a0;
    for (uint64_t k = 0; k + 64 <= n; k += 64) {
        a0 = _mm_add_epi64(a0, _mm_loadu_si128((const __m128i *)(p + k)));
        a1 = _mm_add_epi64(a1, _mm_loadu_si128((const __m128i *)(p + k + 16)));
        a2 = _mm_add_epi64(a2, _mm_loadu_si128((const __m128i *)(p + k + 32)));
        a3 = _mm_add_epi64(a3, _mm_loadu_si128((const __m128i *)(p + k + 48)));
    }
    a0 = _mm_xor_si128(_mm_xor_si128(a0, a1), _mm_xor_si128(a2, a3));
    return (uint64_t)_mm_cvtsi128_si64(a0) ^ (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(a0, a0));
#else
    uint64_t s = 0;
    for (uint64_t k = 0; k + 8 <= n; k += 8) {
        uint64_t w;
        memcpy(&w, p + k, 8);
        s += w;
    }
    return s;
#endif
}

/* chunk c: bytes [c chunk, (c + 1) chunk) of the records laid end to end */
static void rate_chunk(struct rate_pool *P, uint64_t c, int t, int mode)
{
    const uint64_t b0 = c * P->chunk;
    const uint64_t b1 = b0 + P->chunk < P->total ? b0 + P->chunk : P->total;
    const int last = c == P->nchunks - 1;
    uint64_t sum = 0;
    int np = 0;
    for (uint64_t i = rp_first(P, b0); i < P->n; ++i) {
        const uint64_t pi = rp_pos(P, i), li = rp_len(P, i);
        if (!(pi < b1 || (last && pi == b1)))
            break;
        const uint64_t s = pi < b0 ? b0 - pi : 0;
        const uint64_t e = pi + li > b1 ? b1 - pi : li;
        const uint8_t *p = P->base + (P->off ? P->off[i] : i * P->stride) + s;
        if (mode == 3) {
            sum += read_sum(p, e - s);
            continue;
        }
        const uint32_t sd = s == 0 && P->seed ? P->seed[i] : 0;
        const uint32_t v = P->impl == 1 ? oracle_crc32c_hw(sd, p, e - s)
                         : P->impl == 2 ? oracle_crc32c_bitwise(sd, p, e - s)
                                        : oracle_crc32c_sw(sd, p, e - s);
        if (s == 0 && e == li)
            P->out[i] = v;
        else if (np < 2)
            P->piece[c][np++] = (struct rate_piece){i, s, e - s, v};
    }
    P->npiece[c] = np;
    P->sink[8 * t] += sum;
}

static void rate_share(struct rate_pool *P, int t, int mode)
{
    for (;;) {
        const uint64_t c = __atomic_fetch_add(&P->next_chunk, 1, __ATOMIC_RELAXED);
        if (c >= P->nchunks)
            break;
        rate_chunk(P, c, t, mode);
    }
}

static void *rate_worker(void *arg)
{
    struct rate_arg *a = arg;
    struct rate_pool *P = a->pool;
    const int t = a->t;
    const int mode = P->impl == 3 ? 3 : 0;
    if (P->cpus && P->cpus[t] >= 0) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(P->cpus[t], &cs);
        pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
    }
    /* the gate: the thread count (and so every range) is final once it opens */
    pthread_mutex_lock(&P->mu);
    while (!P->go)
        pthread_cond_wait(&P->cv, &P->mu);
    pthread_mutex_unlock(&P->mu);
    for (;;) {
        pthread_barrier_wait(&P->bar);
        if (P->stop)
            break;
        rate_share(P, t, mode);
        pthread_barrier_wait(&P->bar);
        if (t == 0) {
            P->next_chunk = 0; /* the others wait at the next pass's barrier */
            ++P->passes;
            if (oracle_now() - P->t0 >= P->budget)
                P->stop = 1;
        }
    }
    return NULL;
}

/* Returns the seconds the passes took (*passes of them), or -1. */
double oracle_batch_rate(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                         const uint32_t *seed, uint32_t *out, uint64_t n, uint64_t stride,
                         uint64_t fixed_len, int impl, int nthreads, const int *cpus,
                         double budget, uint64_t *passes)
{
    oracle_init_tables();
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    static struct rate_pool P; /* one bench leg at a time */
    memset(&P, 0, sizeof P);
    uint64_t *pos = NULL;
    if (len) {
        pos = malloc((n + 1) * sizeof *pos);
        if (!pos)
            return -1;
        pos[0] = 0;
        for (uint64_t i = 0; i < n; ++i)
            pos[i + 1] = pos[i] + len[i];
    }
    P.base = base;
    P.off = off;
    P.len = len;
    P.pos = pos;
    P.seed = seed;
    P.out = out;
    P.n = n;
    P.stride = stride;
    P.fixed_len = fixed_len;
    P.total = len ? pos[n] : n * fixed_len;
    /* ~16 chunks per thread, at least 256 KiB each (a record cut by a chunk
     * boundary is joined by the zero shift, as a range's were) */
    {
        const uint64_t want = (uint64_t)(nthreads < 1 ? 1 : nthreads) * 16;
        uint64_t ch = (P.total + want - 1) / want;
        if (ch < (256u << 10))
            ch = 256u << 10;
        if ((P.total + ch - 1) / ch > RATE_MAX_CHUNKS)
            ch = (P.total + RATE_MAX_CHUNKS - 1) / RATE_MAX_CHUNKS;
        P.chunk = ch ? ch : 1;
        P.nchunks = P.total ? (P.total + P.chunk - 1) / P.chunk : 1;
    }
    P.impl = impl;
    P.nthreads = nthreads;
    P.cpus = cpus;
    P.budget = budget;
    pthread_mutex_init(&P.mu, NULL);
    pthread_cond_init(&P.cv, NULL);
    pthread_t th[256];
    struct rate_arg args[256];
    int started = 0;
    for (int t = 1; t < nthreads; ++t) {
        args[t] = (struct rate_arg){&P, t};
        if (pthread_create(&th[t], NULL, rate_worker, &args[t]) != 0)
            break;
        started = t;
    }
    nthreads = P.nthreads = started + 1; /* the threads that exist */
    if (pthread_barrier_init(&P.bar, NULL, (unsigned)nthreads) != 0) {
        P.stop = 1; /* workers leave at their first look */
        nthreads = 1;
    }
    pthread_mutex_lock(&P.mu);
    P.go = 1;
    pthread_cond_broadcast(&P.cv);
    pthread_mutex_unlock(&P.mu);
    if (P.stop) {
        for (int t = 1; t <= started; ++t)
            pthread_join(th[t], NULL);
        free(pos);
        return -1;
    }
    args[0] = (struct rate_arg){&P, 0};
    cpu_set_t caller; /* thread 0 is the caller: its own mask comes back after */
    const int have_mask = pthread_getaffinity_np(pthread_self(), sizeof caller, &caller) == 0;
    P.t0 = oracle_now();
    rate_worker(&args[0]);
    const double el = oracle_now() - P.t0;
    if (have_mask)
        pthread_setaffinity_np(pthread_self(), sizeof caller, &caller);
    for (int t = 1; t < nthreads; ++t)
        pthread_join(th[t], NULL);
    pthread_barrier_destroy(&P.bar);
    /* join the pieces of the records the ranges cut, in byte order */
    if (impl != 3) {
        uint64_t cur = UINT64_MAX;
        uint32_t crc = 0;
        for (uint64_t c = 0; c < P.nchunks; ++c)
            for (int k = 0; k < P.npiece[c]; ++k) {
                const struct rate_piece *q = &P.piece[c][k];
                if (q->rec != cur) {
                    cur = q->rec;
                    crc = q->crc;
                } else {
                    crc = oracle_shift(crc, q->len) ^ q->crc;
                }
                if (q->skip + q->len == rp_len(&P, q->rec))
                    out[q->rec] = crc;
            }
    }
    free(pos);
    *passes = P.passes;
    return el;
}
