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
#include <stdint.h>
#include <stddef.h>
#include <string.h>
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
