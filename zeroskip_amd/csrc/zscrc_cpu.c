/*
 * zscrc_cpu.c -- the host-side scalar path of libzscrc.
 *
 * zeroskip calls crc32c_hw ~12 times per transaction on <= 37-byte fields
 * (SURVEY.md sec 3A); shipping those to a GPU would cost tens of microseconds
 * each, so scalar calls below the offload threshold run here on the CPU:
 *   - zscrc_cpu_table : slice-by-8 (8 generated 256-entry tables)
 *   - zscrc_cpu_hw    : SSE4.2 crc32 instruction, three independent streams per
 *                       3*BLK block, merged with the zero-shift operator
 * Both compute exactly the reference's CRC-32C (src/crc32c.c:370-453, :613-645).
 * Tables are generated from the polynomial (zscrc_gf2.c), not transcribed.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#include "zscrc_gf2.h"

static uint32_t g_t8[8][256];     /* g_t8[k][b] = shift(b, k+1) */
static uint32_t g_blk1[1024];     /* shift by BLK1 */
static uint32_t g_blk2[1024];     /* shift by BLK2 */
static int g_sse42;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

enum { BLK1 = 4096, BLK2 = 512 };

static void cpu_init(void)
{
    for (int k = 0; k < 8; ++k)
        for (int b = 0; b < 256; ++b)
            g_t8[k][b] = zs_gf2_shift((uint32_t)b, (uint64_t)k + 1);
    zs_gf2_shift_table(g_blk1, BLK1);
    zs_gf2_shift_table(g_blk2, BLK2);
#if defined(__x86_64__)
    __builtin_cpu_init();
    g_sse42 = __builtin_cpu_supports("sse4.2") != 0;
#endif
}

void zscrc_cpu_init(void) { pthread_once(&g_once, cpu_init); }
int zscrc_cpu_have_sse42(void)
{
    zscrc_cpu_init();
    return g_sse42;
}

static inline uint32_t op_shift(const uint32_t *t, uint32_t r)
{
    return t[r & 0xff] ^ t[256 + ((r >> 8) & 0xff)] ^ t[512 + ((r >> 16) & 0xff)] ^ t[768 + (r >> 24)];
}

/* register-in / register-out slice-by-8 */
static uint32_t reg_table(uint32_t r, const uint8_t *p, size_t n)
{
    while (n && ((uintptr_t)p & 7)) {
        r = (r >> 8) ^ g_t8[0][(r ^ *p++) & 0xff];
        --n;
    }
    while (n >= 8) {
        uint64_t q;
        memcpy(&q, p, 8);
        q ^= r;
        r = g_t8[7][q & 0xff] ^ g_t8[6][(q >> 8) & 0xff] ^ g_t8[5][(q >> 16) & 0xff] ^
            g_t8[4][(q >> 24) & 0xff] ^ g_t8[3][(q >> 32) & 0xff] ^ g_t8[2][(q >> 40) & 0xff] ^
            g_t8[1][(q >> 48) & 0xff] ^ g_t8[0][q >> 56];
        p += 8;
        n -= 8;
    }
    while (n--)
        r = (r >> 8) ^ g_t8[0][(r ^ *p++) & 0xff];
    return r;
}

uint32_t zscrc_cpu_table(uint32_t crc, const void *buf, size_t len)
{
    zscrc_cpu_init();
    return ~reg_table(~crc, (const uint8_t *)buf, len);
}

#if defined(__x86_64__)
__attribute__((target("sse4.2")))
static uint32_t reg_hw(uint32_t r32, const uint8_t *p, size_t n)
{
    uint64_t r = r32;
    while (n && ((uintptr_t)p & 7)) {
        r = __builtin_ia32_crc32qi((uint32_t)r, *p++);
        --n;
    }
#define ZS_STREAMS(BLK, TAB)                                                        \
    while (n >= 3 * (size_t)(BLK)) {                                                \
        uint64_t s1 = 0, s2 = 0;                                                    \
        for (size_t i = 0; i < (BLK); i += 8) {                                     \
            uint64_t a, b, c;                                                       \
            memcpy(&a, p + i, 8);                                                   \
            memcpy(&b, p + (BLK) + i, 8);                                           \
            memcpy(&c, p + 2 * (BLK) + i, 8);                                       \
            r = __builtin_ia32_crc32di(r, a);                                       \
            s1 = __builtin_ia32_crc32di(s1, b);                                     \
            s2 = __builtin_ia32_crc32di(s2, c);                                     \
        }                                                                           \
        r = op_shift(TAB, op_shift(TAB, (uint32_t)r) ^ (uint32_t)s1) ^ (uint32_t)s2; \
        p += 3 * (size_t)(BLK);                                                     \
        n -= 3 * (size_t)(BLK);                                                     \
    }
    ZS_STREAMS(BLK1, g_blk1)
    ZS_STREAMS(BLK2, g_blk2)
#undef ZS_STREAMS
    while (n >= 8) {
        uint64_t a;
        memcpy(&a, p, 8);
        r = __builtin_ia32_crc32di(r, a);
        p += 8;
        n -= 8;
    }
    while (n--)
        r = __builtin_ia32_crc32qi((uint32_t)r, *p++);
    return (uint32_t)r;
}
#endif

uint32_t zscrc_cpu_hw(uint32_t crc, const void *buf, size_t len)
{
    zscrc_cpu_init();
#if defined(__x86_64__)
    if (g_sse42)
        return ~reg_hw(~crc, (const uint8_t *)buf, len);
#endif
    return ~reg_table(~crc, (const uint8_t *)buf, len);
}
