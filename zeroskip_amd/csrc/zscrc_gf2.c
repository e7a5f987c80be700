/* zscrc_gf2.c -- see zscrc_gf2.h. */
#include "zscrc_gf2.h"

/* Multiply two reflected residues.  The loop walks a's coefficients from
 * x^0 (bit 31) upwards while b is multiplied by x at each step. */
uint32_t zs_gf2_mul(uint32_t a, uint32_t b)
{
    uint32_t acc = 0;
    while (a) {
        if (a & 0x80000000u)
            acc ^= b;
        a <<= 1;
        b = (b >> 1) ^ ((b & 1u) ? ZSCRC_POLY : 0u);
    }
    return acc;
}

/* x^(8*2^k) mod P for k = 0..63, built once. */
static uint32_t g_pow2[64];
static int g_pow2_ready;

static void pow2_init(void)
{
    if (g_pow2_ready)
        return;
    uint32_t p = 0x00800000u; /* x^8 */
    for (int k = 0; k < 64; ++k) {
        g_pow2[k] = p;
        p = zs_gf2_mul(p, p);
    }
    g_pow2_ready = 1;
}

uint32_t zs_gf2_xpow8n(uint64_t n)
{
    pow2_init();
    uint32_t r = 0x80000000u; /* x^0 */
    for (int k = 0; n; ++k, n >>= 1)
        if (n & 1)
            r = zs_gf2_mul(r, g_pow2[k]);
    return r;
}

uint32_t zs_gf2_shift(uint32_t reg, uint64_t n)
{
    return n ? zs_gf2_mul(zs_gf2_xpow8n(n), reg) : reg;
}

void zs_gf2_shift_table(uint32_t tab[1024], uint64_t n)
{
    uint32_t m = zs_gf2_xpow8n(n);
    for (int j = 0; j < 4; ++j)
        for (int b = 0; b < 256; ++b)
            tab[j * 256 + b] = zs_gf2_mul(m, (uint32_t)b << (8 * j));
}
