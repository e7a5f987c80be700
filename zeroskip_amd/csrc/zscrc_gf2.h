/*
 * zscrc_gf2.h -- GF(2)[x] / P arithmetic for CRC-32C (Castagnoli, reflected).
 *
 * A CRC register is a residue mod P in reflected bit order (bit 31 = x^0).
 * "Shift by n bytes" = the register after n zero bytes = multiply by x^(8n).
 * This is the operator the reference applies with its 4x256 zero tables
 * (src/crc32c.c:363-367, crc32c_long/short for n = 8192/256); here it is
 * generalised to any n, to tables for any n, and to the combine identity
 *   crc(A||B) = shift(crc(A), |B|) ^ crc(B).
 */
#ifndef ZSCRC_GF2_H
#define ZSCRC_GF2_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZSCRC_POLY 0x82F63B78u

uint32_t zs_gf2_mul(uint32_t a, uint32_t b);        /* a*b mod P            */
uint32_t zs_gf2_xpow8n(uint64_t n);                 /* x^(8n) mod P          */
uint32_t zs_gf2_shift(uint32_t reg, uint64_t n);    /* reg after n zero bytes */
/* tab[j*256 + b] = shift(b << 8j, n): the 4-lookup operator for "n zero bytes". */
void zs_gf2_shift_table(uint32_t tab[1024], uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
