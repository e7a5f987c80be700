/*
 * Mutation fuzzer for libzscrc's host-side zeroskip parsers (TEST
 * INFRASTRUCTURE): zscrc_zs_walk, zscrc_zs_packed_spans, zscrc_zs_records,
 * zscrc_zs_header_crc, zscrc_zs_dotzsdb_crc and the Part-1 CRCs, on
 * corrupted copies of the reference-written fixtures
 * (tests/golden/ref_format/) held in exact-size heap buffers, so an
 * AddressSanitizer build (tests/test_parse_fuzz.py) sees any read past an
 * image.  Checks the outputs' own contract too: every span and record the
 * parsers return lies inside the image.  No GPU call is made.
 *
 * usage: parse_fuzz ITERATIONS SEED FILE...   prints {"iterations": N, ...}
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zscrc.h"

static uint64_t rng_state;

static uint64_t rnd(void)
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static unsigned char *load(const char *path, size_t *n)
{
    FILE *fp = fopen(path, "rb");
    if (!fp)
        return NULL;
    fseek(fp, 0, SEEK_END);
    *n = (size_t)ftell(fp);
    fseek(fp, 0, SEEK_SET);
    unsigned char *p = malloc(*n ? *n : 1);
    if (p && fread(p, 1, *n, fp) != *n) {
        free(p);
        p = NULL;
    }
    fclose(fp);
    return p;
}

static void put_be64(unsigned char *p, uint64_t v)
{
    for (int i = 0; i < 8; ++i)
        p[i] = (unsigned char)(v >> (56 - 8 * i));
}

/* one corrupted copy of src in a fresh exact-size buffer */
static unsigned char *mutate(const unsigned char *src, size_t n, size_t *out_n)
{
    size_t m = n;
    const uint64_t how = rnd() % 6;
    if (how == 0 && n)
        m = (size_t)(rnd() % n); /* truncated */
    else if (how == 1)
        m = n + (size_t)(rnd() % 64); /* trailing bytes */
    unsigned char *p = malloc(m ? m : 1);
    if (!p)
        return NULL;
    memcpy(p, src, m < n ? m : n);
    for (size_t i = n; i < m; ++i)
        p[i] = (unsigned char)rnd();
    const int flips = (int)(rnd() % 8);
    for (int k = 0; k < flips && m; ++k)
        p[rnd() % m] ^= (unsigned char)(1u << (rnd() % 8));
    if (how >= 2 && m >= 8) { /* an 8-byte-aligned word set to an extreme value */
        static const uint64_t ext[] = {0, ~0ull, 0x7fffffffffffffffull, 0x01ffffffffffffffull, 0x04ffffffffffffffull,
                                       0x20ffffff00000000ull, 0x40ffff0000000000ull, 0x0100ffffffffffffull};
        const size_t at = (size_t)(rnd() % (m / 8)) * 8;
        put_be64(p + at, ext[rnd() % 8] ^ (rnd() & 0xff));
    }
    *out_n = m;
    return p;
}

static int check_spans(const uint64_t *off, const uint64_t *len, size_t k, uint64_t size)
{
    for (size_t i = 0; i < k; ++i)
        if (off[i] > size || len[i] > size - off[i])
            return 0;
    return 1;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s ITERATIONS SEED FILE...\n", argv[0]);
        return 2;
    }
    const long iters = strtol(argv[1], NULL, 0);
    rng_state = strtoull(argv[2], NULL, 0) | 1;
    const int nf = argc - 3;
    unsigned char **img = calloc((size_t)nf, sizeof *img);
    size_t *sz = calloc((size_t)nf, sizeof *sz);
    for (int f = 0; f < nf; ++f)
        if (!(img[f] = load(argv[3 + f], &sz[f]))) {
            perror(argv[3 + f]);
            return 2;
        }
    long walks = 0, records = 0, spans = 0, bad = 0;
    for (long it = 0; it < iters; ++it) {
        const int f = (int)(rnd() % (uint64_t)nf);
        size_t n = 0;
        unsigned char *p = mutate(img[f], sz[f], &n);
        if (!p)
            return 2;
        /* the walk */
        const size_t cap = n / 8 + 1;
        uint64_t *off = malloc(cap * 8), *len = malloc(cap * 8);
        size_t nc = 0;
        uint64_t end = 0;
        const int wr = zscrc_zs_walk(p, n, off, len, cap, &nc, &end);
        if (wr >= 0 && (nc > cap || end > n || !check_spans(off, len, nc < cap ? nc : cap, n)))
            ++bad, fprintf(stderr, "walk: out of image (file %d, iter %ld)\n", f, it);
        ++walks;
        /* packed spans */
        uint64_t po[2], pl[2];
        if (zscrc_zs_packed_spans(p, n, po, pl) == ZSCRC_OK && !check_spans(po, pl, 2, n))
            ++bad, fprintf(stderr, "packed_spans: out of image (file %d, iter %ld)\n", f, it);
        ++spans;
        /* records, every kind; a short cap now and then */
        for (int kind = 0; kind < 3; ++kind) {
            const size_t rcap = (rnd() % 4 == 0) ? (size_t)(rnd() % 8) : n / 24 + 2;
            zscrc_zs_record *r = malloc((rcap ? rcap : 1) * sizeof *r);
            size_t nr = 0;
            const int rr = zscrc_zs_records(p, n, kind, r, rcap, &nr);
            if (rr >= 0) {
                const size_t got = nr < rcap ? nr : rcap;
                for (size_t i = 0; i < got; ++i) {
                    const int kok = r[i].key_off <= n && r[i].key_len <= n - r[i].key_off;
                    const int vok = r[i].val_off == ZSCRC_ZS_DELETED ||
                                    (r[i].val_off <= n && r[i].val_len <= n - r[i].val_off);
                    if (!kok || !vok) {
                        ++bad;
                        fprintf(stderr, "records kind %d: out of image (file %d, iter %ld)\n", kind, f, it);
                        break;
                    }
                }
            }
            free(r);
            ++records;
        }
        uint32_t st, cp;
        (void)zscrc_zs_header_crc(p, n, &st, &cp);
        (void)zscrc_zs_dotzsdb_crc(p, n, &st, &cp);
        /* Part 1 over a random slice at a random alignment */
        if (n) {
            const size_t a = (size_t)(rnd() % n), l = (size_t)(rnd() % (n - a + 1));
            if (crc32c_hw(0, p + a, l) != crc32c_sw(0, p + a, l))
                ++bad, fprintf(stderr, "crc32c hw != sw (iter %ld)\n", it);
        }
        free(off);
        free(len);
        free(p);
    }
    printf("{\"iterations\": %ld, \"walks\": %ld, \"packed_spans\": %ld, \"record_lists\": %ld, \"violations\": %ld}\n",
           iters, walks, spans, records, bad);
    for (int f = 0; f < nf; ++f)
        free(img[f]);
    free(img);
    free(sz);
    return bad ? 1 : 0;
}
