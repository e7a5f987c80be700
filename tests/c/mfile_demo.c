/*
 * Append-path demonstrator: the reference's OWN src/mfile.c (with util.c,
 * log.c, cstring.c), compiled unmodified from /root/reference by
 * oracle/Makefile's `ref` target, linked against libzscrc.so instead of
 * src/crc32c.c.  Its crc32_end (src/mfile.c:534-546) calls crc32c_hw through
 * the unchanged symbol; with ZSCRC_GPU_MIN set, the span CRC runs on the GPU.
 *
 * The program appends like zsdb_add / zsdb_commit do (src/zeroskip.c:863-1040):
 * a 40-byte header, crc32_begin, then `pieces` mfile_write calls of `piece`
 * bytes of xorshift64 data (seed 0x9E3779B97F4A7C15), then crc32_end.  It
 * prints one JSON line: the span CRC, the span length, and libzscrc's counters
 * (scalar calls on the CPU / offloaded to the GPU).
 *
 * usage: mfile_demo FILE PIECE_BYTES PIECES [warm]
 *   warm: call zscrc_warmup() first (what a GPU-enabled zeroskip process does
 *   at open), so the offload threshold in force is the warm one.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <libzeroskip/mfile.h>

#include "zscrc.h"

static uint64_t xs = 0x9E3779B97F4A7C15ull;

static void fill(unsigned char *p, uint64_t n)
{
    for (uint64_t i = 0; i < n; i += 8) {
        xs ^= xs << 13;
        xs ^= xs >> 7;
        xs ^= xs << 17;
        uint64_t v = xs;
        memcpy(p + i, &v, n - i < 8 ? n - i : 8);
    }
}

int main(int argc, char **argv)
{
    if (argc != 4 && !(argc == 5 && strcmp(argv[4], "warm") == 0)) {
        fprintf(stderr, "usage: %s FILE PIECE_BYTES PIECES [warm]\n", argv[0]);
        return 2;
    }
    if (argc == 5 && zscrc_warmup() != ZSCRC_OK) {
        fprintf(stderr, "zscrc_warmup: %s\n", zscrc_last_error());
        return 1;
    }
    const uint64_t piece = strtoull(argv[2], NULL, 0), pieces = strtoull(argv[3], NULL, 0);
    struct mfile *mf = NULL;
    if (mfile_open(argv[1], MFILE_RW_CR, &mf) != 0) {
        perror("mfile_open");
        return 1;
    }
    unsigned char hdr[40];
    memset(hdr, 0x5a, sizeof hdr);
    uint64_t nb = 0;
    if (mfile_write(&mf, hdr, sizeof hdr, &nb) != 0)
        return 1;
    unsigned char *buf = malloc(piece ? piece : 1);
    if (!buf)
        return 1;
    uint64_t before[4], after[4];
    zscrc_stats(before);
    crc32_begin(&mf);
    for (uint64_t i = 0; i < pieces; ++i) {
        fill(buf, piece);
        if (mfile_write(&mf, buf, piece, &nb) != 0) {
            perror("mfile_write");
            return 1;
        }
    }
    const uint32_t crc = crc32_end(&mf);
    zscrc_stats(after);
    if (mfile_flush(&mf) != 0 || mfile_close(&mf) != 0)
        return 1;
    printf("{\"crc\": %u, \"span\": %llu, \"cpu_calls\": %llu, \"gpu_calls\": %llu}\n", crc,
           (unsigned long long)(piece * pieces), (unsigned long long)(after[0] - before[0]),
           (unsigned long long)(after[1] - before[1]));
    free(buf);
    return 0;
}
