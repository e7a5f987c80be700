/*
 * crc32bench -- BASELINE config 1 against libzscrc's
 * drop-in symbols: the reference harness's workload (benchmark/crc32bench.c:
 * 65,536 CRCs of its 574-byte text per mode) plus a 1 MiB xorshift64 buffer
 * (seed 0x9E3779B97F4A7C15, tests/golden/datagen.py) hashed R times.
 *
 * Per mode it prints the reference's own line (benchmark/crc32bench.c:52-57:
 * "bytes" there is the SUM of the CRCs, a label bug recorded in SURVEY.md
 * Appendix A) and a corrected line with the byte count and GB/s, then one JSON
 * line.  Modes: hw = crc32c_hw (SSE4.2 3-way path), sw = crc32c_sw
 * (libzscrc: slice-by-8; the reference: slice-by-4), default = crc32c() after crc32c_init (the dispatch), zlib =
 * zlib crc32 (CRC-32, another polynomial: timing context only).  Exit 1 if a
 * CRC differs from the golden value or the three CRC-32C modes disagree.
 *
 * build: gcc -O2 -Iinclude tools/crc32bench.c -Lzeroskip_amd -lzscrc -lz
 *        -Wl,-rpath,$PWD/zeroskip_amd -o tools/crc32bench_bin
 * usage: crc32bench [-r reps_1mib] [-g gpu_min_bytes] [-b route_bytes]
 *
 * -b N (N > 0): the drop-in's routing with a GPU present (tests/
 * test_gpu_c_link.py): crc32c_hw over an N-byte xorshift64 buffer before any
 * device context exists (the cold threshold, 5 GiB by default: the CPU), then
 * zscrc_warmup() and the same call again (the warm threshold, 32 MiB: the
 * GPU), each call's route read from zscrc_stats; both CRCs must agree.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#include "zscrc.h"

/* the 574-byte text of benchmark/crc32bench.c:22 (a test vector) */
static const char TEXT[] =
    "Lorem Ipsum is simply dummy text of the printing and typesetting industry. Lorem Ipsum has been "
    "the industry's standard dummy text ever since the 1500s, when an unknown printer took a galley of "
    "type and scrambled it to make a type specimen book. It has survived not only five centuries, but "
    "also the leap into electronic typesetting, remaining essentially unchanged. It was popularised in "
    "the 1960s with the release of Letraset sheets containing Lorem Ipsum passages, and more recently "
    "with desktop publishing software like Aldus PageMaker including versions of Lorem Ipsum.";
static const uint32_t TEXT_CRC = 1137654557u; /* tests/golden/crc32c_golden.json "crc32bench" */
enum { RUNS = 65536, MIB = 1 << 20 };

typedef uint32_t (*crc_fn)(uint32_t, const void *, size_t);

static uint32_t zlib_crc(uint32_t crc, const void *buf, size_t len)
{
    return (uint32_t)crc32(crc, (const Bytef *)buf, (uInt)len);
}

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

struct result {
    const char *name;
    double text_us, mib_us;
    uint32_t text_crc, mib_crc;
};

static void run(const char *name, crc_fn f, const uint8_t *mib, int reps, struct result *r)
{
    const size_t tl = strlen(TEXT);
    uint32_t sum = 0, last = 0;
    double t0 = now_us();
    for (int i = 0; i < RUNS; ++i) {
        last = f(0, TEXT, tl);
        sum += last;
    }
    double t1 = now_us();
    /* the reference's line, quirk included */
    fprintf(stderr, "%-16s: %u bytes in %.0f \xce\xbcs.\n", name, sum, t1 - t0);
    uint32_t m = 0;
    double t2 = now_us();
    for (int i = 0; i < reps; ++i)
        m = f(0, mib, MIB);
    double t3 = now_us();
    r->name = name;
    r->text_us = t1 - t0;
    r->mib_us = t3 - t2;
    r->text_crc = last;
    r->mib_crc = m;
    printf("%-8s %d x %zu B in %9.0f us = %6.2f GB/s (crc %08x) | %d x 1 MiB in %9.0f us = %6.2f GiB/s "
           "(crc %08x)\n",
           name, RUNS, tl, r->text_us, (double)RUNS * tl / r->text_us / 1e3, last, reps, r->mib_us,
           (double)reps * MIB / (r->mib_us * 1e-6) / (1 << 30), m);
}

int main(int argc, char **argv)
{
    int reps = 2000, opt;
    size_t route = 0;
    while ((opt = getopt(argc, argv, "r:g:b:")) != -1) {
        if (opt == 'r')
            reps = atoi(optarg);
        else if (opt == 'b')
            route = strtoull(optarg, NULL, 0);
        else if (opt == 'g')
            zscrc_set_gpu_min(strtoull(optarg, NULL, 0));
        else {
            fprintf(stderr, "usage: %s [-r reps_1mib] [-g gpu_min_bytes] [-b route_bytes]\n", argv[0]);
            return 2;
        }
    }
    if (reps < 1)
        reps = 1;
    uint8_t *mib = malloc(MIB);
    if (!mib)
        return 2;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < MIB / 8; ++i) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        memcpy(mib + 8 * i, &x, 8); /* little-endian host, as datagen.py */
    }
    crc32c_init();
    struct result r[4];
    run("crc32c_hw", crc32c_hw, mib, reps, &r[0]);
    run("crc32c_sw", crc32c_sw, mib, reps / 10 > 0 ? reps / 10 : 1, &r[1]);
    run("crc32c", crc32c, mib, reps, &r[2]);
    run("zlib crc32", zlib_crc, mib, reps, &r[3]);
    int bad = 0;
    for (int i = 0; i < 3; ++i)
        bad |= r[i].text_crc != TEXT_CRC || r[i].mib_crc != r[0].mib_crc;
    const long cores = sysconf(_SC_NPROCESSORS_ONLN);
    printf("{\"config\": \"config1: crc32bench (574 B x %d) + 1 MiB xorshift64 x R, host CPU, 1 thread\", "
           "\"online_cpus\": %ld, \"threads\": 1, \"ok\": %s",
           RUNS, cores, bad ? "false" : "true");
    for (int i = 0; i < 4; ++i) {
        const int rr = i == 1 ? (reps / 10 > 0 ? reps / 10 : 1) : reps;
        printf(", \"%s\": {\"text_GBs\": %.3f, \"mib_GiBs\": %.3f}", r[i].name,
               (double)RUNS * strlen(TEXT) / r[i].text_us / 1e3,
               (double)rr * MIB / (r[i].mib_us * 1e-6) / (1 << 30));
    }
    if (route) {
        /* routing: cold (no device context yet) then warm (after zscrc_warmup) */
        uint8_t *big = malloc(route);
        if (!big)
            return 2;
        for (size_t i = 0; i < route; i += MIB)
            memcpy(big + i, mib, route - i < MIB ? route - i : MIB);
        uint64_t s0[4], s1[4], s2[4];
        zscrc_stats(s0);
        double t0 = now_us();
        const uint32_t cold = crc32c_hw(0, big, route);
        double t1 = now_us();
        zscrc_stats(s1);
        const int wrc = zscrc_warmup();
        crc32c_hw(0, big, route); /* the offload's buffers and tables warm */
        zscrc_stats(s2);
        const uint64_t off0 = s2[1];
        double t2 = now_us();
        const uint32_t warm = crc32c_hw(0, big, route);
        double t3 = now_us();
        zscrc_stats(s2);
        const int cold_cpu = s1[0] == s0[0] + 1 && s1[1] == s0[1];
        const int warm_gpu = wrc == 0 && s2[1] == off0 + 1;
        bad |= cold != warm || !cold_cpu || !warm_gpu;
        printf(", \"routing\": {\"bytes\": %zu, \"crc\": \"%08x\", \"cold_threshold\": %" PRIu64
               ", \"warm_threshold\": %" PRIu64 ", \"cold_on_cpu\": %s, \"warm_on_gpu\": %s, "
               "\"cold_GBs\": %.2f, \"warm_GBs\": %.2f, \"warmup_rc\": %d}",
               route, warm, zscrc_gpu_min(1), zscrc_gpu_min(0), cold_cpu ? "true" : "false",
               warm_gpu ? "true" : "false", route / (t1 - t0) / 1e3, route / (t3 - t2) / 1e3, wrc);
        printf(", \"ok_all\": %s", bad ? "false" : "true");
        free(big);
    }
    printf("}\n");
    free(mib);
    return bad;
}
