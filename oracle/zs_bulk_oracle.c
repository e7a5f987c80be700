/*
 * zs_bulk_oracle.c -- bulk zeroskip checks and a CPU commit writer for the
 * parity tests and bench.py's post-timing checks (TEST INFRASTRUCTURE ONLY;
 * see zs_oracle.c's header: the product never links or calls this file).
 *
 * Everything here is built on oracle_crc32c_hw and oracle_commit_crc, and
 * restates the reference's code (file:line under /root/reference):
 *   - oracle_walk_image: the record walk of zs_record_read_from_file
 *     (src/zeroskip-record.c:283-331, record lengths :75-181), every commit
 *     re-checked with the WRITER's trailer semantics
 *     (src/zeroskip-file.c:253-350) from crc32c(0, 0, 0) = 0
 *     (src/mfile.c:526-546), as oracle/zs_format.py's walk() does in Python;
 *   - oracle_packed_image: a packed file's pointer-section and records-region
 *     commits (src/zeroskip-packed.c:70-131, :278-339; the records commit
 *     :442 that the reference never re-checks);
 *   - oracle_span_crc: crc32c(0, buf, len) of one long span on T threads,
 *     pieces joined with the zero-shift operator (src/crc32c.c:363-367:
 *     crc(A || B) = shift(crc(A), |B|) ^ crc(B));
 *   - oracle_write_commits: the commit writer (src/zeroskip-file.c:253-350)
 *     for spans whose commit record's type byte is already in place -- the
 *     record (8 or 24 bytes) is written whole, big-endian;
 *   - oracle_commit_crcs: the CRC the writer would store for each span.
 */
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>

uint32_t oracle_crc32c_hw(uint32_t crc, const void *buf, size_t len);
uint32_t oracle_shift(uint32_t reg, uint64_t nbytes);
uint32_t oracle_commit_crc(uint32_t span_crc, uint64_t span_len, int final);

enum { T_KEY = 1, T_VALUE = 2, T_COMMIT = 4, T_2ND = 8, T_FINAL = 16, T_LONG = 32, T_DELETED = 64 };
#define T_LONG_KEY (T_KEY | T_LONG)
#define T_LONG_VALUE (T_VALUE | T_LONG)
#define T_LONG_COMMIT (T_COMMIT | T_LONG)
#define T_LONG_FINAL (T_FINAL | T_LONG)
#define T_LONG_DELETED (T_LONG | T_LONG) /* == 32, as zeroskip-priv.h:119 writes it */
#define MAX_SHORT 16777215ull            /* zeroskip-priv.h:171 */
#define HDR 40u

static uint64_t rd_be64(const uint8_t *p)
{
    uint64_t v;
    memcpy(&v, p, 8);
    return __builtin_bswap64(v);
}

static void wr_be64(uint8_t *p, uint64_t v)
{
    v = __builtin_bswap64(v);
    memcpy(p, &v, 8);
}

static uint64_t rup8(uint64_t n) { return (n + 7) & ~7ull; }

/* --------------------------------------------------------------- threads */
typedef void (*range_fn)(void *ctx, uint64_t lo, uint64_t hi);
struct range_job {
    range_fn fn;
    void *ctx;
    uint64_t lo, hi;
};

static void *range_worker(void *arg)
{
    struct range_job *j = arg;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}

/* fn(ctx, lo, hi) over [0, n) cut into `threads` contiguous ranges */
static int parallel_for(uint64_t n, int threads, range_fn fn, void *ctx)
{
    if (threads < 1)
        threads = 1;
    if (threads > 256)
        threads = 256;
    if ((uint64_t)threads > n)
        threads = n ? (int)n : 1;
    pthread_t th[256];
    struct range_job jobs[256];
    const uint64_t per = (n + threads - 1) / threads;
    int started = 0, rc = 0;
    for (int t = 0; t < threads; ++t) {
        const uint64_t lo = t * per, hi = lo + per < n ? lo + per : n;
        jobs[t] = (struct range_job){fn, ctx, lo, hi};
        if (t == 0 || lo >= hi)
            continue;
        if (pthread_create(&th[t], NULL, range_worker, &jobs[t]) != 0) {
            rc = -1;
            break;
        }
        started = t;
    }
    if (jobs[0].lo < jobs[0].hi)
        range_worker(&jobs[0]);
    for (int t = 1; t <= started; ++t)
        pthread_join(th[t], NULL);
    return rc;
}

/* ---------------------------------------------------------- commit checks */
/* The commit record at `off` after the span [off - len, off): 1 ok, 0 bad,
 * 2 not a commit record / does not fit.  *span_len receives len. */
static int commit_at(const uint8_t *img, uint64_t n, uint64_t off, uint32_t seed, uint64_t *span_len,
                     uint64_t *rec_len)
{
    if (off + 8 > n)
        return 2;
    const uint64_t w0 = rd_be64(img + off);
    const unsigned t = (unsigned)(w0 >> 56);
    if (t == T_COMMIT || t == T_FINAL) {
        const uint64_t len = (w0 >> 32) & 0xFFFFFF;
        if (len > off)
            return 2;
        *span_len = len;
        *rec_len = 8;
        uint32_t c = oracle_crc32c_hw(seed, img + off - len, len);
        const uint64_t w = w0 & 0xFFFFFFFF00000000ull;
        c = oracle_crc32c_hw(c, &w, 8);
        return c == (uint32_t)w0;
    }
    if ((t == T_LONG_COMMIT || t == T_LONG_FINAL) && off + 24 <= n) {
        const uint64_t len = rd_be64(img + off + 8), w2 = rd_be64(img + off + 16);
        if (len > off)
            return 2;
        *span_len = len;
        *rec_len = 24;
        const uint64_t words[3] = {w0, len, w2 & 0xFF00000000000000ull};
        uint32_t c = oracle_crc32c_hw(seed, img + off - len, len);
        c = oracle_crc32c_hw(c, words, 24);
        return c == (uint32_t)w2;
    }
    return 2;
}

/* out[0] commits, out[1] ok, out[2] end offset, out[3] stop reason (0 end of
 * image, 1 truncated record, 2 a type the walk does not advance over, 3 a
 * commit record that does not fit), out[4] file offset of the first bad
 * commit record (~0 none), out[5] its index. */
void oracle_walk_image(const uint8_t *img, uint64_t n, uint64_t out[6])
{
    uint64_t off = HDR, commits = 0, ok = 0, first_bad = ~0ull, first_idx = ~0ull;
    int stop = 0;
    while (off < n) {
        if (off + 8 > n) {
            stop = 1;
            break;
        }
        const uint64_t w0 = rd_be64(img + off);
        const unsigned t = (unsigned)(w0 >> 56);
        if (t == T_KEY || t == T_LONG_KEY) {
            /* key record -> its value record (record.c:75-106, :156-181) */
            uint64_t voff;
            if (t == T_KEY) {
                voff = w0 & 0xFFFFFFFF;
            } else {
                if (off + 24 > n) {
                    stop = 1;
                    break;
                }
                voff = rd_be64(img + off + 16);
            }
            off += voff;
            if (voff == 0 || off + 16 > n) {
                stop = 1;
                break;
            }
            const uint64_t v0 = rd_be64(img + off);
            const uint64_t vlen = (v0 >> 56) == T_VALUE ? (v0 >> 32) & 0xFFFFFF : rd_be64(img + off + 8);
            off += 16 + rup8(vlen);
        } else if (t == T_DELETED || t == T_LONG_DELETED) {
            /* the short delete's key length is stored through a uint16_t
             * (zeroskip-priv.h:124) */
            uint64_t klen;
            if (t == T_DELETED) {
                klen = (w0 >> 40) & 0xFFFF;
            } else {
                if (off + 16 > n) {
                    stop = 1;
                    break;
                }
                klen = rd_be64(img + off + 8);
            }
            off += 24 + rup8(klen);
        } else if (t == T_COMMIT || t == T_LONG_COMMIT) {
            uint64_t sl = 0, rl = 0;
            const int st = commit_at(img, n, off, 0, &sl, &rl);
            if (st == 2) {
                stop = 3;
                break;
            }
            if (st == 1) {
                ok++;
            } else if (first_bad == ~0ull) {
                first_bad = off;
                first_idx = commits;
            }
            commits++;
            off += rl;
        } else { /* FINAL / 2ND_HALF / UNUSED / VALUE: the reference does not advance */
            stop = 2;
            break;
        }
    }
    out[0] = commits;
    out[1] = ok;
    out[2] = off;
    out[3] = (uint64_t)stop;
    out[4] = first_bad;
    out[5] = first_idx;
}

struct walk_ctx {
    const uint64_t *addr, *size;
    uint64_t *out;
};

static void walk_range(void *p, uint64_t lo, uint64_t hi)
{
    struct walk_ctx *c = p;
    for (uint64_t f = lo; f < hi; ++f)
        oracle_walk_image((const uint8_t *)(uintptr_t)c->addr[f], c->size[f], c->out + 6 * f);
}

/* oracle_walk_image over nfiles images (addresses as integers) on T threads */
int oracle_walk_images(const uint64_t *addr, const uint64_t *size, uint64_t nfiles, uint64_t *out, int threads)
{
    struct walk_ctx c = {addr, size, out};
    return parallel_for(nfiles, threads, walk_range, &c);
}

/* --------------------------------------------------------------- spans */
struct span_ctx {
    const uint8_t *buf;
    uint64_t len, per;
    uint32_t *crc;
};

static void span_range(void *p, uint64_t lo, uint64_t hi)
{
    struct span_ctx *c = p;
    for (uint64_t k = lo; k < hi; ++k) {
        const uint64_t a = k * c->per, b = a + c->per < c->len ? a + c->per : c->len;
        c->crc[k] = oracle_crc32c_hw(0, c->buf + a, b - a);
    }
}

/* crc32c(0, buf, len) on T threads: T pieces joined left to right with
 * crc(A || B) = shift(crc(A), |B|) ^ crc(B). */
uint32_t oracle_span_crc(const uint8_t *buf, uint64_t len, int threads)
{
    if (threads < 1)
        threads = 1;
    if (threads > 256)
        threads = 256;
    if (len < (1u << 20) || threads == 1)
        return oracle_crc32c_hw(0, buf, len);
    uint32_t crc[256];
    struct span_ctx c = {buf, len, (len + threads - 1) / threads, crc};
    const uint64_t k = (len + c.per - 1) / c.per;
    parallel_for(k, (int)k, span_range, &c);
    uint32_t r = crc[0];
    for (uint64_t i = 1; i < k; ++i) {
        const uint64_t a = i * c.per, b = a + c.per < len ? a + c.per : len;
        r = oracle_shift(r, b - a) ^ crc[i];
    }
    return r;
}

/* A packed file [Header][records][commit][count][ptrs][final commit]
 * (zeroskip-packed.c:384-473): out[0] pointer-section status (1 ok, 0 bad,
 * 2 layout), out[1] its span offset, out[2] its length, out[3] records-region
 * status, out[4] its span offset, out[5] its length.  The records region is
 * hashed on T threads. */
void oracle_packed_image(const uint8_t *img, uint64_t n, int threads, uint64_t out[6])
{
    for (int i = 0; i < 6; ++i)
        out[i] = 0;
    out[0] = out[3] = 2;
    if (n < HDR + 16)
        return;
    /* the final commit: the last 8 bytes, or 24 when they are a 2ND_HALF word */
    const uint64_t foff = (rd_be64(img + n - 8) >> 56) == T_2ND ? n - 24 : n - 8;
    uint64_t pl = 0, rl = 0;
    out[0] = (uint64_t)commit_at(img, n, foff, 0, &pl, &rl);
    if (out[0] == 2)
        return;
    const uint64_t poff = foff - pl;
    out[1] = poff;
    out[2] = pl;
    if (poff < HDR + 8)
        return;
    const uint64_t roff = (rd_be64(img + poff - 8) >> 56) == T_2ND ? poff - 24 : poff - 8;
    if (roff < HDR || roff + 8 > n)
        return;
    const uint64_t w0 = rd_be64(img + roff);
    const unsigned t = (unsigned)(w0 >> 56);
    uint64_t len, stored;
    uint64_t words[3];
    int nw;
    if (t == T_COMMIT || t == T_FINAL) {
        len = (w0 >> 32) & 0xFFFFFF;
        words[0] = w0 & 0xFFFFFFFF00000000ull;
        nw = 1;
        stored = (uint32_t)w0;
    } else if ((t == T_LONG_COMMIT || t == T_LONG_FINAL) && roff + 24 <= n) {
        len = rd_be64(img + roff + 8);
        const uint64_t w2 = rd_be64(img + roff + 16);
        words[0] = w0;
        words[1] = len;
        words[2] = w2 & 0xFF00000000000000ull;
        nw = 3;
        stored = (uint32_t)w2;
    } else {
        return;
    }
    if (len > roff)
        return;
    out[4] = roff - len;
    out[5] = len;
    uint32_t c = oracle_span_crc(img + roff - len, len, threads);
    c = oracle_crc32c_hw(c, words, 8 * (size_t)nw);
    out[3] = c == stored;
}

/* ------------------------------------------------------------ the writer */
struct commits_ctx {
    uint8_t *base;
    const uint64_t *off, *len;
    uint32_t *crc; /* oracle_commit_crcs */
    int write;
};

static void commits_range(void *p, uint64_t lo, uint64_t hi)
{
    struct commits_ctx *c = p;
    for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t len = c->len[i];
        uint8_t *at = c->base + c->off[i] + len;
        const unsigned t = at[0];
        const int final = (t & T_FINAL) != 0;
        const uint32_t crc = oracle_commit_crc(oracle_crc32c_hw(0, c->base + c->off[i], len), len, final);
        if (c->crc)
            c->crc[i] = crc;
        if (!c->write)
            continue;
        if (len > MAX_SHORT) { /* zeroskip-file.c:266-302 */
            wr_be64(at, (uint64_t)(final ? T_LONG_FINAL : T_LONG_COMMIT) << 56);
            wr_be64(at + 8, len);
            wr_be64(at + 16, ((uint64_t)T_2ND << 56) | crc);
        } else { /* :303-328 */
            wr_be64(at, ((uint64_t)(final ? T_FINAL : T_COMMIT) << 56) | (len << 32) | crc);
        }
    }
}

/* Write the commit record after each span [off[i], +len[i]) of `base`: the
 * record's first byte must already say COMMIT or FINAL (short or long form);
 * the record is (re)written whole for the span length. */
int oracle_write_commits(uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n, int threads)
{
    struct commits_ctx c = {base, off, len, NULL, 1};
    return parallel_for(n, threads, commits_range, &c);
}

/* crc[i] = the CRC the writer stores for span i (its type byte read from the
 * record after it); nothing is written. */
int oracle_commit_crcs(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n, uint32_t *crc,
                       int threads)
{
    struct commits_ctx c = {(uint8_t *)base, off, len, crc, 0};
    return parallel_for(n, threads, commits_range, &c);
}
