/*
 * zscrc_pack.cpp -- packed-file writer with the repack CRCs on the GPU
 * (include/zscrc.h, "Packed-file writer").
 *
 * Byte layout and CRC lifecycle of the reference's repack output:
 *   zs_packed_file_new_from_memtree   src/zeroskip-packed.c:384-473
 *   zs_packed_file_new_from_packed_files                  :617-742
 *   zs_packed_file_write_memtree_record (pointer = offset) :163-176
 *   header                            src/zeroskip-header.c:30-94
 *   key / value / delete records      src/zeroskip-file.c:23-183
 *   commit records (short / long)     src/zeroskip-file.c:253-350
 *   crc32_begin / crc32_end           src/mfile.c:526-546
 * The reference computes the records-region CRC as ONE crc32_end over the
 * mmap'd region after the last record (packed.c:442): gigabytes hashed by one
 * core after all the writing.  Here every record is serialised straight into
 * a pinned staging chunk of a copy-mode zscrc_stream; a full chunk goes to the
 * GPU (H2D + span kernel, asynchronous) while this thread writes it to the
 * file and serialises the next chunk.  The records-region CRC is ready when
 * the last chunk has been written; the pointer section takes the same path.
 */
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/zscrc.h"

extern "C" {
uint8_t *zscrc_internal_stream_stage(zscrc_stream *s, uint64_t *room);
int zscrc_internal_stream_advance(zscrc_stream *s, uint64_t n, int flush, const uint8_t **done, uint64_t *done_n);
}

namespace {

constexpr uint64_t SIGNATURE = 0x5a45524f534b4950ull; /* zeroskip-priv.h:49 */
constexpr uint32_t VERSION = 1;                        /* ZS_VERSION */
constexpr uint64_t HDR = 40;
constexpr uint64_t MAX_SHORT_KEY_LEN = 65535;          /* zeroskip-priv.h */
constexpr uint64_t MAX_SHORT_VAL_LEN = 16777215;       /* zeroskip-priv.h:171 */
enum { T_KEY = 1, T_VALUE = 2, T_COMMIT = 4, T_2ND = 8, T_FINAL = 16, T_LONG = 32, T_DELETED = 64 };

inline void put_be64(uint8_t *p, uint64_t v)
{
    v = __builtin_bswap64(v);
    memcpy(p, &v, 8);
}
inline void put_be32(uint8_t *p, uint32_t v)
{
    v = __builtin_bswap32(v);
    memcpy(p, &v, 4);
}
inline uint64_t rup8(uint64_t n) { return (n + 7) & ~7ull; }

/* The 8- or 24-byte commit record closing a span of span_len bytes whose
 * crc32c(0, span) is span_crc: the writer's semantics (zeroskip-file.c:266-328,
 * trailer words hashed in host order).  Returns its length; *stored = CRC. */
uint64_t commit_record(uint8_t *out, uint32_t span_crc, uint64_t span_len, bool final, uint32_t *stored)
{
    if (span_len > MAX_SHORT_VAL_LEN) {
        const uint64_t t1 = (uint64_t)(final ? T_FINAL | T_LONG : T_COMMIT | T_LONG) << 56;
        const uint64_t t2 = (uint64_t)T_2ND << 56;
        uint32_t c = crc32c_hw(span_crc, &t1, 8);
        c = crc32c_hw(c, &span_len, 8);
        c = crc32c_hw(c, &t2, 8);
        put_be64(out, t1);
        put_be64(out + 8, span_len);
        put_be64(out + 16, t2 | c);
        *stored = c;
        return 24;
    }
    const uint64_t w = ((uint64_t)(final ? T_FINAL : T_COMMIT) << 56) | (span_len << 32);
    const uint32_t c = crc32c_hw(span_crc, &w, 8);
    put_be64(out, w | c);
    *stored = c;
    return 8;
}

} /* namespace */

struct zscrc_packer {
    int fd = -1;
    char *path = nullptr;
    unsigned flags = 0;
    uint64_t chunk = 0;
    zscrc_stream *st = nullptr; /* the span being checksummed (records, then pointers) */
    uint64_t out_off = 0;       /* file offset of the stream's next unwritten chunk */
    uint64_t pos = 0;           /* file offset of the next record byte */
    std::vector<uint64_t> ptrs;
    int err = 0;
};

namespace {

int pk_fail(zscrc_packer *pk, int rc)
{
    if (!pk->err)
        pk->err = rc;
    return pk->err;
}

int write_all(int fd, const uint8_t *p, uint64_t n, uint64_t off)
{
    while (n) {
        const ssize_t w = pwrite(fd, p, n > (1u << 30) ? (1u << 30) : n, (off_t)off);
        if (w < 0 && errno == EINTR)
            continue;
        if (w <= 0)
            return ZSCRC_EINVAL;
        p += w;
        n -= (uint64_t)w;
        off += (uint64_t)w;
    }
    return ZSCRC_OK;
}

/* Hand a chunk the stream just submitted to the file as well. */
int emit_done(zscrc_packer *pk, const uint8_t *done, uint64_t n)
{
    if (!done)
        return ZSCRC_OK;
    int rc = write_all(pk->fd, done, n, pk->out_off);
    pk->out_off += n;
    return rc;
}

/* Append n bytes (src, or zeros when src is NULL) to the current span. */
int put(zscrc_packer *pk, const void *src, uint64_t n)
{
    const uint8_t *s = static_cast<const uint8_t *>(src);
    while (n) {
        uint64_t room = 0;
        uint8_t *dst = zscrc_internal_stream_stage(pk->st, &room);
        if (!dst)
            return pk_fail(pk, ZSCRC_EHIP);
        const uint64_t m = n < room ? n : room;
        if (s) {
            memcpy(dst, s, m);
            s += m;
        } else {
            memset(dst, 0, m);
        }
        const uint8_t *done;
        uint64_t dn;
        int rc = zscrc_internal_stream_advance(pk->st, m, 0, &done, &dn);
        if (!rc)
            rc = emit_done(pk, done, dn);
        if (rc)
            return pk_fail(pk, rc);
        n -= m;
        pk->pos += m;
    }
    return ZSCRC_OK;
}

/* Close the current span: flush its last chunk to the file, fold its CRC. */
int end_span(zscrc_packer *pk, uint32_t *crc)
{
    const uint8_t *done;
    uint64_t dn;
    int rc = zscrc_internal_stream_advance(pk->st, 0, 1, &done, &dn);
    if (!rc)
        rc = emit_done(pk, done, dn);
    const int rc2 = zscrc_stream_final(pk->st, crc);
    pk->st = nullptr;
    return rc ? rc : rc2;
}

void pk_free(zscrc_packer *pk, bool remove_file)
{
    if (pk->st) {
        uint32_t dummy;
        (void)zscrc_stream_final(pk->st, &dummy);
    }
    if (pk->fd >= 0)
        close(pk->fd);
    if (remove_file && pk->path)
        unlink(pk->path);
    free(pk->path);
    delete pk;
}

} /* namespace */

extern "C" {

int zscrc_pack_open(zscrc_packer **out, const char *path, const uint8_t uuid[16], uint32_t startidx,
                    uint32_t endidx, uint64_t chunk_bytes, unsigned flags)
{
    if (!out || !path || !uuid)
        return ZSCRC_EINVAL;
    *out = nullptr;
    zscrc_packer *pk = new (std::nothrow) zscrc_packer;
    if (!pk)
        return ZSCRC_ENOMEM;
    pk->flags = flags;
    pk->chunk = chunk_bytes ? chunk_bytes : (64ull << 20);
    pk->path = strdup(path);
    pk->fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (!pk->path || pk->fd < 0) {
        pk_free(pk, false);
        return ZSCRC_EINVAL;
    }
    /* header: CRC over host-order fields (zeroskip-header.c:30-94) */
    uint8_t h[HDR];
    const uint64_t sig = SIGNATURE;
    uint32_t c = crc32c_hw(0, nullptr, 0);
    c = crc32c_hw(c, &sig, 8);
    c = crc32c_hw(c, &VERSION, 4);
    c = crc32c_hw(c, uuid, 16);
    c = crc32c_hw(c, &startidx, 4);
    c = crc32c_hw(c, &endidx, 4);
    memcpy(h, &sig, 8); /* native order, as zs_header_write stores it */
    put_be32(h + 8, VERSION);
    memcpy(h + 12, uuid, 16);
    put_be32(h + 28, startidx);
    put_be32(h + 32, endidx);
    put_be32(h + 36, c);
    int rc = write_all(pk->fd, h, HDR, 0);
    /* crc32_begin (packed.c:424): the records region starts after the header */
    if (!rc)
        rc = zscrc_stream_open(&pk->st, 0, pk->chunk, 0);
    if (rc) {
        pk_free(pk, true);
        return rc;
    }
    pk->out_off = pk->pos = HDR;
    *out = pk;
    return ZSCRC_OK;
}

int zscrc_pack_add(zscrc_packer *pk, const void *key, uint64_t keylen, const void *val, uint64_t vallen)
{
    if (!pk || (!key && keylen))
        return ZSCRC_EINVAL;
    static const uint8_t empty = 0;
    if (!key)
        key = &empty;
    if (pk->err)
        return pk->err;
    pk->ptrs.push_back(pk->pos); /* zs_packed_file_write_memtree_record: vecu64_append(offset) */
    uint8_t head[24] = {0};
    const uint64_t kbuflen = 24 + rup8(keylen);
    if (!val) {
        /* zs_prepare_delete_key_buf (zeroskip-file.c:137-183).  A long delete
         * leaves its first word unwritten (zero), as the reference does. */
        if (keylen <= MAX_SHORT_KEY_LEN)
            put_be64(head, ((uint64_t)T_DELETED << 56) | (keylen << 40));
        else
            put_be64(head + 8, keylen);
    } else if (keylen > MAX_SHORT_KEY_LEN) {
        put_be64(head, (uint64_t)(T_KEY | T_LONG) << 56); /* zs_prepare_key_buf :59-69 */
        put_be64(head + 8, keylen);
        put_be64(head + 16, kbuflen);
    } else {
        put_be64(head, ((uint64_t)T_KEY << 56) | (keylen << 40) | kbuflen);
    }
    int rc = put(pk, head, 24);
    if (!rc)
        rc = put(pk, key, keylen);
    if (!rc)
        rc = put(pk, nullptr, kbuflen - 24 - keylen);
    if (rc || !val)
        return rc;
    /* zs_prepare_val_buf (zeroskip-file.c:83-133) */
    uint8_t vh[16] = {0};
    if (vallen > MAX_SHORT_VAL_LEN) {
        put_be64(vh, (uint64_t)(T_VALUE | T_LONG) << 56);
        put_be64(vh + 8, vallen);
    } else {
        put_be64(vh, ((uint64_t)T_VALUE << 56) | (vallen << 32));
    }
    rc = put(pk, vh, 16);
    if (!rc)
        rc = put(pk, val, vallen);
    if (!rc)
        rc = put(pk, nullptr, rup8(vallen) - vallen);
    return rc;
}

int zscrc_pack_add_batch(zscrc_packer *pk, const void *keys, const uint64_t *key_off, const uint64_t *key_len,
                         const void *vals, const uint64_t *val_off, const uint64_t *val_len, size_t n)
{
    if (!pk || (n && (!key_off || !key_len || (vals && (!val_off || !val_len)))))
        return ZSCRC_EINVAL;
    const uint8_t *kb = static_cast<const uint8_t *>(keys), *vb = static_cast<const uint8_t *>(vals);
    for (size_t i = 0; i < n; ++i) {
        /* NULL vals: every record a delete; else val_off[i] == ~0 marks one */
        const bool del = !vb || val_off[i] == ~0ull;
        int rc = zscrc_pack_add(pk, kb + key_off[i], key_len[i], del ? nullptr : vb + val_off[i],
                                del ? 0 : val_len[i]);
        if (rc)
            return rc;
    }
    return ZSCRC_OK;
}

int zscrc_pack_abort(zscrc_packer *pk)
{
    /* a partial repack must never look valid: no commits, the file removed
     * (the reference's fail path xunlinks it, src/zeroskip-packed.c:465-466) */
    if (!pk)
        return ZSCRC_EINVAL;
    pk_free(pk, true);
    return ZSCRC_OK;
}

int zscrc_pack_close(zscrc_packer *pk, zscrc_pack_report *rep)
{
    if (!pk)
        return ZSCRC_EINVAL;
    zscrc_pack_report r;
    memset(&r, 0, sizeof r);
    int rc = pk->err;
    /* records-region commit (packed.c:442, zs_file_write_commit_record(f, 0)) */
    uint8_t rec[24];
    if (!rc) {
        r.region_bytes = pk->pos - HDR;
        rc = end_span(pk, &r.region_crc);
    }
    if (!rc) {
        const uint64_t n = commit_record(rec, r.region_crc, r.region_bytes, false, &r.commit_crc);
        rc = write_all(pk->fd, rec, n, pk->pos);
        pk->pos += n;
    }
    /* pointer section: crc32_begin, count, pointers (packed.c:449-453) */
    const uint64_t pstart = pk->pos;
    if (!rc) {
        pk->out_off = pstart;
        const uint64_t pbytes = 8 * ((uint64_t)pk->ptrs.size() + 1);
        rc = zscrc_stream_open(&pk->st, 0, pbytes < pk->chunk ? pbytes : pk->chunk, 0);
    }
    if (!rc) {
        uint8_t w[8];
        put_be64(w, pk->ptrs.size());
        rc = put(pk, w, 8);
        /* big-endian pointers, staged a block at a time */
        std::vector<uint8_t> blk;
        blk.resize(8 * 65536);
        for (size_t i = 0; !rc && i < pk->ptrs.size(); i += 65536) {
            const size_t m = pk->ptrs.size() - i < 65536 ? pk->ptrs.size() - i : 65536;
            for (size_t j = 0; j < m; ++j)
                put_be64(blk.data() + 8 * j, pk->ptrs[i + j]);
            rc = put(pk, blk.data(), 8 * m);
        }
    }
    if (!rc)
        rc = end_span(pk, &r.pointers_crc);
    if (!rc) {
        const uint64_t n = commit_record(rec, r.pointers_crc, pk->pos - pstart, true, &r.final_crc);
        rc = write_all(pk->fd, rec, n, pk->pos);
        pk->pos += n;
    }
    if (!rc && (pk->flags & ZSCRC_PACK_FSYNC) && fsync(pk->fd) != 0)
        rc = ZSCRC_EINVAL;
    r.records = pk->ptrs.size();
    r.file_bytes = pk->pos;
    if (rep)
        *rep = r;
    pk_free(pk, rc != 0);
    return rc;
}

} /* extern "C" */
