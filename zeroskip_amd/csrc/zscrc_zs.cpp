/*
 * zscrc_zs.cpp -- zeroskip file images -> commit span descriptors -> GPU
 * verification (the "next" row of SURVEY.md sec 8f: verify-on-open,
 * `consistent`, repack re-checksum).
 *
 * The record walk is the reference's, restated for the checksum parts only:
 *   walk            src/zeroskip-record.c:283-331 (stops, like the reference,
 *                   at record types it does not advance over)
 *   key + value     src/zeroskip-record.c:75-106,156-181 (value offset from
 *                   the key word, value length from the value word)
 *   delete          src/zeroskip-record.c:183-199 (uint16 key length)
 *   commit          src/zeroskip-record.c:188-273 -- but with the WRITER's
 *                   long-commit trailer (src/zeroskip-file.c:266-302); the
 *                   reference verifier's long branch dereferences a length
 *   packed file     src/zeroskip-packed.c:70-131 (pointer section located from
 *                   the final commit at the end of the file), :278-339
 *   header CRC      src/zeroskip-header.c:105-170 (host-order fields)
 *   .zsdb CRC       src/zeroskip-dotzsdb.c:160-235 (host-order fields)
 * The walk is serial by construction (the next offset depends on the record
 * just parsed), so it runs on the host; every byte of every commit span and
 * every trailer is checksummed and compared on the GPU.
 */
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "../../include/zscrc.h"
#include "zscrc_internal.h"

extern "C" int zscrc_internal_verify_commits(const void *d_image, uint64_t image_size, const uint64_t *d_off,
                                             const uint64_t *d_len, const uint32_t *d_seed, uint32_t *d_crc,
                                             uint32_t *d_status, size_t n, void *stream, int write,
                                             uint64_t max_len);

namespace {

constexpr uint64_t HDR = 40;
constexpr uint64_t SIGNATURE = 0x5a45524f534b4950ull; /* zeroskip-priv.h:49 */
enum {
    T_KEY = 1, T_VALUE = 2, T_COMMIT = 4, T_2ND = 8, T_FINAL = 16, T_LONG = 32, T_DELETED = 64,
    T_LONG_KEY = 33, T_LONG_VALUE = 34, T_LONG_COMMIT = 36, T_LONG_FINAL = 48,
    T_LONG_DELETED_ALIAS = 32, /* REC_TYPE_LONG_DELETED = LONG|LONG (zeroskip-priv.h:119) */
};

inline uint64_t be64(const uint8_t *p)
{
    uint64_t v;
    memcpy(&v, p, 8);
    return __builtin_bswap64(v);
}
inline uint32_t be32(const uint8_t *p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return __builtin_bswap32(v);
}
inline uint64_t rup8(uint64_t n) { return (n + 7) & ~7ull; }

/* Length of the commit record at off and its span; false if not a commit. */
bool commit_at(const uint8_t *img, uint64_t size, uint64_t off, uint64_t *span_len, uint64_t *rec_len)
{
    if (off + 8 > size)
        return false;
    const uint64_t w = be64(img + off);
    const unsigned t = (unsigned)(w >> 56);
    if (t == T_COMMIT || t == T_FINAL) {
        *span_len = (w >> 32) & 0xFFFFFF;
        *rec_len = 8;
    } else if (t == T_LONG_COMMIT || t == T_LONG_FINAL) {
        if (off + 24 > size)
            return false;
        *span_len = be64(img + off + 8);
        *rec_len = 24;
    } else {
        return false;
    }
    return *span_len <= off;
}

} /* namespace */

extern "C" {

int zscrc_zs_walk(const void *image, uint64_t size, uint64_t *span_off, uint64_t *span_len, size_t cap,
                  size_t *n_commits, uint64_t *end_off)
{
    const uint8_t *img = static_cast<const uint8_t *>(image);
    size_t n = 0;
    uint64_t off = HDR;
    int rc = ZSCRC_ZS_END;
    if (!img || size < HDR)
        return ZSCRC_EINVAL;
    /* Every length word comes from the file, which may be corrupt: each step
     * is checked against the bytes left (`room`, never an add that can wrap),
     * so the next offset is always past the current one and inside the image
     * or the walk stops with TRUNCATED. */
    while (off < size) {
        const uint64_t room = size - off;
        if (room < 8) {
            rc = ZSCRC_ZS_TRUNCATED;
            break;
        }
        const uint64_t w = be64(img + off);
        const unsigned t = (unsigned)(w >> 56);
        if (t == T_KEY || t == T_LONG_KEY) {
            uint64_t voff;
            if (t == T_KEY) {
                voff = w & 0xFFFFFFFFull;
            } else {
                if (room < 24) {
                    rc = ZSCRC_ZS_TRUNCATED;
                    break;
                }
                voff = be64(img + off + 16);
            }
            /* the value record (16-byte header) starts voff bytes on */
            if (voff == 0 || voff > room || room - voff < 16) {
                rc = ZSCRC_ZS_TRUNCATED;
                break;
            }
            const uint64_t v = off + voff;
            const uint64_t vw = be64(img + v);
            const uint64_t vlen = (vw >> 56) == T_VALUE ? ((vw >> 32) & 0xFFFFFF) : be64(img + v + 8);
            const uint64_t vroom = size - v - 16;
            if (vlen > vroom || rup8(vlen) > vroom) { /* vlen <= vroom: rup8 cannot wrap */
                rc = ZSCRC_ZS_TRUNCATED;
                break;
            }
            off = v + 16 + rup8(vlen);
        } else if (t == T_DELETED || t == T_LONG_DELETED_ALIAS) {
            if (room < 24) {
                rc = ZSCRC_ZS_TRUNCATED;
                break;
            }
            const uint64_t klen = t == T_DELETED ? ((w >> 40) & 0xFFFF) : be64(img + off + 8);
            if (klen > room - 24 || rup8(klen) > room - 24) {
                rc = ZSCRC_ZS_TRUNCATED;
                break;
            }
            off += 24 + rup8(klen);
        } else if (t == T_COMMIT || t == T_LONG_COMMIT) {
            uint64_t sl, rl;
            if (!commit_at(img, size, off, &sl, &rl)) {
                rc = ZSCRC_ZS_TRUNCATED;
                break;
            }
            if (n < cap) {
                span_off[n] = off - sl;
                span_len[n] = sl;
            }
            ++n;
            off += rl;
        } else {
            rc = ZSCRC_ZS_STOPPED; /* FINAL / 2ND_HALF / UNUSED / VALUE: not advanced over */
            break;
        }
    }
    if (n_commits)
        *n_commits = n;
    if (end_off)
        *end_off = off;
    return n > cap ? ZSCRC_ZS_OVERFLOW : rc;
}

int zscrc_zs_packed_spans(const void *image, uint64_t size, uint64_t span_off[2], uint64_t span_len[2])
{
    const uint8_t *img = static_cast<const uint8_t *>(image);
    if (!img || size < HDR + 16)
        return ZSCRC_EINVAL;
    /* final commit at the end: short FINAL, or LONG_FINAL whose 2ND_HALF word
     * ends the file (get_offset_to_pointers, zeroskip-packed.c:70-131) */
    uint64_t foff = size - 8;
    if ((be64(img + foff) >> 56) == T_2ND)
        foff = size - 24;
    uint64_t sl, rl;
    if (!commit_at(img, size, foff, &sl, &rl) || rl != size - foff)
        return ZSCRC_ZS_TRUNCATED;
    const unsigned ft = (unsigned)(be64(img + foff) >> 56);
    if (ft != T_FINAL && ft != T_LONG_FINAL)
        return ZSCRC_ZS_TRUNCATED;
    span_off[1] = foff - sl;
    span_len[1] = sl;
    /* the records-region commit ends where the pointer section starts */
    const uint64_t pstart = foff - sl;
    if (pstart < HDR + 8)
        return ZSCRC_ZS_TRUNCATED;
    uint64_t roff = pstart - 8;
    if ((be64(img + roff) >> 56) == T_2ND && pstart >= HDR + 24)
        roff = pstart - 24;
    if (!commit_at(img, size, roff, &sl, &rl) || roff + rl != pstart)
        return ZSCRC_ZS_TRUNCATED;
    span_off[0] = roff - sl;
    span_len[0] = sl;
    return ZSCRC_OK;
}

int zscrc_zs_header_crc(const void *image, uint64_t size, uint32_t *stored, uint32_t *computed)
{
    const uint8_t *img = static_cast<const uint8_t *>(image);
    if (!img || size < HDR)
        return ZSCRC_EINVAL;
    uint64_t sig;
    memcpy(&sig, img, 8); /* native byte order (zeroskip-header.c:48) */
    const uint32_t version = be32(img + 8), sidx = be32(img + 28), eidx = be32(img + 32);
    uint32_t c = crc32c_hw(0, 0, 0);
    c = crc32c_hw(c, &sig, 8);
    c = crc32c_hw(c, &version, 4);
    c = crc32c_hw(c, img + 12, 16);
    c = crc32c_hw(c, &sidx, 4);
    c = crc32c_hw(c, &eidx, 4);
    *computed = c;
    *stored = be32(img + 36);
    return sig == SIGNATURE ? ZSCRC_OK : ZSCRC_ZS_BADSIG;
}

int zscrc_zs_dotzsdb_crc(const void *image, uint64_t size, uint32_t *stored, uint32_t *computed)
{
    /* struct dotzsdb (zeroskip-priv.h:83-91, packed): signature u64 (native),
     * offset u64 (BE), uuidstr[37], curidx u32 (BE), crc u32 (BE) = 61 bytes */
    const uint8_t *img = static_cast<const uint8_t *>(image);
    if (!img || size < 61)
        return ZSCRC_EINVAL;
    uint64_t sig;
    memcpy(&sig, img, 8);
    const uint64_t offset = be64(img + 8);
    const uint32_t curidx = be32(img + 53);
    uint32_t c = crc32c_hw(0, 0, 0);
    c = crc32c_hw(c, &sig, 8);
    c = crc32c_hw(c, &offset, 8);
    c = crc32c_hw(c, img + 16, 37);
    c = crc32c_hw(c, &curidx, 4);
    *computed = c;
    *stored = be32(img + 57);
    return sig == SIGNATURE ? ZSCRC_OK : ZSCRC_ZS_BADSIG;
}

int zscrc_device_verify_commits(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                const uint64_t *d_span_len, size_t n, uint32_t *d_crc, uint32_t *d_status,
                                void *stream)
{
    return zscrc_internal_verify_commits(d_image, image_size, d_span_off, d_span_len, nullptr, d_crc, d_status, n,
                                         stream, 0, ZSCRC_LEN_UNBOUNDED);
}

int zscrc_device_verify_commits_seeded(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                       const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                       uint32_t *d_crc, uint32_t *d_status, void *stream)
{
    return zscrc_internal_verify_commits(d_image, image_size, d_span_off, d_span_len, d_seed, d_crc, d_status, n,
                                         stream, 0, ZSCRC_LEN_UNBOUNDED);
}

int zscrc_device_verify_commits_bounded(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                        const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                        uint64_t max_len, uint32_t *d_crc, uint32_t *d_status, void *stream)
{
    return zscrc_internal_verify_commits(d_image, image_size, d_span_off, d_span_len, d_seed, d_crc, d_status, n,
                                         stream, 0, max_len);
}

int zscrc_device_write_commits_bounded(void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                       const uint64_t *d_span_len, size_t n, uint64_t max_len, uint32_t *d_crc,
                                       uint32_t *d_status, void *stream)
{
    return zscrc_internal_verify_commits(d_image, image_size, d_span_off, d_span_len, nullptr, d_crc, d_status, n,
                                         stream, 1, max_len);
}

int zscrc_device_commit_crcs_bounded(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                     const uint64_t *d_span_len, size_t n, uint64_t max_len, uint32_t *d_crc,
                                     uint32_t *d_status, void *stream)
{
    return zscrc_internal_verify_commits(d_image, image_size, d_span_off, d_span_len, nullptr, d_crc, d_status, n,
                                         stream, 2, max_len);
}

int zscrc_device_write_commits(void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                               const uint64_t *d_span_len, size_t n, uint32_t *d_crc, uint32_t *d_status,
                               void *stream)
{
    return zscrc_internal_verify_commits(d_image, image_size, d_span_off, d_span_len, nullptr, d_crc, d_status, n,
                                         stream, 1, ZSCRC_LEN_UNBOUNDED);
}

int zscrc_zs_verify_image(const void *image, uint64_t size, int kind, zscrc_zs_report *rep)
{
    if (!image || !rep)
        return ZSCRC_EINVAL;
    memset(rep, 0, sizeof *rep);
    rep->header_rc = zscrc_zs_header_crc(image, size, &rep->header_stored, &rep->header_computed);
    uint64_t *off = nullptr, *len = nullptr;
    size_t n = 0;
    int rc;
    if (kind == ZSCRC_ZS_PACKED) {
        off = static_cast<uint64_t *>(malloc(2 * sizeof(uint64_t)));
        len = static_cast<uint64_t *>(malloc(2 * sizeof(uint64_t)));
        if (!off || !len) {
            free(off);
            free(len);
            return ZSCRC_ENOMEM;
        }
        rc = zscrc_zs_packed_spans(image, size, off, len);
        n = rc == ZSCRC_OK ? 2 : 0;
        rep->walk_rc = rc;
        rep->end_off = size;
    } else {
        /* a commit needs >= 8 bytes of file: bound the descriptor count */
        const size_t cap = (size_t)(size / 8) + 1;
        off = static_cast<uint64_t *>(malloc(cap * sizeof(uint64_t)));
        len = static_cast<uint64_t *>(malloc(cap * sizeof(uint64_t)));
        if (!off || !len) {
            free(off);
            free(len);
            return ZSCRC_ENOMEM;
        }
        rep->walk_rc = zscrc_zs_walk(image, size, off, len, cap, &n, &rep->end_off);
    }
    rep->n_commits = n;
    rc = ZSCRC_OK;
    if (n) {
        void *dimg = nullptr, *dmeta = nullptr;
        hipError_t e = hipMalloc(&dimg, size);
        if (e == hipSuccess)
            e = hipMalloc(&dmeta, n * 24);
        uint64_t *doff = static_cast<uint64_t *>(dmeta);
        uint64_t *dlen = doff + n;
        uint32_t *dcrc = reinterpret_cast<uint32_t *>(dlen + n);
        uint32_t *dst = dcrc + n;
        if (e == hipSuccess)
            e = hipMemcpy(dimg, image, size, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(doff, off, n * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(dlen, len, n * 8, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            rc = ZSCRC_EHIP;
        } else {
            uint64_t max_len = 0;
            for (size_t i = 0; i < n; ++i)
                max_len = len[i] > max_len ? len[i] : max_len;
            rc = zscrc_device_verify_commits_bounded(dimg, size, doff, dlen, nullptr, n, max_len, dcrc, dst,
                                                     nullptr);
            uint32_t *st = static_cast<uint32_t *>(malloc(n * 4));
            if (!rc && st && hipMemcpy(st, dst, n * 4, hipMemcpyDeviceToHost) == hipSuccess) {
                for (size_t i = 0; i < n; ++i) {
                    if (st[i] != 1) {
                        if (rep->n_bad == 0)
                            rep->first_bad = i;
                        rep->n_bad++;
                    }
                }
            } else if (!rc) {
                rc = ZSCRC_EHIP;
            }
            free(st);
        }
        if (dimg)
            (void)hipFree(dimg);
        if (dmeta)
            (void)hipFree(dmeta);
    }
    free(off);
    free(len);
    return rc;
}

} /* extern "C" */
