/*
 * zs_format_oracle.c -- CPU restatement of the CRC semantics of zeroskip's
 * on-disk records (TEST INFRASTRUCTURE ONLY; see zs_oracle.c header).
 *
 * All fields are hashed in host (little-endian) order, not as the big-endian
 * bytes written to disk, and every value is chained through crc32c_hw:
 *   - short commit: zeroskip-file.c:303-328
 *   - long commit (WRITER semantics, type2 = 2ND_HALF << 56): zeroskip-file.c:266-302
 *     (the long-commit verifier zeroskip-record.c:234-266 is buggy; the packed
 *      verifier zeroskip-packed.c:289-312 agrees with the writer)
 *   - 40-byte file header, CRC over 36 B of host-order fields: zeroskip-header.c:66-76
 *   - .zsdb metadata CRC over 57 B of host-order fields: zeroskip-dotzsdb.c:105-119
 */
#include <stdint.h>
#include <stddef.h>

uint32_t oracle_crc32c_hw(uint32_t crc, const void *buf, size_t len);

enum { REC_COMMIT = 4, REC_2ND_HALF = 8, REC_FINAL = 16, REC_LONG = 32 };
#define MAX_SHORT_VAL_LEN 16777215ull /* zeroskip-priv.h:171 */

/* Stored 32-bit CRC of a commit record whose span CRC is span_crc
 * (crc32c_hw(0, span, span_len)).  final != 0 -> FINAL / LONG_FINAL. */
uint32_t oracle_commit_crc(uint32_t span_crc, uint64_t span_len, int final)
{
    uint64_t v;
    if (span_len > MAX_SHORT_VAL_LEN) {
        uint32_t c;
        v = (uint64_t)(final ? (REC_FINAL | REC_LONG) : (REC_COMMIT | REC_LONG)) << 56;
        c = oracle_crc32c_hw(span_crc, &v, 8);
        v = span_len;
        c = oracle_crc32c_hw(c, &v, 8);
        v = (uint64_t)REC_2ND_HALF << 56;
        return oracle_crc32c_hw(c, &v, 8);
    }
    v = ((uint64_t)(final ? REC_FINAL : REC_COMMIT) << 56) | (span_len << 32);
    return oracle_crc32c_hw(span_crc, &v, 8);
}

/* Header CRC: signature(8, native) || version || uuid(16) || startidx || endidx. */
uint32_t oracle_header_crc(uint64_t signature, uint32_t version, const uint8_t uuid[16],
                           uint32_t startidx, uint32_t endidx)
{
    uint32_t c = oracle_crc32c_hw(0, 0, 0);
    c = oracle_crc32c_hw(c, &signature, 8);
    c = oracle_crc32c_hw(c, &version, 4);
    c = oracle_crc32c_hw(c, uuid, 16);
    c = oracle_crc32c_hw(c, &startidx, 4);
    return oracle_crc32c_hw(c, &endidx, 4);
}

/* .zsdb CRC: signature(8) || offset(8) || uuidstr(37) || curidx(4). */
uint32_t oracle_dotzsdb_crc(uint64_t signature, uint64_t offset, const char uuidstr[37],
                            uint32_t curidx)
{
    uint32_t c = oracle_crc32c_hw(0, 0, 0);
    c = oracle_crc32c_hw(c, &signature, 8);
    c = oracle_crc32c_hw(c, &offset, 8);
    c = oracle_crc32c_hw(c, uuidstr, 37);
    return oracle_crc32c_hw(c, &curidx, 4);
}
