/* Written against include/zscrc.h Part 1 only, calling the library the way
 * zeroskip's sources do (chained crc32c_hw over host-order words,
 * src/zeroskip-file.c:283-318; crc32c_init + crc32c as tests/unit-crc32c.c).
 * Exit 0 iff every result matches the reference's known answers. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/uio.h>

#include "zscrc.h"

int main(void)
{
    int bad = 0;
    crc32c_init();
    uint32_t c1 = crc32c(0, 0, 0);
    c1 = crc32c(c1, "lorem", 5);
    c1 = crc32c(c1, " ipsum", 6);
    bad |= c1 != 0xdfb4e6c9u;                                   /* tests/unit-crc32c.c:36 */
    bad |= crc32c_hw(0, "123456789", 9) != 0xE3069283u;
    bad |= crc32c_sw(0, "123456789", 9) != 0xE3069283u;
    bad |= crc32c_map("lorem ipsum", 11) != 0xdfb4e6c9u;
    bad |= crc32c_buf("lorem ipsum") != 0xdfb4e6c9u;
    char text[] = "lorem ipsum";
    cstring cs = {11, 12, text};
    bad |= crc32c_cstring(&cs) != 0xdfb4e6c9u;
    struct iovec iov[3] = {{text, 3}, {text + 3, 0}, {text + 3, 8}};
    bad |= crc32c_iovec(iov, 3) != 0xdfb4e6c9u;
    /* a short commit trailer chained on a span CRC, as zs_file_write_commit_record */
    uint32_t span = crc32c_hw(0, "lorem ipsum", 11);
    uint64_t val = ((uint64_t)4 << 56) | ((uint64_t)11 << 32);
    uint32_t a = crc32c_hw(span, &val, sizeof val);
    unsigned char whole[19];
    memcpy(whole, "lorem ipsum", 11);
    memcpy(whole + 11, &val, 8);
    bad |= a != crc32c_hw(0, whole, 19);
    bad |= crc32c_combine(crc32c_hw(0, "lorem", 5), crc32c_hw(0, " ipsum", 6), 6) != 0xdfb4e6c9u;
    printf("%s\n", bad ? "FAIL" : "OK");
    return bad;
}
