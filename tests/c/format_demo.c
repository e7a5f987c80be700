/*
 * Format-layer demonstrator (TEST INFRASTRUCTURE ONLY): the reference's OWN
 * writer and verifiers -- src/zeroskip-file.c, zeroskip-record.c,
 * zeroskip-header.c, zeroskip-packed.c and mfile.c (with what they pull from
 * the rest of the library), compiled unmodified from /root/reference by
 * oracle/Makefile's `ref-format` target -- linked against libzscrc.so
 * instead of src/crc32c.c.  Every CRC these
 * sources compute goes through the drop-in crc32c / crc32c_hw symbols.
 * tests/test_reference_format.py drives it and holds oracle/zs_format.py and
 * the product's walk / GPU verifier to what it writes and what it accepts.
 *
 * usage: format_demo write OUT BLOB < OPS
 *   one op per line; key/value bytes are slices of the file BLOB:
 *     H <uuid hex32> <startidx> <endidx>  zs_header_write (zeroskip-header.c:30)
 *     A <koff> <klen> <voff> <vlen>       zsdb_add's file half (zeroskip.c:930-936):
 *                                         crc32_begin unless one is running,
 *                                         zs_file_write_keyval_record
 *     D <koff> <klen>                     zsdb_remove's file half (zeroskip.c:985-987):
 *                                         crc32_begin always, zs_file_write_delete_record
 *     a <koff> <klen> <voff> <vlen>       zs_file_write_keyval_record alone (the packed
 *                                         writer, zeroskip-packed.c:163-176)
 *     d <koff> <klen>                     zs_file_write_delete_record alone
 *     C                                   zs_file_write_commit_record(f, 0)
 *     F                                   zs_file_write_commit_record(f, 1)
 *     B                                   crc32_begin alone (zeroskip-packed.c:424, :449)
 *     P <count> <off>...                  the packed pointer section's words, big-endian
 *   prints {"size": N}
 *
 * usage: format_demo packed FILE
 *   zs_packed_file_open (zeroskip-packed.c:215-365): the header, then the
 *   pointer section's commit -- short or long FINAL, the reference's one
 *   correct long-trailer verifier -- and the pointers.
 *   Prints {"rc": rc, "count": pointers read}.
 *
 * usage: format_demo repack1 OUT UUIDHEX STARTIDX ENDIDX FINALISED...
 *   zsdb_repack's branch 1 (src/zeroskip.c:1460-1505) on the reference's own
 *   code: the finalised files opened (zs_finalised_file_open), ordered and
 *   loaded into the memtree as zsdb_open does (zeroskip.c:749-767: a pqueue by
 *   natural_strcasecmp of the names, list_add_head, loaded in reverse, a later
 *   record of a key replacing an earlier one -- the two 10-line static
 *   callbacks of zeroskip.c:72-96 restated here), then
 *   zs_packed_file_new_from_memtree writes OUT.  Prints {"rc": rc}.
 * usage: format_demo repack2 OUT UUIDHEX STARTIDX ENDIDX PACKED...
 *   Branch 2 (zeroskip.c:1510-1565): the packed files opened
 *   (zs_packed_file_open), ordered and given priorities as zsdb_open does
 *   (zeroskip.c:512-526), the first two of that list merged by
 *   zs_iterator_new + zs_packed_file_new_from_packed_files into OUT.
 *
 * usage: format_demo verify FILE
 *   zs_header_validate (zeroskip-header.c:105), then zs_record_read_from_file
 *   (zeroskip-record.c:283) from offset 40 until the offset stops moving.
 *   Prints one JSON line: the header rc, each short commit's offset and rc,
 *   the long commits met (listed, not verified: zeroskip-record.c:258 hands
 *   the length VALUE to crc32c_hw as a pointer, so the reference's own
 *   verifier cannot run on them), and the offset the walk stopped at.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <libzeroskip/memtree.h>
#include <libzeroskip/mfile.h>
#include <libzeroskip/util.h>
#include <libzeroskip/vecu64.h>
#include <libzeroskip/zeroskip.h>

#include "pqueue.h"
#include "zeroskip-priv.h"

static int hexbyte(const char *s)
{
    unsigned v;
    return sscanf(s, "%2x", &v) == 1 ? (int)v : -1;
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

static int do_write(const char *out, const char *blobpath)
{
    size_t nblob = 0;
    unsigned char *blob = load(blobpath, &nblob);
    if (!blob) {
        perror("blob");
        return 1;
    }
    struct zsdb_file f;
    memset(&f, 0, sizeof f);
    f.type = DB_FTYPE_ACTIVE;
    if (mfile_open(out, MFILE_RW_CR, &f.mf) != 0) {
        perror("mfile_open");
        return 1;
    }
    f.is_open = 1;
    char line[1 << 16];
    int rc = 0;
    while (!rc && fgets(line, sizeof line, stdin)) {
        unsigned long long a, b, c, d;
        char hex[64];
        switch (line[0]) {
        case 'H':
            if (sscanf(line + 1, "%32s %llu %llu", hex, &a, &b) != 3 || strlen(hex) != 32)
                return 2;
            f.header.signature = ZS_SIGNATURE;
            f.header.version = ZS_VERSION;
            for (int i = 0; i < 16; ++i)
                f.header.uuid[i] = (unsigned char)hexbyte(hex + 2 * i);
            f.header.startidx = (uint32_t)a;
            f.header.endidx = (uint32_t)b;
            rc = zs_header_write(&f);
            break;
        case 'A':
        case 'a':
            if (sscanf(line + 1, "%llu %llu %llu %llu", &a, &b, &c, &d) != 4 || a + b > nblob ||
                c + d > nblob)
                return 2;
            if (line[0] == 'A' && !f.mf->compute_crc)
                crc32_begin(&f.mf);
            rc = zs_file_write_keyval_record(&f, blob + a, b, blob + c, d);
            break;
        case 'D':
        case 'd':
            if (sscanf(line + 1, "%llu %llu", &a, &b) != 2 || a + b > nblob)
                return 2;
            if (line[0] == 'D')
                crc32_begin(&f.mf);
            rc = zs_file_write_delete_record(&f, blob + a, b);
            break;
        case 'C':
        case 'F':
            rc = zs_file_write_commit_record(&f, line[0] == 'F');
            break;
        case 'B':
            crc32_begin(&f.mf);
            break;
        case 'P': {
            char *s = line + 1;
            while (!rc && *s && *s != '\n') {
                char *e;
                unsigned long long v = strtoull(s, &e, 10);
                if (e == s)
                    break;
                s = e;
                unsigned char w[8];
                for (int i = 0; i < 8; ++i)
                    w[i] = (unsigned char)(v >> (56 - 8 * i));
                uint64_t nb;
                rc = mfile_write(&f.mf, w, 8, &nb);
            }
            break;
        }
        default:
            return 2;
        }
    }
    if (rc) {
        fprintf(stderr, "reference writer returned %d\n", rc);
        return 1;
    }
    uint64_t size = f.mf->offset;
    if (mfile_flush(&f.mf) != 0 || mfile_close(&f.mf) != 0)
        return 1;
    free(blob);
    printf("{\"size\": %llu}\n", (unsigned long long)size);
    return 0;
}

static int do_verify(const char *path)
{
    struct zsdb_file f;
    memset(&f, 0, sizeof f);
    f.type = DB_FTYPE_ACTIVE;
    if (mfile_open(path, MFILE_RD, &f.mf) != 0) {
        perror("mfile_open");
        return 1;
    }
    f.is_open = 1;
    size_t size = 0;
    mfile_size(&f.mf, &size);
    printf("{\"header\": %d, \"commits\": [", zs_header_validate(&f));
    uint64_t off = ZS_HDR_SIZE;
    const char *sep = "", *why = "end";
    char longs[1 << 14] = "";
    size_t nl = 0;
    while (off + 8 <= size) {
        const unsigned char t = f.mf->ptr[off];
        if (t == REC_TYPE_LONG_COMMIT) {
            nl += (size_t)snprintf(longs + nl, sizeof longs - nl, "%s%llu", nl ? ", " : "",
                                   (unsigned long long)off);
            if (nl >= sizeof longs)
                return 1;
            off += ZS_LONG_COMMIT_REC_SIZE;
            continue;
        }
        const uint64_t before = off;
        const int rc = zs_record_read_from_file(&f, &off, NULL, NULL, NULL);
        if (t == REC_TYPE_COMMIT) {
            printf("%s[%llu, %d]", sep, (unsigned long long)before, rc);
            sep = ", ";
        }
        if (off == before) {
            why = "stopped";
            break;
        }
    }
    printf("], \"long_commits\": [%s], \"stop\": %llu, \"why\": \"%s\"}\n", longs,
           (unsigned long long)off, why);
    mfile_close(&f.mf);
    return 0;
}

/* zeroskip.c:64-70 */
static int dbfname_cmp(const void *d1, const void *d2, void *cbdata)
{
    (void)cbdata;
    return natural_strcasecmp(((const struct zsdb_file *)d1)->fname.buf, ((const struct zsdb_file *)d2)->fname.buf);
}

/* zeroskip.c:72-96 */
static int load_cb(void *data, const unsigned char *key, size_t keylen, const unsigned char *value, size_t vallen)
{
    memtree_replace((struct memtree *)data, record_new(key, keylen, value, vallen, 0));
    return 0;
}

static int load_deleted_cb(void *data, const unsigned char *key, size_t keylen, const unsigned char *value,
                           size_t vallen)
{
    memtree_replace((struct memtree *)data, record_new(key, keylen, value, vallen, 1));
    return 0;
}

static int do_repack(int branch, const char *out, const char *uuidhex, uint32_t sidx, uint32_t eidx, int nf,
                     char **files)
{
    struct zsdb db;
    struct zsdb_priv priv;
    memset(&db, 0, sizeof db);
    memset(&priv, 0, sizeof priv);
    if (strlen(uuidhex) != 32)
        return 2;
    for (int i = 0; i < 16; ++i)
        priv.uuid[i] = (unsigned char)hexbyte(uuidhex + 2 * i);
    priv.open = 1;
    cstring_init(&priv.dbdir, 0);
    db.priv = &priv;
    struct pqueue pq;
    memset(&pq, 0, sizeof pq);
    pq.cmp = dbfname_cmp;
    for (int i = 0; i < nf; ++i) {
        struct zsdb_file *f = NULL;
        const int rc = branch == 1 ? zs_finalised_file_open(files[i], &f) : zs_packed_file_open(files[i], &f);
        if (rc != ZS_OK || !f) {
            printf("{\"rc\": %d, \"open\": \"%s\"}\n", rc, files[i]);
            return 0;
        }
        pqueue_put(&pq, f);
    }
    /* the lists zsdb_open builds: priv->dbfiles.fflist / pflist */
    list_head_init(&priv.dbfiles.fflist);
    list_head_init(&priv.dbfiles.pflist);
    struct list_head *lst = branch == 1 ? &priv.dbfiles.fflist : &priv.dbfiles.pflist;
    while (pq.count) {
        struct zsdb_file *f = pqueue_get(&pq);
        list_add_head(&f->list, lst);
    }
    pqueue_free(&pq);
    struct list_head *pos, *p;
    int rc = ZS_OK, priority = 0;
    struct zsdb_file *nf_out = NULL;
    if (branch == 1) {
        priv.fmemtree = memtree_new(NULL, NULL);
        list_for_each_reverse(pos, lst) {
            struct zsdb_file *f = list_entry(pos, struct zsdb_file, list);
            zs_finalised_file_record_foreach(f, load_cb, load_deleted_cb, priv.fmemtree);
            f->priority = ++priority;
        }
        rc = zs_packed_file_new_from_memtree(out, sidx, eidx, &priv, &nf_out);
    } else {
        list_for_each_forward(pos, lst) {
            struct zsdb_file *f = list_entry(pos, struct zsdb_file, list);
            f->priority = ++priority;
        }
        struct list_head two;
        list_head_init(&two);
        int i = 0;
        list_for_each_forward_safe(pos, p, lst) {
            struct zsdb_file *f = list_entry(pos, struct zsdb_file, list);
            if (i == 2)
                break;
            list_del(pos);
            list_add_head(&f->list, &two);
            ++i;
        }
        struct zsdb_iter *iter = NULL;
        rc = zs_iterator_new(&db, &iter);
        if (rc == ZS_OK)
            rc = zs_packed_file_new_from_packed_files(out, sidx, eidx, &priv, &two, &iter, &nf_out);
        zs_iterator_end(&iter);
    }
    if (nf_out)
        zs_packed_file_close(&nf_out);
    printf("{\"rc\": %d}\n", rc);
    return 0;
}

static int do_packed(const char *path)
{
    struct zsdb_file *f = NULL;
    const int rc = zs_packed_file_open(path, &f);
    unsigned long long count = rc == ZS_OK && f && f->index ? (unsigned long long)f->index->count : 0;
    printf("{\"rc\": %d, \"count\": %llu}\n", rc, count);
    if (rc == ZS_OK && f)
        zs_packed_file_close(&f);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc == 4 && strcmp(argv[1], "write") == 0)
        return do_write(argv[2], argv[3]);
    if (argc == 3 && strcmp(argv[1], "verify") == 0)
        return do_verify(argv[2]);
    if (argc == 3 && strcmp(argv[1], "packed") == 0)
        return do_packed(argv[2]);
    if (argc >= 7 && (strcmp(argv[1], "repack1") == 0 || strcmp(argv[1], "repack2") == 0))
        return do_repack(argv[1][6] - '0', argv[2], argv[3], (uint32_t)strtoul(argv[4], NULL, 0),
                         (uint32_t)strtoul(argv[5], NULL, 0), argc - 6, argv + 6);
    fprintf(stderr, "usage: %s write OUT BLOB < OPS | verify FILE | packed FILE\n", argv[0]);
    return 2;
}
