/*
 * zscrc_repack.cpp -- zsdb_repack (src/zeroskip.c:1419-1571) over a DB
 * directory, in C++, writing through the packed-file writer whose records-
 * region and pointer-section CRCs run on the GPU (zscrc_pack.cpp).
 *
 *   branch 1 (finalised files present): every finalised file's records --
 *     loaded oldest file first, a later record of a key replacing an earlier
 *     one and a delete kept as a delete record (the fmemtree of zsdb_open,
 *     src/zeroskip.c:496-508, load_memtree_record_cb / _deleted_) -- written
 *     in key order (memtree_walk_forward -> zs_packed_file_write_memtree_record,
 *     src/zeroskip-packed.c:163-176, :384-473) into zeroskip-<uuid>-<s>-<e>,
 *     s / e the finalised files' index range (zs_find_index_range_for_files,
 *     :395-425); the finalised files are unlinked (:1489-1497);
 *   branch 2 (no finalised files, two or more packed files): the first two
 *     files of pflist -- which zsdb_open builds newest first (pqueue_get in
 *     natural name order + list_add_head, :512-515), so the two with the
 *     largest indices, although the comment at :1518 says "oldest" -- merged
 *     by the packed-files iterator in key order: on a key present in both,
 *     the file with the larger priority wins, and pflist assigns priorities
 *     1, 2, ... from its head (:520-526), so the older of the two; a winning
 *     delete drops the key (zs_packed_file_new_from_packed_files,
 *     src/zeroskip-packed.c:617-742, `if (data->deleted) continue`); the two
 *     files are unlinked (:1555-1562);
 *   always: .zsdb rewritten with its CRC recomputed (zs_dotzsdb_update_end,
 *     src/zeroskip-dotzsdb.c:477-555: host-order fields hashed, :514-529),
 *     through .zsdb.lock renamed over it.
 *
 * Locking: as zs_dotzsdb_update_begin (src/zeroskip-dotzsdb.c:376-471,
 * file_lock_acquire, src/file-lock.c:128-131), .zsdb.lock is created with
 * O_CREAT | O_EXCL before .zsdb is read or the directory listed, and held
 * until the new .zsdb is renamed from it; a lock already held makes the call
 * return ZSCRC_EBUSY at once (the reference retries with back-off).
 *
 * The packed file is written under a temporary name (".tmp" suffix: not a
 * zeroskip file name) and renamed into place after the sources are unmapped,
 * then the sources are unlinked -- except one whose name the output took.
 * With a single finalised file zeroskip-<uuid>-<i>-<i> the output's name is
 * the source's: the reference then truncates the source it is reading and
 * unlinks the file it just wrote (src/zeroskip.c:1470-1497, survivable there
 * only because the records were copied into its memtree first); here the
 * rename replaces the source and nothing is lost.
 *
 * Records are listed by zscrc_zs_records (C: the record walk of
 * src/zeroskip-record.c:283-331 for active / finalised files, the pointer
 * section for packed files, zeroskip-packed.c:70-131), sorted by key
 * (memcmp_raw, include/libzeroskip/util.h:273-287) with a parallel merge sort
 * on the host, and handed to the writer one record at a time: no Python and
 * no per-record language crossing on the repack path.
 */
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zscrc.h"

namespace {

constexpr uint64_t HDR = 40;
constexpr size_t UUID_CHARS = 36;  /* UUID_STRLEN - 1, zeroskip-priv.h:53 */
constexpr size_t DOTZSDB_SIZE = 61;
enum { T_KEY = 1, T_VALUE = 2, T_COMMIT = 4, T_DELETED = 64, T_LONG = 32 };

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline uint64_t be64(const uint8_t *p)
{
    uint64_t v;
    memcpy(&v, p, 8);
    return __builtin_bswap64(v);
}
inline uint64_t rup8(uint64_t n) { return (n + 7) & ~7ull; }

/* The key (and value) record at `off`; false if it is not one or does not
 * fit the image.  r.val_off = ZSCRC_ZS_DELETED for a delete record. */
bool record_at(const uint8_t *img, uint64_t size, uint64_t off, zscrc_zs_record &r, uint64_t *next)
{
    if (off > size || size - off < 8)
        return false;
    const uint64_t room = size - off;
    const uint64_t w = be64(img + off);
    const unsigned t = (unsigned)(w >> 56);
    if (t == T_KEY || t == (T_KEY | T_LONG)) {
        uint64_t klen, voff;
        if (t == T_KEY) {
            klen = (w >> 40) & 0xFFFF;
            voff = w & 0xFFFFFFFFull;
        } else {
            if (room < 24)
                return false;
            klen = be64(img + off + 8);
            voff = be64(img + off + 16);
        }
        if (klen > room - 24 || voff > room || room - voff < 16 || voff < 24 + klen)
            return false;
        const uint64_t v = off + voff;
        const uint64_t vw = be64(img + v);
        const uint64_t vlen = (vw >> 56) == T_VALUE ? ((vw >> 32) & 0xFFFFFF) : be64(img + v + 8);
        const uint64_t vroom = size - v - 16;
        if (vlen > vroom || rup8(vlen) > vroom)
            return false;
        r.key_off = off + 24;
        r.key_len = klen;
        r.val_off = v + 16;
        r.val_len = vlen;
        *next = v + 16 + rup8(vlen);
        return true;
    }
    if (t == T_DELETED || t == T_LONG) { /* REC_TYPE_LONG_DELETED = LONG | LONG */
        if (room < 24)
            return false;
        const uint64_t klen = t == T_DELETED ? ((w >> 40) & 0xFFFF) : be64(img + off + 8);
        if (klen > room - 24 || rup8(klen) > room - 24)
            return false;
        r.key_off = off + 24;
        r.key_len = klen;
        r.val_off = ZSCRC_ZS_DELETED;
        r.val_len = 0;
        *next = off + 24 + rup8(klen);
        return true;
    }
    return false;
}

int memcmp_raw(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb)
{
    const int c = memcmp(a, b, la < lb ? la : lb);
    if (c)
        return c;
    return la < lb ? -1 : la > lb ? 1 : 0;
}

/* One record of the merge: key / value pointers into a mapped file, and its
 * load order (later replaces earlier). */
struct MRec {
    const uint8_t *k, *v; /* v == nullptr: delete */
    uint64_t kl, vl;
    uint64_t seq;
};

bool mrec_less(const MRec &a, const MRec &b)
{
    const int c = memcmp_raw(a.k, a.kl, b.k, b.kl);
    return c ? c < 0 : a.seq < b.seq;
}

/* Sort by (key, seq): T chunks sorted on T threads, then pairwise merges,
 * each round's merges on threads of their own. */
void parallel_sort(std::vector<MRec> &a, int threads)
{
    const size_t n = a.size();
    const size_t T = (size_t)std::max(1, std::min<int>(threads, (int)(n / 65536) + 1));
    std::vector<size_t> cut(T + 1);
    for (size_t i = 0; i <= T; ++i)
        cut[i] = n * i / T;
    {
        std::vector<std::thread> th;
        for (size_t i = 0; i < T; ++i)
            th.emplace_back([&, i] { std::sort(a.begin() + cut[i], a.begin() + cut[i + 1], mrec_less); });
        for (auto &t : th)
            t.join();
    }
    std::vector<MRec> tmp(n);
    std::vector<MRec> *src = &a, *dst = &tmp;
    while (cut.size() > 2) {
        std::vector<size_t> next;
        std::vector<std::thread> th;
        for (size_t i = 0; i + 1 < cut.size(); i += 2) {
            const size_t lo = cut[i], mid = cut[i + 1], hi = i + 2 < cut.size() ? cut[i + 2] : cut[i + 1];
            next.push_back(lo);
            th.emplace_back([=] {
                std::merge(src->begin() + lo, src->begin() + mid, src->begin() + mid, src->begin() + hi,
                           dst->begin() + lo, mrec_less);
            });
        }
        next.push_back(n);
        for (auto &t : th)
            t.join();
        std::swap(src, dst);
        cut.swap(next);
    }
    if (src != &a)
        a.swap(*src);
}

/* ZSCRC_REPACK_REFERENCE_COMPAT: branch 2 exactly as the reference's
 * packed-files iterator merges (zs_iterator_begin_for_packed_files /
 * zsdb_iter_data_next / zsdb_iter_data_process, src/zeroskip-iterator.c
 * :220-300, driven by zs_packed_file_new_from_packed_files,
 * src/zeroskip-packed.c:617-742).  Each source is a cursor over its records
 * (key order) with a priority (pflist order: 1 = the newest, 2 = the older
 * file) and a `deleted` flag.  The current key of every cursor sits in one
 * ordered table (the iterator's hash table + priority queue); a cursor whose
 * key is already there either takes the entry (higher priority: the other
 * cursor steps on) or steps on itself.  The smallest key is written unless
 * its cursor's flag is set.  The flag is set when a cursor STEPS onto a
 * delete (:258-259) and never cleared, so from a source's first delete after
 * its first record on, none of that source's records is written; a delete as
 * a source's first record is never flagged (begin reads the key without its
 * type) and is written as a delete record.  That loses data; the default
 * merge does not (it keeps every record, the older file winning a key and a
 * winning delete dropping it). */
struct Cursor {
    const uint8_t *img = nullptr;
    const std::vector<zscrc_zs_record> *recs = nullptr;
    int prio = 0;
    size_t pos = 0;
    bool deleted = false, done = false;
};

struct KeyRef {
    const uint8_t *k;
    uint64_t kl;
    bool operator<(const KeyRef &o) const { return memcmp_raw(k, kl, o.k, o.kl) < 0; }
};

void compat_merge(std::vector<Cursor> &cur, std::vector<MRec> &out)
{
    std::map<KeyRef, size_t> table; /* current key -> cursor */
    /* offer cursor c's current key; a cursor that loses steps on (iterative:
     * each live cursor holds at most one entry) */
    auto offer = [&](size_t c) {
        for (;;) {
            Cursor &u = cur[c];
            if (u.done)
                return;
            const zscrc_zs_record &r = (*u.recs)[u.pos];
            const KeyRef key{u.img + r.key_off, r.key_len};
            auto it = table.find(key);
            if (it == table.end()) {
                table.emplace(key, c);
                return;
            }
            size_t loser = c;
            if (u.prio > cur[it->second].prio) {
                loser = it->second;
                table.erase(it);
                table.emplace(key, c);
            }
            /* the loser steps on (zsdb_iter_data_next) */
            Cursor &l = cur[loser];
            if (++l.pos >= l.recs->size()) {
                l.done = true;
                return;
            }
            if ((*l.recs)[l.pos].val_off == ZSCRC_ZS_DELETED)
                l.deleted = true;
            c = loser;
        }
    };
    for (size_t c = 0; c < cur.size(); ++c) {
        cur[c].done = cur[c].recs->empty();
        offer(c);
    }
    uint64_t seq = 0;
    while (!table.empty()) {
        const auto first = table.begin();
        const size_t c = first->second;
        table.erase(first);
        Cursor &u = cur[c];
        if (!u.deleted) {
            const zscrc_zs_record &r = (*u.recs)[u.pos];
            out.push_back({u.img + r.key_off, r.val_off == ZSCRC_ZS_DELETED ? nullptr : u.img + r.val_off,
                           r.key_len, r.val_len, seq++});
        }
        if (++u.pos >= u.recs->size()) {
            u.done = true;
            continue;
        }
        if ((*u.recs)[u.pos].val_off == ZSCRC_ZS_DELETED)
            u.deleted = true;
        offer(c);
    }
}

struct DbFile {
    std::string name;
    int kind = 0;
    unsigned long s = 0, e = 0;
    const uint8_t *img = nullptr;
    size_t size = 0;
};

bool parse_name(const char *n, DbFile &f)
{
    if (strncmp(n, "zeroskip-", 9) != 0 || strlen(n) < 9 + UUID_CHARS + 2)
        return false;
    const char *p = n + 9 + UUID_CHARS;
    if (*p++ != '-' || *p < '0' || *p > '9')
        return false;
    char *q;
    f.s = strtoul(p, &q, 10);
    f.e = f.s;
    f.kind = ZSCRC_ZS_ACTIVE;
    if (*q == '-') {
        p = q + 1;
        if (*p < '0' || *p > '9')
            return false;
        f.e = strtoul(p, &q, 10);
        f.kind = f.e == f.s ? ZSCRC_ZS_FINALISED : ZSCRC_ZS_PACKED;
    }
    if (*q)
        return false;
    f.name = n;
    return true;
}

int hexval(char c)
{
    return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
}

/* uuid_parse of the 36-character form */
bool parse_uuid(const char *s, uint8_t out[16])
{
    int k = 0;
    for (int i = 0; i < 36; ++i) {
        if (i == 8 || i == 13 || i == 18 || i == 23) {
            if (s[i] != '-')
                return false;
            continue;
        }
        const int h = hexval(s[i]), l = i + 1 < 36 ? hexval(s[i + 1]) : -1;
        if (h < 0 || l < 0)
            return false;
        out[k++] = (uint8_t)(h << 4 | l);
        ++i;
    }
    return k == 16;
}

} /* namespace */

extern "C" int zscrc_zs_records(const void *image, uint64_t size, int kind, zscrc_zs_record *recs, size_t cap,
                                size_t *n_records)
{
    const uint8_t *img = static_cast<const uint8_t *>(image);
    if (!img || !n_records || (cap && !recs))
        return ZSCRC_EINVAL;
    size_t n = 0;
    int rc = ZSCRC_ZS_END;
    zscrc_zs_record r;
    uint64_t next;
    if (kind == ZSCRC_ZS_PACKED) {
        uint64_t so[2], sl[2];
        rc = zscrc_zs_packed_spans(image, size, so, sl);
        if (rc)
            return rc < 0 ? rc : (*n_records = 0, rc);
        /* pointer section: BE64 count, then BE64 record offsets */
        const uint64_t poff = so[1], plen = sl[1];
        const uint64_t count = plen >= 8 ? be64(img + poff) : 0;
        if (plen < 8 || count > (plen - 8) / 8) {
            *n_records = 0;
            return ZSCRC_ZS_TRUNCATED;
        }
        for (uint64_t i = 0; i < count; ++i) {
            if (!record_at(img, size, be64(img + poff + 8 + 8 * i), r, &next)) {
                rc = ZSCRC_ZS_TRUNCATED;
                break;
            }
            if (n < cap)
                recs[n] = r;
            ++n;
        }
        *n_records = n;
        return n > cap ? ZSCRC_ZS_OVERFLOW : rc;
    }
    if (size < HDR)
        return ZSCRC_EINVAL;
    uint64_t off = HDR;
    while (off < size) {
        if (size - off < 8) {
            rc = ZSCRC_ZS_TRUNCATED;
            break;
        }
        const unsigned t = img[off];
        if (t == T_COMMIT || t == (T_COMMIT | T_LONG)) {
            const uint64_t rl = t == T_COMMIT ? 8 : 24;
            if (size - off < rl) {
                rc = ZSCRC_ZS_TRUNCATED;
                break;
            }
            off += rl;
            continue;
        }
        if (t != T_KEY && t != (T_KEY | T_LONG) && t != T_DELETED && t != T_LONG) {
            rc = ZSCRC_ZS_STOPPED;
            break;
        }
        if (!record_at(img, size, off, r, &next)) {
            rc = ZSCRC_ZS_TRUNCATED;
            break;
        }
        if (n < cap)
            recs[n] = r;
        ++n;
        off = next;
    }
    *n_records = n;
    return n > cap ? ZSCRC_ZS_OVERFLOW : rc;
}

extern "C" int zscrc_zs_dotzsdb_build(uint64_t offset, const char *uuidstr, uint32_t curidx, uint8_t out[61])
{
    if (!uuidstr || !out)
        return ZSCRC_EINVAL;
    /* zs_dotzsdb_update_end (zeroskip-dotzsdb.c:491-529): native signature,
     * BE64 offset, 37-byte uuid string, BE32 index, BE32 CRC over the
     * host-order fields */
    const uint64_t sig = 0x5a45524f534b4950ull;
    char u[37];
    memset(u, 0, sizeof u);
    memcpy(u, uuidstr, strnlen(uuidstr, 36));
    uint8_t *p = out;
    memcpy(p, &sig, 8);
    const uint64_t o = __builtin_bswap64(offset);
    memcpy(p + 8, &o, 8);
    memcpy(p + 16, u, 37);
    const uint32_t ci = __builtin_bswap32(curidx);
    memcpy(p + 53, &ci, 4);
    uint32_t c = crc32c_hw(0, nullptr, 0);
    c = crc32c_hw(c, &sig, 8);
    c = crc32c_hw(c, &offset, 8);
    c = crc32c_hw(c, u, 37);
    c = crc32c_hw(c, &curidx, 4);
    const uint32_t cb = __builtin_bswap32(c);
    memcpy(p + 57, &cb, 4);
    return ZSCRC_OK;
}

extern "C" int zscrc_zs_repack(const char *dbdir, unsigned flags, int threads, zscrc_repack_report *rep)
{
    if (!dbdir || !rep)
        return ZSCRC_EINVAL;
    memset(rep, 0, sizeof *rep);
    const double t0 = now_s();
    if (threads <= 0) {
        const unsigned h = std::thread::hardware_concurrency();
        threads = h ? (int)std::min(h, 16u) : 4;
        if (const char *e = getenv("OMP_NUM_THREADS"))
            if (atoi(e) > 0)
                threads = std::min(threads, atoi(e));
    }
    const std::string dir(dbdir);
    const std::string lock_path = dir + "/.zsdb.lock", dot_path = dir + "/.zsdb";
    /* the update lock first (zs_dotzsdb_update_begin), held to the end */
    int lockfd = open(lock_path.c_str(), O_WRONLY | O_CREAT | O_EXCL, 0644);
    if (lockfd < 0)
        return errno == EEXIST ? ZSCRC_EBUSY : ZSCRC_EINVAL;
    auto unlock = [&](int code) {
        if (lockfd >= 0) {
            close(lockfd);
            unlink(lock_path.c_str());
            lockfd = -1;
        }
        return code;
    };
    /* .zsdb: zs_dotzsdb_update_begin reads and checks it (:400-446) */
    uint8_t dot[DOTZSDB_SIZE];
    {
        FILE *fp = fopen(dot_path.c_str(), "rb");
        if (!fp)
            return unlock(ZSCRC_EINVAL);
        const size_t got = fread(dot, 1, sizeof dot, fp);
        fclose(fp);
        uint32_t st = 0, cp = 0;
        if (got != sizeof dot || zscrc_zs_dotzsdb_crc(dot, sizeof dot, &st, &cp) != ZSCRC_OK || st != cp)
            return unlock(ZSCRC_EINVAL);
    }
    char uuidstr[37];
    memcpy(uuidstr, dot + 16, 36);
    uuidstr[36] = 0;
    uint8_t uuid[16];
    if (!parse_uuid(uuidstr, uuid))
        return unlock(ZSCRC_EINVAL);
    const uint64_t dot_off = be64(dot + 8);
    uint32_t curidx;
    memcpy(&curidx, dot + 53, 4);
    curidx = __builtin_bswap32(curidx);

    std::vector<DbFile> fin, pk;
    DIR *d = opendir(dbdir);
    if (!d)
        return unlock(ZSCRC_EINVAL);
    for (struct dirent *de; (de = readdir(d)) != nullptr;) {
        DbFile f;
        if (!parse_name(de->d_name, f) || strncmp(de->d_name + 9, uuidstr, UUID_CHARS) != 0)
            continue;
        if (f.kind == ZSCRC_ZS_FINALISED)
            fin.push_back(f);
        else if (f.kind == ZSCRC_ZS_PACKED)
            pk.push_back(f);
    }
    closedir(d);
    auto by_index = [](const DbFile &x, const DbFile &y) { return x.s != y.s ? x.s < y.s : x.e < y.e; };
    std::sort(fin.begin(), fin.end(), by_index);
    std::sort(pk.begin(), pk.end(), by_index);

    std::vector<DbFile> src;
    if (!fin.empty()) {
        rep->branch = 1;
        src = fin; /* oldest first: later records replace earlier ones */
    } else if (pk.size() > 1) {
        rep->branch = 2;
        /* pflist's first two: the two newest; the older one wins a key */
        src.assign(pk.end() - 2, pk.end());
    }
    int rc = ZSCRC_OK;
    for (auto &f : src) {
        const std::string path = dir + "/" + f.name;
        const int fd = open(path.c_str(), O_RDONLY);
        struct stat sb;
        if (fd < 0 || fstat(fd, &sb) != 0) {
            if (fd >= 0)
                close(fd);
            rc = ZSCRC_EINVAL;
            break;
        }
        f.size = (size_t)sb.st_size;
        void *m = f.size ? mmap(nullptr, f.size, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
        close(fd);
        if (m == MAP_FAILED) {
            rc = ZSCRC_EINVAL;
            break;
        }
        f.img = static_cast<const uint8_t *>(m);
        if (f.size)
            (void)madvise(m, f.size, MADV_WILLNEED);
    }
    const double t_open = now_s();

    /* list every source file's records (threads over files) */
    std::vector<std::vector<zscrc_zs_record>> lists(src.size());
    std::vector<int> lrc(src.size(), ZSCRC_OK);
    if (!rc && !src.empty()) {
        std::atomic<size_t> next{0};
        auto work = [&]() {
            for (size_t i; (i = next.fetch_add(1)) < src.size();) {
                const DbFile &f = src[i];
                size_t cap = f.size / 32 + 16, n = 0;
                for (;;) {
                    lists[i].resize(cap);
                    lrc[i] = f.size ? zscrc_zs_records(f.img, f.size, f.kind, lists[i].data(), cap, &n)
                                    : ZSCRC_EINVAL;
                    if (lrc[i] != ZSCRC_ZS_OVERFLOW)
                        break;
                    cap = n;
                }
                lists[i].resize(lrc[i] < 0 ? 0 : n);
            }
        };
        std::vector<std::thread> th;
        for (int i = 0; i < std::min<int>(threads, (int)src.size()); ++i)
            th.emplace_back(work);
        for (auto &t : th)
            t.join();
        for (size_t i = 0; i < src.size(); ++i)
            if (lrc[i] != ZSCRC_ZS_END && lrc[i] != ZSCRC_OK)
                rc = ZSCRC_EINVAL; /* a source that does not parse is not repacked */
    }
    const double t_list = now_s();

    /* merge: one sorted sequence, the winner of every key */
    std::vector<MRec> all;
    const bool compat = rep->branch == 2 && (flags & ZSCRC_REPACK_REFERENCE_COMPAT);
    if (!rc && compat) {
        size_t total = 0;
        for (auto &l : lists)
            total += l.size();
        rep->records_in = total;
        /* pflist order: the newest file first, priority 1; the older, 2 */
        std::vector<Cursor> cur(src.size());
        for (size_t i = 0; i < src.size(); ++i) {
            const size_t fi = src.size() - 1 - i;
            cur[i].img = src[fi].img;
            cur[i].recs = &lists[fi];
            cur[i].prio = (int)i + 1;
        }
        compat_merge(cur, all);
        std::vector<std::vector<zscrc_zs_record>>().swap(lists);
    } else if (!rc) {
        size_t total = 0;
        for (auto &l : lists)
            total += l.size();
        rep->records_in = total;
        all.reserve(total);
        uint64_t seq = 0;
        for (size_t i = 0; i < src.size(); ++i) {
            /* branch 2: the older file (src[0]) wins, so it loads last */
            const size_t fi = rep->branch == 2 ? src.size() - 1 - i : i;
            for (const auto &r : lists[fi])
                all.push_back({src[fi].img + r.key_off,
                               r.val_off == ZSCRC_ZS_DELETED ? nullptr : src[fi].img + r.val_off, r.key_len,
                               r.val_len, seq++});
        }
        std::vector<std::vector<zscrc_zs_record>>().swap(lists);
        parallel_sort(all, threads);
        size_t w = 0;
        for (size_t i = 0; i < all.size(); ++i) {
            const bool last = i + 1 == all.size() ||
                              memcmp_raw(all[i].k, all[i].kl, all[i + 1].k, all[i + 1].kl) != 0;
            if (!last)
                continue; /* a later record of the key replaces it */
            if (rep->branch == 2 && !all[i].v)
                continue; /* a winning delete drops the key */
            all[w++] = all[i];
        }
        all.resize(w);
    }
    const double t_merge = now_s();

    std::string tmp_out;
    if (!rc && rep->branch) {
        uint32_t s = (uint32_t)src[0].s, e = (uint32_t)src[0].e;
        for (const auto &f : src) {
            s = std::min<uint32_t>(s, (uint32_t)f.s);
            e = std::max<uint32_t>(e, (uint32_t)f.e);
        }
        rep->startidx = s;
        rep->endidx = e;
        rep->files_merged = src.size();
        snprintf(rep->path, sizeof rep->path, "%s/zeroskip-%s-%u-%u", dbdir, uuidstr, s, e);
        tmp_out = std::string(rep->path) + ".tmp";
        zscrc_packer *w = nullptr;
        rc = zscrc_pack_open(&w, tmp_out.c_str(), uuid, s, e, 0, flags);
        for (size_t i = 0; !rc && i < all.size(); ++i)
            rc = zscrc_pack_add(w, all[i].k, all[i].kl, all[i].v, all[i].vl);
        if (w) {
            if (rc)
                zscrc_pack_abort(w);
            else
                rc = zscrc_pack_close(w, &rep->pack);
        }
        rep->records_out = rc ? 0 : rep->pack.records;
    }
    const double t_write = now_s();
    for (auto &f : src)
        if (f.img)
            munmap(const_cast<uint8_t *>(f.img), f.size);
    /* the output into place (replacing a source of the same name), then
     * the merged sources go (src/zeroskip.c:1489-1497, :1555-1562) -- never
     * the output itself */
    if (!rc && rep->branch && rename(tmp_out.c_str(), rep->path) != 0)
        rc = ZSCRC_EINVAL;
    if (rc && !tmp_out.empty())
        unlink(tmp_out.c_str());
    if (!rc)
        for (auto &f : src) {
            const std::string path = dir + "/" + f.name;
            if (path != rep->path)
                unlink(path.c_str());
        }
    /* zs_dotzsdb_update_end: .zsdb rewritten into the held lock file, CRC
     * recomputed, renamed over .zsdb (file_lock_rename) */
    if (!rc) {
        uint8_t out[DOTZSDB_SIZE];
        zscrc_zs_dotzsdb_build(dot_off, uuidstr, curidx, out);
        bool ok = write(lockfd, out, sizeof out) == (ssize_t)sizeof out;
        if (flags & ZSCRC_PACK_FSYNC)
            ok = ok && fsync(lockfd) == 0;
        /* ZSCRC_FAULT=dotzsdb_rename: the rename fails (fault injection for
         * tests/test_gpu_repack.py; nothing else reads it) */
        const char *fault = getenv("ZSCRC_FAULT");
        const bool renamed = ok && !(fault && !strcmp(fault, "dotzsdb_rename")) &&
                             rename(lock_path.c_str(), dot_path.c_str()) == 0;
        close(lockfd);
        lockfd = -1;
        if (!renamed) {
            /* the lock file was not renamed into place: it must not outlive
             * the call (a stale .zsdb.lock refuses every later update) */
            unlink(lock_path.c_str());
            rc = ZSCRC_EINVAL;
        }
        rep->dotzsdb_crc = be64(out + 53) & 0xFFFFFFFFull;
    }
    unlock(rc);
    rep->list_s = t_list - t_open;
    rep->merge_s = t_merge - t_list;
    rep->write_s = t_write - t_merge;
    rep->total_s = now_s() - t0;
    return rc;
}
