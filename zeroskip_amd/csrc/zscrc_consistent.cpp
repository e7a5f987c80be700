/*
 * zscrc_consistent.cpp -- `consistent` for one process / one GPU, in C, for
 * the reference's own entry points: zsdb_consistent (src/zeroskip.c:1399-1407,
 * ZS_NOTIMPLEMENTED there) and `zeroskip consistent` (tool/cmd-consistent.c:
 * 23-49, which only parses options).  Same checks as the multi-GPU driver
 * zeroskip_amd/consistent.py:
 *   .zsdb          signature + CRC (src/zeroskip-dotzsdb.c:105-119)
 *   every file     header signature + CRC (src/zeroskip-header.c:105-170)
 *                  named like interpret_db_filename (src/zeroskip.c:200-235)
 *   active /       the record walk (src/zeroskip-record.c:283-331) and every
 *   finalised      commit CRC, writer semantics (src/zeroskip-file.c:253-350)
 *   packed         records-region commit + pointer-section commit
 *                  (src/zeroskip-packed.c:70-131, :278-339, :442)
 * Files are memory-mapped, walked on the host, staged to the GPU in groups of
 * up to ZSCRC_CONSISTENT_GROUP bytes (default 8 GiB) and every commit of a
 * group is verified in one device pass.  Zero-length commits that hash the
 * previous span's register (zs_active_file_finalise after a committed
 * transaction, src/zeroskip-active.c:122 + src/mfile.c:534-546) are counted
 * apart as stale_empty_commits.
 */
#include <hip/hip_runtime.h>

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/zscrc.h"


namespace {

constexpr size_t UUID_CHARS = 36; /* UUID_STRLEN - 1, zeroskip-priv.h:53 */

struct DbFile {
    std::string name;
    int kind = 0;
    unsigned long s = 0, e = 0;
    const uint8_t *img = nullptr;
    size_t size = 0;
    std::vector<uint64_t> off, len; /* commit spans */
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

void note(zscrc_consistent_report *rep, const std::string &file, uint64_t off, const char *what)
{
    if (!rep->first_bad[0])
        snprintf(rep->first_bad, sizeof rep->first_bad, "%s:%llu: %s", file.c_str(),
                 (unsigned long long)off, what);
}

/* Verify the commits of files[a, b) in one device pass. */
int verify_group(std::vector<DbFile> &files, size_t a, size_t b, zscrc_consistent_report *rep)
{
    std::vector<size_t> base(b - a);
    size_t total = 0, ncommit = 0;
    for (size_t i = a; i < b; ++i) {
        base[i - a] = total;
        total += (files[i].size + 255) & ~size_t(255);
        ncommit += files[i].off.size();
    }
    if (!ncommit)
        return ZSCRC_OK;
    uint8_t *dimg = nullptr;
    uint64_t *dmeta = nullptr;
    hipError_t e = hipMalloc(&dimg, total);
    if (e == hipSuccess)
        e = hipMalloc(&dmeta, ncommit * 24);
    std::vector<uint64_t> hoff(ncommit), hlen(ncommit);
    std::vector<uint32_t> hfile(ncommit);
    size_t k = 0;
    for (size_t i = a; i < b && e == hipSuccess; ++i) {
        e = hipMemcpy(dimg + base[i - a], files[i].img, files[i].size, hipMemcpyHostToDevice);
        for (size_t c = 0; c < files[i].off.size(); ++c, ++k) {
            hoff[k] = files[i].off[c] + base[i - a];
            hlen[k] = files[i].len[c];
            hfile[k] = (uint32_t)i;
        }
    }
    uint64_t *doff = dmeta, *dlen = dmeta + ncommit;
    uint32_t *dcrc = reinterpret_cast<uint32_t *>(dlen + ncommit), *dst = dcrc + ncommit;
    if (e == hipSuccess)
        e = hipMemcpy(doff, hoff.data(), ncommit * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(dlen, hlen.data(), ncommit * 8, hipMemcpyHostToDevice);
    int rc = e == hipSuccess ? ZSCRC_OK : ZSCRC_EHIP;
    std::vector<uint32_t> st(ncommit);
    uint64_t max_len = 0;
    for (uint64_t l : hlen)
        max_len = l > max_len ? l : max_len;
    if (!rc)
        rc = zscrc_device_verify_commits_bounded(dimg, total, doff, dlen, nullptr, ncommit, max_len, dcrc, dst,
                                                 nullptr);
    if (!rc && hipMemcpy(st.data(), dst, ncommit * 4, hipMemcpyDeviceToHost) != hipSuccess)
        rc = ZSCRC_EHIP;
    /* zero-length mismatches right after a commit of the same file: the
     * finalise quirk if the stored CRC continues from the previous span's CRC
     * (stored = crc32c(crc32c(0, previous span), trailer)).  Re-verified on the
     * device: CRC the previous spans, then verify seeded with them. */
    std::vector<size_t> cand;
    for (size_t i = 1; !rc && i < ncommit; ++i)
        if (st[i] != 1 && hlen[i] == 0 && hfile[i - 1] == hfile[i])
            cand.push_back(i);
    std::vector<uint32_t> st2(cand.size());
    if (!rc && !cand.empty()) {
        const size_t m = cand.size();
        std::vector<uint64_t> q(4 * m);
        uint64_t prev_max = 0;
        for (size_t c = 0; c < m; ++c) {
            prev_max = hlen[cand[c] - 1] > prev_max ? hlen[cand[c] - 1] : prev_max;
            q[c] = hoff[cand[c] - 1];
            q[m + c] = hlen[cand[c] - 1];
            q[2 * m + c] = hoff[cand[c]];
            q[3 * m + c] = hlen[cand[c]];
        }
        uint64_t *dq = nullptr;
        uint32_t *dprev = nullptr;
        e = hipMalloc(&dq, 4 * m * 8 + 3 * m * 4);
        if (e == hipSuccess) {
            dprev = reinterpret_cast<uint32_t *>(dq + 4 * m);
            e = hipMemcpy(dq, q.data(), 4 * m * 8, hipMemcpyHostToDevice);
        }
        rc = e == hipSuccess ? ZSCRC_OK : ZSCRC_EHIP;
        if (!rc)
            rc = zscrc_device_batch_bounded(dimg, dq, dq + m, nullptr, dprev, m, 0, prev_max, nullptr);
        if (!rc) /* the candidates are zero-length spans */
            rc = zscrc_device_verify_commits_bounded(dimg, total, dq + 2 * m, dq + 3 * m, dprev, m, 0, dprev + m,
                                                     dprev + 2 * m, nullptr);
        if (!rc && hipMemcpy(st2.data(), dprev + 2 * m, m * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = ZSCRC_EHIP;
        if (dq)
            (void)hipFree(dq);
    }
    if (dimg)
        (void)hipFree(dimg);
    if (dmeta)
        (void)hipFree(dmeta);
    if (rc)
        return rc;
    rep->commits += ncommit;
    rep->bytes += total;
    size_t c = 0;
    for (size_t i = 0; i < ncommit; ++i) {
        if (st[i] == 1)
            continue;
        if (c < cand.size() && cand[c] == i && st2[c++] == 1) {
            rep->stale_empty_commits++;
            continue;
        }
        const DbFile &f = files[hfile[i]];
        rep->bad_commits++;
        note(rep, f.name, hoff[i] - base[hfile[i] - a] + hlen[i], "commit CRC mismatch");
    }
    return ZSCRC_OK;
}

} /* namespace */

extern "C" int zscrc_zs_consistent(const char *dbdir, zscrc_consistent_report *rep)
{
    if (!dbdir || !rep)
        return ZSCRC_EINVAL;
    memset(rep, 0, sizeof *rep);
    rep->dotzsdb = -1;
    DIR *d = opendir(dbdir);
    if (!d)
        return ZSCRC_EINVAL;
    std::vector<DbFile> files;
    std::vector<uint8_t> dot;
    const std::string dir(dbdir);
    int rc = ZSCRC_OK;
    for (struct dirent *de; (de = readdir(d)) != nullptr;) {
        const std::string path = dir + "/" + de->d_name;
        struct stat sb;
        if (stat(path.c_str(), &sb) != 0 || !S_ISREG(sb.st_mode))
            continue;
        if (strcmp(de->d_name, ".zsdb") == 0) {
            FILE *fp = fopen(path.c_str(), "rb");
            if (fp) {
                dot.resize((size_t)sb.st_size);
                if (fread(dot.data(), 1, dot.size(), fp) != dot.size())
                    dot.clear();
                fclose(fp);
            }
            continue;
        }
        DbFile f;
        if (!parse_name(de->d_name, f))
            continue;
        f.size = (size_t)sb.st_size;
        if (f.size) {
            const int fd = open(path.c_str(), O_RDONLY);
            void *m = fd >= 0 ? mmap(nullptr, f.size, PROT_READ, MAP_PRIVATE, fd, 0) : MAP_FAILED;
            if (fd >= 0)
                close(fd);
            if (m == MAP_FAILED) {
                rc = ZSCRC_EINVAL;
                break;
            }
            f.img = static_cast<const uint8_t *>(m);
        }
        files.push_back(std::move(f));
    }
    closedir(d);
    std::sort(files.begin(), files.end(), [](const DbFile &x, const DbFile &y) {
        return x.s != y.s ? x.s < y.s : x.e != y.e ? x.e < y.e : x.name < y.name;
    });

    if (!dot.empty()) {
        uint32_t st = 0, cp = 0;
        rep->dotzsdb = zscrc_zs_dotzsdb_crc(dot.data(), dot.size(), &st, &cp) == ZSCRC_OK && st == cp;
    }
    /* host: headers, walks, packed layouts */
    for (auto &f : files) {
        if (rc)
            break;
        rep->files++;
        uint32_t st = 0, cp = 0;
        if (zscrc_zs_header_crc(f.img, f.size, &st, &cp) != ZSCRC_OK || st != cp) {
            rep->header_errors++;
            note(rep, f.name, 0, "header");
        }
        if (f.kind == ZSCRC_ZS_PACKED) {
            uint64_t o[2], l[2];
            if (f.size >= 56 && zscrc_zs_packed_spans(f.img, f.size, o, l) == ZSCRC_OK) {
                f.off.assign(o, o + 2);
                f.len.assign(l, l + 2);
            } else {
                rep->walk_errors++;
                note(rep, f.name, 0, "packed layout");
            }
            continue;
        }
        const size_t cap = f.size / 8 + 1;
        f.off.resize(cap);
        f.len.resize(cap);
        size_t n = 0;
        uint64_t end = 0;
        const int w = f.size ? zscrc_zs_walk(f.img, f.size, f.off.data(), f.len.data(), cap, &n, &end)
                             : ZSCRC_ZS_TRUNCATED;
        f.off.resize(w >= 0 ? n : 0);
        f.len.resize(w >= 0 ? n : 0);
        if (w != ZSCRC_ZS_END) {
            rep->walk_errors++;
            note(rep, f.name, end, "record walk stopped");
        }
    }
    /* device: commits, in groups */
    uint64_t group = 8ull << 30;
    if (const char *g = getenv("ZSCRC_CONSISTENT_GROUP"))
        group = strtoull(g, nullptr, 0);
    for (size_t a = 0; a < files.size() && !rc;) {
        size_t b = a, bytes = 0;
        while (b < files.size() && (b == a || bytes + files[b].size <= group))
            bytes += files[b++].size;
        rc = verify_group(files, a, b, rep);
        a = b;
    }
    for (auto &f : files)
        if (f.img)
            munmap(const_cast<uint8_t *>(f.img), f.size);
    rep->consistent = !rc && rep->dotzsdb == 1 && !rep->bad_commits && !rep->header_errors &&
                      !rep->walk_errors;
    return rc;
}
