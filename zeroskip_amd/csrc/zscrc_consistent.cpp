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
 * Files are memory-mapped and handed to zscrc_zs_verify_files
 * (zscrc_files.cpp): threaded host walks, pinned staging and H2D copies
 * overlapped with per-group device verification.  Zero-length commits that hash the
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
    /* headers, walks and every commit: the end-to-end pipeline */
    if (!rc && !files.empty()) {
        std::vector<const void *> imgs(files.size());
        std::vector<uint64_t> sizes(files.size());
        std::vector<int> kinds(files.size());
        for (size_t i = 0; i < files.size(); ++i) {
            imgs[i] = files[i].img;
            sizes[i] = files[i].size;
            kinds[i] = files[i].kind;
        }
        zscrc_files_report fr;
        rc = zscrc_zs_verify_files(imgs.data(), sizes.data(), kinds.data(), files.size(), 0, &fr);
        if (!rc) {
            rep->files = fr.files;
            rep->commits = fr.commits;
            rep->bytes = fr.bytes;
            rep->bad_commits = fr.bad_commits;
            rep->stale_empty_commits = fr.stale_empty_commits;
            rep->header_errors = fr.header_errors;
            rep->walk_errors = fr.walk_errors;
            if (fr.first_bad_what) {
                static const char *what[] = {"", "header", "record walk stopped", "commit CRC mismatch"};
                const DbFile &f = files[fr.first_bad_file];
                note(rep, f.name, fr.first_bad_off,
                     f.kind == ZSCRC_ZS_PACKED && fr.first_bad_what == ZSCRC_FILES_BAD_WALK
                         ? "packed layout" : what[fr.first_bad_what]);
            }
        }
    }
    for (auto &f : files)
        if (f.img)
            munmap(const_cast<uint8_t *>(f.img), f.size);
    rep->consistent = !rc && rep->dotzsdb == 1 && !rep->bad_commits && !rep->header_errors &&
                      !rep->walk_errors;
    return rc;
}
