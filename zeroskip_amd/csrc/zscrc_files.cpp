/*
 * zscrc_files.cpp -- verify every CRC of a set of host-resident zeroskip file
 * images (mmap'd files: verify-on-open of a whole DB, `consistent`), end to
 * end: host memory -> GPUs -> verdict.  Declared in include/zscrc.h
 * (zscrc_zs_verify_files); zscrc_zs_consistent runs on it.
 *
 * What is checked is the reference's: the header CRC (src/zeroskip-header.c:
 * 105-170), the record walk (src/zeroskip-record.c:283-331) and every commit
 * CRC with the writer's trailer semantics (src/zeroskip-file.c:253-350) for
 * active / finalised files, and the records-region + pointer-section commits
 * of packed files (src/zeroskip-packed.c:70-131, :278-339, :442).
 *
 * Devices: every entry of the device list (zscrc_set_devices, env
 * ZSCRC_DEVICES="0,1,..."; default every visible gfx950 device) is a "slot"
 * with its own host thread, staging slots, streams and device buffer.  An
 * entry may repeat (ZSCRC_DEVICES=0,0 rehearses two slots on one GPU).
 *
 * Plan (the byte-weight cut of zeroskip_amd/consistent.py:168-213, in C):
 *   * the DB is a sequence of units: a whole active / finalised file (or a
 *     packed file whose layout does not parse), or, for a packed file, its
 *     records region and its tail (region commit + pointer section + final
 *     commit);
 *   * the W bytes are cut into one range of W / S bytes per slot; a unit
 *     goes to the slot holding its middle, except records regions, which are
 *     cut at the slot bounds (4 KiB aligned) into pieces;
 *   * each slot's units run in groups of at most `group` bytes (env
 *     ZSCRC_FILES_GROUP, default 8 GiB, at most half the device's free memory
 *     at the call; records-region pieces are cut to fit): the device buffer is
 *     reused from group to group, so a DB larger than HBM is checked in
 *     bounded memory;
 *   * a records-region piece is checksummed as a raw span on its slot's GPU
 *     (zscrc_device_span: every CU, no per-record work); after every slot has
 *     finished, the host folds each region's piece registers in order,
 *     reg = shift(reg, |piece|) ^ raw (zscrc_shift, GF(2)), and checks the
 *     region's commit trailer -- 8 or 24 bytes -- with crc32c_hw.
 *
 * Pipeline of one group on one slot:
 *   * the group's byte ranges are laid out back to back (256-byte aligned) in
 *     the slot's device buffer, cut into pieces of `slot` bytes;
 *   * a pool of host threads takes tasks in order -- the copy of 4 MiB
 *     sub-ranges of piece p into pinned staging slot p % NSLOT (once the
 *     slot's previous H2D copy has left), then the walks of the files ending
 *     in piece p (header CRC, commit spans);
 *   * the slot's thread issues piece p's H2D copy on a copy stream as soon as
 *     its sub-ranges are staged; when the last byte is on the device, the
 *     group's commits are verified in one bounded launch and its region
 *     pieces checksummed on a compute stream;
 *   * zero-length commits that chain from the previous span's CRC (the
 *     finalise quirk, src/zeroskip-active.c:122 + src/mfile.c:534-546) are
 *     re-verified with that CRC as the seed and counted apart.
 * Pinned slots, pinned descriptor blocks and the device buffer are cached per
 * slot between calls (the buffer is at most one group; zscrc_release_cache()
 * frees everything).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zscrc.h"

namespace {

constexpr int NSLOT = 4;
constexpr uint64_t ALIGN = 256;
constexpr uint64_t SUB = 4ull << 20;      /* bytes per copy task */
constexpr int MAX_SLOTS = 64;             /* entries of the device list */
constexpr uint64_t SPLIT_ALIGN = 4096;    /* records-region cuts */
constexpr uint64_t GROUP_DEFAULT = 8ull << 30;

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

/* ------------------------------------------------------------ device list */
std::mutex g_dev_mu;
std::vector<int> g_devices; /* empty = default */
bool g_devices_set = false;

bool gfx950(int dev)
{
    hipDeviceProp_t p;
    return hipGetDeviceProperties(&p, dev) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

/* The slots of this call: the caller's list, else ZSCRC_DEVICES, else every
 * visible gfx950 device. */
int device_list(std::vector<int> &out)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return ZSCRC_ENODEV;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    out.clear();
    if (g_devices_set) {
        out = g_devices;
    } else if (const char *e = getenv("ZSCRC_DEVICES")) {
        for (const char *p = e; *p;) {
            char *q;
            const long v = strtol(p, &q, 10);
            if (q == p)
                return ZSCRC_EINVAL;
            out.push_back((int)v);
            p = *q == ',' ? q + 1 : q;
            if (*q && *q != ',')
                return ZSCRC_EINVAL;
        }
    } else {
        for (int d = 0; d < count && (int)out.size() < MAX_SLOTS; ++d)
            if (gfx950(d))
                out.push_back(d);
    }
    if (out.empty() || out.size() > (size_t)MAX_SLOTS)
        return ZSCRC_ENODEV;
    for (int d : out)
        if (d < 0 || d >= count || !gfx950(d))
            return ZSCRC_ENODEV;
    return ZSCRC_OK;
}

/* ------------------------------------------------------------ per-slot cache */
struct Cache {
    std::mutex mu;
    int dev = -1;
    uint64_t slot_bytes = 0;
    uint8_t *slot[NSLOT] = {};
    uint8_t *dimg = nullptr;
    uint64_t dimg_bytes = 0;
    /* commit descriptors: pinned SoA arrays (written by the walkers), their
     * device copy and the device results */
    uint64_t dcap = 0;
    uint64_t *h_off = nullptr, *h_len = nullptr;
    uint32_t *h_st = nullptr;
    uint8_t *ddesc = nullptr;
    uint64_t ddesc_bytes = 0;
    uint64_t *h_bad = nullptr; /* pinned: the verdict's count + listed indices */
    uint8_t *dq = nullptr;     /* device: the stale-commit re-verification batch */
    uint64_t dq_bytes = 0;
    /* copy and compute streams and their events, kept across calls (creating
     * and destroying them per group cost milliseconds per call) */
    hipStream_t cs = nullptr, ks = nullptr;
    hipEvent_t slot_ev[NSLOT] = {};
    hipEvent_t done_ev = nullptr;
};
Cache g_cache[MAX_SLOTS];

void sync_free(Cache &c)
{
    for (hipStream_t s : {c.cs, c.ks})
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    for (auto &e : c.slot_ev)
        if (e)
            (void)hipEventDestroy(e);
    if (c.done_ev)
        (void)hipEventDestroy(c.done_ev);
    c.cs = c.ks = nullptr;
    for (auto &e : c.slot_ev)
        e = nullptr;
    c.done_ev = nullptr;
}

int ensure_sync(Cache &c)
{
    if (c.cs && c.ks && c.done_ev)
        return ZSCRC_OK;
    sync_free(c);
    hipError_t e = hipStreamCreateWithFlags(&c.cs, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&c.ks, hipStreamNonBlocking);
    for (int k = 0; e == hipSuccess && k < NSLOT; ++k)
        e = hipEventCreateWithFlags(&c.slot_ev[k], hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&c.done_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        sync_free(c);
        return ZSCRC_EHIP;
    }
    return ZSCRC_OK;
}

/* commits a group's verdict lists (more mismatches: the per-commit status
 * arrays instead) */
constexpr uint64_t VCAP = 65536;

void cache_free(Cache &c)
{
    if (c.dev >= 0)
        (void)hipSetDevice(c.dev);
    for (int k = 0; k < NSLOT; ++k)
        if (c.slot[k])
            (void)hipHostFree(c.slot[k]);
    if (c.h_off)
        (void)hipHostFree(c.h_off);
    if (c.h_len)
        (void)hipHostFree(c.h_len);
    if (c.h_st)
        (void)hipHostFree(c.h_st);
    if (c.dimg)
        (void)hipFree(c.dimg);
    if (c.ddesc)
        (void)hipFree(c.ddesc);
    if (c.h_bad)
        (void)hipHostFree(c.h_bad);
    if (c.dq)
        (void)hipFree(c.dq);
    sync_free(c);
    const int dev = c.dev;
    c.dev = dev; /* keep the binding; everything else reset */
    c.slot_bytes = 0;
    for (auto &s : c.slot)
        s = nullptr;
    c.dimg = nullptr;
    c.dimg_bytes = 0;
    c.dcap = 0;
    c.h_off = c.h_len = nullptr;
    c.h_st = nullptr;
    c.ddesc = nullptr;
    c.ddesc_bytes = 0;
    c.h_bad = nullptr;
    c.dq = nullptr;
    c.dq_bytes = 0;
}

int grow_dev(uint8_t **p, uint64_t *have, uint64_t need)
{
    if (*have >= need)
        return ZSCRC_OK;
    if (*p)
        (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    need += need / 8;
    if (hipMalloc(reinterpret_cast<void **>(p), need) != hipSuccess)
        return ZSCRC_ENOMEM;
    *have = need;
    return ZSCRC_OK;
}

int ensure_slots(Cache &c, uint64_t slot_bytes)
{
    if (c.slot_bytes >= slot_bytes)
        return ZSCRC_OK;
    for (int k = 0; k < NSLOT; ++k) {
        if (c.slot[k])
            (void)hipHostFree(c.slot[k]);
        c.slot[k] = nullptr;
    }
    c.slot_bytes = 0;
    for (int k = 0; k < NSLOT; ++k)
        if (hipHostMalloc(reinterpret_cast<void **>(&c.slot[k]), slot_bytes, hipHostMallocDefault) != hipSuccess)
            return ZSCRC_ENOMEM;
    c.slot_bytes = slot_bytes;
    return ZSCRC_OK;
}

/* Pinned descriptor arrays for at least `count` commits (contents dropped). */
int ensure_desc(Cache &c, uint64_t count)
{
    if (c.dcap >= count)
        return ZSCRC_OK;
    if (c.h_off)
        (void)hipHostFree(c.h_off);
    if (c.h_len)
        (void)hipHostFree(c.h_len);
    if (c.h_st)
        (void)hipHostFree(c.h_st);
    c.h_off = c.h_len = nullptr;
    c.h_st = nullptr;
    c.dcap = 0;
    count += count / 4 + 1024;
    if (hipHostMalloc(reinterpret_cast<void **>(&c.h_off), 8 * count, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&c.h_len), 8 * count, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&c.h_st), 4 * count, hipHostMallocDefault) != hipSuccess)
        return ZSCRC_ENOMEM;
    c.dcap = count;
    if (!c.h_bad &&
        hipHostMalloc(reinterpret_cast<void **>(&c.h_bad), 8 * (VCAP + 1), hipHostMallocDefault) != hipSuccess)
        return ZSCRC_ENOMEM;
    return ZSCRC_OK;
}

/* ------------------------------------------------------------ the plan */
enum { EXT_FILE = 0, EXT_PIECE = 1, EXT_TAIL = 2 };

/* One contiguous byte range [lo, hi) of one file, checked on one slot. */
struct Ext {
    size_t file = 0;
    int what = EXT_FILE;
    uint64_t lo = 0, hi = 0;
    int slot = 0;
    uint32_t piece = 0;             /* EXT_PIECE: index within its region */
    /* per call, within its group */
    uint64_t dev_off = 0;           /* where its bytes go in the device buffer */
    std::vector<uint64_t> off, len; /* commit spans while walking (file offsets) */
    uint64_t ncommit = 0;
    uint64_t pos = 0;               /* its commits: [pos, pos + ncommit) of the descriptor arrays */
    bool placed = false;            /* written to the pinned arrays by its walker */
    uint64_t max_len = 0, min_len = ~0ull;
    uint32_t raw = 0;               /* EXT_PIECE: raw register of its bytes */
};

struct FileInfo {
    bool split = false;             /* packed file checked as region pieces + tail */
    uint64_t roff = 0, rlen = 0, poff = 0, plen = 0;
    int header_bad = 0;
    int walk_rc = 0;                /* ZSCRC_ZS_END, or ZSCRC_OK for a packed file's layout */
    uint64_t walk_end = 0;
};

/* Shared verdict accumulator (slot threads). */
struct Acc {
    std::mutex mu;
    uint64_t commits = 0, bad = 0, stale = 0;
    uint64_t first_file = ~0ull, first_off = 0;
    int first_what = 0;
    void first(uint64_t f, uint64_t off, int what)
    {
        if (f < first_file || (f == first_file && off < first_off)) {
            first_file = f;
            first_off = off;
            first_what = what;
        }
    }
};

void walk_ext(const uint8_t *img, uint64_t size, int kind, FileInfo &fi, Ext &x)
{
    size_t n = 0;
    if (x.what == EXT_PIECE)
        return;
    uint32_t st = 0, cp = 0;
    fi.header_bad = size < 40 || zscrc_zs_header_crc(img, size, &st, &cp) != ZSCRC_OK || st != cp;
    if (x.what == EXT_TAIL) {
        /* the pointer section's commit; the region's is folded on the host */
        fi.walk_rc = ZSCRC_OK;
        fi.walk_end = size;
        x.off.assign(1, fi.poff);
        x.len.assign(1, fi.plen);
        n = 1;
    } else if (kind == ZSCRC_ZS_PACKED) {
        /* a packed file whose layout does not parse: reported, nothing hashed */
        uint64_t o[2], l[2];
        fi.walk_rc = size >= 56 ? zscrc_zs_packed_spans(img, size, o, l) : ZSCRC_ZS_TRUNCATED;
        if (fi.walk_rc == ZSCRC_OK)
            fi.walk_rc = ZSCRC_ZS_TRUNCATED; /* not reached: parsed layouts are split */
        fi.walk_end = size;
    } else if (size < 40) {
        fi.walk_rc = ZSCRC_ZS_TRUNCATED;
    } else {
        size_t cap = (size_t)(size / 256) + 64; /* grown on overflow */
        for (;;) {
            x.off.resize(cap);
            x.len.resize(cap);
            fi.walk_rc = zscrc_zs_walk(img, size, x.off.data(), x.len.data(), cap, &n, &fi.walk_end);
            if (fi.walk_rc != ZSCRC_ZS_OVERFLOW)
                break;
            cap = n + 64;
        }
        if (fi.walk_rc < 0)
            n = 0;
    }
    x.off.resize(n);
    x.len.resize(n);
    x.ncommit = n;
    for (size_t i = 0; i < n; ++i) {
        x.max_len = std::max(x.max_len, x.len[i]);
        x.min_len = std::min(x.min_len, x.len[i]);
    }
}

/* The walker's spans -> descriptor arrays at pos (device offsets). */
void place(Ext &x, uint64_t *h_off, uint64_t *h_len)
{
    for (uint64_t i = 0; i < x.ncommit; ++i) {
        h_off[x.pos + i] = x.dev_off + (x.off[i] - x.lo);
        h_len[x.pos + i] = x.len[i];
    }
    x.placed = true;
    std::vector<uint64_t>().swap(x.off);
    std::vector<uint64_t>().swap(x.len);
}

/* Commit record at file offset `off` after a span whose crc32c(0, span) is
 * span_crc, checked with the writer's trailer words (zeroskip-file.c:266-302,
 * host-order words as hashed there): 1 match, 0 mismatch, 2 no commit record. */
int host_commit_check(const uint8_t *img, uint64_t size, uint64_t off, uint32_t span_crc)
{
    if (off > size || size - off < 8)
        return 2;
    const uint64_t w0 = be64(img + off);
    const unsigned t = (unsigned)(w0 >> 56);
    if (t == 4 || t == 16) { /* COMMIT / FINAL */
        const uint64_t w = w0 & 0xFFFFFFFF00000000ull;
        return crc32c_hw(span_crc, &w, 8) == (uint32_t)w0;
    }
    if ((t == 36 || t == 48) && size - off >= 24) { /* LONG_COMMIT / LONG_FINAL */
        const uint64_t w2 = be64(img + off + 16);
        const uint64_t w[3] = {w0, be64(img + off + 8), w2 & 0xFF00000000000000ull};
        return crc32c_hw(span_crc, w, 24) == (uint32_t)w2;
    }
    return 2;
}

struct Call {
    const void *const *images;
    const uint64_t *sizes;
    const int *kinds;
    size_t n;
    std::vector<FileInfo> fi;
    std::vector<Ext> ext;
    Acc acc;
    uint64_t slot_bytes = 64ull << 20;
    bool direct = false;
    double copy_s = 0, tail_s = 0;
    std::mutex tmu;
};

/* One group of one slot: stage, copy, walk, verify, report.  Runs on the
 * slot's thread with its device current and its cache locked. */
int run_group(Call &C, Cache &cache, std::vector<Ext *> &G, int threads)
{
    const size_t ng = G.size();
    uint64_t total = 0, est = 1024;
    for (Ext *x : G) {
        x->dev_off = total;
        total += (x->hi - x->lo + ALIGN - 1) & ~(ALIGN - 1);
        est += (x->what == EXT_FILE ? (x->hi - x->lo) / 256 : 0) + 4;
    }
    const uint64_t slot = C.slot_bytes;
    int rc = C.direct ? ZSCRC_OK : ensure_slots(cache, slot);
    if (!rc)
        rc = grow_dev(&cache.dimg, &cache.dimg_bytes, std::max<uint64_t>(total, ALIGN));
    if (!rc && cache.dcap == 0)
        rc = ensure_desc(cache, est); /* later calls keep what the largest needed */
    if (rc)
        return rc;
    const uint64_t npiece = (total + slot - 1) / slot;

    struct Task {
        int walk;    /* 1 walk, 0 copy */
        uint64_t a;  /* extent (in G), or piece */
        uint64_t b;  /* sub-range of the piece */
    };
    std::vector<Task> tasks;
    tasks.reserve(ng + npiece * (slot / SUB) + 1);
    std::vector<std::atomic<int>> left(npiece);
    size_t qf = 0; /* extents whose walks are queued */
    if (!C.direct) {
        /* each piece's copy tasks, then the walks of the extents that end in
         * it -- the PCIe stream starts at once and the walks overlap it (all
         * walks first held every copy back ~25 ms on 10 M commits) */
        for (uint64_t p = 0; p < npiece; ++p) {
            const uint64_t len = std::min(total, (p + 1) * slot) - p * slot;
            left[p] = (int)((len + SUB - 1) / SUB);
            for (uint64_t s = 0; s < (uint64_t)left[p]; ++s)
                tasks.push_back({0, p, s});
            for (; qf < ng && G[qf]->dev_off + (G[qf]->hi - G[qf]->lo) <= (p + 1) * slot; ++qf)
                tasks.push_back({1, qf, 0});
        }
    }
    /* every extent is walked, also when nothing is copied (empty files) */
    for (; qf < ng; ++qf)
        tasks.push_back({1, qf, 0});

    if (!rc)
        rc = ensure_sync(cache);
    hipStream_t cs = cache.cs, ks = cache.ks;
    hipEvent_t *slot_ev = cache.slot_ev, done_ev = cache.done_ev;

    std::atomic<uint64_t> next{0};
    std::atomic<int> stop{0};
    /* slot of piece p is free for its copy tasks once piece p - NSLOT's H2D
     * copy has completed: free_upto = (last such piece) + 1 */
    std::atomic<int64_t> free_upto{NSLOT};
    std::atomic<size_t> walks_left{ng};
    std::atomic<uint64_t> dpos{0};          /* descriptor bump index */
    std::atomic<uint64_t> max_len{0}, min_len{~0ull};
    const uint64_t dcap = cache.dcap;

    auto worker = [&]() {
        for (;;) {
            const uint64_t t = next.fetch_add(1, std::memory_order_relaxed);
            if (t >= tasks.size())
                return;
            const Task tk = tasks[t];
            if (tk.walk) {
                Ext &x = *G[tk.a];
                walk_ext(static_cast<const uint8_t *>(C.images[x.file]), C.sizes[x.file], C.kinds[x.file],
                         C.fi[x.file], x);
                uint64_t m = max_len.load(std::memory_order_relaxed);
                while (x.max_len > m && !max_len.compare_exchange_weak(m, x.max_len))
                    ;
                m = min_len.load(std::memory_order_relaxed);
                while (x.min_len < m && !min_len.compare_exchange_weak(m, x.min_len))
                    ;
                /* descriptors straight into the pinned arrays (any order:
                 * results go back by position) */
                x.pos = dpos.fetch_add(x.ncommit, std::memory_order_relaxed);
                if (x.pos + x.ncommit <= dcap)
                    place(x, cache.h_off, cache.h_len);
                walks_left.fetch_sub(1, std::memory_order_acq_rel);
                continue;
            }
            const uint64_t p = tk.a;
            while (free_upto.load(std::memory_order_acquire) <= (int64_t)p) {
                if (stop.load(std::memory_order_relaxed))
                    return;
                std::this_thread::yield();
            }
            const uint64_t base = p * slot;
            const uint64_t lo = base + tk.b * SUB;
            const uint64_t hi = std::min(std::min(total, base + slot), lo + SUB);
            uint8_t *dst = cache.slot[p % NSLOT] - base;
            /* the extents overlapping [lo, hi) (each padded to ALIGN with zeros) */
            size_t f = std::upper_bound(G.begin(), G.end(), lo,
                                        [](uint64_t v, const Ext *q) { return v < q->dev_off; }) -
                       G.begin();
            f = f ? f - 1 : 0;
            for (uint64_t at = lo; f < ng && at < hi; ++f) {
                const Ext &x = *G[f];
                const uint64_t fa = x.dev_off, fb = fa + (x.hi - x.lo);
                const uint64_t pe = std::min(hi, fa + ((x.hi - x.lo + ALIGN - 1) & ~(ALIGN - 1)));
                if (pe <= at)
                    continue;
                const uint64_t a = std::max(at, fa), b = std::min(pe, fb);
                if (a < b)
                    memcpy(dst + a, static_cast<const uint8_t *>(C.images[x.file]) + x.lo + (a - fa), b - a);
                const uint64_t z = std::max(at, fb);
                if (z < pe)
                    memset(dst + z, 0, pe - z);
                at = pe;
            }
            left[p].fetch_sub(1, std::memory_order_acq_rel);
        }
    };
    const double t_start = now_s();
    std::vector<std::thread> pool;
    if (!rc)
        for (int i = 0; i < threads; ++i)
            pool.emplace_back(worker);

    /* Descriptors go to the device on the copy stream, between data pieces,
     * as soon as every walk is in; a walk that did not fit the cached pinned
     * arrays (first call, or a larger group) makes them grow here, once. */
    uint64_t ncommit = 0;
    bool desc_sent = false;
    uint64_t *doff = nullptr, *dlen = nullptr;
    uint32_t *dcrc = nullptr, *dst = nullptr, *draw = nullptr;
    std::vector<Ext *> pieces;
    for (Ext *x : G)
        if (x->what == EXT_PIECE)
            pieces.push_back(x);
    auto send_desc = [&]() -> int {
        ncommit = dpos.load();
        if (ncommit > dcap) {
            /* nothing reads the old arrays yet: regrow and place every extent */
            std::vector<uint64_t> oo(cache.h_off, cache.h_off + std::min(ncommit, dcap));
            std::vector<uint64_t> ol(cache.h_len, cache.h_len + std::min(ncommit, dcap));
            int r = ensure_desc(cache, ncommit);
            if (r)
                return r;
            for (Ext *x : G) {
                if (x->placed) {
                    memcpy(cache.h_off + x->pos, oo.data() + x->pos, 8 * x->ncommit);
                    memcpy(cache.h_len + x->pos, ol.data() + x->pos, 8 * x->ncommit);
                } else {
                    place(*x, cache.h_off, cache.h_len);
                }
            }
        }
        /* + the verdict (count + VCAP indices) after the raw registers */
        int r = grow_dev(&cache.ddesc, &cache.ddesc_bytes, 24 * ncommit + 4 * pieces.size() + 8 * (VCAP + 2) + 1024);
        if (r)
            return r;
        doff = reinterpret_cast<uint64_t *>(cache.ddesc);
        dlen = doff + ncommit;
        dcrc = reinterpret_cast<uint32_t *>(dlen + ncommit);
        dst = dcrc + ncommit;
        draw = dst + ncommit;
        if (ncommit && (hipMemcpyAsync(doff, cache.h_off, 8 * ncommit, hipMemcpyHostToDevice, cs) != hipSuccess ||
                        hipMemcpyAsync(dlen, cache.h_len, 8 * ncommit, hipMemcpyHostToDevice, cs) != hipSuccess))
            return ZSCRC_EHIP;
        desc_sent = true;
        return ZSCRC_OK;
    };

    if (C.direct) {
        /* pageable H2D straight from the images: runs of extents adjacent
         * both in host memory and in the device layout go as one copy */
        for (size_t f = 0; !rc && f < ng;) {
            const uint8_t *src = static_cast<const uint8_t *>(C.images[G[f]->file]) + G[f]->lo;
            uint64_t bytes = G[f]->hi - G[f]->lo;
            size_t g = f + 1;
            while (g < ng &&
                   static_cast<const uint8_t *>(C.images[G[g]->file]) + G[g]->lo == src + bytes &&
                   G[g]->dev_off == G[f]->dev_off + bytes) {
                bytes += G[g]->hi - G[g]->lo;
                ++g;
            }
            if (bytes && hipMemcpyAsync(cache.dimg + G[f]->dev_off, src, bytes, hipMemcpyHostToDevice, cs) !=
                             hipSuccess)
                rc = ZSCRC_EHIP;
            if (!rc && !desc_sent && walks_left.load(std::memory_order_acquire) == 0)
                rc = send_desc();
            f = g;
        }
    }
    for (uint64_t p = 0; !C.direct && !rc && p < npiece; ++p) {
        while (left[p].load(std::memory_order_acquire) > 0)
            std::this_thread::yield();
        const int k = (int)(p % NSLOT);
        const uint64_t lo = p * slot, hi = std::min(total, lo + slot);
        if (hipMemcpyAsync(cache.dimg + lo, cache.slot[k], hi - lo, hipMemcpyHostToDevice, cs) != hipSuccess ||
            hipEventRecord(slot_ev[k], cs) != hipSuccess) {
            rc = ZSCRC_EHIP;
            break;
        }
        if (!desc_sent && walks_left.load(std::memory_order_acquire) == 0)
            rc = send_desc();
        /* the next piece's slot: free once piece p + 1 - NSLOT's copy is done */
        if (!rc && p + 1 >= (uint64_t)NSLOT && p + 1 < npiece) {
            if (hipEventSynchronize(slot_ev[(p + 1) % NSLOT]) != hipSuccess) {
                rc = ZSCRC_EHIP;
                break;
            }
            free_upto.store((int64_t)p + 2, std::memory_order_release);
        }
    }
    if (rc)
        stop = 1;
    for (auto &t : pool)
        t.join();
    pool.clear();
    if (!rc && !desc_sent)
        rc = send_desc();
    /* the group's commits in one verify, its region pieces as raw spans, once
     * the last byte is on the device */
    if (!rc && (hipEventRecord(done_ev, cs) != hipSuccess || hipStreamWaitEvent(ks, done_ev, 0) != hipSuccess))
        rc = ZSCRC_EHIP;
    /* the verdict: a count and the indices of the commits that do not
     * verify -- no per-commit output, no 4 B per commit back over PCIe and
     * no host scan of them (the per-commit arrays only when more than VCAP
     * commits fail) */
    uint64_t *d_nbad = reinterpret_cast<uint64_t *>(
        (reinterpret_cast<uintptr_t>(draw + pieces.size()) + 7) & ~uintptr_t(7));
    const uint64_t vcap = std::min<uint64_t>(VCAP, ncommit);
    if (!rc && ncommit) {
        /* the walks' length range: classes outside it get no launch */
        rc = zscrc_device_verify_commits_verdict_range(cache.dimg, total, doff, dlen, nullptr, ncommit,
                                                       std::min(min_len.load(), max_len.load()), max_len.load(),
                                                       d_nbad, d_nbad + 1, vcap, ks);
        if (!rc && hipMemcpyAsync(cache.h_bad, d_nbad, 8 * (vcap + 1), hipMemcpyDeviceToHost, ks) != hipSuccess)
            rc = ZSCRC_EHIP;
    }
    std::vector<uint32_t> raw(pieces.size());
    if (!rc && !pieces.empty()) {
        /* up to 8 pieces in one segment launch + one fold launch */
        const void *bufs[8];
        uint64_t lens[8];
        size_t i = 0;
        while (!rc && i < pieces.size()) {
            size_t k = 0;
            while (k < 8 && i + k < pieces.size() && pieces[i + k]->hi - pieces[i + k]->lo >= (16u << 10)) {
                bufs[k] = cache.dimg + pieces[i + k]->dev_off;
                lens[k] = pieces[i + k]->hi - pieces[i + k]->lo;
                ++k;
            }
            if (k >= 2) {
                rc = zscrc_device_spans(bufs, lens, nullptr, draw + i, k, ZSCRC_RAW, ks);
                i += k;
            } else {
                rc = zscrc_device_span(cache.dimg + pieces[i]->dev_off, pieces[i]->hi - pieces[i]->lo, 0, draw + i,
                                       nullptr, ZSCRC_RAW, ks);
                ++i;
            }
        }
        if (!rc && hipMemcpyAsync(raw.data(), draw, 4 * raw.size(), hipMemcpyDeviceToHost, ks) != hipSuccess)
            rc = ZSCRC_EHIP;
    }
    if (!rc && hipStreamSynchronize(cs) != hipSuccess)
        rc = ZSCRC_EHIP;
    const double t_copied = now_s();
    if (!rc && hipStreamSynchronize(ks) != hipSuccess)
        rc = ZSCRC_EHIP;
    const double t_verified = now_s();
    for (size_t i = 0; !rc && i < pieces.size(); ++i)
        pieces[i]->raw = raw[i];

    /* mismatches (status != 1), by descriptor position -> extent */
    std::vector<uint64_t> badpos;
    if (!rc && ncommit) {
        const uint64_t nbad = cache.h_bad[0];
        if (nbad <= vcap) {
            badpos.assign(cache.h_bad + 1, cache.h_bad + 1 + nbad);
            std::sort(badpos.begin(), badpos.end());
        } else {
            /* more than the list holds: every commit's status */
            rc = zscrc_device_verify_commits_bounded(cache.dimg, total, doff, dlen, nullptr, ncommit, max_len.load(),
                                                     dcrc, dst, ks);
            if (!rc && (hipMemcpyAsync(cache.h_st, dst, 4 * ncommit, hipMemcpyDeviceToHost, ks) != hipSuccess ||
                        hipStreamSynchronize(ks) != hipSuccess))
                rc = ZSCRC_EHIP;
            const uint32_t *st = cache.h_st;
            for (uint64_t i = 0; !rc && i < ncommit; ++i)
                if (st[i] != 1)
                    badpos.push_back(i);
        }
    }
    std::vector<std::pair<uint64_t, size_t>> by_pos; /* (pos, extent) of extents with commits */
    if (!badpos.empty()) {
        for (size_t f = 0; f < ng; ++f)
            if (G[f]->ncommit)
                by_pos.push_back({G[f]->pos, f});
        std::sort(by_pos.begin(), by_pos.end());
    }
    auto ext_of = [&](uint64_t i) -> Ext & {
        auto it = std::upper_bound(by_pos.begin(), by_pos.end(), std::make_pair(i, ~size_t(0)));
        return *G[(it - 1)->second];
    };
    /* stale zero-length commits: chained from the previous span's CRC */
    std::vector<uint64_t> cand;
    for (uint64_t i : badpos) {
        if (cache.h_len[i] == 0 && i > ext_of(i).pos)
            cand.push_back(i);
    }
    std::vector<uint32_t> st2(cand.size());
    if (!rc && !cand.empty()) {
        const size_t m = cand.size();
        std::vector<uint64_t> q(4 * m);
        uint64_t prev_max = 0;
        for (size_t c = 0; c < m; ++c) {
            const uint64_t i = cand[c];
            prev_max = std::max(prev_max, cache.h_len[i - 1]);
            q[c] = cache.h_off[i - 1];
            q[m + c] = cache.h_len[i - 1];
            q[2 * m + c] = cache.h_off[i];
            q[3 * m + c] = cache.h_len[i];
        }
        /* a cached device buffer: a hipMalloc / hipFree per call cost a
         * device-wide synchronisation each */
        rc = grow_dev(&cache.dq, &cache.dq_bytes, 4 * m * 8 + 3 * m * 4);
        uint64_t *dq = rc ? nullptr : reinterpret_cast<uint64_t *>(cache.dq);
        uint32_t *dprev = dq ? reinterpret_cast<uint32_t *>(dq + 4 * m) : nullptr;
        if (!rc && hipMemcpyAsync(dq, q.data(), 4 * m * 8, hipMemcpyHostToDevice, ks) != hipSuccess)
            rc = ZSCRC_EHIP;
        if (!rc)
            rc = zscrc_device_batch_bounded(cache.dimg, dq, dq + m, nullptr, dprev, m, 0, prev_max, ks);
        if (!rc)
            rc = zscrc_device_verify_commits_bounded(cache.dimg, total, dq + 2 * m, dq + 3 * m, dprev, m, 0,
                                                     dprev + m, dprev + 2 * m, ks);
        if (!rc && (hipMemcpyAsync(st2.data(), dprev + 2 * m, m * 4, hipMemcpyDeviceToHost, ks) != hipSuccess ||
                    hipStreamSynchronize(ks) != hipSuccess))
            rc = ZSCRC_EHIP;
    }
    if (!rc) {
        std::lock_guard<std::mutex> lk(C.acc.mu);
        C.acc.commits += ncommit;
        size_t c = 0;
        for (uint64_t i : badpos) {
            while (c < cand.size() && cand[c] < i)
                ++c;
            if (c < cand.size() && cand[c] == i && st2[c] == 1) {
                C.acc.stale++;
                continue;
            }
            C.acc.bad++;
            const Ext &x = ext_of(i);
            C.acc.first(x.file, cache.h_off[i] - x.dev_off + x.lo + cache.h_len[i], ZSCRC_FILES_BAD_COMMIT);
        }
    }
    /* nothing of this group left queued on the cached streams (error paths
     * included) before the buffers serve another group */
    for (hipStream_t q : {cs, ks})
        if (q && hipStreamSynchronize(q) != hipSuccess && !rc)
            rc = ZSCRC_EHIP;
    {
        std::lock_guard<std::mutex> lk(C.tmu);
        C.copy_s = std::max(C.copy_s, t_copied - t_start);
        C.tail_s = std::max(C.tail_s, t_verified - t_copied);
    }
    return rc;
}

} /* namespace */

extern "C" int zscrc_set_devices(const int *ids, int n)
{
    if (n < 0 || n > MAX_SLOTS || (n && !ids))
        return ZSCRC_EINVAL;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    g_devices.assign(ids, ids + n);
    g_devices_set = n > 0;
    return ZSCRC_OK;
}

extern "C" int zscrc_files_devices(int *ids, int cap)
{
    std::vector<int> d;
    const int rc = device_list(d);
    if (rc)
        return rc;
    for (int i = 0; i < cap && i < (int)d.size(); ++i)
        ids[i] = d[i];
    return (int)d.size();
}

extern "C" void zs_fill_release_cache(void);
extern "C" void zs_scalar_release_cache(void);

extern "C" void zscrc_release_cache(void)
{
    int cur = -1;
    (void)hipGetDevice(&cur);
    for (auto &c : g_cache) {
        std::lock_guard<std::mutex> lk(c.mu);
        cache_free(c);
    }
    if (cur >= 0)
        (void)hipSetDevice(cur);
    zs_fill_release_cache();   /* zscrc_zs_fill_commits' pipeline */
    zs_scalar_release_cache(); /* the drop-in symbols' offload stream */
}

extern "C" int zscrc_zs_verify_files(const void *const *images, const uint64_t *sizes, const int *kinds, size_t n,
                                     int threads, zscrc_files_report *rep)
{
    if (!rep || (n && (!images || !sizes || !kinds)))
        return ZSCRC_EINVAL;
    memset(rep, 0, sizeof *rep);
    rep->first_bad_file = ~0ull;
    const double t0 = now_s();
    std::vector<int> devs;
    int rc = device_list(devs);
    if (rc)
        return rc;
    const int S = (int)devs.size();
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return ZSCRC_ENODEV;
    if (threads <= 0) {
        const unsigned h = std::thread::hardware_concurrency();
        threads = h ? (int)std::min(h, 16u) : 4;
        if (const char *e = getenv("OMP_NUM_THREADS"))
            if (atoi(e) > 0)
                threads = std::min(threads, atoi(e));
    }
    rep->threads = threads;
    rep->devices = S;

    Call C;
    C.images = images;
    C.sizes = sizes;
    C.kinds = kinds;
    C.n = n;
    C.fi.resize(n);
    if (const char *e = getenv("ZSCRC_FILES_SLOT"))
        C.slot_bytes = std::max<uint64_t>(SUB, strtoull(e, nullptr, 0));
    C.slot_bytes = (C.slot_bytes + SUB - 1) / SUB * SUB;
    /* staged (default): host threads copy into pinned staging slots, the
     * copy stream DMAs those; ZSCRC_FILES_STAGE=0: pageable H2D copies
     * straight from the images, the host threads only walk (measured slower:
     * config 4 BATCHED 39 vs 47 GB/s, a DB directory 17 vs 44 GB/s,
     * profiles/r02/e2e_v2.jsonl) */
    const char *stage_env = getenv("ZSCRC_FILES_STAGE");
    C.direct = stage_env && atoi(stage_env) == 0;
    rep->staged = C.direct ? 0 : 1;

    /* group bound: env, and at most half of what each slot's device can hold */
    uint64_t group = GROUP_DEFAULT;
    if (const char *e = getenv("ZSCRC_FILES_GROUP"))
        group = std::max<uint64_t>(1u << 20, strtoull(e, nullptr, 0));
    for (int s = 0; s < S; ++s) {
        size_t fr = 0, tot = 0;
        if (hipSetDevice(devs[s]) != hipSuccess || hipMemGetInfo(&fr, &tot) != hipSuccess) {
            (void)hipSetDevice(cur);
            return ZSCRC_EHIP;
        }
        /* slots sharing a device share its memory */
        const uint64_t share = (uint64_t)std::count(devs.begin(), devs.end(), devs[s]);
        uint64_t held = 0;
        if (g_cache[s].dev == devs[s])
            held = g_cache[s].dimg_bytes;
        group = std::min<uint64_t>(group, (fr / share + held) / 2);
    }
    (void)hipSetDevice(cur);
    group = std::max<uint64_t>(group & ~(SPLIT_ALIGN - 1), SPLIT_ALIGN);

    /* units in file order; packed files with a parsed layout split */
    struct Unit {
        size_t file;
        int what;
        uint64_t lo, hi;
    };
    std::vector<Unit> seq;
    uint64_t W = 0;
    for (size_t f = 0; f < n; ++f) {
        const uint8_t *img = static_cast<const uint8_t *>(images[f]);
        FileInfo &fi = C.fi[f];
        if (kinds[f] == ZSCRC_ZS_PACKED && sizes[f] >= 56) {
            uint64_t o[2], l[2];
            if (zscrc_zs_packed_spans(img, sizes[f], o, l) == ZSCRC_OK) {
                fi.split = true;
                fi.roff = o[0];
                fi.rlen = l[0];
                fi.poff = o[1];
                fi.plen = l[1];
                const uint64_t rend = fi.roff + fi.rlen;
                if (fi.rlen)
                    seq.push_back({f, EXT_PIECE, fi.roff, rend});
                seq.push_back({f, EXT_TAIL, rend, sizes[f]});
                W += sizes[f] - fi.roff;
                continue;
            }
        }
        seq.push_back({f, EXT_FILE, 0, sizes[f]});
        W += sizes[f];
    }
    std::vector<uint64_t> bound(S + 1);
    for (int s = 0; s <= S; ++s)
        bound[s] = (uint64_t)((unsigned __int128)W * s / S);
    auto slot_of = [&](uint64_t x) {
        int s = 0;
        while (s + 1 < S && bound[s + 1] <= x)
            ++s;
        return s;
    };
    uint64_t at = 0;
    for (const Unit &u : seq) {
        const uint64_t w = u.hi - u.lo;
        if (u.what != EXT_PIECE) {
            Ext x;
            x.file = u.file;
            x.what = u.what;
            x.lo = u.lo;
            x.hi = u.hi;
            x.slot = slot_of(at + w / 2);
            C.ext.push_back(std::move(x));
        } else {
            /* cut at the slot bounds, then into pieces of at most `group` */
            std::vector<uint64_t> cuts{u.lo};
            for (int s = 1; s < S; ++s)
                if (at < bound[s] && bound[s] < at + w) {
                    const uint64_t c = u.lo + (bound[s] - at) / SPLIT_ALIGN * SPLIT_ALIGN;
                    if (cuts.back() < c && c < u.hi)
                        cuts.push_back(c);
                }
            cuts.push_back(u.hi);
            uint32_t idx = 0;
            for (size_t i = 0; i + 1 < cuts.size(); ++i) {
                const uint64_t a = cuts[i], b = cuts[i + 1];
                const int s = slot_of(at + (a - u.lo) + (b - a) / 2);
                const uint64_t k = (b - a + group - 1) / group;
                const uint64_t step = ((b - a) / k + SPLIT_ALIGN - 1) / SPLIT_ALIGN * SPLIT_ALIGN;
                for (uint64_t c = a; c < b; c += step) {
                    Ext x;
                    x.file = u.file;
                    x.what = EXT_PIECE;
                    x.lo = c;
                    x.hi = std::min(b, c + step);
                    x.slot = s;
                    x.piece = idx++;
                    C.ext.push_back(std::move(x));
                }
            }
        }
        at += w;
    }

    /* every slot on its own thread: its extents in groups of <= group bytes */
    const int per = std::max(2, threads / S);
    std::vector<int> src(S, ZSCRC_OK);
    auto run_slot = [&](int s) {
        Cache &cache = g_cache[s];
        std::lock_guard<std::mutex> lk(cache.mu);
        if (cache.dev != devs[s]) {
            cache_free(cache);
            cache.dev = devs[s];
        }
        if (hipSetDevice(devs[s]) != hipSuccess) {
            src[s] = ZSCRC_EHIP;
            return;
        }
        std::vector<Ext *> G;
        uint64_t gbytes = 0;
        auto flush = [&]() {
            if (!G.empty() && !src[s])
                src[s] = run_group(C, cache, G, per);
            G.clear();
            gbytes = 0;
        };
        for (Ext &x : C.ext) {
            if (x.slot != s)
                continue;
            const uint64_t b = (x.hi - x.lo + ALIGN - 1) & ~(ALIGN - 1);
            if (!G.empty() && gbytes + b > group)
                flush();
            G.push_back(&x);
            gbytes += b;
        }
        flush();
        /* the buffer never holds more than one group; beyond that, free it */
        if (cache.dimg_bytes > group + group / 8) {
            (void)hipFree(cache.dimg);
            cache.dimg = nullptr;
            cache.dimg_bytes = 0;
        }
    };
    if (S == 1) {
        run_slot(0);
    } else {
        std::vector<std::thread> th;
        for (int s = 0; s < S; ++s)
            th.emplace_back(run_slot, s);
        for (auto &t : th)
            t.join();
    }
    (void)hipSetDevice(cur);
    for (int s = 0; s < S; ++s)
        if (src[s] && !rc)
            rc = src[s];
    if (rc)
        return rc;

    /* records regions: fold the pieces' raw registers in order, check the
     * region's commit trailer on the host */
    std::vector<std::vector<const Ext *>> reg(n);
    for (const Ext &x : C.ext)
        if (x.what == EXT_PIECE)
            reg[x.file].push_back(&x);
    Acc &A = C.acc;
    for (size_t f = 0; f < n; ++f) {
        const FileInfo &fi = C.fi[f];
        if (!fi.split)
            continue;
        std::sort(reg[f].begin(), reg[f].end(), [](const Ext *a, const Ext *b) { return a->lo < b->lo; });
        uint32_t r = 0xFFFFFFFFu; /* crc32c(0, ...) starts from ~0 */
        for (const Ext *x : reg[f])
            r = zscrc_shift(r, x->hi - x->lo) ^ x->raw;
        const int st = host_commit_check(static_cast<const uint8_t *>(images[f]), sizes[f], fi.roff + fi.rlen,
                                         r ^ 0xFFFFFFFFu);
        A.commits++;
        if (st != 1) {
            A.bad++;
            A.first(f, fi.roff + fi.rlen, ZSCRC_FILES_BAD_COMMIT);
        }
    }
    /* verdicts; the first problem in file order */
    rep->files = n;
    rep->commits = A.commits;
    rep->bad_commits = A.bad;
    rep->stale_empty_commits = A.stale;
    rep->first_bad_file = A.first_file;
    rep->first_bad_off = A.first_off;
    rep->first_bad_what = A.first_what;
    for (size_t f = 0; f < n; ++f) {
        rep->bytes += sizes[f];
        if (C.fi[f].header_bad) {
            rep->header_errors++;
            A.first(f, 0, ZSCRC_FILES_BAD_HEADER);
        }
        if (C.fi[f].walk_rc != (kinds[f] == ZSCRC_ZS_PACKED ? ZSCRC_OK : ZSCRC_ZS_END)) {
            rep->walk_errors++;
            A.first(f, C.fi[f].walk_end, ZSCRC_FILES_BAD_WALK);
        }
    }
    rep->first_bad_file = A.first_file;
    rep->first_bad_off = A.first_off;
    rep->first_bad_what = A.first_what;
    rep->copy_s = C.copy_s;
    rep->verify_tail_s = C.tail_s;
    rep->total_s = now_s() - t0;
    return ZSCRC_OK;
}
