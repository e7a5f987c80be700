/*
 * zscrc_files.cpp -- verify every CRC of a set of host-resident zeroskip file
 * images (mmap'd files: verify-on-open of a whole DB, `consistent`), end to
 * end: host memory -> GPU -> verdict.  Declared in include/zscrc.h
 * (zscrc_zs_verify_files); zscrc_zs_consistent runs on it.
 *
 * What is checked is the reference's: the header CRC (src/zeroskip-header.c:
 * 105-170), the record walk (src/zeroskip-record.c:283-331) and every commit
 * CRC with the writer's trailer semantics (src/zeroskip-file.c:253-350) for
 * active / finalised files, and the records-region + pointer-section commits
 * of packed files (src/zeroskip-packed.c:70-131, :278-339, :442).
 *
 * Pipeline (one call):
 *   * the files are laid out back to back (256-byte aligned) in one device
 *     buffer, whose byte range is cut into pieces of `slot` bytes;
 *   * a pool of host threads takes tasks in order -- first every file's walk
 *     (header CRC, commit spans), then the copy of 4 MiB sub-ranges of piece p
 *     into pinned staging slot p % NSLOT, once the slot's previous H2D copy
 *     has left;
 *   * the calling thread issues piece p's H2D copy on a copy stream as soon
 *     as its sub-ranges are staged; whenever the bytes and walks of further
 *     files are complete, their commits are verified on a compute stream in
 *     one bounded launch -- PCIe transfer, host copies and GPU verification
 *     overlap;
 *   * zero-length commits that chain from the previous span's CRC (the
 *     finalise quirk, src/zeroskip-active.c:122 + src/mfile.c:534-546) are
 *     re-verified at the end with that CRC as the seed and counted apart.
 * Pinned slots, pinned descriptor blocks and the device buffer are cached per
 * device between calls.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/zscrc.h"

namespace {

constexpr int NSLOT = 4;
constexpr uint64_t ALIGN = 256;
constexpr uint64_t SUB = 4ull << 20; /* bytes per copy task */
constexpr int MAX_DEV = 64;

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

/* Per-device cache. */
struct Cache {
    std::mutex mu;
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
};
Cache g_cache[MAX_DEV];

int grow_dev(uint8_t **p, uint64_t *have, uint64_t need)
{
    if (*have >= need)
        return ZSCRC_OK;
    if (*p)
        (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    need += need / 4;
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
    return ZSCRC_OK;
}

struct FileState {
    uint64_t dev_off = 0;           /* where its bytes go in the device buffer */
    std::vector<uint64_t> off, len; /* commit spans while walking (file offsets) */
    uint64_t ncommit = 0;
    uint64_t pos = 0;               /* its commits: [pos, pos + ncommit) of the descriptor arrays */
    bool placed = false;            /* written to the pinned arrays by its walker */
    uint64_t max_len = 0;
    int header_bad = 0;
    int walk_rc = 0;                /* ZSCRC_ZS_END, or ZSCRC_OK for a packed file's layout */
    uint64_t walk_end = 0;
};

void walk_file(const uint8_t *img, uint64_t size, int kind, FileState &fs)
{
    uint32_t st = 0, cp = 0;
    fs.header_bad = size < 40 || zscrc_zs_header_crc(img, size, &st, &cp) != ZSCRC_OK || st != cp;
    size_t n = 0;
    if (kind == ZSCRC_ZS_PACKED) {
        uint64_t o[2], l[2];
        fs.walk_rc = size >= 56 ? zscrc_zs_packed_spans(img, size, o, l) : ZSCRC_ZS_TRUNCATED;
        fs.walk_end = size;
        if (fs.walk_rc == ZSCRC_OK) {
            fs.off.assign(o, o + 2);
            fs.len.assign(l, l + 2);
            n = 2;
        }
    } else if (size < 40) {
        fs.walk_rc = ZSCRC_ZS_TRUNCATED;
    } else {
        size_t cap = (size_t)(size / 256) + 64; /* grown on overflow */
        for (;;) {
            fs.off.resize(cap);
            fs.len.resize(cap);
            fs.walk_rc = zscrc_zs_walk(img, size, fs.off.data(), fs.len.data(), cap, &n, &fs.walk_end);
            if (fs.walk_rc != ZSCRC_ZS_OVERFLOW)
                break;
            cap = n + 64;
        }
        if (fs.walk_rc < 0)
            n = 0;
    }
    fs.off.resize(n);
    fs.len.resize(n);
    fs.ncommit = n;
    for (size_t i = 0; i < n; ++i)
        fs.max_len = std::max(fs.max_len, fs.len[i]);
}

/* The walker's spans -> descriptor arrays at pos (device offsets). */
void place(FileState &fs, uint64_t *h_off, uint64_t *h_len)
{
    for (uint64_t i = 0; i < fs.ncommit; ++i) {
        h_off[fs.pos + i] = fs.dev_off + fs.off[i];
        h_len[fs.pos + i] = fs.len[i];
    }
    fs.placed = true;
    std::vector<uint64_t>().swap(fs.off);
    std::vector<uint64_t>().swap(fs.len);
}

} /* namespace */

extern "C" int zscrc_zs_verify_files(const void *const *images, const uint64_t *sizes, const int *kinds, size_t n,
                                     int threads, zscrc_files_report *rep)
{
    if (!rep || (n && (!images || !sizes || !kinds)))
        return ZSCRC_EINVAL;
    memset(rep, 0, sizeof *rep);
    rep->first_bad_file = ~0ull;
    const double t0 = now_s();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV)
        return ZSCRC_ENODEV;
    if (threads <= 0) {
        const unsigned h = std::thread::hardware_concurrency();
        threads = h ? (int)std::min(h, 16u) : 4;
        if (const char *e = getenv("OMP_NUM_THREADS"))
            if (atoi(e) > 0)
                threads = std::min(threads, atoi(e));
    }
    rep->threads = threads;
    std::vector<FileState> fs(n);
    uint64_t total = 0, est = 1024;
    for (size_t i = 0; i < n; ++i) {
        fs[i].dev_off = total;
        total += (sizes[i] + ALIGN - 1) & ~(ALIGN - 1);
        est += sizes[i] / 256 + 4;
    }
    uint64_t slot = 64ull << 20;
    if (const char *e = getenv("ZSCRC_FILES_SLOT"))
        slot = std::max<uint64_t>(SUB, strtoull(e, nullptr, 0));
    slot = (slot + SUB - 1) / SUB * SUB;
    /* staged (default): host threads copy into pinned staging slots, the
     * copy stream DMAs those; ZSCRC_FILES_STAGE=0: pageable H2D copies
     * straight from the images, the host threads only walk (measured slower:
     * config 4 BATCHED 39 vs 47 GB/s, a DB directory 17 vs 44 GB/s,
     * profiles/r02/e2e_v2.jsonl) */
    const char *stage_env = getenv("ZSCRC_FILES_STAGE");
    const bool direct = stage_env && atoi(stage_env) == 0;
    rep->staged = direct ? 0 : 1;
    Cache &cache = g_cache[dev];
    std::lock_guard<std::mutex> lk(cache.mu);
    int rc = direct ? ZSCRC_OK : ensure_slots(cache, slot);
    if (!rc)
        rc = grow_dev(&cache.dimg, &cache.dimg_bytes, std::max<uint64_t>(total, ALIGN));
    if (!rc && cache.dcap == 0)
        rc = ensure_desc(cache, est); /* later calls keep what the largest needed */
    if (rc)
        return rc;
    const uint64_t npiece = (total + slot - 1) / slot;

    struct Task {
        int walk;    /* 1 walk, 0 copy */
        uint64_t a;  /* file, or piece */
        uint64_t b;  /* sub-range of the piece */
    };
    std::vector<Task> tasks;
    tasks.reserve(n + npiece * (slot / SUB));
    std::vector<std::atomic<int>> left(npiece);
    if (direct) {
        /* the copies are the driver's (pageable H2D straight from the
         * images): the pool only walks */
        for (size_t f = 0; f < n; ++f)
            tasks.push_back({1, f, 0});
    } else {
        /* staged: each piece's copy tasks, then the walks of the files that
         * end in it -- the PCIe stream starts at once and the walks overlap
         * it (all walks first held every copy back ~25 ms on 10 M commits) */
        size_t f = 0;
        for (uint64_t p = 0; p < npiece; ++p) {
            const uint64_t len = std::min(total, (p + 1) * slot) - p * slot;
            left[p] = (int)((len + SUB - 1) / SUB);
            for (uint64_t s = 0; s < (uint64_t)left[p]; ++s)
                tasks.push_back({0, p, s});
            for (; f < n && (fs[f].dev_off + sizes[f] <= (p + 1) * slot || p + 1 == npiece); ++f)
                tasks.push_back({1, f, 0});
        }
    }

    hipStream_t cs = nullptr, ks = nullptr;
    hipEvent_t slot_ev[NSLOT] = {}, done_ev = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&ks, hipStreamNonBlocking);
    for (int k = 0; e == hipSuccess && k < NSLOT; ++k)
        e = hipEventCreateWithFlags(&slot_ev[k], hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&done_ev, hipEventDisableTiming);
    if (e != hipSuccess)
        rc = ZSCRC_EHIP;

    std::atomic<uint64_t> next{0};
    std::atomic<int> stop{0};
    /* slot of piece p is free for its copy tasks once piece p - NSLOT's H2D
     * copy has completed: free_upto = (last such piece) + 1 */
    std::atomic<int64_t> free_upto{NSLOT};
    std::atomic<size_t> walks_left{n};
    std::atomic<uint64_t> dpos{0};          /* descriptor bump index */
    std::atomic<uint64_t> max_len{0};
    const uint64_t dcap = cache.dcap;

    auto worker = [&]() {
        for (;;) {
            const uint64_t t = next.fetch_add(1, std::memory_order_relaxed);
            if (t >= tasks.size())
                return;
            const Task tk = tasks[t];
            if (tk.walk) {
                FileState &f = fs[tk.a];
                walk_file(static_cast<const uint8_t *>(images[tk.a]), sizes[tk.a], kinds[tk.a], f);
                uint64_t m = max_len.load(std::memory_order_relaxed);
                while (f.max_len > m && !max_len.compare_exchange_weak(m, f.max_len))
                    ;
                /* descriptors straight into the pinned arrays (any file order:
                 * results go back by position) */
                f.pos = dpos.fetch_add(f.ncommit, std::memory_order_relaxed);
                if (f.pos + f.ncommit <= dcap)
                    place(f, cache.h_off, cache.h_len);
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
            /* the files overlapping [lo, hi) (each padded to ALIGN with zeros) */
            size_t f = std::upper_bound(fs.begin(), fs.end(), lo,
                                        [](uint64_t v, const FileState &q) { return v < q.dev_off; }) -
                       fs.begin();
            f = f ? f - 1 : 0;
            for (uint64_t at = lo; f < n && at < hi; ++f) {
                const uint64_t fa = fs[f].dev_off, fb = fa + sizes[f];
                const uint64_t pe = std::min(hi, fa + ((sizes[f] + ALIGN - 1) & ~(ALIGN - 1)));
                if (pe <= at)
                    continue;
                const uint64_t a = std::max(at, fa), b = std::min(pe, fb);
                if (a < b)
                    memcpy(dst + a, static_cast<const uint8_t *>(images[f]) + (a - fa), b - a);
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
     * arrays (first call, or a larger DB) makes them grow here, once. */
    uint64_t ncommit = 0;
    bool desc_sent = false;
    uint64_t *doff = nullptr, *dlen = nullptr;
    uint32_t *dcrc = nullptr, *dst = nullptr;
    auto send_desc = [&]() -> int {
        ncommit = dpos.load();
        if (ncommit > dcap) {
            /* nothing reads the old arrays yet: regrow and place every file */
            std::vector<std::pair<uint64_t, uint64_t>> keep; /* placed files' old ranges */
            std::vector<uint64_t> oo(cache.h_off, cache.h_off + std::min(ncommit, dcap));
            std::vector<uint64_t> ol(cache.h_len, cache.h_len + std::min(ncommit, dcap));
            int r = ensure_desc(cache, ncommit);
            if (r)
                return r;
            for (auto &f : fs) {
                if (f.placed) {
                    memcpy(cache.h_off + f.pos, oo.data() + f.pos, 8 * f.ncommit);
                    memcpy(cache.h_len + f.pos, ol.data() + f.pos, 8 * f.ncommit);
                } else {
                    place(f, cache.h_off, cache.h_len);
                }
            }
        }
        int r = grow_dev(&cache.ddesc, &cache.ddesc_bytes, 24 * ncommit + 1024);
        if (r)
            return r;
        doff = reinterpret_cast<uint64_t *>(cache.ddesc);
        dlen = doff + ncommit;
        dcrc = reinterpret_cast<uint32_t *>(dlen + ncommit);
        dst = dcrc + ncommit;
        if (ncommit && (hipMemcpyAsync(doff, cache.h_off, 8 * ncommit, hipMemcpyHostToDevice, cs) != hipSuccess ||
                        hipMemcpyAsync(dlen, cache.h_len, 8 * ncommit, hipMemcpyHostToDevice, cs) != hipSuccess))
            return ZSCRC_EHIP;
        desc_sent = true;
        return ZSCRC_OK;
    };

    if (direct) {
        /* runs of files adjacent both in host memory and in the device
         * layout go as one copy */
        for (size_t f = 0; !rc && f < n;) {
            size_t g = f + 1;
            uint64_t bytes = sizes[f];
            while (g < n && static_cast<const uint8_t *>(images[g]) ==
                                static_cast<const uint8_t *>(images[g - 1]) + sizes[g - 1] &&
                   fs[g].dev_off == fs[g - 1].dev_off + sizes[g - 1]) {
                bytes += sizes[g];
                ++g;
            }
            if (bytes && hipMemcpyAsync(cache.dimg + fs[f].dev_off, images[f], bytes, hipMemcpyHostToDevice, cs) !=
                             hipSuccess)
                rc = ZSCRC_EHIP;
            if (!rc && !desc_sent && walks_left.load(std::memory_order_acquire) == 0)
                rc = send_desc();
            f = g;
        }
    }
    for (uint64_t p = 0; !direct && !rc && p < npiece; ++p) {
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
    /* one verify over every commit once the last byte is on the device */
    if (!rc && (hipEventRecord(done_ev, cs) != hipSuccess || hipStreamWaitEvent(ks, done_ev, 0) != hipSuccess))
        rc = ZSCRC_EHIP;
    const double t_issued = now_s();
    if (!rc && ncommit) {
        rc = zscrc_device_verify_commits_bounded(cache.dimg, total, doff, dlen, nullptr, ncommit, max_len.load(),
                                                 dcrc, dst, ks);
        if (!rc && hipMemcpyAsync(cache.h_st, dst, 4 * ncommit, hipMemcpyDeviceToHost, ks) != hipSuccess)
            rc = ZSCRC_EHIP;
    }
    if (!rc && hipStreamSynchronize(cs) != hipSuccess)
        rc = ZSCRC_EHIP;
    const double t_copied = now_s();
    if (!rc && hipStreamSynchronize(ks) != hipSuccess)
        rc = ZSCRC_EHIP;
    const double t_verified = now_s();
    (void)t_issued;

    /* mismatches (status != 1), by descriptor position -> file */
    std::vector<uint64_t> badpos;
    if (!rc) {
        const uint32_t *st = cache.h_st;
        for (uint64_t i = 0; i < ncommit; ++i)
            if (st[i] != 1)
                badpos.push_back(i);
    }
    std::vector<std::pair<uint64_t, size_t>> by_pos; /* (pos, file) of files with commits */
    if (!badpos.empty()) {
        for (size_t f = 0; f < n; ++f)
            if (fs[f].ncommit)
                by_pos.push_back({fs[f].pos, f});
        std::sort(by_pos.begin(), by_pos.end());
    }
    auto file_of = [&](uint64_t i) -> size_t {
        auto it = std::upper_bound(by_pos.begin(), by_pos.end(), std::make_pair(i, ~size_t(0)));
        return (it - 1)->second;
    };
    /* stale zero-length commits: chained from the previous span's CRC */
    std::vector<uint64_t> cand;
    for (uint64_t i : badpos) {
        const size_t f = file_of(i);
        if (cache.h_len[i] == 0 && i > fs[f].pos)
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
        uint64_t *dq = nullptr;
        e = hipMalloc(&dq, 4 * m * 8 + 3 * m * 4);
        uint32_t *dprev = e == hipSuccess ? reinterpret_cast<uint32_t *>(dq + 4 * m) : nullptr;
        if (e == hipSuccess)
            e = hipMemcpy(dq, q.data(), 4 * m * 8, hipMemcpyHostToDevice);
        rc = e == hipSuccess ? ZSCRC_OK : ZSCRC_EHIP;
        if (!rc)
            rc = zscrc_device_batch_bounded(cache.dimg, dq, dq + m, nullptr, dprev, m, 0, prev_max, nullptr);
        if (!rc)
            rc = zscrc_device_verify_commits_bounded(cache.dimg, total, dq + 2 * m, dq + 3 * m, dprev, m, 0,
                                                     dprev + m, dprev + 2 * m, nullptr);
        if (!rc && hipMemcpy(st2.data(), dprev + 2 * m, m * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = ZSCRC_EHIP;
        if (dq)
            (void)hipFree(dq);
    }
    /* verdicts; the first problem in file order */
    if (!rc) {
        auto first = [&](uint64_t f, uint64_t off, int what) {
            if (f < rep->first_bad_file || (f == rep->first_bad_file && off < rep->first_bad_off)) {
                rep->first_bad_file = f;
                rep->first_bad_off = off;
                rep->first_bad_what = what;
            }
        };
        rep->files = n;
        rep->commits = ncommit;
        for (size_t f = 0; f < n; ++f) {
            rep->bytes += sizes[f];
            if (fs[f].header_bad) {
                rep->header_errors++;
                first(f, 0, ZSCRC_FILES_BAD_HEADER);
            }
            if (fs[f].walk_rc != (kinds[f] == ZSCRC_ZS_PACKED ? ZSCRC_OK : ZSCRC_ZS_END)) {
                rep->walk_errors++;
                first(f, fs[f].walk_end, ZSCRC_FILES_BAD_WALK);
            }
        }
        size_t c = 0;
        for (uint64_t i : badpos) {
            while (c < cand.size() && cand[c] < i)
                ++c;
            if (c < cand.size() && cand[c] == i && st2[c] == 1) {
                rep->stale_empty_commits++;
                continue;
            }
            rep->bad_commits++;
            const size_t f = file_of(i);
            first(f, cache.h_off[i] - fs[f].dev_off + cache.h_len[i], ZSCRC_FILES_BAD_COMMIT);
        }
    }
    for (int k = 0; k < NSLOT; ++k)
        if (slot_ev[k])
            (void)hipEventDestroy(slot_ev[k]);
    if (done_ev)
        (void)hipEventDestroy(done_ev);
    if (cs)
        (void)hipStreamDestroy(cs);
    if (ks)
        (void)hipStreamDestroy(ks);
    const double t1 = now_s();
    rep->copy_s = t_copied - t_start;
    rep->verify_tail_s = t_verified - t_copied;
    rep->total_s = t1 - t0;
    return rc;
}
