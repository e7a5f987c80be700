/*
 * zscrc_fill.cpp -- the commit writer for images that live in host memory
 * (include/zscrc.h, zscrc_zs_fill_commits): every commit CRC of a log image
 * computed on the GPU and written into the caller's image on the host.
 *
 * The reference writer builds each commit record on the host and
 * mfile_write()s it (src/zeroskip-file.c:253-350: crc32_end over the span,
 * the trailer words, the BE64 record).  The GPU only has to return the CRCs:
 * the image goes host -> device once, 4 bytes per commit come back, and host
 * threads patch the 32-bit CRC fields -- not the whole image back over PCIe
 * (the in-place device writer, zscrc_device_write_commits, is for images
 * that already live on the GPU).
 *
 * Pipeline (one call, the current device; spans sorted and disjoint):
 *   * the commits are cut into chunks of about `chunk` bytes of image
 *     (env ZSCRC_FILL_CHUNK, default 64 MiB), found by binary search on the
 *     span ends; a commit whose extent alone exceeds a chunk goes to the long
 *     list (below);
 *   * host threads take tasks in order: the chunk's span descriptors as
 *     32-bit (offset in chunk, length) pairs into pinned memory, and -- for a
 *     pageable image -- the copy of the chunk into one of four pinned staging
 *     slots (a pinned image is copied straight from the caller's memory);
 *   * the calling thread issues, per chunk, on three streams: the H2D copy of
 *     the chunk and its descriptors; the descriptor widening + commit kernel
 *     in CRC-array mode (zscrc_device_commit_crcs_bounded: one coalesced
 *     4-byte result per commit, nothing stored into the device copy); the D2H
 *     copy of the CRCs.  Device buffers rotate over three chunks, so chunk k's
 *     D2H, chunk k+1's kernel and chunk k+2's H2D overlap;
 *   * host threads patch chunk k's CRC fields (BE32 at +4 of a short commit
 *     record, +20 of a long one) once its D2H has landed, while later chunks
 *     are on the wire;
 *   * long commits: crc32c of the span streamed through the GPU in chunks
 *     (zscrc_stream_*), the trailer words and the patch on the host.
 * The commit record's header words (type, and the lengths) must already be in
 * the image, as for zscrc_device_write_commits; a span with no commit record
 * after it inside the image is counted and left alone.
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

extern "C" int zs_launch_widen_desc(const uint32_t *pairs, uint64_t *off, uint64_t *len, uint64_t n,
                                    hipStream_t stream);

namespace {

constexpr int NSLOT = 4;            /* pinned staging slots (pageable images)   */
constexpr int RING = 3;             /* device buffers: H2D / kernel / D2H overlap */
constexpr uint64_t SUB = 4ull << 20; /* bytes per staging copy task            */
constexpr uint64_t CHUNK_DEFAULT = 64ull << 20;
constexpr uint64_t MAX_SHORT = 16777215ull; /* zeroskip-priv.h:171 */
enum { T_COMMIT = 4, T_FINAL = 16, T_LONG_COMMIT = 36, T_LONG_FINAL = 48 };

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

/* Bytes of the commit record at `at` (8 short, 24 long), 0 = none inside the
 * image. */
inline uint64_t rec_len(const uint8_t *img, uint64_t size, uint64_t at)
{
    if (at > size || size - at < 8)
        return 0;
    const unsigned t = img[at];
    if (t == T_COMMIT || t == T_FINAL)
        return 8;
    if ((t == T_LONG_COMMIT || t == T_LONG_FINAL) && size - at >= 24)
        return 24;
    return 0;
}

/* Cached per device: staging slots, descriptor and CRC arrays (pinned and
 * device), the device image ring. */
struct Cache {
    std::mutex mu;
    uint64_t slot_bytes = 0;
    uint8_t *slot[NSLOT] = {};
    uint64_t ring_bytes = 0;
    uint8_t *dring[RING] = {};
    uint64_t ring_commits = 0;
    uint32_t *dpairs[RING] = {};
    uint64_t *doff[RING] = {};
    uint64_t *dlen[RING] = {};
    uint32_t *dcrc[RING] = {};
    uint64_t host_commits = 0;
    uint32_t *hpairs = nullptr; /* 2 x n */
    uint32_t *hcrc = nullptr;   /* n */
    /* copy / kernel / copy-back streams and per-chunk events, kept across
     * calls: creating and destroying them per call cost milliseconds */
    hipStream_t cs = nullptr, ks = nullptr, os = nullptr;
    std::vector<hipEvent_t> h2d, kern, d2h;
};

int ensure_sync(Cache &c, size_t nk)
{
    if (!c.cs && (hipStreamCreateWithFlags(&c.cs, hipStreamNonBlocking) != hipSuccess ||
                  hipStreamCreateWithFlags(&c.ks, hipStreamNonBlocking) != hipSuccess ||
                  hipStreamCreateWithFlags(&c.os, hipStreamNonBlocking) != hipSuccess)) {
        for (hipStream_t *s : {&c.cs, &c.ks, &c.os}) {
            if (*s)
                (void)hipStreamDestroy(*s);
            *s = nullptr;
        }
        return ZSCRC_EHIP;
    }
    while (c.h2d.size() < nk) {
        hipEvent_t a = nullptr, b = nullptr, d = nullptr;
        if (hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&d, hipEventDisableTiming) != hipSuccess) {
            for (hipEvent_t x : {a, b, d})
                if (x)
                    (void)hipEventDestroy(x);
            return ZSCRC_EHIP;
        }
        c.h2d.push_back(a);
        c.kern.push_back(b);
        c.d2h.push_back(d);
    }
    return ZSCRC_OK;
}
constexpr int MAX_DEV = 64;
Cache g_cache[MAX_DEV];

int ensure(Cache &c, bool staged, uint64_t chunk_bytes, uint64_t chunk_commits, uint64_t n)
{
    if (staged && c.slot_bytes < chunk_bytes) {
        for (auto &s : c.slot) {
            if (s)
                (void)hipHostFree(s);
            s = nullptr;
        }
        c.slot_bytes = 0;
        for (auto &s : c.slot)
            if (hipHostMalloc(reinterpret_cast<void **>(&s), chunk_bytes, hipHostMallocDefault) != hipSuccess)
                return ZSCRC_ENOMEM;
        c.slot_bytes = chunk_bytes;
    }
    if (c.ring_bytes < chunk_bytes + 256) {
        for (auto &b : c.dring) {
            if (b)
                (void)hipFree(b);
            b = nullptr;
        }
        c.ring_bytes = 0;
        for (auto &b : c.dring)
            if (hipMalloc(&b, chunk_bytes + 256) != hipSuccess)
                return ZSCRC_ENOMEM;
        c.ring_bytes = chunk_bytes + 256;
    }
    if (c.ring_commits < chunk_commits) {
        for (int r = 0; r < RING; ++r) {
            if (c.dpairs[r])
                (void)hipFree(c.dpairs[r]);
            c.dpairs[r] = nullptr;
        }
        c.ring_commits = 0;
        const uint64_t m = chunk_commits + chunk_commits / 4 + 64;
        for (int r = 0; r < RING; ++r) {
            /* pairs (8 B) + off (8) + len (8) + crc (4) per commit */
            uint8_t *p = nullptr;
            if (hipMalloc(&p, 28 * m + 64) != hipSuccess)
                return ZSCRC_ENOMEM;
            c.dpairs[r] = reinterpret_cast<uint32_t *>(p);
            c.doff[r] = reinterpret_cast<uint64_t *>(p + 8 * m);
            c.dlen[r] = c.doff[r] + m;
            c.dcrc[r] = reinterpret_cast<uint32_t *>(c.dlen[r] + m);
        }
        c.ring_commits = m;
    }
    if (c.host_commits < n) {
        if (c.hpairs)
            (void)hipHostFree(c.hpairs);
        if (c.hcrc)
            (void)hipHostFree(c.hcrc);
        c.hpairs = nullptr;
        c.hcrc = nullptr;
        c.host_commits = 0;
        const uint64_t m = n + n / 4 + 1024;
        if (hipHostMalloc(reinterpret_cast<void **>(&c.hpairs), 8 * m, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&c.hcrc), 4 * m, hipHostMallocDefault) != hipSuccess)
            return ZSCRC_ENOMEM;
        c.host_commits = m;
    }
    return ZSCRC_OK;
}

struct Chunk {
    uint64_t i0, i1;   /* commits [i0, i1) */
    uint64_t lo, hi;   /* image bytes [lo, hi), lo 4-aligned */
};

bool is_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

} /* namespace */

extern "C" int zscrc_zs_fill_commits(void *image, uint64_t size, const uint64_t *span_off, const uint64_t *span_len,
                                     size_t n, uint64_t max_len, int threads, zscrc_fill_report *rep)
{
    if (!rep || (n && (!image || !span_off || !span_len)))
        return ZSCRC_EINVAL;
    memset(rep, 0, sizeof *rep);
    const double t0 = now_s();
    uint8_t *img = static_cast<uint8_t *>(image);
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
    threads = std::max(2, threads);
    rep->threads = threads;
    if (n == 0) {
        rep->total_s = now_s() - t0;
        return ZSCRC_OK;
    }
    uint64_t chunk = CHUNK_DEFAULT;
    if (const char *e = getenv("ZSCRC_FILL_CHUNK"))
        chunk = std::max<uint64_t>(64u << 10, strtoull(e, nullptr, 0));
    chunk = std::min<uint64_t>((chunk + 4095) & ~4095ull, 1ull << 31); /* 32-bit offsets within a chunk */

    /* the plan: chunks by binary search over the span ends (sorted and
     * disjoint spans have non-decreasing ends); longer commits apart */
    auto span_end = [&](uint64_t i) { return span_off[i] + span_len[i]; };
    std::vector<Chunk> chunks;
    std::vector<uint64_t> longs;
    uint64_t max_commits = 0, max_bytes = 0;
    for (uint64_t i0 = 0; i0 < n;) {
        if (span_off[i0] > size || span_len[i0] > size - span_off[i0])
            return ZSCRC_EINVAL;
        const uint64_t lo = span_off[i0] & ~3ull;
        if (span_end(i0) + 24 - lo > chunk) {
            longs.push_back(i0++);
            continue;
        }
        /* first i > i0 whose span (+ a long record) would leave the chunk */
        uint64_t a = i0 + 1, b = n;
        while (a < b) {
            const uint64_t m = a + (b - a) / 2;
            if (span_end(m) + 24 - lo <= chunk)
                a = m + 1;
            else
                b = m;
        }
        const uint64_t i1 = a;
        const uint64_t last = span_end(i1 - 1);
        if (span_off[i1 - 1] > size || span_len[i1 - 1] > size - span_off[i1 - 1] || last < lo)
            return ZSCRC_EINVAL; /* unsorted: the plan's search met a span behind the chunk */
        const uint64_t hi = std::min(size, last + std::max<uint64_t>(rec_len(img, size, last), 8));
        chunks.push_back({i0, i1, lo, hi});
        max_commits = std::max(max_commits, i1 - i0);
        max_bytes = std::max(max_bytes, hi - lo);
        i0 = i1;
    }
    const bool staged = !is_pinned(image);
    rep->staged = staged ? 1 : 0;
    rep->chunks = chunks.size();

    Cache &c = g_cache[dev];
    std::lock_guard<std::mutex> lk(c.mu);
    int rc = chunks.empty() ? ZSCRC_OK : ensure(c, staged, (max_bytes + 4095) & ~4095ull, max_commits, n);
    if (rc)
        return rc;
    max_len = std::min<uint64_t>(max_len, MAX_SHORT);

    const size_t nk = chunks.size();
    if (!rc && nk)
        rc = ensure_sync(c, nk);
    hipStream_t cs = c.cs, ks = c.ks, os = c.os;
    const std::vector<hipEvent_t> &h2d = c.h2d, &kern = c.kern, &d2h = c.d2h;

    /* tasks, in order: chunk k's descriptors and staging copies; chunk k's
     * patches after chunk k + LAG's copies (its D2H is queued by then) */
    struct Task {
        int kind;      /* 0 descriptors, 1 staging copy, 2 patch, 3 validate */
        uint64_t k;    /* chunk */
        uint64_t a, b; /* copy: bytes [a, b) of the chunk; patch: commits [a, b) */
    };
    std::vector<Task> tasks;
    /* first: every span's bounds and order, in slices over the workers; no
     * patch touches the image before all slices passed, so invalid input
     * fails with the image unmodified (the copies and kernels only read it) */
    const uint64_t nval = std::min<uint64_t>((uint64_t)threads, n);
    for (uint64_t v = 0; v < nval; ++v)
        tasks.push_back({3, 0, n * v / nval, n * (v + 1) / nval});
    std::vector<std::atomic<int>> ready(nk); /* tasks left before chunk k can be issued */
    constexpr uint64_t PATCH_SUB = 1u << 16;
    const uint64_t LAG = NSLOT;
    auto add_patches = [&](uint64_t k) {
        for (uint64_t a = chunks[k].i0; a < chunks[k].i1; a += PATCH_SUB)
            tasks.push_back({2, k, a, std::min(chunks[k].i1, a + PATCH_SUB)});
    };
    for (uint64_t k = 0; k < nk; ++k) {
        const Chunk &ch = chunks[k];
        int cnt = 1;
        tasks.push_back({0, k, 0, 0});
        if (staged)
            for (uint64_t a = 0; a < ch.hi - ch.lo; a += SUB, ++cnt)
                tasks.push_back({1, k, a, std::min(ch.hi - ch.lo, a + SUB)});
        ready[k] = cnt;
        if (k >= LAG)
            add_patches(k - LAG);
    }
    for (uint64_t k = nk > LAG ? nk - LAG : 0; k < nk; ++k)
        add_patches(k);

    std::vector<char> chunk_ok(nk, 0); /* its spans sorted and disjoint: written by its descriptor task */
    std::atomic<uint64_t> next{0};
    std::atomic<int64_t> issued{0};  /* chunks whose copies / kernel / D2H are queued */
    std::atomic<int> stop{0}, bad_order{0};
    std::atomic<uint64_t> validated{0}; /* validation slices done */
    std::atomic<uint64_t> patched{0}, norec{0};
    auto wait_issued = [&](int64_t k) -> bool { /* chunk k queued (its events recorded) */
        while (issued.load(std::memory_order_acquire) <= k) {
            if (stop.load(std::memory_order_relaxed))
                return false;
            std::this_thread::yield();
        }
        return true;
    };
    auto worker = [&]() {
        for (;;) {
            const uint64_t t = next.fetch_add(1, std::memory_order_relaxed);
            if (t >= tasks.size())
                return;
            const Task tk = tasks[t];
            if (tk.kind == 3) {
                bool ok = true;
                for (uint64_t i = tk.a; ok && i < tk.b; ++i)
                    ok = span_off[i] <= size && span_len[i] <= size - span_off[i] &&
                         (i == 0 || span_off[i] >= span_end(i - 1));
                if (!ok)
                    bad_order = 1;
                validated.fetch_add(1, std::memory_order_release);
                continue;
            }
            const Chunk &ch = chunks[tk.k];
            if (tk.kind == 0) {
                uint32_t *p = c.hpairs + 2 * ch.i0;
                uint64_t prev = ch.i0 ? span_end(ch.i0 - 1) : 0;
                bool ok = true;
                for (uint64_t i = ch.i0; i < ch.i1; ++i) {
                    ok = ok && span_off[i] >= prev && span_len[i] <= size - span_off[i];
                    prev = span_end(i);
                    p[0] = (uint32_t)(span_off[i] - ch.lo);
                    p[1] = (uint32_t)span_len[i];
                    p += 2;
                }
                chunk_ok[tk.k] = ok; /* published by the release below, read after `issued` */
                if (!ok)
                    bad_order = 1;
            } else if (tk.kind == 1) {
                /* slot k % NSLOT is free once chunk k - NSLOT's H2D is done */
                const int64_t k = (int64_t)tk.k;
                if (k >= NSLOT) {
                    if (!wait_issued(k - NSLOT))
                        return;
                    (void)hipEventSynchronize(h2d[k - NSLOT]);
                }
                memcpy(c.slot[k % NSLOT] + tk.a, img + ch.lo + tk.a, tk.b - tk.a);
            } else {
                if (!wait_issued((int64_t)tk.k))
                    return;
                (void)hipEventSynchronize(d2h[tk.k]);
                while (validated.load(std::memory_order_acquire) < nval) {
                    if (stop.load(std::memory_order_relaxed))
                        return;
                    std::this_thread::yield();
                }
                if (!chunk_ok[tk.k] || bad_order.load(std::memory_order_relaxed))
                    continue; /* unsorted / overlapping spans: nothing written, the call fails */
                uint64_t done = 0, none = 0;
                for (uint64_t i = tk.a; i < tk.b; ++i) {
                    const uint64_t at = span_end(i);
                    const uint64_t rl = rec_len(img, size, at);
                    if (!rl) {
                        ++none;
                        continue;
                    }
                    const uint32_t v = __builtin_bswap32(c.hcrc[i]);
                    memcpy(img + at + (rl == 8 ? 4 : 20), &v, 4);
                    ++done;
                }
                patched += done;
                norec += none;
                continue;
            }
            ready[tk.k].fetch_sub(1, std::memory_order_acq_rel);
        }
    };
    std::vector<std::thread> pool;
    if (!rc)
        for (int i = 0; i < threads; ++i)
            pool.emplace_back(worker);

    double t_h2d = t0;
    auto wait_ready = [&](size_t k) {
        while (ready[k].load(std::memory_order_acquire) > 0)
            std::this_thread::yield();
    };
    for (size_t k = 0; !rc && k < nk; ++k) {
        const Chunk &ch = chunks[k];
        const int r = (int)(k % RING);
        const uint64_t m = ch.i1 - ch.i0;
        const uint64_t shift = ch.lo & 255; /* the image's alignment within 256 B, kept on the device */
        uint8_t *dimg = c.dring[r] + shift;
        /* ring buffer r is free once chunk k - RING's kernel and D2H are done */
        if (k >= (size_t)RING && (hipStreamWaitEvent(cs, kern[k - RING], 0) != hipSuccess ||
                                  hipStreamWaitEvent(cs, d2h[k - RING], 0) != hipSuccess))
            rc = ZSCRC_EHIP;
        /* a pinned image goes on the wire before its descriptors are built;
         * a staged one once its slot is filled (the slot copies are in ready) */
        if (staged)
            wait_ready(k);
        const void *src = staged ? static_cast<const void *>(c.slot[k % NSLOT]) : img + ch.lo;
        if (!rc && hipMemcpyAsync(dimg, src, ch.hi - ch.lo, hipMemcpyHostToDevice, cs) != hipSuccess)
            rc = ZSCRC_EHIP;
        if (k == 0)
            rep->setup_s = now_s() - t0;
        if (!staged)
            wait_ready(k);
        if (!rc && (hipMemcpyAsync(c.dpairs[r], c.hpairs + 2 * ch.i0, 8 * m, hipMemcpyHostToDevice, cs) !=
                        hipSuccess ||
                    hipEventRecord(h2d[k], cs) != hipSuccess))
            rc = ZSCRC_EHIP;
        if (!rc && hipStreamWaitEvent(ks, h2d[k], 0) != hipSuccess)
            rc = ZSCRC_EHIP;
        if (!rc && zs_launch_widen_desc(c.dpairs[r], c.doff[r], c.dlen[r], m, ks))
            rc = ZSCRC_EHIP;
        if (!rc)
            rc = zscrc_device_commit_crcs_bounded(dimg, ch.hi - ch.lo, c.doff[r], c.dlen[r], m, max_len, c.dcrc[r],
                                                  nullptr, ks);
        if (!rc && (hipEventRecord(kern[k], ks) != hipSuccess || hipStreamWaitEvent(os, kern[k], 0) != hipSuccess ||
                    hipMemcpyAsync(c.hcrc + ch.i0, c.dcrc[r], 4 * m, hipMemcpyDeviceToHost, os) != hipSuccess ||
                    hipEventRecord(d2h[k], os) != hipSuccess))
            rc = ZSCRC_EHIP;
        if (!rc)
            issued.store((int64_t)k + 1, std::memory_order_release);
        rep->bytes += ch.hi - ch.lo;
        rep->desc_bytes += 8 * m;
    }
    if (!rc && nk && hipEventSynchronize(h2d[nk - 1]) != hipSuccess)
        rc = ZSCRC_EHIP;
    t_h2d = now_s();
    if (rc)
        stop = 1;
    for (auto &t : pool)
        t.join();
    /* every queued copy and kernel drained before the call returns (an error
     * part-way leaves work queued on the cached streams otherwise) */
    if (cs && ks && os &&
        (hipStreamSynchronize(cs) != hipSuccess || hipStreamSynchronize(ks) != hipSuccess ||
         hipStreamSynchronize(os) != hipSuccess) && !rc)
        rc = ZSCRC_EHIP;
    if (!rc && bad_order)
        rc = ZSCRC_EINVAL; /* unsorted or overlapping spans: the image was not patched */

    /* long commits: the span streamed through the GPU, trailer on the host
     * (zeroskip-file.c:266-302 / :303-328) */
    for (size_t j = 0; !rc && j < longs.size(); ++j) {
        const uint64_t i = longs[j];
        const uint64_t at = span_end(i);
        const uint64_t rl = rec_len(img, size, at);
        if (!rl) {
            ++norec;
            continue;
        }
        zscrc_stream *s = nullptr;
        uint32_t span_crc = 0;
        rc = zscrc_stream_open(&s, 0, chunk, ZSCRC_STREAM_NOCOPY);
        if (!rc)
            rc = zscrc_stream_update(s, img + span_off[i], span_len[i]);
        if (s) {
            const int r2 = zscrc_stream_final(s, &span_crc);
            rc = rc ? rc : r2;
        }
        if (rc)
            break;
        uint32_t crc;
        if (rl == 8) {
            const uint64_t w = be64(img + at) & 0xFFFFFFFF00000000ull;
            crc = crc32c_hw(span_crc, &w, 8);
        } else {
            const uint64_t w[3] = {be64(img + at), be64(img + at + 8), be64(img + at + 16) & 0xFF00000000000000ull};
            crc = crc32c_hw(span_crc, w, 24);
        }
        const uint32_t v = __builtin_bswap32(crc);
        memcpy(img + at + (rl == 8 ? 4 : 20), &v, 4);
        ++patched;
        rep->bytes += span_len[i] + rl;
    }
    rep->commits = patched.load();
    rep->no_record = norec.load();
    rep->long_commits = longs.size();
    rep->h2d_s = t_h2d - t0;
    rep->total_s = now_s() - t0;
    return rc;
}

/* zscrc_release_cache(): every device's staging slots, device ring, pinned
 * per-commit arrays, streams and events (each cache under its own lock). */
extern "C" void zs_fill_release_cache(void)
{
    int cur = -1;
    (void)hipGetDevice(&cur);
    for (int d = 0; d < MAX_DEV; ++d) {
        Cache &c = g_cache[d];
        std::lock_guard<std::mutex> lk(c.mu);
        if (!c.cs && !c.slot_bytes && !c.ring_bytes && !c.ring_commits && !c.host_commits)
            continue;
        (void)hipSetDevice(d);
        for (hipStream_t *st : {&c.cs, &c.ks, &c.os})
            if (*st) {
                (void)hipStreamSynchronize(*st);
                (void)hipStreamDestroy(*st);
                *st = nullptr;
            }
        for (auto *v : {&c.h2d, &c.kern, &c.d2h}) {
            for (hipEvent_t e : *v)
                (void)hipEventDestroy(e);
            v->clear();
        }
        for (auto &p : c.slot) {
            if (p)
                (void)hipHostFree(p);
            p = nullptr;
        }
        for (auto &p : c.dring) {
            if (p)
                (void)hipFree(p);
            p = nullptr;
        }
        for (int r = 0; r < RING; ++r) {
            if (c.dpairs[r])
                (void)hipFree(c.dpairs[r]);
            c.dpairs[r] = nullptr;
            c.doff[r] = c.dlen[r] = nullptr;
            c.dcrc[r] = nullptr;
        }
        if (c.hpairs)
            (void)hipHostFree(c.hpairs);
        if (c.hcrc)
            (void)hipHostFree(c.hcrc);
        c.hpairs = c.hcrc = nullptr;
        c.slot_bytes = c.ring_bytes = c.ring_commits = c.host_commits = 0;
    }
    if (cur >= 0)
        (void)hipSetDevice(cur);
}
