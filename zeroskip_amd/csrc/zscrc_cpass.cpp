/*
 * zscrc_cpass.cpp -- the device pass of `consistent` (zeroskip_amd/
 * consistent.py run()) as one C call over a prepared, device-resident DB
 * share: the commits of active / finalised files as ONE verdict batch
 * (zscrc_device_verify_commits_verdict: commit_kernel, no per-commit output),
 * the raw spans (records-region pieces, pointer sections) checksummed
 * (zscrc_device_spans), one post kernel (cpass_post_kernel: the finalise
 * quirk told from bad commits, the whole spans' commit trailers checked --
 * src/zeroskip-file.c:266-302, src/zeroskip-active.c:122, src/mfile.c:534-546)
 * and ONE device->host copy of a small block.  The reference's
 * zsdb_consistent (src/zeroskip.c:1399-1407) is a stub; this is the
 * multi-rank driver's inner loop, repeated per pass without host work
 * beyond reading the block.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/zscrc.h"
#include "zscrc_internal.h"

extern "C" {
const uint32_t *zscrc_internal_gtab(void);
int zs_launch_cpass_post(const zs::CPassArgs *a, const zs::SpanFolds *fs, uint32_t nfold, const uint32_t *gtab,
                         hipStream_t stream, hipEvent_t done);
int zscrc_internal_spans_private(const void *const *d_bufs, const uint64_t *lens, uint32_t *d_out, size_t k,
                                 unsigned flags, uint32_t *part, uint64_t part_words, void *stream,
                                 zs::SpanFolds *defer_folds);
int zscrc_internal_verdict_prezeroed(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                     const uint64_t *d_span_len, size_t n, uint64_t max_len, uint64_t *d_nbad,
                                     uint64_t *d_bad, size_t cap, void *stream);
uint32_t zs_gf2_xpow8n(uint64_t n);
uint32_t zs_gf2_mul(uint32_t a, uint32_t b);
}

namespace {

constexpr uint64_t LIST_CAP = 4096; /* bad-list entries copied back per pass */

} /* namespace */

struct zscrc_cpass {
    zscrc_cpass_spec spec;
    int dev = 0; /* the device current at create: every buffer lives there */
    std::vector<uint64_t> span_off, span_len;
    std::vector<int64_t> span_commit;
    /* device block: [0] nbad, [1] nstale, [2] the post kernel's workgroup
     * ticket, then span_raw[64] (u32), span_status[64] (i32),
     * flags[LIST_CAP] (u32), bad[LIST_CAP] (u64) (written by the post
     * kernel); a host slot has the same layout ([2] unused) */
    /* two device blocks, used by consecutive passes in turn: a pass's post
     * kernel zeroes the other block's counters for the next pass, so no
     * memset launch precedes a pass (two fill kernels of ~4.5 us and their
     * gaps per pass until then) */
    uint8_t *dblk = nullptr;   /* 2 x BLK */
    int blk_next = 0;
    uint8_t *hblk = nullptr;   /* NSLOT host blocks (zscrc_cpass_submit / _collect) */
    hipEvent_t done[2] = {};   /* each slot's completion */
    /* passes in stream order (the blocks' counters are zeroed by the
     * previous pass): a pass enqueued on another stream than the previous
     * one first waits for everything already on that stream (`order`,
     * recorded there only then -- nothing extra per pass on one stream) */
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    hipEvent_t order = nullptr;
    hipEvent_t wait[2] = {};   /* what collect waits on: done[], or the caller's end event */
    bool pending[2] = {};
    /* the digest row (zscrc_cpass_set_row / _submit_row) */
    bool have_row = false;
    zs::CPassRowArgs row = {};
    int64_t *dpiece = nullptr;
    uint64_t *dbad_full = nullptr; /* the verdict's list (cap entries) */
    uint64_t cap = 0;
    int64_t *dspan_commit = nullptr;
    uint32_t *dspan_init = nullptr;
    /* the multi-span launches' segment registers: the handle's own, so a
     * pass needs no ordering event on the device's shared scratch (its
     * record put ~6 us between the folds and the post kernel) */
    uint32_t *dpart = nullptr;
    uint64_t part_words = 0;
    /* one stream: the raw spans on a second stream beside the verdict batch
     * measured slower (config 5: 1.659 vs 1.542 ms per pass,
     * profiles/r03/cpass_streams.jsonl) */
};

namespace {

constexpr size_t NCOUNT = 3, OFF_RAW = 32, OFF_ST = OFF_RAW + 4 * zs::CPASS_SPANS, OFF_FLAGS = OFF_ST + 4 * zs::CPASS_SPANS,
                 OFF_BAD = OFF_FLAGS + 4 * LIST_CAP, BLK = OFF_BAD + 8 * LIST_CAP;

constexpr int NSLOT = 2;

void cpass_free(zscrc_cpass *p)
{
    /* a submitted pass not yet collected may still be writing its host slot
     * and the device blocks; its completion may be the caller's event, which
     * the caller may have recorded again or destroyed: wait for the device */
    if (p->pending[0] || p->pending[1])
        (void)hipDeviceSynchronize();
    for (hipEvent_t &e : p->done)
        if (e) {
            (void)hipEventSynchronize(e);
            (void)hipEventDestroy(e);
        }
    if (p->order)
        (void)hipEventDestroy(p->order);
    if (p->dblk)
        (void)hipFree(p->dblk);
    if (p->hblk)
        (void)hipHostFree(p->hblk);
    if (p->dbad_full)
        (void)hipFree(p->dbad_full);
    if (p->dspan_commit)
        (void)hipFree(p->dspan_commit);
    if (p->dpiece)
        (void)hipFree(p->dpiece);
    if (p->dpart)
        (void)hipFree(p->dpart);
    delete p;
}

} /* namespace */

extern "C" int zscrc_cpass_create(zscrc_cpass **out, const zscrc_cpass_spec *spec)
{
    if (!out || !spec || (spec->n && (!spec->d_image || !spec->d_off || !spec->d_len || !spec->d_file)) ||
        spec->nspans > ZSCRC_CPASS_SPANS || (spec->nspans && (!spec->span_off || !spec->span_len || !spec->span_commit)))
        return ZSCRC_EINVAL;
    *out = nullptr;
    if (!zscrc_internal_gtab())
        return ZSCRC_ENODEV;
    zscrc_cpass *p = new zscrc_cpass;
    p->spec = *spec;
    if (hipGetDevice(&p->dev) != hipSuccess) {
        delete p;
        return ZSCRC_ENODEV;
    }
    p->span_off.assign(spec->span_off, spec->span_off + spec->nspans);
    p->span_len.assign(spec->span_len, spec->span_len + spec->nspans);
    p->span_commit.assign(spec->span_commit, spec->span_commit + spec->nspans);
    p->spec.span_off = p->span_off.data();
    p->spec.span_len = p->span_len.data();
    p->spec.span_commit = p->span_commit.data();
    for (size_t k = 0; k < spec->nspans; ++k)
        if (p->span_len[k] == 0 || p->span_off[k] + p->span_len[k] > spec->image_size) {
            cpass_free(p);
            return ZSCRC_EINVAL;
        }
    /* the verdict keeps up to `cap` indices; the block copies LIST_CAP */
    p->cap = std::max<uint64_t>(LIST_CAP, std::min<uint64_t>(spec->n, 1u << 20));
    std::vector<uint32_t> init(spec->nspans);
    for (size_t k = 0; k < spec->nspans; ++k)
        init[k] = zs_gf2_mul(0xFFFFFFFFu, zs_gf2_xpow8n(p->span_len[k]));
    hipError_t e = hipMalloc(&p->dblk, 2 * BLK);
    if (e == hipSuccess)
        e = hipMemset(p->dblk, 0, 2 * BLK); /* both blocks' counters start at 0 */
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void **>(&p->hblk), NSLOT * BLK, hipHostMallocDefault);
    for (int k = 0; k < NSLOT && e == hipSuccess; ++k)
        e = hipEventCreateWithFlags(&p->done[k], hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&p->order, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipMalloc(&p->dbad_full, 8 * p->cap);
    if (e == hipSuccess)
        e = hipMalloc(&p->dspan_commit, (8 + 4) * zs::CPASS_SPANS);
    /* segment registers of the multi-span launches: any segment size is at
     * least 1 KiB (SEG_MIN), so this bounds every launch shape the tuning
     * can pick */
    for (size_t k = 0; k < spec->nspans; ++k)
        p->part_words += (p->span_len[k] + 1023) / 1024;
    if (e == hipSuccess && p->part_words)
        e = hipMalloc(&p->dpart, 4 * p->part_words);
    if (e != hipSuccess) {
        cpass_free(p);
        return ZSCRC_ENOMEM;
    }
    p->dspan_init = reinterpret_cast<uint32_t *>(p->dspan_commit + zs::CPASS_SPANS);
    if (spec->nspans &&
        (hipMemcpy(p->dspan_commit, p->span_commit.data(), 8 * spec->nspans, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(p->dspan_init, init.data(), 4 * spec->nspans, hipMemcpyHostToDevice) != hipSuccess)) {
        cpass_free(p);
        return ZSCRC_EHIP;
    }
    /* max_len selects which length classes the verdict launches (a range
     * that holds: the classes above it get no launch), so it must bound every
     * span: the lengths are read back once here and the bound used is their
     * true maximum -- a caller's under-stated max_len cannot leave long
     * commits unchecked (an over-stated one would only cost time) */
    if (spec->n) {
        std::vector<uint64_t> lens(spec->n);
        if (hipMemcpy(lens.data(), spec->d_len, 8 * spec->n, hipMemcpyDeviceToHost) != hipSuccess) {
            cpass_free(p);
            return ZSCRC_EHIP;
        }
        p->spec.max_len = *std::max_element(lens.begin(), lens.end());
    }
    *out = p;
    return ZSCRC_OK;
}

namespace {

int cpass_submit(zscrc_cpass *p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, int slot);
int cpass_collect(zscrc_cpass *p, int slot, zscrc_cpass_result *res);

/* the pass runs on the device it was created on (its buffers and the
 * operator table the kernels read are that device's), whatever device the
 * caller has current; the caller's device is restored */
struct OnDevice {
    int cur = -1;
    int dev;
    bool ok;
    explicit OnDevice(int d) : dev(d)
    {
        ok = hipGetDevice(&cur) == hipSuccess && (cur == dev || hipSetDevice(dev) == hipSuccess);
    }
    ~OnDevice()
    {
        if (ok && cur != dev)
            (void)hipSetDevice(cur);
    }
};

} /* namespace */

extern "C" int zscrc_cpass_run(zscrc_cpass *p, void *stream, zscrc_cpass_result *res)
{
    return zscrc_cpass_run_timed(p, stream, nullptr, nullptr, res);
}

extern "C" int zscrc_cpass_run_timed(zscrc_cpass *p, void *stream, void *start_event, void *end_event,
                                     zscrc_cpass_result *res)
{
    if (!p || !res)
        return ZSCRC_EINVAL;
    OnDevice od(p->dev);
    if (!od.ok)
        return ZSCRC_EHIP;
    /* a synchronous pass takes a free slot; one still holding an uncollected
     * pass is collected first (its result dropped) */
    const int slot = p->pending[0] && !p->pending[1] ? 1 : 0;
    zscrc_cpass_result tmp;
    if (p->pending[slot])
        (void)cpass_collect(p, slot, &tmp);
    const int rc = cpass_submit(p, static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(start_event),
                                static_cast<hipEvent_t>(end_event), slot);
    return rc ? rc : cpass_collect(p, slot, res);
}

extern "C" int zscrc_cpass_submit(zscrc_cpass *p, void *stream, void *start_event, void *end_event, int slot)
{
    if (!p || slot < 0 || slot >= NSLOT || p->pending[slot])
        return ZSCRC_EINVAL;
    OnDevice od(p->dev);
    if (!od.ok)
        return ZSCRC_EHIP;
    return cpass_submit(p, static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(start_event),
                        static_cast<hipEvent_t>(end_event), slot);
}

extern "C" int zscrc_cpass_collect(zscrc_cpass *p, int slot, zscrc_cpass_result *res)
{
    if (!p || !res || slot < 0 || slot >= NSLOT || !p->pending[slot])
        return ZSCRC_EINVAL;
    OnDevice od(p->dev);
    if (!od.ok)
        return ZSCRC_EHIP;
    return cpass_collect(p, slot, res);
}

extern "C" int zscrc_cpass_set_row(zscrc_cpass *p, const zscrc_cpass_row_spec *rs)
{
    if (!p || !rs || (p->spec.n && !rs->d_rec) || (p->spec.nspans && (!rs->piece_fid || !rs->piece_code)) ||
        rs->pmax < p->spec.nspans || rs->listed == 0)
        return ZSCRC_EINVAL;
    OnDevice od(p->dev);
    if (!od.ok)
        return ZSCRC_EHIP;
    std::vector<int64_t> meta(3 * std::max<size_t>(p->spec.nspans, 1));
    for (size_t k = 0; k < p->spec.nspans; ++k) {
        meta[3 * k] = rs->piece_fid[k];
        meta[3 * k + 1] = rs->piece_code[k];
        meta[3 * k + 2] = (int64_t)p->span_len[k];
    }
    if (!p->dpiece && hipMalloc(&p->dpiece, 3 * 8 * zs::CPASS_SPANS) != hipSuccess)
        return ZSCRC_ENOMEM;
    if (hipMemcpy(p->dpiece, meta.data(), 8 * meta.size(), hipMemcpyHostToDevice) != hipSuccess)
        return ZSCRC_EHIP;
    zs::CPassRowArgs &a = p->row;
    memset(&a, 0, sizeof a);
    a.blk = p->dblk; /* set per pass: the block it used */
    a.off_raw = OFF_RAW;
    a.off_st = OFF_ST;
    a.off_flags = OFF_FLAGS;
    a.off_bad = OFF_BAD;
    a.list_cap = (uint32_t)LIST_CAP;
    a.commits = p->spec.n;
    a.file = p->spec.d_file;
    a.rec = rs->d_rec;
    a.piece = p->dpiece;
    a.nspans = (uint32_t)p->spec.nspans;
    a.listed = rs->listed;
    a.pmax = rs->pmax;
    for (int k = 0; k < 4; ++k)
        a.checked[k] = rs->checked[k];
    p->have_row = true;
    return ZSCRC_OK;
}

namespace {
int cpass_enqueue(zscrc_cpass *p, hipStream_t s, hipEvent_t ev0, uint8_t **blk, uint8_t *host,
                  int64_t *d_row = nullptr, hipEvent_t done = nullptr);
}

extern "C" int zscrc_cpass_submit_row(zscrc_cpass *p, void *stream, void *start_event, void *end_event,
                                      int64_t *d_row)
{
    if (!p || !d_row || !p->have_row)
        return ZSCRC_EINVAL;
    OnDevice od(p->dev);
    if (!od.ok)
        return ZSCRC_EHIP;
    hipStream_t s = static_cast<hipStream_t>(stream);
    uint8_t *blk = nullptr;
    /* the post kernel's last workgroup builds the row: no launch of its own;
     * the end event completes with the post kernel's dispatch */
    return cpass_enqueue(p, s, static_cast<hipEvent_t>(start_event), &blk, nullptr, d_row,
                         static_cast<hipEvent_t>(end_event));
}

namespace {

/* Enqueue one pass on s: the verdict batch, the raw spans, the post kernel
 * and the copy of the small block into host slot `slot`; nothing waits. */
int cpass_submit(zscrc_cpass *p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, int slot)
{
    uint8_t *blk = nullptr;
    /* the post kernel writes the listed part of the verdict, the count and
     * the span registers straight into the pinned host slot: no copy back
     * (a blit launch and ~12 us of gap per pass) */
    /* the end event completes with the post kernel's own dispatch: the
     * device's part of the pass, without the host's wait and the list
     * sorting.  The caller's end event doubles as the slot's completion;
     * otherwise the slot's own */
    p->wait[slot] = ev1 ? ev1 : p->done[slot];
    int rc = cpass_enqueue(p, s, ev0, &blk, p->hblk + slot * BLK, nullptr, p->wait[slot]);
    if (!rc)
        p->pending[slot] = true;
    return rc;
}

/* The pass's kernels: verdict batch, raw spans, post kernel, into the next
 * of the two device blocks (*blk).  Passes must follow one another in
 * stream order (one stream, or the caller's own ordering): the blocks'
 * counters are zeroed by the previous pass. */
int cpass_enqueue(zscrc_cpass *p, hipStream_t s, hipEvent_t ev0, uint8_t **blk, uint8_t *host, int64_t *d_row,
                  hipEvent_t done)
{
    if (p->have_last && s != p->last_stream &&
        (hipEventRecord(p->order, p->last_stream) != hipSuccess || hipStreamWaitEvent(s, p->order, 0) != hipSuccess))
        return ZSCRC_EHIP;
    p->last_stream = s;
    p->have_last = true;
    if (ev0 && hipEventRecord(ev0, s) != hipSuccess)
        return ZSCRC_EHIP;
    const zscrc_cpass_spec &sp = p->spec;
    uint8_t *b = p->dblk + p->blk_next * BLK, *other = p->dblk + (p->blk_next ^ 1) * BLK;
    p->blk_next ^= 1;
    *blk = b;
    uint64_t *d_nbad = reinterpret_cast<uint64_t *>(b);
    uint32_t *d_raw = reinterpret_cast<uint32_t *>(b + OFF_RAW);
    int rc = zscrc_internal_verdict_prezeroed(sp.d_image, sp.image_size, sp.d_off, sp.d_len, sp.n, sp.max_len,
                                              d_nbad, p->dbad_full, p->cap, s);
    /* raw spans: up to 8 of >= 16 KiB per launch pair, else one by one.
     * When they all make one multi-span launch (config 5: two records
     * regions, two pointer sections) and no row is built, its folds run in
     * the post kernel (nfold): a launch fewer per pass. */
    const uint8_t *img = static_cast<const uint8_t *>(sp.d_image);
    zs::SpanFolds folds;
    uint32_t nfold = 0;
    bool defer = !d_row && sp.nspans >= 2 && sp.nspans <= (size_t)zs::SPANS_MAX;
    for (size_t i = 0; defer && i < sp.nspans; ++i)
        defer = p->span_len[i] >= (16u << 10);
    for (size_t i = 0; !rc && i < sp.nspans;) {
        const void *bufs[8];
        uint64_t lens[8];
        size_t k = 0;
        while (k < 8 && i + k < sp.nspans && p->span_len[i + k] >= (16u << 10)) {
            bufs[k] = img + p->span_off[i + k];
            lens[k] = p->span_len[i + k];
            ++k;
        }
        if (k >= 2) {
            zs::SpanFolds *df = defer && k == sp.nspans ? &folds : nullptr;
            rc = zscrc_internal_spans_private(bufs, lens, d_raw + i, k, ZSCRC_RAW, p->dpart, p->part_words, s, df);
            if (rc == ZSCRC_EINVAL) /* a tuning without the one-launch shape: the shared path */
                rc = zscrc_device_spans(bufs, lens, nullptr, d_raw + i, k, ZSCRC_RAW, s);
            else if (!rc && df)
                nfold = (uint32_t)k;
            i += k;
        } else {
            rc = zscrc_device_span(img + p->span_off[i], p->span_len[i], 0, d_raw + i, nullptr, ZSCRC_RAW, s);
            ++i;
        }
    }
    if (!rc) {
        zs::CPassArgs a;
        memset(&a, 0, sizeof a);
        a.base = img;
        a.img_size = sp.image_size;
        a.off = sp.d_off;
        a.len = sp.d_len;
        a.file = sp.d_file;
        a.nbad = reinterpret_cast<const unsigned long long *>(d_nbad);
        a.bad = p->dbad_full;
        a.cap = p->cap;
        uint8_t *o = host ? host : b; /* where the listed verdict goes */
        a.flags = reinterpret_cast<uint32_t *>(o + OFF_FLAGS);
        a.bad_out = reinterpret_cast<uint64_t *>(o + OFF_BAD);
        if (host) {
            a.host_nbad = reinterpret_cast<uint64_t *>(host);
            a.host_raw = reinterpret_cast<uint32_t *>(host + OFF_RAW);
        }
        a.out_cap = LIST_CAP;
        a.nstale = reinterpret_cast<unsigned long long *>(b + 8);
        a.ticket = reinterpret_cast<unsigned long long *>(b + 16);
        a.next_counters = reinterpret_cast<unsigned long long *>(other);
        a.nspans = (uint32_t)sp.nspans;
        a.span_raw = d_raw;
        a.span_commit = p->dspan_commit;
        a.span_init = p->dspan_init;
        a.span_status = reinterpret_cast<int32_t *>(o + OFF_ST);
        if (d_row) {
            a.row = p->row;
            a.row.blk = b;
            a.row.row = d_row;
        }
        if (zs_launch_cpass_post(&a, &folds, nfold, zscrc_internal_gtab(), s, done))
            rc = ZSCRC_EHIP;
    }
    if (rc) { /* a pass cut short did not zero the next block: start both over */
        (void)hipMemsetAsync(b, 0, 8 * NCOUNT, s);
        (void)hipMemsetAsync(other, 0, 8 * NCOUNT, s);
    }
    return rc;
}

/* Wait for slot's copy back and read its block. */
int cpass_collect(zscrc_cpass *p, int slot, zscrc_cpass_result *res)
{
    p->pending[slot] = false;
    if (hipEventSynchronize(p->wait[slot]) != hipSuccess)
        return ZSCRC_EHIP;
    const zscrc_cpass_spec &sp = p->spec;
    const uint8_t *blk = p->hblk + slot * BLK;
    const uint64_t nbad = reinterpret_cast<const uint64_t *>(blk)[0];
    /* the device's stale count over every classified entry (the post
     * kernel's last workgroup), not a recount of the listed flags: the same
     * number the device row carries, whatever order the entries were listed
     * in */
    const uint64_t nstale = reinterpret_cast<const uint64_t *>(blk)[1];
    const uint32_t *flags = reinterpret_cast<const uint32_t *>(blk + OFF_FLAGS);
    const uint64_t *bad = reinterpret_cast<const uint64_t *>(blk + OFF_BAD);
    memset(res, 0, sizeof *res);
    const uint64_t nl = std::min<uint64_t>(nbad, LIST_CAP);
    res->complete = nbad <= LIST_CAP;
    std::vector<uint64_t> b, st, und;
    for (uint64_t k = 0; k < nl; ++k)
        (flags[k] == 1 ? st : flags[k] == 2 ? und : b).push_back(bad[k]);
    std::sort(b.begin(), b.end());
    std::sort(st.begin(), st.end());
    std::sort(und.begin(), und.end());
    res->n_stale = nstale;
    res->n_bad = nbad - nstale; /* undecided ones included: the host may move them */
    res->n_undecided = und.size();
    res->n_listed_bad = std::min<uint64_t>(b.size(), ZSCRC_CPASS_LIST);
    res->n_listed_stale = std::min<uint64_t>(st.size(), ZSCRC_CPASS_LIST);
    std::copy(b.begin(), b.begin() + res->n_listed_bad, res->bad);
    std::copy(st.begin(), st.begin() + res->n_listed_stale, res->stale);
    for (size_t k = 0; k < und.size() && k < ZSCRC_CPASS_SPANS; ++k)
        res->undecided[k] = und[k];
    memcpy(res->span_raw, blk + OFF_RAW, 4 * sp.nspans);
    memcpy(res->span_status, blk + OFF_ST, 4 * sp.nspans);
    return ZSCRC_OK;
}

} /* namespace */

extern "C" void zscrc_cpass_destroy(zscrc_cpass *p)
{
    if (!p)
        return;
    int cur = -1;
    const bool sw = hipGetDevice(&cur) == hipSuccess && cur != p->dev && hipSetDevice(p->dev) == hipSuccess;
    cpass_free(p);
    if (sw)
        (void)hipSetDevice(cur);
}
