/*
 * zscrc_api.cpp -- the C ABI of libzscrc (declared in include/zscrc.h).
 *
 * Part 1 re-exports the reference's checksum symbols (crc32c_hw et al.,
 * /root/reference/include/libzeroskip/crc32c.h:15-24) with identical
 * semantics.  Part 2 drives the gfx950 kernels in zscrc_kernels.hip.
 *
 * Per HIP device the library keeps one context: the 36 KiB operator-table
 * block (zscrc_internal.h GT_*), the CU count that sizes the persistent grid,
 * and growable scratch for spans and host-staged batches.
 */
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/zscrc.h"
#include "zscrc_gf2.h"
#include "zscrc_internal.h"

extern "C" {
uint32_t zscrc_cpu_table(uint32_t crc, const void *buf, size_t len);
uint32_t zscrc_cpu_hw(uint32_t crc, const void *buf, size_t len);
int zscrc_cpu_have_sse42(void);
void zscrc_cpu_init(void);
int zs_launch_team(int g, int fixed, int depth, const zs::BatchDesc *d, const uint32_t *gtab, int grid,
                   hipStream_t stream);
int zs_launch_span_fold(const zs::SpanFold *f, const uint32_t *gtab, hipStream_t stream);
int zs_launch_short(int fixed, int pf, const zs::BatchDesc *d, const uint32_t *gtab, int grid, hipStream_t stream);
int zs_launch_stream_read(const void *buf, uint64_t n, uint32_t *out, int grid, hipStream_t stream);
int zs_set_wave_times(uint64_t *p);
int zs_set_classify_times(uint64_t *p);
int zs_launch_classify(const zs::Classify *c, hipStream_t stream);
int zs_launch_part_fold(const zs::BatchDesc *d, int nd, const uint32_t *gtab, hipStream_t stream);
int zs_launch_plan(const zs::PlanArgs *a, hipStream_t stream);
int zs_launch_burst(int fixed, int xp, int nb, const zs::BatchDesc *d, const uint32_t *gtab, int grid,
                    hipStream_t stream);
int zs_launch_multi(const zs::BatchDesc *d, const zs::MultiBatch *m, const uint32_t *gtab, int grid,
                    hipStream_t stream);
int zs_launch_xteam(int depth, const zs::BatchDesc *d, const uint32_t *gtab, int grid, hipStream_t stream);
int zs_launch_commit(const zs::BatchDesc *d, const uint32_t *gtab, int grid, hipStream_t stream);
int zs_launch_commit_scatter(uint8_t *base, const uint64_t *off, const uint64_t *len, const uint32_t *crc,
                             const uint32_t *status, uint64_t n, uint32_t *user_status, int ncu, hipStream_t stream);
int zs_launch_qdyn(const zs::BatchDesc *bd, const zs::QDyn *q, uint32_t K, uint32_t K_last, const uint32_t *gtab,
                   int grid, hipStream_t stream);
int zs_launch_xparts(const zs::BatchDesc *d, const uint32_t *gtab, int grid, int deal, hipStream_t stream);
int zs_launch_nbv(const zs::XParts *p, const uint32_t *gtab, int grid, hipStream_t stream);
int zs_launch_spans(const zs::XDesc *x, const zs::XMulti *m, const zs::SpanFolds *fs, const uint32_t *gtab,
                    int grid, int deal, hipStream_t stream);
int zs_launch_mismatch_rows(const uint32_t *st, const uint32_t *crc, const int64_t *end, const uint8_t *img,
                            uint64_t img_size, uint64_t n, int64_t *hdr, int64_t *rows, uint32_t cap,
                            hipStream_t stream);
}

namespace {

constexpr int MAX_DEV = 64;
/* spans below SPAN_SPLIT_MIN: one whole-wave team; longer: segments of at
 * least SEG_MIN over every CU (a lone 320 KB or 1.5 MB span ran as one wave's
 * or 23 teams' serial walk: 0.1-0.25 ms) */
constexpr uint64_t SPAN_SPLIT_MIN = 16u << 10;
constexpr uint64_t SEG_MIN = 1u << 10;

thread_local char t_err[256];
std::atomic<uint64_t> g_stat[4];
/* Scalar offload thresholds of the drop-in symbols (crc32c_hw & co.): a call
 * of at least g_gpu_min bytes goes to the GPU once this process has a device
 * context (warm), at least g_gpu_min_cold before (the first offloaded call
 * pays HIP init, ~0.1-0.2 s).  Defaults are the crossovers measured against
 * one CPU core on a pageable buffer (tools/probes/crossover.py,
 * profiles/r04/crossover.jsonl); env ZSCRC_GPU_MIN sets both (0 = never),
 * ZSCRC_GPU_MIN_COLD the cold one alone. */
/* measured: warm, the GPU wins from 32 MiB (0.85 vs 1.26 ms; 16 MiB level,
 * 0.446 vs 0.432); cold, the first call costs ~0.106 s more (4 GiB: 0.184 s
 * vs 0.077 warm), so it wins from ~4.6 GiB (24 GB/s on one core against
 * 55.6 GB/s) */
constexpr uint64_t GPU_MIN_WARM_DEFAULT = 32ull << 20;
constexpr uint64_t GPU_MIN_COLD_DEFAULT = 5ull << 30;
std::atomic<uint64_t> g_gpu_min{GPU_MIN_WARM_DEFAULT};
std::atomic<uint64_t> g_gpu_min_cold{GPU_MIN_COLD_DEFAULT};
std::atomic<bool> g_warm{false}; /* a device context exists in this process */
std::atomic<uint64_t> g_g1_max{640};
std::atomic<uint64_t> g_g16_max{1u << 20};
std::atomic<int> g_split_team{64}; /* team size on split long records */
/* 2-lane teams on fixed-stride records: 0 = automatic (128-byte-aligned
 * records of 128..1024 bytes), 1 = never, 2 = every record <= g1_max */
std::atomic<int> g_small_team{0};
/* coalesced non-temporal whole-wave teams (xteam_kernel) on fixed-stride
 * records of at least g_xteam_min bytes: 0 = off, 1 = on (same-box
 * interleaved A/B, profiles/r02/xteam_ab.jsonl: 1 MiB records 0.64-0.68 ms
 * per 4 GiB against 0.73-0.77 for team<64>; on 64 KiB records (config 3)
 * within -4..+8 % of team<16> from box to box, so team<16> keeps those) */
std::atomic<int> g_xteam{1};
/* tuning bits copied into every BatchDesc (zs::BatchDesc::opt; env ZSCRC_OPT) */
std::atomic<uint32_t> g_opt{0};
std::atomic<uint64_t> g_xteam_min{256u << 10};
/* spans on xteam_kernel: segments per wave, dealt per workgroup by an LDS
 * counter (env ZSCRC_XDEAL, at most 16, which zscrc_span_scratch_bytes
 * covers; 0 or tuning bit 1 << 26: the static walk's two per wave) */
constexpr uint32_t XDEAL_MAX = 16;
std::atomic<uint32_t> g_xdeal{XDEAL_MAX};
uint32_t xdeal_for(uint32_t opt)
{
    return (opt & zs::OPT_XSTATIC) ? 0u : g_xdeal.load();
}
/* coalesced non-temporal 16-lane teams (qteam_kernel) in place of
 * team_kernel<16>'s two-level walk on equal-length fixed-stride records of
 * >= g_qteam_min bytes: 0 = off, 1 = on */
std::atomic<int> g_qteam{1};
/* qteam from 2 KiB records (tools/probes/qteam_ab.py, profiles/r02/qteam_ab_small.jsonl:
 * 2 KiB 0.789 vs 0.824 ms per 4 GiB, 4 KiB 0.665 vs 0.756, 8 KiB 0.661 vs
 * 0.736; ~1 KiB loses, 1.53 vs 1.32); env ZSCRC_QTEAM_MIN */
std::atomic<uint64_t> g_qteam_min{2048};
std::atomic<int> g_span_team{16}; /* team size on span segments (16 or 64; 16: 3 GiB 5.56 -> 5.71 TB/s) */
int g_strict = 0;
/* record-walk override per team size (index 0/1/2 = G 1/16/64): -1 = automatic
 * (walk_for), 0 = two-level loop, 1/2 = flattened loop with a 1/2-item ring;
 * G = 1 only: 3..8 = short_kernel (per-lane records; next piece loaded if it
 * exists / always four loads / two pieces ahead / bursts of 2, 3, 4 pieces),
 * 9 = burst_kernel (a record's pieces loaded at once, next record in flight),
 * 10 = burst_kernel with quad-cooperative loads and a lane transpose */
std::atomic<int> g_depth[3] = {{-1}, {-1}, {-1}};

struct DevCtx {
    std::recursive_mutex mu;
    bool ready = false;
    int ncu = 0;
    uint32_t *gtab = nullptr;
    uint32_t *sink = nullptr;  /* 4 KiB a kernel's masked-off stores go to */
    void *scratch = nullptr;   /* span partials */
    size_t scratch_bytes = 0;
    void *stage = nullptr;     /* host-batch staging */
    size_t stage_bytes = 0;
    void *classes = nullptr;   /* class lists + counters of variable batches */
    size_t classes_bytes = 0;
    void *parts = nullptr;     /* part registers of split long records */
    void *qparts = nullptr;    /* qteam_dyn_kernel: part registers */
    size_t qparts_bytes = 0;
    void *rlist = nullptr;     /* split commit batches: leftover-round count + list */
    size_t rlist_bytes = 0;
    void *wbuf = nullptr;      /* two-pass commit writer: statuses (+ CRCs) */
    size_t wbuf_bytes = 0;
    size_t parts_bytes = 0;
    hipEvent_t last = nullptr; /* end of the last scratch user's work ... */
    hipStream_t last_stream = nullptr; /* ... enqueued on this stream */
    bool last_valid = false;
    /* verdict counters published by commit_kernel's last workgroup: four
     * (count, workgroups done) pairs per stream that used one, 0 at rest --
     * calls on one stream are ordered, so a stream's own pair needs no
     * event (verdict_slot) */
    unsigned long long *vctr = nullptr;
    /* class-3-only verdicts (xteam_kernel MODE 3 + nbv_fold_kernel): part
     * registers per segment, then the commits' starts; used under the
     * scratch's cross-stream ordering */
    uint32_t *nbv = nullptr;
    hipStream_t vctr_stream[64] = {};
    uint32_t vctr_turn[64] = {};
    int vctr_n = 0;
};
DevCtx g_ctx[MAX_DEV];
std::once_flag g_env_once;

void set_err(const char *what, hipError_t e)
{
    snprintf(t_err, sizeof t_err, "%s: %s", what, e == hipSuccess ? "ok" : hipGetErrorString(e));
}

void env_init()
{
    const char *s = getenv("ZSCRC_GPU_MIN");
    if (s)
        g_gpu_min = g_gpu_min_cold = strtoull(s, nullptr, 0);
    s = getenv("ZSCRC_GPU_MIN_COLD");
    if (s && g_gpu_min)
        g_gpu_min_cold = strtoull(s, nullptr, 0);
    s = getenv("ZSCRC_STRICT");
    g_strict = s && *s && *s != '0';
    s = getenv("ZSCRC_G1_MAX");
    if (s)
        g_g1_max = strtoull(s, nullptr, 0);
    s = getenv("ZSCRC_SPLIT_TEAM");
    if (s && (atoi(s) == 16 || atoi(s) == 64))
        g_split_team = atoi(s);
    s = getenv("ZSCRC_SMALL_TEAM");
    if (s && atoi(s) >= 0 && atoi(s) <= 2)
        g_small_team = atoi(s);
    s = getenv("ZSCRC_SPAN_TEAM");
    if (s && (atoi(s) == 16 || atoi(s) == 64))
        g_span_team = atoi(s);
    s = getenv("ZSCRC_G16_MAX");
    if (s)
        g_g16_max = strtoull(s, nullptr, 0);
    s = getenv("ZSCRC_XTEAM");
    if (s && atoi(s) >= 0 && atoi(s) <= 1)
        g_xteam = atoi(s);
    s = getenv("ZSCRC_OPT");
    if (s)
        g_opt = (uint32_t)strtoul(s, nullptr, 0);
    s = getenv("ZSCRC_QTEAM_MIN");
    if (s)
        g_qteam_min = strtoull(s, nullptr, 0);
    s = getenv("ZSCRC_QTEAM");
    if (s && atoi(s) >= 0 && atoi(s) <= 1)
        g_qteam = atoi(s);
    s = getenv("ZSCRC_XTEAM_MIN");
    if (s)
        g_xteam_min = strtoull(s, nullptr, 0);
    if ((s = getenv("ZSCRC_XDEAL")))
        g_xdeal = (uint32_t)std::min<unsigned long>(strtoul(s, nullptr, 0), XDEAL_MAX);
}

bool is_gfx950(int dev)
{
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess)
        return false;
    return strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

void build_gtab(uint32_t *t)
{
    zs_gf2_shift_table(t + GT_S4, 4);
    zs_gf2_shift_table(t + GT_U16, 4 + 15 * 64);
    zs_gf2_shift_table(t + GT_U64, 4 + 63 * 64);
    for (int k = 0; k < 6; ++k)
        zs_gf2_shift_table(t + GT_Z + 1024 * k, 64ull << k);
    for (int k = 0; k < 64; ++k)
        t[GT_POW2 + k] = zs_gf2_xpow8n(1ull << k);
    zs_gf2_shift_table(t + GT_U2, 4 + 64);
    zs_gf2_shift_table(t + GT_Z192, 192);
}

/* Context of the current device, initialised on first use. */
int get_ctx(DevCtx **out)
{
    std::call_once(g_env_once, env_init);
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess || dev < 0 || dev >= MAX_DEV) {
        set_err("hipGetDevice", e);
        return ZSCRC_ENODEV;
    }
    DevCtx &c = g_ctx[dev];
    std::lock_guard<std::recursive_mutex> lk(c.mu);
    if (c.ready) {
        *out = &c;
        return ZSCRC_OK;
    }
    if (!is_gfx950(dev)) {
        snprintf(t_err, sizeof t_err, "device %d is not gfx950 (MI355X)", dev);
        return ZSCRC_ENODEV;
    }
    int ncu = 0;
    e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess || ncu <= 0) {
        set_err("hipDeviceGetAttribute(CU count)", e);
        return ZSCRC_EHIP;
    }
    static uint32_t host_tab[GT_WORDS];
    static std::once_flag tab_once;
    std::call_once(tab_once, [] { build_gtab(host_tab); });
    e = hipMalloc(&c.gtab, sizeof host_tab);
    if (e != hipSuccess) {
        set_err("hipMalloc(tables)", e);
        return ZSCRC_ENOMEM;
    }
    e = hipMemcpy(c.gtab, host_tab, sizeof host_tab, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_err("hipMemcpy(tables)", e);
        return ZSCRC_EHIP;
    }
    e = hipMalloc(&c.sink, 4096);
    if (e != hipSuccess) {
        set_err("hipMalloc(sink)", e);
        return ZSCRC_ENOMEM;
    }
    c.ncu = ncu;
    c.ready = true;
    g_warm = true;
    *out = &c;
    return ZSCRC_OK;
}

int grow(void **p, size_t *have, size_t need)
{
    if (*have >= need)
        return ZSCRC_OK;
    if (*p)
        (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    size_t n = need + need / 4;
    hipError_t e = hipMalloc(p, n);
    if (e != hipSuccess) {
        set_err("hipMalloc(scratch)", e);
        return ZSCRC_ENOMEM;
    }
    *have = n;
    return ZSCRC_OK;
}

/* The scratch buffers (class lists, part registers, span partials) are
 * shared by every call on a device.  A call on another stream than the last
 * user's waits for that user's work (hipStreamWaitEvent) -- concurrent calls
 * on two streams would otherwise race on the lists.  Call with c->mu held for
 * the whole enqueue.  Streams under hipGraph capture are left alone (an
 * event recorded outside the capture cannot be waited on inside it). */
bool capturing(hipStream_t s)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

int scratch_acquire(DevCtx *c, hipStream_t s)
{
    if (!c->last_valid || c->last_stream == s || capturing(s))
        return ZSCRC_OK;
    hipError_t e = hipStreamWaitEvent(s, c->last, 0);
    if (e != hipSuccess) {
        set_err("hipStreamWaitEvent(scratch)", e);
        return ZSCRC_EHIP;
    }
    return ZSCRC_OK;
}

int scratch_release(DevCtx *c, hipStream_t s)
{
    if (capturing(s)) {
        c->last_valid = false;
        return ZSCRC_OK;
    }
    hipError_t e = hipSuccess;
    if (!c->last)
        e = hipEventCreateWithFlags(&c->last, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipEventRecord(c->last, s);
    if (e != hipSuccess) {
        set_err("hipEventRecord(scratch)", e);
        c->last_valid = false;
        return ZSCRC_EHIP;
    }
    c->last_stream = s;
    c->last_valid = true;
    return ZSCRC_OK;
}

/* Team size for n fixed-stride records of `len` bytes at `stride` from
 * `base` (profiles/r01/team_sweep.jsonl, same-GPU A/B of G 1 / 2 / 16):
 *  - 2-lane teams where every record starts and ends on a 128-byte line
 *    (each lane reads one half of each line: 4.7-5.3 TB/s from 128 B to
 *    1 KiB, vs 2.8-4.6 one lane per record and 0.7-5.1 with 16 lanes);
 *    unaligned records leave the two lanes' 64-byte pieces straddling lines
 *    and one lane a piece behind, and lose to one lane per record;
 *  - one lane per record up to g1_max (640) bytes;
 *  - 16-lane teams above it (best from ~700 B unaligned), which keep four
 *    records per wave in flight, when there are enough records to give every
 *    team one; otherwise whole-wave teams. */
int team_for(uint64_t len, uint64_t n, int ncu, uint64_t stride, uintptr_t base)
{
    const int st = g_small_team;
    if (st == 2 && len <= g_g1_max)
        return 2;
    if (st == 0 && len >= 128 && len <= 1024 && ((len | stride | base) & 127) == 0)
        return 2;
    if (len <= g_g1_max)
        return 1;
    if (g_xteam && len >= g_xteam_min && len > g_g1_max)
        return 64; /* xteam_kernel: coalesced non-temporal whole-wave teams */
    if (len <= g_g16_max && n >= (uint64_t)ncu * 16 * 4)
        return 16;
    return 64;
}

zs::BatchDesc make_desc()
{
    zs::BatchDesc d;
    memset(&d, 0, sizeof d);
    d.last_len = ~0ull;
    d.len_lo = 0;
    d.len_hi = ~0ull;
    d.opt = g_opt;
    return d;
}

/* Record walk by record length (profiles/r01/sweep_walks.jsonl, same-GPU A/B):
 * records >= 8 KiB: the two-level loop (G16 on 64 KiB chunks reads at the
 * streaming-read ceiling); shorter records: the flattened (record, step) loop,
 * whose register ring keeps loads in flight across record boundaries -- two
 * items deep where the batch is fixed-stride, except 4-8 KiB G16 records. */
int walk_for(int g, int fixed, uint64_t len)
{
    if (g == 1) /* record bursts with quad-cooperative loads (burst_kernel,
                 * walk 10) for records over 64 bytes and variable batches;
                 * one-piece fixed-stride records: the piece walk
                 * (tools/probes/g1_sweep.py, profiles/r01/mid_sweep.jsonl) */
        return fixed && len <= 64 ? 3 : 10;
    if (len >= 8192)
        return 0;
    if (!fixed)
        return 1;
    return (g == 16 && len > 2048) ? 1 : 2;
}

/* qteam_kernel's preconditions: every record the same length (>= g_qteam_min)
 * and 4-byte phase, lane offsets within 32 bits */
bool qteam_fits(const zs::BatchDesc &d)
{
    return d.fixed_len >= g_qteam_min && d.fixed_len >= 1024 && (d.last_len == ~0ull || d.last_len == d.fixed_len) &&
           (d.stride & 3) == 0 &&
           d.stride <= (1ull << 30);
}

/* Big qteam batches: records cut into parts dealt per workgroup (config 3
 * 0.640 -> 0.633 ms, 16 KiB records -2.9 %, 4 KiB -2.3 %, interleaved,
 * profiles/r04/ab_config3_qdeal.jsonl); small ones keep the static walk (the
 * fold launch is ~1 % of a 4 GiB pass).  Tuning bit 1 << 24: never, 1 << 25:
 * always. */
bool qdeal_for(const DevCtx *c, const zs::BatchDesc &d)
{
    if (d.opt & (1u << 24))
        return false;
    const uint64_t ngroups = (d.n + 3) / 4;
    return (d.opt & (1u << 25)) || (d.n * d.fixed_len >= (1ull << 30) && ngroups >= 2ull * c->ncu * 16);
}

/* qteam_dyn_kernel's parts: P 1 KiB steps each (env ZSCRC_QDYN_P, default
 * 16), np per record; whether a workgroup's part registers fit its LDS (a
 * workgroup's records -- 16 groups per ceil(ngroups / waves) -- x np), so
 * it folds its own records at its end and no second launch runs. */
struct QdynShape {
    uint32_t P, np;
    uint64_t tail, ngroups;
    bool lds_fold;
};

QdynShape qdyn_shape(const DevCtx *c, const zs::BatchDesc &d)
{
    QdynShape q;
    q.P = 16;
    if (const char *e = getenv("ZSCRC_QDYN_P")) {
        const unsigned long v = strtoul(e, nullptr, 0);
        if (v >= 1 && v <= 4096)
            q.P = (uint32_t)v;
    }
    const uint64_t ph = reinterpret_cast<uintptr_t>(d.base) & 3;
    const uint64_t span = ((ph + d.fixed_len) & ~uint64_t(3)) - ph;
    const uint64_t S = (span + 1023) / 1024;
    q.tail = d.fixed_len - span;
    q.np = (uint32_t)((S + q.P - 1) / q.P);
    q.ngroups = (d.n + 3) / 4;
    const uint64_t nw = (uint64_t)c->ncu * 16;
    q.lds_fold = !(d.opt & zs::OPT_QFOLD_LAUNCH) && 4 * 16 * ((q.ngroups + nw - 1) / nw) * q.np <= zs::QDYN_LDS_PARTS;
    return q;
}

/* qteam with each workgroup's units dealt to its waves: every record cut
 * into np parts, folded per record in the kernel (LDS) or by a second
 * launch (qfold_kernel). */
int launch_qdyn(DevCtx *c, const zs::BatchDesc &d, hipStream_t s)
{
    const QdynShape sh = qdyn_shape(c, d);
    const uint32_t P = sh.P, np = sh.np;
    const uint64_t tail = sh.tail, ngroups = sh.ngroups;
    /* a workgroup's slots: its groups x np (32-bit) */
    if (ngroups / ((uint64_t)c->ncu * 16) * np >= (1ull << 31))
        return ZSCRC_EINVAL;
    const uint32_t K = zs_gf2_xpow8n(1024ull * P), K_last = zs_gf2_xpow8n(1024ull * P + tail);
    if (sh.lds_fold) {
        zs::QDyn q;
        memset(&q, 0, sizeof q);
        q.P = P;
        q.np = np;
        q.lds_fold = 1;
        q.K = K;
        q.K_last = K_last;
        if (zs_launch_qdyn(&d, &q, K, K_last, c->gtab, c->ncu, s)) {
            set_err("qteam dyn launch", hipGetLastError());
            return ZSCRC_EHIP;
        }
        g_stat[2]++;
        return ZSCRC_OK;
    }
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    int rc = scratch_acquire(c, s);
    if (rc)
        return rc;
    rc = grow(&c->qparts, &c->qparts_bytes, (size_t)d.n * np * sizeof(uint32_t));
    if (!rc) {
        zs::QDyn q;
        memset(&q, 0, sizeof q);
        q.part_out = static_cast<uint32_t *>(c->qparts);
        q.P = P;
        q.np = np;
        if (zs_launch_qdyn(&d, &q, K, K_last, c->gtab, c->ncu, s)) {
            set_err("qteam dyn launch", hipGetLastError());
            rc = ZSCRC_EHIP;
        } else {
            g_stat[2]++;
        }
    }
    const int rc2 = scratch_release(c, s);
    return rc ? rc : rc2;
}

int launch(DevCtx *c, int g, const zs::BatchDesc &d, hipStream_t s, int depth_hint = -1)
{
    /* fixed-stride form when no per-record arrays are involved */
    const int fixed = !d.desc && !d.off && !d.len && !d.seed && !d.commit && d.len_lo == 0 && d.len_hi == ~0ull;
    const uint64_t typical = fixed ? d.fixed_len : (d.len_lo > 0 ? d.len_lo : 1);
    int depth = g == 2 ? -1 : g_depth[g == 1 ? 0 : g == 16 ? 1 : 2].load();
    if (depth < 0)
        depth = depth_hint >= 0 ? depth_hint : walk_for(g, fixed, typical);
    if (g != 1 && depth > 2)
        depth = 2;
    if (!fixed && depth == 2)
        depth = 1;
    zs::BatchDesc dx = d;
    /* pieces per burst: a fixed-stride record spans at most ceil(len/64) */
    const int nb = fixed && d.fixed_len <= 64 && d.last_len == ~0ull ? 1
                   : fixed && d.fixed_len <= 128 && d.last_len == ~0ull ? 2 : 5;
    const int xt = g_xteam;
    const bool xteam = g == 64 && fixed && xt && g_depth[2] < 0 && depth_hint < 0 && d.fixed_len >= g_xteam_min;
    const bool qteam = g == 16 && fixed && g_qteam && g_depth[1] < 0 && depth_hint < 0 && qteam_fits(d);
    if (qteam && qdeal_for(c, d))
        return launch_qdyn(c, d, s);
    int rc = qteam       ? zs_launch_xteam(16, &d, c->gtab, c->ncu, s)
             : xteam     ? zs_launch_xteam(xt, &d, c->gtab, c->ncu, s)
             : depth >= 9 ? zs_launch_burst(fixed, depth == 10, nb, &dx, c->gtab, c->ncu, s)
             : depth >= 3 ? zs_launch_short(fixed, depth - 3, &dx, c->gtab, c->ncu, s)
                        : zs_launch_team(g, fixed, depth, &d, c->gtab, c->ncu, s);
    if (rc) {
        set_err("team kernel launch", hipGetLastError());
        return ZSCRC_EHIP;
    }
    g_stat[2]++;
    return ZSCRC_OK;
}

/* A variable-length batch: a device-side classify kernel sorts the records
 * into four length classes (lists + counts stay on the device: no host
 * round trip), then one persistent launch per class walks its list:
 *   <= g1_max          one lane per record, flattened walk
 *   <= 8 KiB           16-lane teams, flattened walk
 *   <= g16_max         16-lane teams, two-level walk
 *   longer             whole-wave teams
 * Classes 2-3 with fewer records than two per team are cut into equal parts
 * (unit ~ class bytes / items wanted, plan_kernel) and a fold kernel combines
 * each record's part registers. */
int launch_classes_locked(DevCtx *c, zs::BatchDesc d, hipStream_t s, uint64_t g1, uint64_t g16, uint64_t min_len,
                          uint64_t max_len, bool range_holds);

/* A bounded commit batch (every span within the one-lane bound): commit_kernel
 * -- run rounds, verdicts, rounds dealt per workgroup.  Batches of at least
 * 12 rounds per wave run on the run-only form (zscrc_kernels.hip,
 * commit_kernel RO: 16 waves per CU), which hashes its other rounds one lane
 * per commit.  Tuning bits: 1 << 29 = commit_kernel alone, 16384 = the
 * run-only kernel lists its other rounds and commit_kernel takes them in a
 * second launch. */
int launch_commit_two_pass(DevCtx *c, zs::BatchDesc d, hipStream_t s);

int launch_commit(DevCtx *c, zs::BatchDesc d, hipStream_t s)
{
    const uint64_t nr = (d.n + 63) / 64;
    const bool split = !(d.opt & zs::OPT_NO_RUNSPLIT) && nr >= (uint64_t)c->ncu * 12 && nr < (1ull << 32);
    if (d.commit == 2 && split && (d.opt & zs::OPT_WRITE_TWO_PASS) && !(d.opt & zs::OPT_RO_LIST))
        return launch_commit_two_pass(c, d, s);
    if (!split || !(d.opt & zs::OPT_RO_LIST)) {
        d.round_mode = split ? 3 : 0;
        if (zs_launch_commit(&d, c->gtab, c->ncu, s)) {
            set_err("commit kernel launch", hipGetLastError());
            return ZSCRC_EHIP;
        }
        g_stat[2]++;
        return ZSCRC_OK;
    }
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    int rc = scratch_acquire(c, s);
    if (!rc)
        rc = grow(&c->rlist, &c->rlist_bytes, 4 * (nr + 1));
    if (!rc) {
        uint32_t *cnt = static_cast<uint32_t *>(c->rlist);
        hipError_t e = hipMemsetAsync(cnt, 0, sizeof(uint32_t), s);
        if (e != hipSuccess) {
            set_err("hipMemsetAsync(round count)", e);
            rc = ZSCRC_EHIP;
        }
        d.round_count = cnt;
        d.round_list = cnt + 1;
        for (int mode = 1; !rc && mode <= 2; ++mode) {
            d.round_mode = mode;
            if (zs_launch_commit(&d, c->gtab, c->ncu, s)) {
                set_err("commit kernel launch", hipGetLastError());
                rc = ZSCRC_EHIP;
            } else {
                g_stat[2]++;
            }
        }
    }
    const int rc2 = scratch_release(c, s);
    return rc ? rc : rc2;
}

/* The bounded commit writer in two passes (tuning bit 512, measured and not
 * the default): the run-only commit_kernel computes the CRCs (commit mode 4,
 * the image only read) into the caller's d_crc or a scratch array,
 * commit_scatter_kernel stores them into the image.  Config 4's 10 M fields:
 * 1.025 ms (0.540 CRC array + ~0.485 scatter) against 0.977 for the stores
 * from inside the read pass (interleaved, profiles/r05/writer_ab.jsonl): the
 * scattered field writes cost the same wherever they are issued. */
int launch_commit_two_pass(DevCtx *c, zs::BatchDesc d, hipStream_t s)
{
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    int rc = scratch_acquire(c, s);
    const size_t n = d.n;
    if (!rc)
        rc = grow(&c->wbuf, &c->wbuf_bytes, (d.out ? 4 : 8) * n);
    if (!rc) {
        uint32_t *st = static_cast<uint32_t *>(c->wbuf);
        uint32_t *crc = d.out ? d.out : st + n;
        uint32_t *user_status = d.status;
        zs::BatchDesc dc = d;
        dc.commit = 4;
        dc.out = crc;
        dc.status = st;
        dc.round_mode = 3;
        if (zs_launch_commit(&dc, c->gtab, c->ncu, s) ||
            zs_launch_commit_scatter(const_cast<uint8_t *>(d.base), d.off, d.len, crc, st, n, user_status, c->ncu,
                                     s)) {
            set_err("commit writer launch", hipGetLastError());
            rc = ZSCRC_EHIP;
        } else {
            g_stat[2] += 2;
        }
    }
    const int rc2 = scratch_release(c, s);
    return rc ? rc : rc2;
}

/* The verdict counter pair of stream s (nullptr: none -- the caller zeroes
 * its counter with a fill launch as before).  Pairs are 128 bytes apart;
 * up to 64 streams get one.  Config 4's bench batch: the fill launch and its
 * gap (~5 us of a 0.52 ms call) gone.  Round 5's form of this shared one
 * pair between streams and ordered it with the scratch event -- whose
 * marker packet cost more than the fill (profiles/r05/verdict_publish/).
 * Pairs are keyed by the stream handle, four per stream used in turn: a
 * stream destroyed while one of its verdicts still runs (hipStreamDestroy
 * need not drain it) and a new stream given the same handle would share
 * a pair only after four of the new stream's calls ran in that time. */
unsigned long long *verdict_slot(DevCtx *c, hipStream_t s)
{
    const char *e = getenv("ZSCRC_VERDICT_MEMSET"); /* A/B: the fill launch */
    if ((e && *e == '1') || capturing(s))
        return nullptr;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!c->vctr) {
        void *p = nullptr;
        if (hipMalloc(&p, 64 * 4 * 128) != hipSuccess)
            return nullptr;
        c->vctr = static_cast<unsigned long long *>(p);
    }
    int k = 0;
    while (k < c->vctr_n && c->vctr_stream[k] != s)
        ++k;
    if (k == c->vctr_n) {
        if (c->vctr_n == 64)
            return nullptr;
        /* the stream's four pairs zeroed on the stream itself, ahead of
         * their first use (once per stream, no device-wide wait) */
        if (hipMemsetAsync(c->vctr + 16 * 4 * k, 0, 4 * 128, s) != hipSuccess)
            return nullptr;
        c->vctr_stream[c->vctr_n++] = s;
    }
    const uint32_t turn = c->vctr_turn[k]++ & 3;
    return c->vctr + 16 * (4 * k + turn);
}

/* max_len: a bound on the lengths -- at most g1_max, one kernel straight
 * over the caller's arrays (correct for any length: a wrong bound costs only
 * time).  range_holds: [min_len, max_len] is a range the caller guarantees
 * (the host walk that found the spans knows it; the _range entry point's
 * contract), and the length classes outside it get no launch -- a record
 * outside a wrong range would go unprocessed, so without that guarantee
 * (the _bounded entry points, whose results never depend on the bound) every
 * class is launched. */
int launch_classes(DevCtx *c, zs::BatchDesc d, hipStream_t s, uint64_t max_len = ZSCRC_LEN_UNBOUNDED,
                   uint64_t min_len = 0, bool range_holds = false)
{
    const uint64_t g1 = g_g1_max, g16 = g_g16_max;
    {
        /* the caller bounds every length by one-lane records: burst_kernel
         * straight over the caller's arrays, no classify (it is correct for
         * any length, so a wrong bound costs only time) */
        const int w0 = g_depth[0];
        const bool direct = max_len <= g1 && (w0 < 0 || w0 >= 9);
        const bool commit_direct = max_len <= g1 && d.commit && !d.desc && !(d.opt & 32768) && w0 < 0;
        if (d.bad_count && commit_direct && !d.bad_prezeroed && !(d.opt & zs::OPT_RO_LIST) &&
            d.n < (1ull << 32)) {
            /* one commit_kernel launch: it counts into this stream's pair
             * and its last workgroup publishes the count -- no fill launch */
            unsigned long long *pair = verdict_slot(c, s);
            if (pair) {
                d.bad_publish = d.bad_count;
                d.bad_count = pair;
                d.bad_prezeroed = 1;
            }
        }
        if (d.bad_count && direct && !d.bad_prezeroed) {
            /* verdict batch without classify: zero its counter here (the
             * classify launch does it otherwise) */
            hipError_t e = hipMemsetAsync(d.bad_count, 0, sizeof(uint64_t), s);
            if (e != hipSuccess) {
                set_err("hipMemsetAsync(verdict count)", e);
                return ZSCRC_EHIP;
            }
        }
        if (commit_direct)
            return launch_commit(c, d, s); /* bounded commit batch */
        if (max_len <= g1 && (w0 < 0 || w0 >= 9))
            return launch(c, 1, d, s, walk_for(1, 0, 1));
    }
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    int rc = scratch_acquire(c, s);
    if (!rc)
        rc = launch_classes_locked(c, d, s, g1, g16, range_holds ? min_len : 0,
                                   range_holds ? max_len : ZSCRC_LEN_UNBOUNDED, range_holds);
    const int rc2 = scratch_release(c, s);
    return rc ? rc : rc2;
}

/* batches up to this many records classify in one single-block launch */
constexpr uint64_t SMALL_CLASSIFY = 16384;

int launch_classes_locked(DevCtx *c, zs::BatchDesc d, hipStream_t s, uint64_t g1, uint64_t g16, uint64_t min_len,
                          uint64_t max_len, bool range_holds)
{
    (void)range_holds; /* (min_len, max_len) are 0 / unbounded unless it holds */
    const uint64_t n = d.n;
    uint64_t b1 = g16 < 8191 ? g16 : 8191;
    if (b1 < g1)
        b1 = g1;
    const uint64_t b2 = g16 > b1 ? g16 : b1;
    /* classes buffer: [0,32) class sizes + scatter cursors, [32,64) class
     * byte totals, [64,160) split plans, [256, ...) class-sorted descriptors */
    constexpr size_t HEAD = 256;
    const size_t list_bytes = HEAD + n * sizeof(zs::RecDesc);
    const int gs = g_split_team;
    /* split target per class: two items per team of the launch */
    auto split_items = [&](int g) { return 2u * (uint32_t)c->ncu * 16u * (uint32_t)(64 / g); };
    const size_t T = split_items(16) > split_items(gs) ? split_items(16) : split_items(gs);
    /* class 3 on xteam_kernel's parts mode: a segment plan of one segment per
     * wave, or xdeal per wave dealt per workgroup */
    const bool xparts = g_xteam && !(d.opt & 65536);
    const bool xseg = xparts && !(d.opt & (256 | 131072));
    /* dealt segment plans (16 per wave) measured slower on NOTBATCHED: the
     * single-block plan of ~67 k parts 27 -> 85 us, the parts' geometry loads
     * and the fold outweigh the balance (0.559 -> 0.603 ms interleaved,
     * profiles/r04/ab_notbatched_xdeal.jsonl); tuning bit 1 << 27 for A/B */
    const uint32_t xdeal = xseg && (d.opt & zs::OPT_XDEAL_PARTS) ? xdeal_for(d.opt) : 0u;
    const size_t nseg3 = (size_t)c->ncu * 16u * (xdeal ? xdeal : 1u);
    const size_t P3 = 2 * T > T + nseg3 ? 2 * T : T + nseg3;
    /* parts buffer: class 2 part registers (< 2T), part_rec (< 2T),
     * part_base (< T); class 3 part registers and part_rec (< P3 each: at
     * most T records + one part per segment), part_base (< T); class 3's
     * segment plan: rec_start (< T records, 64-bit) and seg_first (nseg3 + 1) */
    const size_t part_bytes = (5 * T + 2 * P3 + T + 2 * T + nseg3 + 64) * sizeof(uint32_t);
    {
        int rc = grow(&c->classes, &c->classes_bytes, list_bytes);
        if (!rc)
            rc = grow(&c->parts, &c->parts_bytes, part_bytes);
        if (rc)
            return rc;
    }
    uint32_t *cnt = static_cast<uint32_t *>(c->classes);
    uint64_t *cbytes = reinterpret_cast<uint64_t *>(static_cast<char *>(c->classes) + 32);
    zs::SplitPlan *plans = reinterpret_cast<zs::SplitPlan *>(static_cast<char *>(c->classes) + 64);
    zs::RecDesc *desc = reinterpret_cast<zs::RecDesc *>(static_cast<char *>(c->classes) + HEAD);
    const int team[4] = {1, 16, 16, gs};
    const int walk[4] = {-1, 1, 0, 0};
    /* classes 2-3 with fewer records than two per team are cut into equal
     * parts (a lone 1 MiB record would otherwise be one team's serial walk; a
     * few 3 GiB regions beside small records would leave most teams idle),
     * folded per record afterwards.  Class 3 (> g16_max): parts on
     * xteam_kernel's coalesced whole-wave teams, every record through the
     * part fold. */
    zs::PlanArgs pa[2];
    uint32_t *part_out[2];
    for (int k = 2; k < 4; ++k) {
        zs::PlanArgs &p = pa[k - 2];
        memset(&p, 0, sizeof p);
        p.count = cnt;
        p.bytes = cbytes;
        p.desc = desc;
        p.klass = (uint32_t)k;
        p.target = split_items(team[k]);
        if (k == 3 && g_xteam && (d.opt & 131072))
            p.target *= 2; /* four parts per wave (A/B) */
        p.unit_min = (uint64_t)team[k] * 64 * 16; /* 16 steps of the team */
        p.always_split = k == 3 && xparts ? 1u : 0u;
        p.gtab = c->gtab;
        p.plan = plans;
        const size_t cap = k == 3 ? P3 : 2 * T;
        part_out[k - 2] = static_cast<uint32_t *>(c->parts) + (k == 3 ? 5 * T : 0);
        p.part_rec = part_out[k - 2] + cap;
        p.part_base = p.part_rec + cap;
        if (k == 3 && xseg) {
            /* class 3 on xteam_kernel: a segment per wave of its grid, or
             * xdeal per wave dealt per workgroup */
            uint32_t *ext = p.part_base + T;
            p.nseg = (uint32_t)nseg3;
            /* test hook: fewer segments than waves (several records per
             * segment at small sizes) */
            if (const char *e = getenv("ZSCRC_XSEGS")) {
                const unsigned long v = strtoul(e, nullptr, 0);
                if (v >= 1 && v < p.nseg)
                    p.nseg = (uint32_t)v;
            }
            /* part_base / rec_start hold T records: count <= T, and the parts
             * (<= count + nseg <= T + nseg3) fit P3 */
            p.max_parts = (uint32_t)(T + p.nseg);
            p.rec_start = reinterpret_cast<uint64_t *>(ext);
            p.seg_first = ext + 2 * T;
        }
    }
    zs::Classify cl;
    memset(&cl, 0, sizeof cl);
    cl.off = d.off;
    cl.len = d.len;
    cl.seed = d.seed;
    cl.n = n;
    cl.bound[0] = g1;
    cl.bound[1] = b1;
    cl.bound[2] = b2;
    cl.count = cnt;
    cl.bytes = cbytes;
    cl.desc = desc;
    cl.commit = d.commit != 0;
    cl.img_size = d.img_size;
    cl.zero_count = d.bad_count;
    /* a verdict batch whose range starts above class 0: no class-0 launch,
     * the scatter counts out-of-image commits into the verdict */
    if (d.commit && d.bad_count && min_len > g1) {
        cl.verdict_nocommit = 1;
        cl.bad_idx = d.bad_idx;
        cl.bad_cap = d.bad_cap;
    }
    {
        /* class 0 goes to burst_kernel (walk 9, the default), which walks
         * the caller's arrays and skips longer records: no class-0 list */
        const int w0 = g_depth[0];
        cl.direct_ok = g1 > 0 && (w0 < 0 || w0 >= 9);
    }
    /* small batches: one single-block classify launch that also writes the
     * counters and both plans (no memset, no second pass, no plan launches) */
    cl.single = n <= SMALL_CLASSIFY && !(d.opt & 524288) ? 1 : 0;
    /* a verdict batch whose range is all class 3, on a segment plan: the
     * fused single pass (Classify::only3; tuning bit 1 << 28: off) */
    cl.only3 = cl.single && cl.verdict_nocommit && min_len > b2 && xseg && pa[1].nseg &&
                       !(d.opt & zs::OPT_NO_ONLY3)
                   ? 1
                   : 0;
    /* a class-3-only verdict of at most NBV_MAX commits in two launches
     * instead of three: every workgroup of xteam_kernel MODE 3 scans the
     * commits' lengths itself while its tables fill (no classify launch), a
     * wave finishes the commits inside its segment and stores the parts of
     * longer ones, nbv_fold_kernel folds those.  NOTBATCHED interleaved:
     * 0.5122 against 0.5266 ms (tuning bit
     * OPT_NO_NBV: the three launches).  A wave holds its segment's part
     * registers in one register across the wave: at most NBV_PARTS_MAX
     * parts per segment, which the range bounds (a segment of G bytes meets
     * at most G / min_len + 2 commits) */
    auto nbv_parts_fit = [&]() {
        if (!min_len || max_len > UINT64_MAX / 2 / n)
            return false;
        uint64_t G = (n * max_len + nseg3 - 1) / nseg3;
        G = (G + 63) & ~63ull;
        if (G < pa[1].unit_min)
            G = pa[1].unit_min;
        return G / min_len + 2 <= zs::NBV_PARTS_MAX;
    };
    if (cl.only3 && n <= zs::NBV_MAX && !(d.opt & zs::OPT_NO_NBV) && !d.bad_prezeroed && d.off && d.len &&
        pa[1].nseg == nseg3 && nseg3 == (size_t)c->ncu * 16 && nbv_parts_fit()) {
        unsigned long long *pair = verdict_slot(c, s);
        if (pair) {
            if (!c->nbv) {
                void *p = nullptr;
                const size_t bytes = 2 * nseg3 * sizeof(uint32_t) + (zs::NBV_MAX + 1) * sizeof(uint64_t);
                hipError_t e = hipMalloc(&p, bytes);
                if (e != hipSuccess) {
                    if (p)
                        (void)hipFree(p);
                    set_err("nbv buffers", e);
                    return ZSCRC_EHIP;
                }
                c->nbv = static_cast<uint32_t *>(p);
            }
            zs::XParts x;
            memset(&x, 0, sizeof x);
            x.base = d.base;
            x.xor_io = d.xor_io;
            x.off3 = d.off;
            x.len3 = d.len;
            x.seed3 = d.seed;
            x.n3 = n;
            x.img_size = d.img_size;
            x.nbv = c->nbv;
            x.rstart = reinterpret_cast<uint64_t *>(c->nbv + 2 * nseg3);
            x.vpair = pair;
            x.publish = d.bad_count;
            x.bad_idx = d.bad_idx;
            x.bad_cap = d.bad_cap;
            x.nseg = (uint32_t)nseg3;
            x.unit_min = pa[1].unit_min;
            if (zs_launch_nbv(&x, c->gtab, c->ncu, s)) {
                set_err("nbv launch", hipGetLastError());
                return ZSCRC_EHIP;
            }
            g_stat[2] += 2; /* the hashing launch and its fold */
            return ZSCRC_OK;
        }
    }
    if (cl.single) {
        cl.plan[0] = pa[0];
        cl.plan[1] = pa[1];
    } else {
        hipError_t e = hipMemsetAsync(cnt, 0, HEAD, s);
        if (e != hipSuccess) {
            set_err("hipMemsetAsync(class counters)", e);
            return ZSCRC_EHIP;
        }
    }
    for (int pass = 0; pass < (cl.single ? 1 : 2); ++pass) {
        cl.pass = pass;
        if (zs_launch_classify(&cl, s)) {
            set_err("classify launch", hipGetLastError());
            return ZSCRC_EHIP;
        }
        g_stat[2]++;
    }
    d.len_lo = 0;
    d.len_hi = ~0ull;
    d.desc = desc;
    d.class_count = cnt;
    /* class 3 first: its long launch is queued while the host still submits
     * the small ones, which then run back to back behind it (the parts
     * buffers are per class); the folds last */
    zs::BatchDesc fold[2];
    int nfold = 0;
    /* class k holds lengths in (lower[k], upper[k]]; out-of-image commits
     * are class 0 (length 0) */
    const uint64_t lower[4] = {0, g1, b1, b2}, upper[4] = {g1, b1, b2, ~0ull};
    for (const int k : {3, 0, 1, 2}) {
        const bool empty = (k > 0 && upper[k] < min_len) || (k == 0 && min_len > g1 && (!d.commit || cl.verdict_nocommit)) ||
                           (k > 0 && lower[k] >= max_len);
        if (empty)
            continue; /* the caller's range rules this class out: no launch */
        zs::BatchDesc dk = d;
        dk.klass = (uint32_t)k;
        if (k == 0 && cl.direct_ok)
            dk.direct_max = g1;
        if (k >= 2) {
            if (!cl.single) {
                if (zs_launch_plan(&pa[k - 2], s)) {
                    set_err("split plan launch", hipGetLastError());
                    return ZSCRC_EHIP;
                }
                g_stat[2]++;
            }
            dk.split = 1;
            dk.plan = plans;
            dk.part_base = pa[k - 2].part_base;
            dk.part_rec = pa[k - 2].part_rec;
            dk.rec_start = pa[k - 2].rec_start;
            dk.seg_first = pa[k - 2].seg_first;
            dk.part_out = part_out[k - 2];
        }
        int rc;
        if (k == 3 && xparts) {
            rc = zs_launch_xparts(&dk, c->gtab, c->ncu, xdeal != 0, s) ? ZSCRC_EHIP : ZSCRC_OK;
            if (rc)
                set_err("xparts launch", hipGetLastError());
            else
                g_stat[2]++;
        } else {
            rc = launch(c, team[k], dk, s, walk[k]);
        }
        if (rc)
            return rc;
        if (k >= 2)
            fold[nfold++] = dk;
    }
    /* both split classes' folds in one launch */
    if (nfold) {
        if (zs_launch_part_fold(fold, nfold, c->gtab, s)) {
            set_err("part fold launch", hipGetLastError());
            return ZSCRC_EHIP;
        }
        g_stat[2]++;
    }
    return ZSCRC_OK;
}

/* Span over [d_buf, d_buf+len): split across the chip, fold on the GPU. */
int span_impl(DevCtx *c, const void *d_buf, uint64_t len, uint32_t seed, uint32_t *d_out,
              void *scratch, unsigned flags, hipStream_t s)
{
    const uint32_t xio = (flags & ZSCRC_RAW) ? 0u : 0xffffffffu;
    zs::BatchDesc d = make_desc();
    if (len < SPAN_SPLIT_MIN) {
        d.base = static_cast<const uint8_t *>(d_buf);
        d.n = 1;
        d.fixed_len = len;
        d.fixed_seed = seed;
        d.xor_io = xio;
        d.out = d_out;
        return launch(c, len <= g_g1_max ? 1 : 64, d, s);
    }
    int g = g_span_team;
    uint64_t nteams = (uint64_t)c->ncu * 16 * (64 / g);
    /* two segments per wave of >= g_xteam_min bytes: the coalesced
     * whole-wave teams (xteam_kernel); else two per 16-lane team */
    const uint64_t xseg = ((len + 2 * c->ncu * 16 - 1) / (2 * (uint64_t)c->ncu * 16) + 4095) & ~4095ull;
    if (g_xteam && xseg >= g_xteam_min) {
        g = 64;
        nteams = (uint64_t)c->ncu * 16;
    }
    /* xteam: g_xdeal segments per wave dealt per workgroup (else two) */
    const uint32_t deal = g == 64 ? xdeal_for(d.opt) : 0u;
    const uint64_t per_wave = deal > 2 ? deal : 2;
    uint64_t seg = (len + per_wave * nteams - 1) / (per_wave * nteams);
    seg = (seg + 1023) & ~1023ull;
    if (seg < SEG_MIN)
        seg = SEG_MIN;
    const uint64_t w = (len + seg - 1) / seg;
    uint32_t *part = static_cast<uint32_t *>(scratch);
    if (!part) {
        int rc = grow(&c->scratch, &c->scratch_bytes, w * 4);
        if (rc)
            return rc;
        part = static_cast<uint32_t *>(c->scratch);
    }
    d.base = static_cast<const uint8_t *>(d_buf);
    d.n = w;
    d.stride = seg;
    d.fixed_len = seg;
    d.last_len = len - (w - 1) * seg;
    d.fixed_seed = 0;
    d.xor_io = 0;
    d.out = part;
    int rc;
    if (deal) { /* the segments are shorter than launch()'s xteam bound */
        d.opt |= zs::OPT_XDEAL;
        rc = zs_launch_xteam(g_xteam, &d, c->gtab, c->ncu, s) ? ZSCRC_EHIP : ZSCRC_OK;
        if (rc)
            set_err("span launch", hipGetLastError());
        else
            g_stat[2]++;
    } else {
        rc = launch(c, g, d, s);
    }
    if (rc)
        return rc;
    zs::SpanFold f;
    memset(&f, 0, sizeof f);
    f.part = part;
    f.out = d_out;
    f.w = (uint32_t)w;
    f.k = zs_gf2_xpow8n(seg);
    f.kp2[0] = f.k;
    for (int b = 1; b < 32; ++b)
        f.kp2[b] = zs_gf2_mul(f.kp2[b - 1], f.kp2[b - 1]);
    f.x_last = zs_gf2_xpow8n(d.last_len);
    f.x_total = zs_gf2_xpow8n(len);
    f.r0 = seed ^ xio;
    f.xor_out = xio;
    /* the fold kernel XORs its block partials into *d_out: preset it to the
     * constant terms */
    hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_out),
                                     (int)(zs_gf2_mul(f.r0, f.x_total) ^ f.xor_out), 1, s);
    if (e != hipSuccess) {
        set_err("hipMemsetD32Async(span result)", e);
        return ZSCRC_EHIP;
    }
    if (zs_launch_span_fold(&f, c->gtab, s)) {
        set_err("span fold launch", hipGetLastError());
        return ZSCRC_EHIP;
    }
    g_stat[2]++;
    return ZSCRC_OK;
}

/* Scalar call offloaded to the GPU: the chunked copy/CRC pipeline of Part 4
 * straight from the caller's memory, on a stream object cached per device
 * (buffers, streams and events opened once; per call only the copies, the
 * launches and one synchronisation).  Pieces of len / 8 (4-64 MiB) keep the
 * H2D copy of piece k+1 beside the CRC of piece k for mid-size calls.
 * Returns false to fall back to the CPU (no device, an error, or another
 * thread using this device's offload right now). */
struct ScalarOffload {
    std::mutex mu;
    zscrc_stream *s = nullptr;
};
ScalarOffload g_scalar[MAX_DEV];
int stream_submit(zscrc_stream *s, const void *src, uint64_t n);
int stream_collect(zscrc_stream *s, uint32_t *crc);
void stream_reset(zscrc_stream *s, uint32_t seed);
void stream_set_piece(zscrc_stream *s, uint64_t piece);
void stream_free(zscrc_stream *s);

bool gpu_scalar(uint32_t crc, const void *buf, size_t len, uint32_t *res)
{
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV)
        return false;
    ScalarOffload &so = g_scalar[dev];
    std::unique_lock<std::mutex> lk(so.mu, std::try_to_lock);
    if (!lk.owns_lock())
        return false;
    if (!so.s && zscrc_stream_open(&so.s, crc, 64ull << 20, ZSCRC_STREAM_NOCOPY)) {
        so.s = nullptr;
        return false;
    }
    zscrc_stream *s = so.s;
    stream_reset(s, crc);
    stream_set_piece(s, (len / 8 + 4095) & ~4095ull);
    const int rc = zscrc_stream_update(s, buf, len);
    uint32_t r = 0;
    const int rc2 = stream_collect(s, &r);
    if (rc || rc2) {
        /* a failed pass: drop the cached stream (the next call reopens) */
        stream_free(s);
        so.s = nullptr;
        return false;
    }
    *res = r;
    return true;
}

} /* namespace */

/* zscrc_release_cache(): the scalar offload's cached stream objects (three
 * 64 MiB device buffers each), every device. */
extern "C" void zs_scalar_release_cache(void)
{
    int cur = -1;
    (void)hipGetDevice(&cur);
    for (int d = 0; d < MAX_DEV; ++d) {
        ScalarOffload &so = g_scalar[d];
        std::lock_guard<std::mutex> lk(so.mu);
        if (!so.s)
            continue;
        (void)hipSetDevice(d);
        stream_free(so.s);
        so.s = nullptr;
    }
    if (cur >= 0)
        (void)hipSetDevice(cur);
}

/* ====================================================== Part 1: reference API */
extern "C" {

void crc32c_init(void)
{
    std::call_once(g_env_once, env_init);
    zscrc_cpu_init();
}

uint32_t crc32c_sw(uint32_t crc, const void *buf, size_t len)
{
    g_stat[0]++;
    return zscrc_cpu_table(crc, buf, len);
}

uint32_t crc32c_hw(uint32_t crc, const void *buf, size_t len)
{
    std::call_once(g_env_once, env_init);
    const uint64_t gmin = g_warm ? g_gpu_min.load() : g_gpu_min_cold.load();
    if (gmin && g_gpu_min && len >= gmin && buf) {
        uint32_t r;
        if (gpu_scalar(crc, buf, len, &r)) {
            g_stat[1]++;
            return r;
        }
        if (g_strict) {
            fprintf(stderr, "libzscrc: GPU offload failed (%s) and ZSCRC_STRICT is set\n", t_err);
            abort();
        }
    }
    g_stat[0]++;
    return zscrc_cpu_hw(crc, buf, len);
}

uint32_t crc32c(uint32_t crc, const void *buf, size_t len) { return crc32c_hw(crc, buf, len); }

uint32_t crc32c_map(const char *base, unsigned len) { return crc32c(0, base, (size_t)len); }

uint32_t crc32c_cstring(const cstring *buf) { return crc32c_map(buf->buf, (unsigned)buf->len); }

uint32_t crc32c_buf(const char *buf) { return crc32c_map(buf, (unsigned)strlen(buf)); }

uint32_t crc32c_iovec(struct iovec *iov, int iovcnt)
{
    uint32_t crc = 0;
    for (int i = 0; i < iovcnt; ++i)
        if (iov[i].iov_len)
            crc = crc32c(crc, iov[i].iov_base, iov[i].iov_len);
    return crc;
}

/* ============================================================ Part 2: new API */
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    return zs_gf2_shift(crc_a, len_b) ^ crc_b;
}

uint32_t zscrc_shift(uint32_t reg, uint64_t nbytes) { return zs_gf2_shift(reg, nbytes); }

int zscrc_device_batch(const void *d_base, const uint64_t *d_off, const uint64_t *d_len,
                       const uint32_t *d_seed, uint32_t *d_out, size_t n, unsigned flags,
                       void *stream)
{
    return zscrc_device_batch_bounded(d_base, d_off, d_len, d_seed, d_out, n, flags, ZSCRC_LEN_UNBOUNDED,
                                      stream);
}

int zscrc_device_batch_bounded(const void *d_base, const uint64_t *d_off, const uint64_t *d_len,
                               const uint32_t *d_seed, uint32_t *d_out, size_t n, unsigned flags,
                               uint64_t max_len, void *stream)
{
    if (n == 0)
        return ZSCRC_OK;
    if (!d_base || !d_off || !d_len || !d_out)
        return ZSCRC_EINVAL;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    zs::BatchDesc d = make_desc();
    d.base = static_cast<const uint8_t *>(d_base);
    d.off = d_off;
    d.len = d_len;
    d.seed = d_seed;
    d.out = d_out;
    d.n = n;
    d.xor_io = (flags & ZSCRC_RAW) ? 0u : 0xffffffffu;
    return launch_classes(c, d, s, max_len);
}

int zscrc_device_fixed(const void *d_base, uint64_t stride, uint64_t len, uint32_t seed,
                       uint32_t *d_out, size_t n, unsigned flags, void *stream)
{
    if (n == 0)
        return ZSCRC_OK;
    if (!d_base || !d_out)
        return ZSCRC_EINVAL;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    zs::BatchDesc d = make_desc();
    d.base = static_cast<const uint8_t *>(d_base);
    d.stride = stride;
    d.fixed_len = len;
    d.fixed_seed = seed;
    d.out = d_out;
    d.n = n;
    d.xor_io = (flags & ZSCRC_RAW) ? 0u : 0xffffffffu;
    return launch(c, team_for(len, n, c->ncu, stride, reinterpret_cast<uintptr_t>(d_base)), d,
                  static_cast<hipStream_t>(stream));
}

int zscrc_device_fixed_multi(const void *const *d_bases, uint32_t *const *d_outs, size_t k, uint64_t stride,
                             uint64_t len, uint32_t seed, size_t n, unsigned flags, void *stream)
{
    if (n == 0 || k == 0)
        return ZSCRC_OK;
    if (!d_bases || !d_outs || k > ZSCRC_MULTI_MAX)
        return ZSCRC_EINVAL;
    for (size_t b = 0; b < k; ++b)
        if (!d_bases[b] || !d_outs[b])
            return ZSCRC_EINVAL;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (len > 64) {
        /* multi-piece records: one launch per batch (each already long) */
        for (size_t b = 0; b < k && !rc; ++b)
            rc = zscrc_device_fixed(d_bases[b], stride, len, seed, d_outs[b], n, flags, stream);
        return rc;
    }
    zs::BatchDesc d = make_desc();
    d.stride = stride;
    d.fixed_len = len;
    d.fixed_seed = seed;
    d.n = n;
    d.xor_io = (flags & ZSCRC_RAW) ? 0u : 0xffffffffu;
    zs::MultiBatch m;
    memset(&m, 0, sizeof m);
    m.nb = (uint32_t)k;
    m.sink = c->sink;
    for (size_t b = 0; b < k; ++b) {
        m.base[b] = static_cast<const uint8_t *>(d_bases[b]);
        m.out[b] = d_outs[b];
    }
    if (zs_launch_multi(&d, &m, c->gtab, c->ncu, s)) {
        set_err("multi kernel launch", hipGetLastError());
        return ZSCRC_EHIP;
    }
    g_stat[2]++;
    return ZSCRC_OK;
}

size_t zscrc_span_scratch_bytes(uint64_t len)
{
    (void)len;
    /* <= 2 segments per 16-lane team, or XDEAL_MAX per whole-wave team, on 256 CUs */
    return 4u * (XDEAL_MAX * 256u * 16u + 16u);
}

int zscrc_device_span(const void *d_buf, uint64_t len, uint32_t seed, uint32_t *d_out,
                      void *scratch, unsigned flags, void *stream)
{
    if (!d_out || (!d_buf && len))
        return ZSCRC_EINVAL;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (scratch) /* the caller's own partials buffer */
        return span_impl(c, d_buf, len, seed, d_out, scratch, flags, s);
    rc = scratch_acquire(c, s);
    if (!rc)
        rc = span_impl(c, d_buf, len, seed, d_out, nullptr, flags, s);
    const int rc2 = scratch_release(c, s);
    return rc ? rc : rc2;
}

/* The multi-span launch's segment size and segment count (its partial
 * registers) for spans of these lengths. */
static uint64_t spans_seg(const DevCtx *c, uint64_t total)
{
    /* one segment size for every span (g_xdeal segments per wave in all,
     * dealt per workgroup; or two, static), so a short span is as many
     * segments as its length needs, not one wave's walk */
    /* at most 4 segments per wave here: on config 5's shape (two 3 GiB
     * regions + two pointer sections) 4 per wave 1.014 ms, static 1.021, 16
     * per wave 1.028; a lone 3 GiB span wants 16 (0.502 against 0.523)
     * (interleaved, profiles/r04/ab_spans_xdeal.jsonl) */
    const uint32_t deal = std::min<uint32_t>(xdeal_for(g_opt), 4u);
    const uint64_t target = (uint64_t)(deal > 2 ? deal : 2) * (uint64_t)c->ncu * 16;
    uint64_t seg = ((total + target - 1) / target + 1023) & ~1023ull;
    return seg < SEG_MIN ? SEG_MIN : seg;
}

/* part_own != NULL (zscrc_cpass, which owns it and orders its own passes):
 * the segments' partial registers go there, not to the device's shared
 * scratch, so the call needs no scratch ordering -- its event record put a
 * ~6 us gap before the next launch on the stream (config 5's pass,
 * profiles/r06/config5/rt5). */
static int device_spans(const void *const *d_bufs, const uint64_t *lens, const uint32_t *seeds, uint32_t *d_out,
                        size_t k, unsigned flags, void *stream, uint32_t *part_own, uint64_t part_words,
                        zs::SpanFolds *defer_folds = nullptr)
{
    if (k == 0)
        return ZSCRC_OK;
    if (!d_bufs || !lens || !d_out)
        return ZSCRC_EINVAL;
    uint64_t total = 0;
    bool multi = k <= (size_t)zs::SPANS_MAX && g_xteam;
    for (size_t i = 0; i < k; ++i) {
        if (!d_bufs[i] && lens[i])
            return ZSCRC_EINVAL;
        if (lens[i] < SPAN_SPLIT_MIN)
            multi = false;
        total += lens[i];
    }
    if (!multi && part_own)
        return ZSCRC_EINVAL; /* the private form is the one-launch shape only */
    if (!multi) { /* short spans or many: one call each */
        for (size_t i = 0; i < k; ++i) {
            const int rc = zscrc_device_span(d_bufs[i], lens[i], seeds ? seeds[i] : 0u, d_out + i, nullptr, flags,
                                             stream);
            if (rc)
                return rc;
        }
        return ZSCRC_OK;
    }
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t xio = (flags & ZSCRC_RAW) ? 0u : 0xffffffffu;
    const uint32_t deal = std::min<uint32_t>(xdeal_for(g_opt), 4u);
    const uint64_t seg = spans_seg(c, total);
    zs::XMulti m;
    memset(&m, 0, sizeof m);
    zs::SpanFolds fs;
    memset(&fs, 0, sizeof fs);
    m.k = (uint32_t)k;
    uint64_t w = 0;
    for (size_t i = 0; i < k; ++i) {
        const uint64_t W = (lens[i] + seg - 1) / seg;
        m.base[i] = static_cast<const uint8_t *>(d_bufs[i]);
        m.seg[i] = seg;
        m.last[i] = lens[i] - (W - 1) * seg;
        m.first[i] = w;
        m.out[i] = d_out + i;
        w += W;
    }
    m.first[k] = w;
    if (part_own && w > part_words)
        return ZSCRC_EINVAL;
    if (!part_own && (rc = scratch_acquire(c, s)))
        return rc;
    if (!part_own)
        rc = grow(&c->scratch, &c->scratch_bytes, w * 4);
    if (!rc) {
        uint32_t *part = part_own ? part_own : static_cast<uint32_t *>(c->scratch);
        const uint32_t kseg = zs_gf2_xpow8n(seg);
        for (size_t i = 0; i < k; ++i) {
            zs::SpanFold &f = fs.f[i];
            f.part = part + m.first[i];
            f.out = d_out + i;
            f.w = (uint32_t)(m.first[i + 1] - m.first[i]);
            f.k = kseg;
            f.kp2[0] = kseg;
            for (int b = 1; b < 32; ++b)
                f.kp2[b] = zs_gf2_mul(f.kp2[b - 1], f.kp2[b - 1]);
            f.x_last = zs_gf2_xpow8n(m.last[i]);
            f.x_total = zs_gf2_xpow8n(lens[i]);
            f.r0 = (seeds ? seeds[i] : 0u) ^ xio;
            f.xor_out = xio;
            m.preset[i] = zs_gf2_mul(f.r0, f.x_total) ^ f.xor_out;
        }
        zs::XDesc x;
        memset(&x, 0, sizeof x);
        x.base = m.base[0];
        x.out = part;
        x.n = w;
        x.stride = seg;
        x.fixed_len = seg;
        x.last_len = seg;
        if (defer_folds) /* the caller's kernel folds them (zscrc_cpass's post kernel) */
            *defer_folds = fs;
        if (zs_launch_spans(&x, &m, defer_folds ? nullptr : &fs, c->gtab, c->ncu, deal != 0, s)) {
            set_err("multi-span launch", hipGetLastError());
            rc = ZSCRC_EHIP;
        } else {
            g_stat[2] += 2;
            g_stat[3] += total;
        }
    }
    if (part_own)
        return rc;
    const int rc2 = scratch_release(c, s);
    return rc ? rc : rc2;
}

int zscrc_device_spans(const void *const *d_bufs, const uint64_t *lens, const uint32_t *seeds, uint32_t *d_out,
                       size_t k, unsigned flags, void *stream)
{
    return device_spans(d_bufs, lens, seeds, d_out, k, flags, stream, nullptr, 0);
}

/* For zscrc_cpass: the one-launch multi-span call into the caller's own
 * buffer of segment registers (part_words of them). */
extern "C" int zscrc_internal_spans_private(const void *const *d_bufs, const uint64_t *lens, uint32_t *d_out, size_t k,
                                            unsigned flags, uint32_t *part, uint64_t part_words, void *stream,
                                            zs::SpanFolds *defer_folds)
{
    if (!part)
        return ZSCRC_EINVAL;
    return device_spans(d_bufs, lens, nullptr, d_out, k, flags, stream, part, part_words, defer_folds);
}

int zscrc_device_mismatch_rows(const uint32_t *d_status, const uint32_t *d_crc, const int64_t *d_span_end,
                               const void *d_image, uint64_t image_size, size_t n, int64_t *d_hdr,
                               int64_t *d_rows, uint32_t cap, void *stream)
{
    if (!d_hdr || (n && (!d_status || !d_crc || !d_span_end || !d_image || !image_size || (cap && !d_rows))))
        return ZSCRC_EINVAL;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipMemsetAsync(d_hdr, 0, sizeof(int64_t), s);
    if (e != hipSuccess) {
        set_err("hipMemsetAsync(mismatch count)", e);
        return ZSCRC_EHIP;
    }
    if (n == 0)
        return ZSCRC_OK;
    if (zs_launch_mismatch_rows(d_status, d_crc, d_span_end, static_cast<const uint8_t *>(d_image), image_size, n,
                                d_hdr, d_rows, cap, s)) {
        set_err("mismatch rows launch", hipGetLastError());
        return ZSCRC_EHIP;
    }
    g_stat[2]++;
    return ZSCRC_OK;
}

int zscrc_host_batch(const void *base, const uint64_t *off, const uint64_t *len,
                     const uint32_t *seed, uint32_t *out, size_t n)
{
    if (n == 0)
        return ZSCRC_OK;
    if (!base || !off || !len || !out)
        return ZSCRC_EINVAL;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    uint64_t lo = ~0ull, hi = 0;
    for (size_t i = 0; i < n; ++i) {
        if (off[i] < lo)
            lo = off[i];
        if (off[i] + len[i] > hi)
            hi = off[i] + len[i];
    }
    if (hi < lo)
        hi = lo;
    const uint64_t data = (hi - lo + 15) & ~15ull;
    const uint64_t need = data + n * (8 + 8 + 4 + 4) + 64;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if ((rc = grow(&c->stage, &c->stage_bytes, need)))
        return rc;
    uint8_t *dbase = static_cast<uint8_t *>(c->stage);
    uint64_t *doff = reinterpret_cast<uint64_t *>(dbase + data);
    uint64_t *dlen = doff + n;
    uint32_t *dseed = reinterpret_cast<uint32_t *>(dlen + n);
    uint32_t *dout = dseed + n;
    uint64_t *hoff = static_cast<uint64_t *>(malloc(n * 8));
    if (!hoff)
        return ZSCRC_ENOMEM;
    for (size_t i = 0; i < n; ++i)
        hoff[i] = off[i] - lo;
    hipError_t e = hipMemcpy(dbase, static_cast<const uint8_t *>(base) + lo, hi - lo,
                             hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(doff, hoff, n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(dlen, len, n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess && seed)
        e = hipMemcpy(dseed, seed, n * 4, hipMemcpyHostToDevice);
    free(hoff);
    if (e != hipSuccess) {
        set_err("hipMemcpy H2D", e);
        return ZSCRC_EHIP;
    }
    zs::BatchDesc d = make_desc();
    d.base = dbase;
    d.off = doff;
    d.len = dlen;
    d.seed = seed ? dseed : nullptr;
    d.out = dout;
    d.n = n;
    d.xor_io = 0xffffffffu;
    if ((rc = launch_classes(c, d, nullptr)))
        return rc;
    e = hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        set_err("hipMemcpy D2H", e);
        return ZSCRC_EHIP;
    }
    for (size_t i = 0; i < n; ++i)
        g_stat[3] += len[i];
    return ZSCRC_OK;
}

int zscrc_diag_wave_times(void *d_buf)
{
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    if (zs_set_wave_times(static_cast<uint64_t *>(d_buf))) {
        set_err("hipMemcpyToSymbol(zs_wave_times)", hipGetLastError());
        return ZSCRC_EHIP;
    }
    return ZSCRC_OK;
}

int zscrc_diag_classify_times(void *d_buf)
{
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    if (zs_set_classify_times(static_cast<uint64_t *>(d_buf))) {
        set_err("hipMemcpyToSymbol(zs_classify_times)", hipGetLastError());
        return ZSCRC_EHIP;
    }
    return ZSCRC_OK;
}

int zscrc_diag_stream_read(const void *d_buf, uint64_t len, void *d_scratch4, int grid_mult, void *stream)
{
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    if (grid_mult < 1)
        grid_mult = 1;
    if (zs_launch_stream_read(d_buf, len, static_cast<uint32_t *>(d_scratch4), c->ncu * grid_mult,
                              static_cast<hipStream_t>(stream))) {
        set_err("stream read launch", hipGetLastError());
        return ZSCRC_EHIP;
    }
    return ZSCRC_OK;
}

int zscrc_internal_verify_commits(const void *d_image, uint64_t image_size, const uint64_t *d_off,
                                  const uint64_t *d_len, const uint32_t *d_seed, uint32_t *d_crc,
                                  uint32_t *d_status, size_t n, void *stream, int write, uint64_t max_len)
{
    if (n == 0)
        return ZSCRC_OK;
    /* write: 0 verify, 1 write in place, 2 the writer's CRCs into d_crc only */
    if (!d_image || !d_off || !d_len || (write != 1 && !d_crc) || (!write && !d_status))
        return ZSCRC_EINVAL;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    zs::BatchDesc d = make_desc();
    d.base = static_cast<const uint8_t *>(d_image);
    d.off = d_off;
    d.len = d_len;
    d.seed = d_seed;
    d.out = d_crc;
    d.status = d_status;
    d.commit = write == 2 ? 3u : write ? 2u : 1u;
    d.img_size = image_size;
    d.n = n;
    d.xor_io = 0xffffffffu;
    return launch_classes(c, d, static_cast<hipStream_t>(stream), max_len);
}

/* The verdict for zscrc_cpass: *d_nbad was zeroed on the stream by the
 * previous pass's post kernel, so the bounded direct launch needs no memset
 * (a fill launch of ~4.5 us plus its gap per pass). */
extern "C" int zscrc_internal_verdict_prezeroed(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                                const uint64_t *d_span_len, size_t n, uint64_t max_len,
                                                uint64_t *d_nbad, uint64_t *d_bad, size_t cap, void *stream)
{
    if (!d_nbad || (cap && !d_bad) || (n && (!d_image || !d_span_off || !d_span_len)))
        return ZSCRC_EINVAL;
    if (n == 0)
        return ZSCRC_OK; /* the count stays 0 */
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    zs::BatchDesc d = make_desc();
    d.base = static_cast<const uint8_t *>(d_image);
    d.off = d_span_off;
    d.len = d_span_len;
    d.commit = 1;
    d.img_size = image_size;
    d.n = n;
    d.xor_io = 0xffffffffu;
    d.bad_count = reinterpret_cast<unsigned long long *>(d_nbad);
    d.bad_idx = d_bad;
    d.bad_cap = cap;
    d.bad_prezeroed = 1;
    /* max_len is the pass's own host walk's: the range holds */
    return launch_classes(c, d, static_cast<hipStream_t>(stream), max_len, 0, true);
}

static int verdict_impl(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                        const uint64_t *d_span_len, const uint32_t *d_seed, size_t n, uint64_t min_len,
                        uint64_t max_len, uint64_t *d_nbad, uint64_t *d_bad, size_t cap, void *stream,
                        bool range_holds);

int zscrc_device_verify_commits_verdict(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                        const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                        uint64_t max_len, uint64_t *d_nbad, uint64_t *d_bad, size_t cap,
                                        void *stream)
{
    /* max_len a bound the results never depend on (as _bounded) */
    return verdict_impl(d_image, image_size, d_span_off, d_span_len, d_seed, n, 0, max_len, d_nbad, d_bad, cap,
                        stream, false);
}

int zscrc_device_verify_commits_verdict_range(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                              const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                              uint64_t min_len, uint64_t max_len, uint64_t *d_nbad, uint64_t *d_bad,
                                              size_t cap, void *stream)
{
    /* the caller guarantees the range */
    return verdict_impl(d_image, image_size, d_span_off, d_span_len, d_seed, n, min_len, max_len, d_nbad, d_bad,
                        cap, stream, true);
}

static int verdict_impl(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                        const uint64_t *d_span_len, const uint32_t *d_seed, size_t n, uint64_t min_len,
                        uint64_t max_len, uint64_t *d_nbad, uint64_t *d_bad, size_t cap, void *stream,
                        bool range_holds)
{
    if (min_len > max_len)
        return ZSCRC_EINVAL;
    if (!d_nbad || (cap && !d_bad) || (n && (!d_image || !d_span_off || !d_span_len)))
        return ZSCRC_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_nbad, 0, sizeof(uint64_t), s);
        if (e != hipSuccess) {
            set_err("hipMemsetAsync(verdict count)", e);
            return ZSCRC_EHIP;
        }
        return ZSCRC_OK;
    }
    /* *d_nbad is zeroed on the stream by launch_classes (a memset before a
     * direct launch, or the first classify launch) */
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    zs::BatchDesc d = make_desc();
    d.base = static_cast<const uint8_t *>(d_image);
    d.off = d_span_off;
    d.len = d_span_len;
    d.seed = d_seed;
    d.commit = 1;
    d.img_size = image_size;
    d.n = n;
    d.xor_io = 0xffffffffu;
    d.bad_count = reinterpret_cast<unsigned long long *>(d_nbad);
    d.bad_idx = d_bad;
    d.bad_cap = cap;
    return launch_classes(c, d, s, max_len, min_len, range_holds);
}

const char *zscrc_last_error(void) { return t_err; }

void zscrc_stats(uint64_t out[4])
{
    for (int i = 0; i < 4; ++i)
        out[i] = g_stat[i];
}

void zscrc_set_gpu_min(uint64_t min_bytes)
{
    std::call_once(g_env_once, env_init);
    g_gpu_min = min_bytes;
    g_gpu_min_cold = min_bytes;
}

void zscrc_set_gpu_min_pair(uint64_t warm, uint64_t cold)
{
    std::call_once(g_env_once, env_init);
    g_gpu_min = warm;
    g_gpu_min_cold = cold;
}

uint64_t zscrc_gpu_min(int cold)
{
    std::call_once(g_env_once, env_init);
    return cold ? g_gpu_min_cold.load() : g_gpu_min.load();
}

int zscrc_warmup(void)
{
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV)
        return ZSCRC_ENODEV;
    ScalarOffload &so = g_scalar[dev];
    std::lock_guard<std::mutex> lk(so.mu);
    if (!so.s && (rc = zscrc_stream_open(&so.s, 0, 64ull << 20, ZSCRC_STREAM_NOCOPY)) != ZSCRC_OK)
        so.s = nullptr;
    return rc;
}

void zscrc_set_prefetch(int g, int depth)
{
    if (depth < -1 || depth > (g == 1 ? 10 : 2))
        return;
    if (g == 1)
        g_depth[0] = depth;
    else if (g == 16)
        g_depth[1] = depth;
    else if (g == 64)
        g_depth[2] = depth;
}

int zscrc_team_for(uint64_t len, uint64_t n)
{
    DevCtx *c;
    if (get_ctx(&c))
        return 0;
    return team_for(len, n, c->ncu, len, 0);
}

void zscrc_set_small_team(int mode)
{
    std::call_once(g_env_once, env_init);
    if (mode >= 0 && mode <= 2)
        g_small_team = mode;
}

void zscrc_set_xteam(int mode, uint64_t min_len)
{
    std::call_once(g_env_once, env_init);
    if (mode >= 0 && mode <= 1)
        g_xteam = mode;
    g_xteam_min = min_len;
}

const char *zscrc_fixed_kernel(const void *d_base, uint64_t stride, uint64_t len, size_t n)
{
    DevCtx *c;
    if (get_ctx(&c))
        return "none";
    zs::BatchDesc d = make_desc();
    d.base = static_cast<const uint8_t *>(d_base);
    d.stride = stride;
    d.fixed_len = len;
    d.n = n;
    const int g = team_for(len, n, c->ncu, stride, reinterpret_cast<uintptr_t>(d_base));
    if (g == 64 && g_xteam && g_depth[2] < 0 && len >= g_xteam_min)
        return "xteam_kernel";
    if (g == 16 && g_qteam && g_depth[1] < 0 && qteam_fits(d))
        return !qdeal_for(c, d) ? "qteam_kernel"
               : qdyn_shape(c, d).lds_fold ? "qteam_dyn_kernel" : "qteam_dyn_kernel+qfold_kernel";
    static const char *names[] = {"team_kernel<1>/short_kernel/burst_kernel", "team_kernel<2>",
                                  "team_kernel<16>", "team_kernel<64>"};
    return names[g == 1 ? 0 : g == 2 ? 1 : g == 16 ? 2 : 3];
}

int zscrc_xteam_for(uint64_t len, uint64_t n)
{
    DevCtx *c;
    if (get_ctx(&c))
        return 0;
    return team_for(len, n, c->ncu, len, 0) == 64 && g_xteam && g_depth[2] < 0 && len >= g_xteam_min ? g_xteam.load()
                                                                                                        : 0;
}

unsigned zscrc_set_xdeal(unsigned per_wave)
{
    std::call_once(g_env_once, env_init);
    return g_xdeal.exchange(std::min<unsigned>(per_wave, XDEAL_MAX));
}

void zscrc_set_qteam(int mode)
{
    std::call_once(g_env_once, env_init);
    if (mode >= 0 && mode <= 1)
        g_qteam = mode;
}

void zscrc_set_opt(unsigned bits)
{
    std::call_once(g_env_once, env_init);
    g_opt = bits;
}

void zscrc_set_teams(uint64_t g1_max, uint64_t g16_max)
{
    std::call_once(g_env_once, env_init);
    g_g1_max = g1_max;
    g_g16_max = g16_max;
}

/* The current device's operator tables (for the host objects in other
 * translation units, e.g. zscrc_cpass.cpp); NULL without a device. */
const uint32_t *zscrc_internal_gtab(void)
{
    DevCtx *c;
    return get_ctx(&c) ? nullptr : c->gtab;
}

int zscrc_abi_version(void)
{
    return ZSCRC_ABI_VERSION;
}

int zscrc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    int k = 0;
    for (int i = 0; i < n; ++i)
        k += is_gfx950(i);
    return k;
}

/* ============================================= Part 4: host byte streams */
/*
 * Incremental CRC of a host byte stream on the GPU -- the shape of zeroskip's
 * crc32_begin / mfile_write / crc32_end (src/mfile.c:270-290, :526-546) and
 * of repack's one huge records-region CRC (src/zeroskip-packed.c:442).
 * Bytes are cut into fixed chunks; each chunk is copied host->device on a
 * copy stream and its RAW register computed on a compute stream (span
 * kernel), NSLOT chunks in flight, so PCIe transfer, CRC and the caller's
 * production of the next bytes overlap.  final() folds the chunk registers on
 * the host: reg = shift(reg, len_k) ^ raw_k, then the initial register.
 */
} /* extern "C" */

struct zscrc_stream {
    static constexpr int NSLOT = 3;
    DevCtx *c = nullptr;
    int dev = 0;
    unsigned flags = 0;
    hipStream_t cs = nullptr, ks = nullptr; /* copy / compute */
    uint32_t seed = 0;
    uint64_t chunk = 0;
    uint8_t *dbuf[NSLOT] = {};
    uint8_t *hpin[NSLOT] = {};
    void *scr[NSLOT] = {};
    hipEvent_t copied[NSLOT] = {}, done[NSLOT] = {};
    bool used[NSLOT] = {};
    uint32_t *dparts = nullptr;
    size_t cap = 0;
    std::vector<uint64_t> lens;
    int slot = 0;
    uint64_t fill = 0;   /* copy mode: bytes staged in hpin[slot] */
    uint64_t total = 0;
    uint64_t piece = 0;  /* NOCOPY: bytes per submitted piece (<= chunk; 0 = chunk) */
    int err = 0;
};

namespace {

int stream_fail(zscrc_stream *s, const char *what, hipError_t e)
{
    set_err(what, e);
    s->err = ZSCRC_EHIP;
    return s->err;
}

/* Queue chunk `idx` = n bytes at src (device-visible after the copy) in slot k. */
int stream_submit(zscrc_stream *s, const void *src, uint64_t n)
{
    const int k = s->slot;
    const size_t idx = s->lens.size();
    hipError_t e;
    if (idx >= s->cap) {
        /* grow the device register array (rare: doubles) */
        size_t ncap = s->cap ? 2 * s->cap : 4096;
        uint32_t *np = nullptr;
        if ((e = hipStreamSynchronize(s->ks)) != hipSuccess)
            return stream_fail(s, "hipStreamSynchronize", e);
        if ((e = hipMalloc(&np, ncap * 4)) != hipSuccess)
            return stream_fail(s, "hipMalloc(stream registers)", e);
        if (s->dparts) {
            (void)hipMemcpy(np, s->dparts, s->cap * 4, hipMemcpyDeviceToDevice);
            (void)hipFree(s->dparts);
        }
        s->dparts = np;
        s->cap = ncap;
    }
    /* the slot's device buffer is free once its previous CRC finished */
    if (s->used[k] && (e = hipStreamWaitEvent(s->cs, s->done[k], 0)) != hipSuccess)
        return stream_fail(s, "hipStreamWaitEvent", e);
    if ((e = hipMemcpyAsync(s->dbuf[k], src, n, hipMemcpyHostToDevice, s->cs)) != hipSuccess)
        return stream_fail(s, "hipMemcpyAsync H2D", e);
    if ((e = hipEventRecord(s->copied[k], s->cs)) != hipSuccess ||
        (e = hipStreamWaitEvent(s->ks, s->copied[k], 0)) != hipSuccess)
        return stream_fail(s, "stream event", e);
    {
        std::lock_guard<std::recursive_mutex> lk(s->c->mu);
        int rc = span_impl(s->c, s->dbuf[k], n, 0, s->dparts + idx, s->scr[k], ZSCRC_RAW, s->ks);
        if (rc)
            return s->err = rc;
    }
    if ((e = hipEventRecord(s->done[k], s->ks)) != hipSuccess)
        return stream_fail(s, "hipEventRecord", e);
    s->used[k] = true;
    s->lens.push_back(n);
    s->total += n;
    g_stat[3] += n;
    s->slot = (k + 1) % zscrc_stream::NSLOT;
    return ZSCRC_OK;
}

void stream_free(zscrc_stream *s)
{
    if (s->cs)
        (void)hipStreamSynchronize(s->cs);
    if (s->ks)
        (void)hipStreamSynchronize(s->ks);
    for (int k = 0; k < zscrc_stream::NSLOT; ++k) {
        if (s->dbuf[k])
            (void)hipFree(s->dbuf[k]);
        if (s->scr[k])
            (void)hipFree(s->scr[k]);
        if (s->hpin[k])
            (void)hipHostFree(s->hpin[k]);
        if (s->copied[k])
            (void)hipEventDestroy(s->copied[k]);
        if (s->done[k])
            (void)hipEventDestroy(s->done[k]);
    }
    if (s->dparts)
        (void)hipFree(s->dparts);
    if (s->cs)
        (void)hipStreamDestroy(s->cs);
    if (s->ks)
        (void)hipStreamDestroy(s->ks);
    delete s;
}

} /* namespace */

extern "C" {

int zscrc_stream_open(zscrc_stream **out, uint32_t seed, uint64_t chunk_bytes, unsigned flags)
{
    if (!out)
        return ZSCRC_EINVAL;
    *out = nullptr;
    DevCtx *c;
    int rc = get_ctx(&c);
    if (rc)
        return rc;
    zscrc_stream *s = new (std::nothrow) zscrc_stream;
    if (!s)
        return ZSCRC_ENOMEM;
    s->c = c;
    s->flags = flags;
    s->seed = seed;
    s->chunk = chunk_bytes ? ((chunk_bytes + 4095) & ~4095ull) : (64ull << 20);
    hipError_t e = hipGetDevice(&s->dev);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&s->cs, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&s->ks, hipStreamNonBlocking);
    for (int k = 0; e == hipSuccess && k < zscrc_stream::NSLOT; ++k) {
        e = hipMalloc(&s->dbuf[k], s->chunk);
        if (e == hipSuccess)
            e = hipMalloc(&s->scr[k], zscrc_span_scratch_bytes(s->chunk));
        if (e == hipSuccess && !(flags & ZSCRC_STREAM_NOCOPY))
            e = hipHostMalloc(reinterpret_cast<void **>(&s->hpin[k]), s->chunk, hipHostMallocDefault);
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&s->copied[k], hipEventDisableTiming);
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&s->done[k], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        set_err("zscrc_stream_open", e);
        stream_free(s);
        return ZSCRC_ENOMEM;
    }
    *out = s;
    return ZSCRC_OK;
}

int zscrc_stream_update(zscrc_stream *s, const void *buf, size_t len)
{
    if (!s || (!buf && len))
        return ZSCRC_EINVAL;
    if (s->err)
        return s->err;
    const uint8_t *p = static_cast<const uint8_t *>(buf);
    if (s->flags & ZSCRC_STREAM_NOCOPY) {
        /* straight from the caller's (unchanging) memory, chunk by chunk */
        const uint64_t pc = s->piece && s->piece < s->chunk ? s->piece : s->chunk;
        while (len) {
            const uint64_t n = len < pc ? len : pc;
            int rc = stream_submit(s, p, n);
            if (rc)
                return rc;
            p += n;
            len -= n;
        }
        return ZSCRC_OK;
    }
    while (len) {
        const int k = s->slot;
        if (s->fill == 0 && s->used[k]) {
            /* the staging buffer is free once its copy has left */
            hipError_t e = hipEventSynchronize(s->copied[k]);
            if (e != hipSuccess)
                return stream_fail(s, "hipEventSynchronize", e);
        }
        const uint64_t n = len < s->chunk - s->fill ? len : s->chunk - s->fill;
        memcpy(s->hpin[k] + s->fill, p, n);
        s->fill += n;
        p += n;
        len -= n;
        if (s->fill == s->chunk) {
            s->fill = 0;
            int rc = stream_submit(s, s->hpin[k], s->chunk);
            if (rc)
                return rc;
        }
    }
    return ZSCRC_OK;
}

/* Producer side without the update() copy (zscrc_pack.cpp): the caller
 * serialises bytes straight into the stream's pinned staging.  stage()
 * returns the free part of the current slot (waiting until the slot's
 * previous copy has left); advance(n) marks n of them written and, when the
 * slot is full (or on flush), submits it and hands it back in *done so the
 * caller can also write it elsewhere (a file) before staging NSLOT more
 * chunks.  Copy-mode streams only. */
uint8_t *zscrc_internal_stream_stage(zscrc_stream *s, uint64_t *room)
{
    if (!s || s->err || (s->flags & ZSCRC_STREAM_NOCOPY))
        return nullptr;
    const int k = s->slot;
    if (s->fill == 0 && s->used[k]) {
        hipError_t e = hipEventSynchronize(s->copied[k]);
        if (e != hipSuccess) {
            stream_fail(s, "hipEventSynchronize", e);
            return nullptr;
        }
    }
    *room = s->chunk - s->fill;
    return s->hpin[k] + s->fill;
}

int zscrc_internal_stream_advance(zscrc_stream *s, uint64_t n, int flush, const uint8_t **done, uint64_t *done_n)
{
    *done = nullptr;
    *done_n = 0;
    if (s->err)
        return s->err;
    if (n > s->chunk - s->fill)
        return ZSCRC_EINVAL;
    s->fill += n;
    if (s->fill == s->chunk || (flush && s->fill)) {
        const int k = s->slot;
        const uint64_t m = s->fill;
        s->fill = 0;
        int rc = stream_submit(s, s->hpin[k], m);
        if (rc)
            return rc;
        *done = s->hpin[k];
        *done_n = m;
    }
    return ZSCRC_OK;
}

} /* extern "C" */

namespace {

/* The CRC of everything submitted (final() without the free): the chunk
 * registers folded on the host, reg = shift(reg, len_k) ^ raw_k. */
int stream_collect(zscrc_stream *s, uint32_t *crc)
{
    int rc = s->err;
    if (!rc && s->fill) {
        const uint64_t n = s->fill;
        s->fill = 0;
        rc = stream_submit(s, s->hpin[s->slot], n);
    }
    std::vector<uint32_t> raw(s->lens.size());
    if (!rc && !raw.empty()) {
        hipError_t e = hipStreamSynchronize(s->ks);
        if (e == hipSuccess)
            e = hipMemcpy(raw.data(), s->dparts, raw.size() * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess)
            rc = stream_fail(s, "stream final", e);
    }
    if (!rc && crc) {
        const uint64_t l0 = s->lens.empty() ? s->chunk : s->lens[0];
        const uint32_t kx = zs_gf2_xpow8n(l0);
        uint32_t reg = 0;
        for (size_t i = 0; i < raw.size(); ++i)
            reg = (s->lens[i] == l0 ? zs_gf2_mul(reg, kx) : zs_gf2_shift(reg, s->lens[i])) ^ raw[i];
        reg ^= zs_gf2_shift(s->seed ^ 0xffffffffu, s->total);
        *crc = reg ^ 0xffffffffu;
    }
    return rc;
}

/* A finished stream ready for the next span from `seed`: its buffers,
 * streams and events are kept (the scalar offload reuses one per device --
 * opening a stream allocates and freeing it synchronises the device, ~7 ms
 * per call, profiles/r04/crossover_before.jsonl). */
void stream_reset(zscrc_stream *s, uint32_t seed)
{
    s->seed = seed;
    s->lens.clear();
    s->slot = 0;
    s->fill = 0;
    s->total = 0;
    s->err = 0;
}

/* NOCOPY pieces of `piece` bytes, within [4 MiB, chunk] */
void stream_set_piece(zscrc_stream *s, uint64_t piece)
{
    s->piece = piece < (4ull << 20) ? (4ull << 20) : piece > s->chunk ? s->chunk : piece;
}

} /* namespace */

extern "C" {

int zscrc_stream_final(zscrc_stream *s, uint32_t *crc)
{
    if (!s)
        return ZSCRC_EINVAL;
    const int rc = stream_collect(s, crc);
    stream_free(s);
    return rc;
}

} /* extern "C" */
