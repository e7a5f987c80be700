/*
 * zscrc.h -- C ABI of libzscrc, the MI355X-native CRC-32C engine for zeroskip.
 *
 * Part 1 is a drop-in for the reference's checksum API: same names, same
 * signatures, same results, so zeroskip's src/ files link unchanged once
 * src/crc32c.c is dropped from libzeroskip_la_SOURCES (src/Makefile.am:47).
 * Part 2 is the new batched / device-resident API (status-returning).
 *
 * No HIP or torch types appear here: device pointers are plain pointers,
 * a stream is an opaque `void *` (a hipStream_t, NULL = default stream).
 */
#ifndef ZSCRC_H
#define ZSCRC_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of this header.  4: the drop-in symbols offload large calls to
 * the GPU by default (32 MiB once a device context exists, 5 GiB before one;
 * earlier versions never offloaded unless asked -- INTEGRATION.md 2), and
 * zscrc_release_cache() also frees the fill and scalar-offload caches.
 * 3: round-3 ABI (zscrc_files_report.devices,
 * the device-slot API); 2 added image_size / d_status to the commit entry
 * points.  A caller built against this header checks at startup that
 * zscrc_abi_version() == ZSCRC_ABI_VERSION: a library of another version
 * has other struct layouts or argument lists. */
#define ZSCRC_ABI_VERSION 4
int zscrc_abi_version(void);

/* zeroskip's string type (reference include/libzeroskip/cstring.h:23-29). */
#ifndef _CSTRING_H_
struct _cstring {
    size_t len;
    size_t alloc;
    char *buf;
};
typedef struct _cstring cstring;
#endif

/* ======================================================================
 * Part 1 -- reference API (include/libzeroskip/crc32c.h:15-24,
 * exported by src/libzeroskip.symbols:113-120).  crc = 0 starts a new CRC;
 * a previous result chains: crc32c(crc32c(0,A),B) == crc32c(0,A||B).
 * These never fail (the reference has no error channel).
 * ====================================================================== */

/* replaces src/crc32c.c:668-673 (CPU feature probe; also warms the GPU context
 * when ZSCRC_GPU_MIN enables offload) */
void crc32c_init(void);
/* replaces src/crc32c.c:613-645 (portable table path) */
uint32_t crc32c_sw(uint32_t crc, const void *buf, size_t len);
/* replaces src/crc32c.c:370-453; called directly by mfile.c:538,
 * zeroskip-file.c:283-318, zeroskip-record.c:212-259, zeroskip-header.c:45-161,
 * zeroskip-packed.c:298-327, zeroskip-dotzsdb.c:106-525 */
uint32_t crc32c_hw(uint32_t crc, const void *buf, size_t len);
/* replaces src/crc32c.c:675-684 */
uint32_t crc32c(uint32_t crc, const void *buf, size_t len);
/* replaces src/crc32c.c:686-689 */
uint32_t crc32c_map(const char *base, unsigned len);
/* replaces src/crc32c.c:703-706 */
uint32_t crc32c_cstring(const cstring *buf);
/* replaces src/crc32c.c:708-711 */
uint32_t crc32c_buf(const char *buf);
/* replaces src/crc32c.c:691-701 */
uint32_t crc32c_iovec(struct iovec *iov, int iovcnt);

/* ======================================================================
 * Part 2 -- new API.
 * ====================================================================== */

enum zscrc_status {
    ZSCRC_OK = 0,
    ZSCRC_EINVAL = -1,   /* bad argument                     */
    ZSCRC_ENODEV = -2,   /* no usable gfx950 device          */
    ZSCRC_EHIP = -3,     /* HIP runtime error (see zscrc_last_error) */
    ZSCRC_ENOMEM = -4,   /* device or pinned allocation failed */
    ZSCRC_EBUSY = -5,    /* a lock is held by someone else (zscrc_zs_repack: .zsdb.lock) */
};

/* flags */
#define ZSCRC_RAW 1u /* seeds/outputs are raw registers: no pre/post inversion */

/* crc(A||B) from crc(A), crc(B) and |B|.  Generalises crc32c_shift
 * (src/crc32c.c:363-367) to any length. */
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
/* raw register after `nbytes` zero bytes (x^(8n) mod P multiply) */
uint32_t zscrc_shift(uint32_t reg, uint64_t nbytes);

/* Device-resident batch.  Every pointer is a device pointer on the current
 * HIP device.  Record i is d_base[d_off[i] .. d_off[i]+d_len[i]); d_seed may
 * be NULL (seed 0).  d_out[i] = crc32c(seed_i, record_i).  Asynchronous on
 * `stream`; returns after launch. */
int zscrc_device_batch(const void *d_base, const uint64_t *d_off, const uint64_t *d_len,
                       const uint32_t *d_seed, uint32_t *d_out, size_t n,
                       unsigned flags, void *stream);

/* As zscrc_device_batch, with a caller-known bound on the record lengths:
 * max_len >= every d_len[i] (ZSCRC_LEN_UNBOUNDED: none known).  A bound of
 * short records (<= 640 bytes by default) skips the device-side length
 * classification: one kernel over the caller's arrays.  Results never depend
 * on the bound; a wrong one costs only time. */
#define ZSCRC_LEN_UNBOUNDED UINT64_MAX
int zscrc_device_batch_bounded(const void *d_base, const uint64_t *d_off, const uint64_t *d_len,
                               const uint32_t *d_seed, uint32_t *d_out, size_t n, unsigned flags,
                               uint64_t max_len, void *stream);

/* Device-resident fixed-stride batch: record i = d_base[i*stride .. +len). */
int zscrc_device_fixed(const void *d_base, uint64_t stride, uint64_t len, uint32_t seed,
                       uint32_t *d_out, size_t n, unsigned flags, void *stream);

/* K device-resident fixed-stride batches in one call: batch b is
 * d_bases[b][i*stride .. +len) for i < n, results to d_outs[b][i] (as
 * zscrc_device_fixed).  d_bases / d_outs are HOST arrays of k <= ZSCRC_MULTI_MAX
 * device pointers.  Records of <= 64 bytes (BASELINE config 2) run as ONE
 * persistent launch over all k batches: the launch, the operator-table fill
 * and the HBM ramp are paid once instead of k times; longer records run one
 * launch per batch. */
#define ZSCRC_MULTI_MAX 64
int zscrc_device_fixed_multi(const void *const *d_bases, uint32_t *const *d_outs, size_t k, uint64_t stride,
                             uint64_t len, uint32_t seed, size_t n, unsigned flags, void *stream);

/* One long device-resident span, split over every CU and folded on the GPU.
 * d_out (device, 1 word) receives crc32c(seed, span).  `scratch` may be NULL
 * (library-owned) or a device buffer of zscrc_span_scratch_bytes(len). */
size_t zscrc_span_scratch_bytes(uint64_t len);
int zscrc_device_span(const void *d_buf, uint64_t len, uint32_t seed, uint32_t *d_out,
                      void *scratch, unsigned flags, void *stream);

/* Device: k spans in one launch pair (segments of every span over every CU,
 * then one fold launch for all): d_out[i] = crc32c(seeds[i], d_bufs[i],
 * lens[i]) (seeds NULL = 0; ZSCRC_RAW: raw registers).  k <= 8 spans of
 * >= 16 KiB each; otherwise one zscrc_device_span per span.  The library's
 * scratch, like zscrc_device_span with scratch NULL. */
int zscrc_device_spans(const void *const *d_bufs, const uint64_t *lens, const uint32_t *seeds, uint32_t *d_out,
                       size_t k, unsigned flags, void *stream);

/* Device post-pass of a commit verification (consistent): for every commit
 * i with d_status[i] != 1, one row of 18 int64 -- i, d_crc[i-1] (d_crc[0]
 * for i = 0), the 8 image bytes at d_span_end[i] and the 8 at
 * d_span_end[i-1] (each clamped to the image) -- in any order; *d_hdr = the
 * number of such commits (rows past cap are counted, not written). */
int zscrc_device_mismatch_rows(const uint32_t *d_status, const uint32_t *d_crc, const int64_t *d_span_end,
                               const void *d_image, uint64_t image_size, size_t n, int64_t *d_hdr,
                               int64_t *d_rows, uint32_t cap, void *stream);

/* Host-resident batch: copies [min off, max off+len) to the device, runs the
 * batch, copies results back.  Synchronous.  The PCIe-bound path. */
int zscrc_host_batch(const void *base, const uint64_t *off, const uint64_t *len,
                     const uint32_t *seed, uint32_t *out, size_t n);

/* Diagnostics. */
const char *zscrc_last_error(void);
/* counters: [0] scalar calls on CPU, [1] scalar calls offloaded,
 * [2] kernel launches, [3] bytes checksummed on the GPU */
void zscrc_stats(uint64_t out[4]);
/* Scalar offload of the drop-in symbols (crc32c_hw, crc32c, map / buf /
 * cstring / iovec): a call of at least the threshold runs on the GPU
 * (falling back to the CPU silently if that fails, unless ZSCRC_STRICT=1).
 * Two thresholds: the warm one once this process has a device context, the
 * cold one before (the first GPU call pays HIP init).  Defaults: the
 * crossovers against one CPU core measured on MI355X (DESIGN.md §8,
 * profiles/r04/crossover.jsonl); env ZSCRC_GPU_MIN sets both, 0 = never;
 * ZSCRC_GPU_MIN_COLD the cold one alone.  zscrc_set_gpu_min sets both. */
void zscrc_set_gpu_min(uint64_t min_bytes);
/* warm / cold thresholds apart (warm 0 = never offload) */
void zscrc_set_gpu_min_pair(uint64_t warm, uint64_t cold);
/* the threshold in force: cold != 0 -> before any device context exists */
uint64_t zscrc_gpu_min(int cold);
/* Create the current device's context and the scalar-offload buffers now
 * (a zeroskip process that wants large crc32_end calls offloaded from the
 * first one: call it at open).  0 or a negative status. */
int zscrc_warmup(void);
/* team size tuning: records <= g1_max bytes (default 640) use one lane each,
 * <= g16_max (default 1 MiB) a 16-lane team, larger a 64-lane (whole
 * wavefront) team. */
void zscrc_set_teams(uint64_t g1_max, uint64_t g16_max);
/* tuning: 2-lane teams on fixed-stride batches -- 0 = automatic (records of
 * 128..1024 bytes whose length, stride and base are multiples of 128; the
 * default), 1 = never, 2 = every record <= g1_max */
void zscrc_set_small_team(int mode);
/* tuning: record walk for team size g (1, 16 or 64): -1 = automatic (default),
 * 0 = two-level loop, 1 / 2 = flattened (record, step) loop with a 1- / 2-item
 * register ring; g = 1 only: 3..8 = per-lane short-record kernel (next
 * piece loaded when it exists / always / two pieces ahead / bursts of 2, 3,
 * 4 pieces), 9 / 10 = record bursts with per-lane / quad-cooperative loads */
void zscrc_set_prefetch(int g, int depth);
/* team size the fixed-stride path picks for n packed records of len bytes
 * from a 128-byte-aligned base (1/2/16/64; 0 if no device) */
int zscrc_team_for(uint64_t len, uint64_t n);
/* tuning: coalesced non-temporal whole-wave teams (xteam_kernel) on
 * fixed-stride records of at least min_len bytes (default 256 KiB): mode 0 =
 * off, 1 = on (default; env ZSCRC_XTEAM, ZSCRC_XTEAM_MIN) */
void zscrc_set_xteam(int mode, uint64_t min_len);
/* tuning: coalesced non-temporal 16-lane teams (qteam_kernel) in place of
 * team_kernel<16> on equal-length fixed-stride records of >= 2 KiB (stride a
 * multiple of 4): mode 0 = off, 1 = on (env ZSCRC_QTEAM) */
void zscrc_set_qteam(int mode);
/* tuning: spans on xteam_kernel cut into per_wave segments per wave, dealt to
 * each workgroup's waves by an LDS counter (default 16, the most; a
 * multi-span launch, zscrc_device_spans, takes at most 4; env ZSCRC_XDEAL);
 * 0 = the static walk, two contiguous segments per wave.  Returns the
 * previous setting. */
unsigned zscrc_set_xdeal(unsigned per_wave);
/* tuning bits (env ZSCRC_OPT), for A/B runs: 1 = hash five-piece record
 * bursts as one chain instead of three; 2 = 64-byte record batches of
 * zscrc_device_fixed_multi by the per-lane piece walk instead of coalesced
 * chunks; 64 = a _verdict_range batch of long commits only (at most 4,096)
 * through the classify, parts and fold launches (default: two launches
 * without the classify); the rest are listed in
 * zscrc_internal.h (BatchDesc::opt).  Results never depend on them. */
void zscrc_set_opt(unsigned bits);
/* the xteam mode the fixed-stride path uses for n packed records of len
 * bytes (0 = another kernel, or no device) */
int zscrc_xteam_for(uint64_t len, uint64_t n);
/* name of the kernel zscrc_device_fixed launches for this batch shape
 * (diagnostic; "none" if no device) */
const char *zscrc_fixed_kernel(const void *d_base, uint64_t stride, uint64_t len, size_t n);
/* Diagnostic: fully coalesced non-temporal streaming read of len bytes
 * (multiple of 4096) -- the measured HBM read ceiling on this GPU (grid =
 * grid_mult x CUs of 1024 threads).  d_scratch4: 4 writable device bytes. */
int zscrc_diag_stream_read(const void *d_buf, uint64_t len, void *d_scratch4, int grid_mult,
                           void *stream);
/* Diagnostic: per-wave timestamps of xteam_kernel launches on the current
 * device -- d_buf (device, 32 bytes per wave of the grid: entry, after the
 * LDS table fill, end, in s_memrealtime ticks of 100 MHz, and the wave's
 * record / part count) or NULL to stop. */
int zscrc_diag_wave_times(void *d_buf);
/* Diagnostic: phase end times of the single-block classify + plan launch of
 * variable commit batches (<= 16,384 records) -- d_buf (device, 8 x 8 bytes:
 * entry, count pass, scatter, plan table, plan scan, plan tail, plan write,
 * end; s_memrealtime ticks of 100 MHz) or NULL to stop. */
int zscrc_diag_classify_times(void *d_buf);
/* Number of gfx950 devices visible (0 if none / no HIP runtime). */
int zscrc_device_count(void);

/* Host byte streams: crc32c(seed, everything passed to update), computed on
 * the GPU chunk by chunk while the caller keeps producing bytes (the shape
 * of crc32_begin / mfile_write / crc32_end, src/mfile.c:270-290, :526-546,
 * and of repack's records-region CRC, src/zeroskip-packed.c:442).  Default:
 * update() copies into pinned staging, the caller may reuse its buffer on
 * return.  ZSCRC_STREAM_NOCOPY: the GPU copies straight from the caller's
 * memory, which must stay valid and unchanged until final() (an append-only
 * mmap).  chunk_bytes 0 = 64 MiB.  final() always frees the stream. */
typedef struct zscrc_stream zscrc_stream;
#define ZSCRC_STREAM_NOCOPY 1u
int zscrc_stream_open(zscrc_stream **s, uint32_t seed, uint64_t chunk_bytes, unsigned flags);
int zscrc_stream_update(zscrc_stream *s, const void *buf, size_t len);
int zscrc_stream_final(zscrc_stream *s, uint32_t *crc);

/* ======================================================================
 * Part 3 -- zeroskip file images (verify-on-open / `consistent` / repack).
 * A commit's CRC covers its span (the bytes since crc32_begin, ending where
 * the commit record starts) followed by the commit record's host-order
 * trailer words (src/zeroskip-file.c:253-350).
 * ====================================================================== */

/* walk / parse results (>= 0) */
#define ZSCRC_ZS_END 0        /* walked to the end of the image            */
#define ZSCRC_ZS_STOPPED 1    /* stopped at a record type the reference walk
                               * does not advance over (record.c:314-325)  */
#define ZSCRC_ZS_TRUNCATED 2  /* a record runs past the end of the image   */
#define ZSCRC_ZS_OVERFLOW 3   /* more commits than `cap`; *n_commits = all  */
#define ZSCRC_ZS_BADSIG 4     /* header signature is not "ZEROSKIP"         */

/* file kinds */
#define ZSCRC_ZS_ACTIVE 0
#define ZSCRC_ZS_FINALISED 1
#define ZSCRC_ZS_PACKED 2

/* Walk an active or finalised file image from its 40-byte header
 * (zeroskip-record.c:283-331) and list every commit's span [off, off+len);
 * the commit record starts at off+len. */
int zscrc_zs_walk(const void *image, uint64_t size, uint64_t *span_off, uint64_t *span_len, size_t cap,
                  size_t *n_commits, uint64_t *end_off);
/* Packed file: [0] = records-region commit span, [1] = pointer-section span
 * (zeroskip-packed.c:70-131, :278-339). */
int zscrc_zs_packed_spans(const void *image, uint64_t size, uint64_t span_off[2], uint64_t span_len[2]);
/* 40-byte header CRC over host-order fields (zeroskip-header.c:105-170). */
int zscrc_zs_header_crc(const void *image, uint64_t size, uint32_t *stored, uint32_t *computed);
/* 61-byte .zsdb CRC over host-order fields (zeroskip-dotzsdb.c:160-235). */
int zscrc_zs_dotzsdb_crc(const void *image, uint64_t size, uint32_t *stored, uint32_t *computed);
/* Device: verify n commits of a device-resident image of image_size bytes.
 * Commit i's span is [d_span_off[i], +d_span_len[i]) and its commit record
 * starts right after it.  d_crc[i] = computed commit CRC, d_status[i] = 1
 * match / 0 mismatch / 2 no commit record there -- also when the span, the
 * 8-byte commit word or a long commit's 24 bytes do not lie inside the image:
 * nothing outside [d_image, d_image + image_size) is ever read. */
int zscrc_device_verify_commits(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                const uint64_t *d_span_len, size_t n, uint32_t *d_crc, uint32_t *d_status,
                                void *stream);

/* Device: as zscrc_device_verify_commits, but span i's CRC continues from
 * d_seed[i] (a crc32c value, crc32c(d_seed[i], span) chaining) instead of
 * crc32c(0, 0, 0) = 0.  Resolves the reference's zero-length finalise commit
 * (zeroskip-file.c:253-350 after crc32_end without crc32_begin, mfile.c:534-546):
 * its stored CRC continues from the previous span's CRC.  d_seed NULL = 0. */
int zscrc_device_verify_commits_seeded(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                       const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                       uint32_t *d_crc, uint32_t *d_status, void *stream);

/* Device: zscrc_device_verify_commits_seeded (d_seed may be NULL) with a
 * caller-known bound on the span lengths, as zscrc_device_batch_bounded --
 * the host walk that found the commits knows it. */
int zscrc_device_verify_commits_bounded(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                        const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                        uint64_t max_len, uint32_t *d_crc, uint32_t *d_status, void *stream);

/* Device verdict of n commits (the verifier's question: is every commit
 * good, and which are not?): as zscrc_device_verify_commits_bounded (d_seed
 * may be NULL; max_len a bound on the span lengths, ZSCRC_LEN_UNBOUNDED if
 * none is known -- results never depend on it), but no per-commit output -- *d_nbad (device) = the number
 * of commits whose status would not be 1 (mismatch, or no commit record in
 * the image), and d_bad (device, cap entries) receives the indices of the
 * first cap of them found, in no particular order.  A clean batch writes
 * nothing but the count.  *d_nbad holds the count once the batch is done
 * (in stream order); until then it may hold anything (a bounded batch's
 * kernel counts into a small library counter of the stream's and writes
 * *d_nbad at its end: no zeroing launch before it). */
int zscrc_device_verify_commits_verdict(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                        const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                        uint64_t max_len, uint64_t *d_nbad, uint64_t *d_bad, size_t cap,
                                        void *stream);

/* As zscrc_device_verify_commits_verdict with a caller-known range
 * min_len <= every span length <= max_len (the walk that found the commits
 * knows both): the length classes the range rules out get no launch --
 * NOTBATCHED's ~2 MiB commits run the classify, the long-record parts and
 * their fold only; a range above the 16-lane bound on a batch of at most
 * 16,384 commits classifies in one fused pass (no count or scatter pass).
 * Commits outside the image still count as bad.  The range must hold (a span
 * outside it may go unverified). */
int zscrc_device_verify_commits_verdict_range(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                              const uint64_t *d_span_len, const uint32_t *d_seed, size_t n,
                                              uint64_t min_len, uint64_t max_len, uint64_t *d_nbad, uint64_t *d_bad,
                                              size_t cap, void *stream);

/* Device: compute n commit CRCs (the writer's side, zeroskip-file.c:253-350)
 * and store each one big-endian into its commit record; d_crc[i] receives it.
 * The commit record's header word (type, and for long commits the length
 * words) must already be in the image: only the CRC field is written.
 * d_status (may be NULL): 1 written, 2 not written (no commit record there,
 * or outside the image -- nothing outside the image is read or written).
 * d_crc may be NULL (the CRCs only go into the image). */
int zscrc_device_write_commits(void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                               const uint64_t *d_span_len, size_t n, uint32_t *d_crc, uint32_t *d_status,
                               void *stream);
/* As zscrc_device_write_commits with a caller-known bound on the span
 * lengths (see zscrc_device_batch_bounded). */
int zscrc_device_write_commits_bounded(void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                       const uint64_t *d_span_len, size_t n, uint64_t max_len, uint32_t *d_crc,
                                       uint32_t *d_status, void *stream);

/* Device: the writer's commit CRCs out of place -- d_crc[i] = the CRC
 * zscrc_device_write_commits would store for span i (type read from its
 * commit record), one coalesced 4-byte result per commit; the image is only
 * read (nothing is stored into it).  d_status (may be NULL): 1 a commit
 * record is there, 2 none (or not inside the image).  For images that live
 * in host memory (zscrc_zs_fill_commits): only the CRCs come back over PCIe,
 * the host patches its own image, as the reference writer builds the commit
 * record on the host (src/zeroskip-file.c:315-331). */
int zscrc_device_commit_crcs_bounded(const void *d_image, uint64_t image_size, const uint64_t *d_span_off,
                                     const uint64_t *d_span_len, size_t n, uint64_t max_len, uint32_t *d_crc,
                                     uint32_t *d_status, void *stream);

/* The commit writer for an image in HOST memory (a log file being written,
 * or a whole mmap'd log): every commit CRC computed on the current GPU and
 * stored big-endian into the caller's image (BE32 at +4 of a short commit
 * record, +20 of a long one) -- only the CRCs cross PCIe back, the image is
 * copied to the device once, pipelined in chunks (ZSCRC_FILL_CHUNK, default
 * 64 MiB) with host threads patching earlier chunks.  Span i is
 * [span_off[i], +span_len[i]) of the image; spans sorted and disjoint
 * (ZSCRC_EINVAL otherwise, with the image left unmodified: every span is
 * checked before the first CRC is stored); the commit record's header words must already be
 * in the image (zscrc_device_write_commits' contract), a span without one is
 * counted in no_record and left alone.  max_len: a bound on the span lengths
 * or ZSCRC_LEN_UNBOUNDED; spans longer than a chunk are streamed through the
 * GPU (zscrc_stream_*).  A pinned image (hipHostMalloc / hipHostRegister) is
 * copied straight from the caller's memory, a pageable one through pinned
 * staging filled by `threads` host threads (0 = up to 16).  Synchronous. */
typedef struct zscrc_fill_report {
    uint64_t commits;          /* CRCs written into the image                */
    uint64_t no_record;        /* spans with no commit record after them      */
    uint64_t long_commits;     /* spans streamed on their own                 */
    uint64_t bytes;            /* image bytes sent to the GPU                 */
    uint64_t desc_bytes;       /* descriptor bytes sent (8 per commit)        */
    uint64_t chunks;
    int32_t staged;            /* 1 pageable image via pinned staging, 0 direct */
    int32_t threads;
    double h2d_s;              /* until the last chunk was on the GPU         */
    double total_s;
    double setup_s;            /* until the first chunk's copy was queued     */
} zscrc_fill_report;
int zscrc_zs_fill_commits(void *image, uint64_t size, const uint64_t *span_off, const uint64_t *span_len,
                          size_t n, uint64_t max_len, int threads, zscrc_fill_report *rep);

typedef struct zscrc_zs_report {
    int header_rc;            /* zscrc_zs_header_crc result */
    uint32_t header_stored, header_computed;
    int walk_rc;              /* zscrc_zs_walk / packed_spans result */
    uint64_t end_off;         /* where the walk ended */
    uint64_t n_commits;       /* commits checked on the GPU */
    uint64_t n_bad;           /* commits whose CRC does not match */
    uint64_t first_bad;       /* index of the first bad commit */
} zscrc_zs_report;

/* Host convenience: header check on the CPU, walk, copy the image to the
 * current device, verify every commit there.  Synchronous. */
int zscrc_zs_verify_image(const void *image, uint64_t size, int kind, zscrc_zs_report *rep);

/* `consistent` for one process / one GPU (zsdb_consistent,
 * src/zeroskip.c:1399-1407, and tool/cmd-consistent.c:23-49 are stubs in the
 * reference): every .zsdb / header / commit CRC of the DB directory,
 * recomputed; commits on the GPU.  The multi-GPU driver is
 * zeroskip_amd/consistent.py. */
typedef struct zscrc_consistent_report {
    uint64_t files;               /* zeroskip-* files checked                    */
    uint64_t commits;             /* commit CRCs recomputed on the GPU           */
    uint64_t bytes;               /* file bytes staged to the GPU                */
    uint64_t bad_commits;         /* stored CRC != recomputed                    */
    uint64_t stale_empty_commits; /* zero-length finalise commits hashed from the
                                   * previous span (src/mfile.c:534-546 quirk)  */
    uint64_t header_errors;       /* bad signature or header CRC                 */
    uint64_t walk_errors;         /* record walk stopped early / packed layout   */
    int dotzsdb;                  /* 1 ok, 0 bad, -1 missing                     */
    int consistent;               /* 1 if every check passed                     */
    char first_bad[512];          /* "file:offset: what" of the first problem    */
} zscrc_consistent_report;
int zscrc_zs_consistent(const char *dbdir, zscrc_consistent_report *rep);

/* The device pass of `consistent` over a prepared, device-resident share of
 * a DB (zeroskip_amd/consistent.py's inner loop, in C): the commits of
 * active / finalised files as ONE verdict batch (no per-commit output), up
 * to ZSCRC_CPASS_SPANS raw spans (records-region pieces, pointer sections),
 * one post kernel -- zero-length finalise commits that chain from the
 * previous span's CRC (src/zeroskip-active.c:122 + src/mfile.c:534-546)
 * told from bad ones, the commit trailer after every span whose commit
 * record is in the image checked (src/zeroskip-file.c:266-302) -- and ONE
 * small device->host copy.  All pointers named d_* are device pointers. */
#define ZSCRC_CPASS_SPANS 64
#define ZSCRC_CPASS_LIST 1000
typedef struct zscrc_cpass zscrc_cpass;
typedef struct zscrc_cpass_spec {
    const void *d_image;
    uint64_t image_size;
    size_t n;                     /* commits                                     */
    const uint64_t *d_off;        /* commit spans: image offsets / lengths       */
    const uint64_t *d_len;
    const uint32_t *d_file;       /* file id of each commit                      */
    uint64_t max_len;             /* bound on the span lengths (the host walk's);
                                   * create reads d_len back once and uses the
                                   * true maximum, so a wrong value is harmless.
                                   * d_off / d_len must not change after create
                                   * (the image's bytes may)                      */
    size_t nspans;                /* raw spans                                   */
    const uint64_t *span_off;     /* host arrays: image offset, length, and the  */
    const uint64_t *span_len;     /* image offset of the span's commit record   */
    const int64_t *span_commit;   /* (-1: not in this image -- a split piece)    */
} zscrc_cpass_spec;
typedef struct zscrc_cpass_result {
    uint64_t n_bad;               /* commits that do not verify (undecided incl.),
                                   * minus n_stale                                 */
    uint64_t n_stale;             /* finalise-quirk commits among the first
                                   * min(mismatches, max(4096, min(n, 2^20)))
                                   * the verdict kept -- all of them unless more
                                   * than that many commits mismatch.  The same
                                   * count the digest row carries, independent of
                                   * the order the device listed mismatches in.    */
    uint64_t n_undecided;         /* zero-length commits after a long span or with a
                                   * long trailer: the caller decides (indices below) */
    int32_t complete;             /* 0: more mismatches than one pass lists (4096):
                                   * n_bad + n_stale is still the exact mismatch
                                   * count and n_stale as above, but WHICH ones
                                   * bad[] / stale[] / undecided[] hold depends on
                                   * the order the device found them -- decide such
                                   * a pass another way (consistent.py: the torch
                                   * path)                                          */
    int32_t pad_;
    uint64_t n_listed_bad, n_listed_stale;
    uint64_t bad[ZSCRC_CPASS_LIST];        /* commit indices, ascending, undecided excl. */
    uint64_t stale[ZSCRC_CPASS_LIST];
    uint64_t undecided[ZSCRC_CPASS_SPANS];
    uint32_t span_raw[ZSCRC_CPASS_SPANS];  /* raw register of each span (from 0)         */
    int32_t span_status[ZSCRC_CPASS_SPANS]; /* 1 ok, 0 mismatch, 2 no commit record,
                                             * -1 not checked (span_commit -1)            */
} zscrc_cpass_result;
/* The pass is bound to the device current at create (its buffers live
 * there); run and destroy switch to it and restore the caller's device. */
int zscrc_cpass_create(zscrc_cpass **p, const zscrc_cpass_spec *spec);
/* Synchronous on `stream` (NULL = default). */
int zscrc_cpass_run(zscrc_cpass *p, void *stream, zscrc_cpass_result *res);
/* As zscrc_cpass_run; start_event / end_event (hipEvent_t, may be NULL) are
 * recorded on `stream` before the first launch and right after the copy back
 * is enqueued -- the device's part of the pass, without the host's wait. */
int zscrc_cpass_run_timed(zscrc_cpass *p, void *stream, void *start_event, void *end_event,
                          zscrc_cpass_result *res);
/* The pass in two halves, so the host's reading of pass k overlaps the
 * device's pass k + 1: submit enqueues everything on `stream` (events as
 * zscrc_cpass_run_timed) with the copy back into host slot `slot` (0 or 1)
 * and returns at once; collect waits for that slot's copy and fills `res`.
 * A slot holds one submitted pass until it is collected (ZSCRC_EINVAL
 * otherwise).  Passes run in submission order: a pass enqueued on a stream
 * other than the previous pass's first waits (on the device) for what was
 * already on that stream, which must still exist.  A submit's end_event
 * (may be NULL) is also what its collect waits on: record it again only
 * after that collect. */
int zscrc_cpass_submit(zscrc_cpass *p, void *stream, void *start_event, void *end_event, int slot);
int zscrc_cpass_collect(zscrc_cpass *p, int slot, zscrc_cpass_result *res);
/* The pass's digest as a fixed-shape int64 row in DEVICE memory, for ranks
 * that all-gather their digests over RCCL (one collective, one copy to the
 * host, no host round trip inside the pass): [commits, n_bad, n_stale,
 * listed bad, listed stale, pieces, flags (1 more mismatches than the pass
 * lists, 2 commits left undecided: the caller decides them itself)], then
 * `listed` (file id, record offset) pairs of bad commits in ascending commit
 * order, `listed` pairs of stale finalise commits, and `pmax` (file id, piece
 * code, length, raw register) quadruples -- the span's own piece code and
 * raw register when span_commit was -1, else checked[0..3] (ok, bad, tail
 * ok, tail bad; a tail = piece code -1) and 0.  Row length: 7 + 4 listed +
 * 4 pmax. */
typedef struct zscrc_cpass_row_spec {
    const int64_t *d_rec;      /* device, n: each commit's record offset in its file */
    const int64_t *piece_fid;  /* host, nspans: file id of each span              */
    const int64_t *piece_code; /* host, nspans: piece index (>= 0) or -1 (tail)   */
    uint32_t listed;           /* pairs per list (<= ZSCRC_CPASS_LIST is what the pass keeps) */
    uint32_t pmax;             /* piece slots (>= nspans)                          */
    int64_t checked[4];
} zscrc_cpass_row_spec;
int zscrc_cpass_set_row(zscrc_cpass *p, const zscrc_cpass_row_spec *spec);
/* Enqueue one pass and its row into d_row (device, row length int64);
 * nothing is copied to the host and nothing waits.  The row is built by the
 * pass's post kernel (its last workgroup): no launch of its own. */
int zscrc_cpass_submit_row(zscrc_cpass *p, void *stream, void *start_event, void *end_event, int64_t *d_row);
void zscrc_cpass_destroy(zscrc_cpass *p);

/* End to end from host memory: every CRC of n zeroskip file images (mmap'd
 * files; kinds[i] = ZSCRC_ZS_ACTIVE / _FINALISED / _PACKED) -- header, record
 * walk and every commit of active / finalised files, records-region and
 * pointer-section commits of packed files.  Multi-GPU in one process: the
 * DB's bytes are cut into one equal share per device slot (records regions
 * of packed files split across slots, their piece registers folded on the
 * host with zscrc_shift); each slot checks its share in groups of at most
 * ZSCRC_FILES_GROUP bytes (default 8 GiB, at most half the device's free
 * memory).  `threads` host threads in all (0 = up to 16) walk the files and
 * copy them into pinned staging; the H2D copies and the verification
 * overlap with that work.  Synchronous. */
#define ZSCRC_FILES_BAD_HEADER 1
#define ZSCRC_FILES_BAD_WALK 2
#define ZSCRC_FILES_BAD_COMMIT 3
typedef struct zscrc_files_report {
    uint64_t files, commits, bytes;
    uint64_t bad_commits;         /* stored CRC != recomputed                    */
    uint64_t stale_empty_commits; /* zero-length commits hashed from the previous
                                   * span's CRC (src/mfile.c:534-546 quirk)      */
    uint64_t header_errors;       /* bad signature or header CRC                 */
    uint64_t walk_errors;         /* walk stopped early / packed layout          */
    uint64_t first_bad_file;      /* file index of the first problem, ~0 = none  */
    uint64_t first_bad_off;       /* its offset: commit record / walk stop / 0   */
    int32_t first_bad_what;       /* ZSCRC_FILES_BAD_*, 0 = none                 */
    int32_t threads;              /* host threads used                           */
    int32_t staged;               /* 1: copies through pinned staging (ZSCRC_FILES_STAGE=1),
                                   * 0: pageable H2D straight from the images    */
    double copy_s;                /* start of the pipeline -> last byte on the GPU */
    double verify_tail_s;         /* last byte on the GPU -> every verdict back  */
    double total_s;               /* the whole call                              */
    int32_t devices;              /* device slots used (zscrc_set_devices)       */
} zscrc_files_report;
int zscrc_zs_verify_files(const void *const *images, const uint64_t *sizes, const int *kinds, size_t n,
                          int threads, zscrc_files_report *rep);
/* Device slots of zscrc_zs_verify_files / zscrc_zs_consistent: n device ids
 * (an id may repeat: two slots on one GPU); n = 0 restores the default --
 * env ZSCRC_DEVICES ("0,1,2"), else every visible gfx950 device. */
int zscrc_set_devices(const int *ids, int n);
/* The slots a call would use now: writes up to cap ids, returns their count
 * (or a negative status). */
int zscrc_files_devices(int *ids, int cap);
/* Frees the pinned staging, device buffers, streams and events the library
 * keeps between calls: the file APIs', zscrc_zs_fill_commits' and the
 * drop-in symbols' scalar offload (the next call that needs them allocates
 * them again). */
void zscrc_release_cache(void);

/* Packed-file writer: the repack output path with its CRCs on the GPU.
 * Same byte layout and CRC lifecycle as zs_packed_file_new_from_memtree
 * (src/zeroskip-packed.c:384-473; from_packed_files :617-742):
 *   header (CRC over host-order fields, zeroskip-header.c:30-94)
 *   crc32_begin; records in caller order, pointer i = file offset of record i
 *   records-region commit (short, or long above 16 MiB: zeroskip-file.c:253-350)
 *   crc32_begin; count + pointers (big-endian); final commit.
 * Records are serialised straight into pinned staging chunks; each full chunk
 * is copied to the GPU and checksummed there while the host writes it to the
 * file and serialises the next one -- the reference's one huge crc32_end over
 * the records region (packed.c:442, mfile.c:534-546) never runs on the CPU.
 * Keys must arrive in key order (the caller's merge, as memtree_walk_forward
 * hands them over).  chunk_bytes 0 = 64 MiB. */
typedef struct zscrc_packer zscrc_packer;
#define ZSCRC_PACK_FSYNC 1u /* fsync the file on close (mfile_flush's msync) */
int zscrc_pack_open(zscrc_packer **pk, const char *path, const uint8_t uuid[16], uint32_t startidx,
                    uint32_t endidx, uint64_t chunk_bytes, unsigned flags);
/* key/value record (zs_file_write_keyval_record, zeroskip-file.c:188-247), or
 * a delete record when val is NULL (zs_file_write_delete_record, :352+) */
int zscrc_pack_add(zscrc_packer *pk, const void *key, uint64_t keylen, const void *val, uint64_t vallen);
/* n records in one call (no per-record crossing of a language boundary):
 * record i = key bytes keys + key_off[i] (key_len[i]) and value vals +
 * val_off[i] (val_len[i]); vals NULL, or val_off[i] == ~0, writes a delete. */
int zscrc_pack_add_batch(zscrc_packer *pk, const void *keys, const uint64_t *key_off, const uint64_t *key_len,
                         const void *vals, const uint64_t *val_off, const uint64_t *val_len, size_t n);
typedef struct zscrc_pack_report {
    uint64_t records;       /* pointers written                          */
    uint64_t region_bytes;  /* records region (span of the first commit) */
    uint64_t file_bytes;    /* size of the packed file                   */
    uint32_t region_crc;    /* crc32c(0, records region)                 */
    uint32_t pointers_crc;  /* crc32c(0, count + pointers)               */
    uint32_t commit_crc;    /* stored CRC of the records-region commit   */
    uint32_t final_crc;     /* stored CRC of the final commit            */
} zscrc_pack_report;
/* Writes the commits and the pointer section, closes the file and frees the
 * writer (also on error, after which the file is removed). */
int zscrc_pack_close(zscrc_packer *pk, zscrc_pack_report *rep);
/* Abandons a packing: frees the writer and removes the file without writing
 * any commit (a partial repack never looks valid). */
int zscrc_pack_abort(zscrc_packer *pk);

/* Record lister: the key / value (or delete) records of a file image --
 * active / finalised: the record walk (zeroskip-record.c:283-331), commits
 * skipped; packed: the pointer section's order (zeroskip-packed.c:70-131).
 * Offsets are into the image; val_off == ZSCRC_ZS_DELETED marks a delete.
 * Returns ZSCRC_ZS_END (walked to the end; packed: ZSCRC_OK), STOPPED,
 * TRUNCATED, or OVERFLOW with *n_records = all records when cap is short. */
#define ZSCRC_ZS_DELETED UINT64_MAX
typedef struct zscrc_zs_record {
    uint64_t key_off, key_len, val_off, val_len;
} zscrc_zs_record;
int zscrc_zs_records(const void *image, uint64_t size, int kind, zscrc_zs_record *recs, size_t cap,
                     size_t *n_records);
/* The 61-byte .zsdb of zs_dotzsdb_update_end (zeroskip-dotzsdb.c:477-555),
 * CRC over the host-order fields. */
int zscrc_zs_dotzsdb_build(uint64_t offset, const char *uuidstr, uint32_t curidx, uint8_t out[61]);

/* zsdb_repack (src/zeroskip.c:1419-1571) over a DB directory, in one call:
 * finalised files present -> all of them merged (later record of a key
 * wins, deletes kept) into one packed file; else two or more packed files
 * -> the first two of the reference's pflist (the two newest; the older of
 * the two wins a key present in both, a winning delete drops the key); the
 * merged sources unlinked; .zsdb rewritten with its CRC.  The DB's update
 * lock, .zsdb.lock, is created with O_EXCL before anything is read and held
 * until the new .zsdb is renamed from it (zs_dotzsdb_update_begin / _end):
 * ZSCRC_EBUSY if it is already held.  The packed file is written as
 * "<path>.tmp" and renamed into place before any source is unlinked (a
 * source of the same name -- one finalised file -- is replaced, never
 * unlinked).  Keys sorted on
 * `threads` host threads (0 = up to 16); the packed file's records-region
 * and pointer CRCs computed on the GPU (zscrc_pack_*).  flags:
 * ZSCRC_PACK_FSYNC. */
typedef struct zscrc_repack_report {
    int32_t branch;             /* 0 nothing to pack, 1 finalised files, 2 packed files */
    uint32_t startidx, endidx;  /* index range of the new packed file            */
    uint64_t files_merged;
    uint64_t records_in;        /* records listed from the sources               */
    uint64_t records_out;       /* records written                               */
    uint32_t dotzsdb_crc;       /* CRC of the rewritten .zsdb                     */
    zscrc_pack_report pack;     /* the writer's report                           */
    double list_s, merge_s, write_s, total_s;
    char path[4096];            /* the new packed file                           */
} zscrc_repack_report;
/* ZSCRC_REPACK_REFERENCE_COMPAT (flags): branch 2 writes the reference's
 * bytes exactly, including its loss of records: the reference's packed-file
 * iterator sets its `deleted` flag on the first delete it steps onto and never
 * clears it (src/zeroskip-iterator.c:258-259), so every later record of that
 * source is dropped, and a delete that is a source's first record is written
 * as a delete record.  Without the flag (the default) every record is kept:
 * the older file wins a key in both, a winning delete drops the key -- the
 * same bytes as the reference whenever the two files hold no delete. */
#define ZSCRC_REPACK_REFERENCE_COMPAT 2u
int zscrc_zs_repack(const char *dbdir, unsigned flags, int threads, zscrc_repack_report *rep);

#ifdef __cplusplus
}
#endif
#endif /* ZSCRC_H */
