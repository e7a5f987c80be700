/* zscrc_internal.h -- structures shared by the kernels and the host API. */
#ifndef ZSCRC_INTERNAL_H
#define ZSCRC_INTERNAL_H

#include <stdint.h>

/* Global operator-table block (uint32 words), built on the host per device. */
enum {
    GT_S4 = 0,       /* shift(b<<8j, 4): slice-by-4 tables, j = byte position */
    GT_U16 = 1024,   /* shift(b<<8j, 4 + 15*64): word then skip, 16-lane team */
    GT_U64 = 2048,   /* shift(b<<8j, 4 + 63*64): word then skip, 64-lane team */
    GT_Z = 3072,     /* GT_Z + k*1024: shift(b<<8j, 64<<k), k = 0..5          */
    GT_POW2 = 3072 + 6 * 1024, /* 64 words: x^(8*2^k) mod P, k = 0..63          */
    GT_U2 = 3072 + 6 * 1024 + 64, /* shift(b<<8j, 4 + 64): word then skip, 2-lane team */
    GT_Z192 = 3072 + 6 * 1024 + 64 + 1024, /* shift(b<<8j, 192): run rounds of burst_kernel */
    GT_WORDS = 3072 + 6 * 1024 + 64 + 2 * 1024,
};

namespace zs {

struct RecDesc;

struct BatchDesc {
    const uint8_t *base;
    const uint64_t *off;  /* NULL -> rec * stride        */
    const uint64_t *len;  /* NULL -> fixed_len           */
    const uint32_t *seed; /* NULL -> fixed_seed          */
    uint32_t *out;
    uint64_t n;
    uint64_t stride;
    uint64_t fixed_len;
    uint64_t last_len;    /* ~0 = none; else length of record n-1 */
    uint64_t len_lo;      /* process records with len_lo <= len <= len_hi */
    uint64_t len_hi;
    uint32_t fixed_seed;
    uint32_t xor_io;      /* 0xFFFFFFFF standard CRC, 0 raw registers */
    /* zeroskip commits: commit = 1 (verify) / 2 (write) / 3 (the writer's
     * CRCs, out of place): record i is the span of a commit record that
     * starts right after it; out[i] receives the commit CRC (span +
     * host-order trailer words); verify: status[i] 1 = matches the stored
     * CRC, 0 = mismatch, 2 = no commit record there; write: the CRC is stored
     * big-endian into the commit record; 3: out[] only (status 1 / 2 as the
     * writer's), nothing stored into the image; 4: as 3 with status 3 for a
     * long commit record (the two-pass writer's first pass). */
    uint32_t commit;
    uint32_t *status;     /* may be NULL */
    /* commit mode: bytes of the image at base.  A span whose commit word
     * (8 bytes, 24 for a long commit) does not lie inside the image gets
     * status 2 and nothing outside the image is read or written. */
    uint64_t img_size;
    /* variable batches: class-sorted record descriptors built on the device
     * by classify_kernel; this launch covers class `klass`, i.e. entries
     * [sum(class_count[<klass]), +class_count[klass]) */
    const struct RecDesc *desc;
    const uint32_t *class_count;
    uint32_t klass;
    /* class 0 of a variable batch, direct_max != 0: the class kernel walks the
     * caller's off/len/seed arrays itself and skips records longer than
     * direct_max (the other classes' kernels take them); no class-0 list */
    uint64_t direct_max;
    /* split != 0: this class may be split into parts (plan_kernel decides
     * from the class's record count and bytes, plan[klass]); part p of
     * record part_rec[p] covers part p - part_base[rec] of it (split_part:
     * the first part the rest of len / unit, then unit bytes each);
     * raw part registers go to part_out[p], part_fold_kernel folds them */
    uint32_t split;
    uint32_t opt;         /* tuning bits: 1 = no three-chain five-piece bursts, 2 = no multi64_kernel,
                             64 = class-3-only range verdicts through the classify, parts and
                             fold launches instead of xteam_kernel MODE 3 + nbv_fold_kernel
                             (OPT_NO_NBV),
                             4 / 8 = qteam_kernel with XOR3 grouping 1 / 2,
                             16 = team_kernel<16>'s two-level walk with XOR3 grouping 2,
                             1024 = direct burst batches without the descriptor prefetch,
                             2048 = no run rounds in commit bursts,
                             4096 / 8192 = diagnostics of the run rounds (no chains / no
                             trailer and result stores; results wrong),
                             32768 = bounded commit batches on burst_kernel instead of
                             commit_kernel, 65536 = split class 3 on team_kernel<64>
                             instead of xteam_kernel's parts mode, 131072 = four parts
                             per wave there instead of two (no segment plan), 256 = class 3
                             parts cut per record instead of the segment plan
                             (SplitPlan::seg), 262144 = diagnostic: multi64_kernel
                             stores its results into one L2-resident window (wrong results),
                             524288 = small variable batches classify in two multi-block
                             passes and plan launches instead of one single-block launch,
                             1 << 20 = diagnostic: multi64 without hashing (the load + store
                             shape alone, wrong results), 1 << 21 = multi64d_kernel (results
                             staged in LDS per group of chunks, one contiguous write),
                             1 << 22 = commit_kernel with static rounds (not dealt per
                             workgroup), 1 << 23 = multi64_kernel's static walk (chunks not
                             dealt per workgroup), 1 << 24 = qteam_kernel's static walk on big
                             batches too (not parts dealt per workgroup: qteam_dyn_kernel +
                             qfold_kernel), 1 << 25 = parts dealt on small batches too,
                             1 << 26 = spans on xteam_kernel's static walk (two segments per
                             wave, not 16 dealt per workgroup), 1 << 27 = class-3 segment
                             plans dealt per workgroup too (g_xdeal segments per wave; default
                             one per wave, static), 1 << 28 = no fused class-3-only classify
                             (Classify::only3), 1 << 29 = bounded commit batches on one
                             commit_kernel (not the run-only kernel), 16384 = the run-only
                             kernel lists its other rounds for a second commit_kernel launch
                             (instead of hashing them one lane per commit), 1 << 31 = the
                             run-only kernel at 12 waves per CU (not 16);
                             OPT_XDEAL (1 << 30) is set
                             by the span launches themselves, not a tuning bit */
    uint32_t *part_out;
    /* commit verdict mode (bad_count != NULL): no per-record out / status;
     * every commit whose status is not 1 is counted in *bad_count and its
     * index stored in bad_idx[<bad_cap] (any order) */
    unsigned long long *bad_count;
    uint32_t bad_prezeroed;  /* verdict: *bad_count already 0 on the stream (no memset launch) */
    uint64_t *bad_idx;
    uint64_t bad_cap;
    const struct SplitPlan *plan;
    const uint32_t *part_base;
    const uint32_t *part_rec;
    /* segment plans (SplitPlan::seg): each record's first byte in the
     * class's bytes laid end to end (part_fold_kernel's last-part shift) */
    const uint64_t *rec_start;
    const uint32_t *seg_first; /* segment plans: first part of segment w */
    /* commit_kernel's run-only form (16 waves per CU): round_mode 3 = every
     * round that is not a run round hashed one lane per commit in the same
     * launch; 1 = such rounds appended to round_list (*round_count, zeroed
     * before) and 2 = commit_kernel takes its rounds from that list */
    int round_mode;
    uint32_t *round_list;
    uint32_t *round_count;
    /* commit_kernel verdict without a zeroing launch: bad_count points at a
     * library counter pair that is 0 at rest (count, then workgroups done);
     * the last workgroup out moves the count to *bad_publish (the caller's)
     * and leaves both at 0 */
    unsigned long long *bad_publish;
};

/* A fixed-stride batch for xteam_kernel (what it reads of a BatchDesc: few
 * kernel arguments, few SGPRs).  last_len = fixed_len when there is none. */
struct XDesc {
    const uint8_t *base;
    uint32_t *out;
    uint64_t n;
    uint64_t stride;
    uint64_t fixed_len;
    uint64_t last_len;
    uint32_t seed;
    uint32_t xor_io;
};

/* qteam_dyn_kernel (tuning bit 1 << 24): records cut into np parts of P
 * 1 KiB steps, each workgroup's units dealt by an LDS counter */
struct QDyn {
    uint32_t *part_out; /* raw register of part p of record r at r * np + p */
    uint32_t P;         /* 1 KiB steps per part (part 0: the rest)          */
    uint32_t np;        /* parts per record                                */
    /* lds_fold != 0: the part registers stay in LDS (a workgroup's records
     * x np fit QDYN_LDS_PARTS) and each workgroup folds its own records at
     * its end with K / K_last -- no part_out, no qfold_kernel launch */
    uint32_t lds_fold;
    uint32_t K, K_last;
};
/* part registers a qteam_dyn_kernel workgroup can hold in LDS: the 12 KiB
 * after fill_lds<16>'s four Z tables, less the 16 bytes of its counter */
constexpr uint32_t QDYN_LDS_PARTS = (163840u - (135168u + 4u * 4096u) - 16u) / 4u;
constexpr uint32_t OPT_QFOLD_LAUNCH = 32u; /* tuning: qteam_dyn's fold as a second launch */
constexpr uint32_t OPT_WRITE_TWO_PASS = 512u; /* tuning: bounded commit writer as CRC array + scatter launch */

/* Up to SPANS_MAX spans in one xteam_kernel launch (zscrc_device_spans):
 * span s is segments [first[s], first[s+1]) of the launch, seg[s] bytes each
 * from base[s], the last one last[s]; block 0 presets *out[s] = preset[s]
 * (the constant terms the fold XORs into). */
constexpr int SPANS_MAX = 8;
constexpr uint32_t OPT_XSTATIC = 1u << 26; /* tuning: spans on the static walk           */
constexpr uint32_t OPT_XDEAL_PARTS = 1u << 27; /* tuning: class-3 segment plans dealt too */
constexpr uint32_t OPT_NO_ONLY3 = 1u << 28;    /* tuning: no fused class-3-only classify */
constexpr uint32_t OPT_NO_RUNSPLIT = 1u << 29; /* tuning: bounded commit batches in one commit_kernel */
constexpr uint32_t OPT_RO12 = 1u << 31;        /* tuning: the run-only commit_kernel at 12 waves per CU */
constexpr uint32_t OPT_RO_LIST = 1u << 14;     /* tuning: its other rounds listed for a second launch */
constexpr uint32_t OPT_XDEAL = 1u << 30;   /* internal: this batch is a span's dealt segments */
struct XMulti {
    uint32_t k;
    uint32_t preset[SPANS_MAX];
    const uint8_t *base[SPANS_MAX];
    uint64_t seg[SPANS_MAX];
    uint64_t last[SPANS_MAX];
    uint64_t first[SPANS_MAX + 1];
    uint32_t *out[SPANS_MAX];
};

/* Parts of a split length class for xteam_kernel (MODE 2): part w of the
 * class list's record part_rec[w] covers bytes [(w - part_base[rec]) * unit,
 * +unit) (the last part the rest); raw registers to part_out[w] (folded by
 * part_fold_kernel); the count of parts comes from plan[klass] on the device. */
struct XParts {
    const uint8_t *base;
    const struct RecDesc *desc;
    const uint32_t *class_count;
    uint32_t klass;
    uint32_t xor_io;
    const struct SplitPlan *plan;
    const uint32_t *part_base;
    const uint32_t *part_rec;
    uint32_t *part_out;
    const uint64_t *rec_start; /* segment plans: see SplitPlan::seg */
    const uint32_t *seg_first; /* segment plans: first part of segment w */
    uint32_t seg;              /* the plan's seg (read on the device)     */
    uint32_t first_rec;        /* the class's first record in desc (device) */
    uint64_t U;                /* the plan's unit / segment bytes (device)  */
    /* MODE 3, a class-3-only commit verdict in one launch (no classify, no
     * plan, no fold launch): every workgroup scans the caller's lengths
     * itself, wave w hashes segment w of the commits' bytes laid end to end;
     * a commit in one segment is finished by its wave; a longer one's parts
     * are stored (head[j]: a commit's first part, cont[j]: the part at
     * segment j's start) for nbv_fold_kernel, which folds and checks them.
     * The verdict counts into vpair (count, blocks done; 0 at rest); the
     * fold launch's last block moves the count to *publish. */
    const uint64_t *off3, *len3;
    const uint32_t *seed3; /* NULL: seed 0 */
    uint64_t n3, img_size;
    uint32_t *nbv;    /* head[nseg], then cont[nseg] */
    uint64_t *rstart; /* the commits' starts end to end, [n3] = their total */
    unsigned long long *vpair, *publish;
    uint64_t *bad_idx;
    uint64_t bad_cap;
    uint32_t nseg;
    uint64_t unit_min;
    uint64_t seg_lo, seg_hi, G; /* per wave, set on the device */
};
/* MODE 3's commit limit: four lengths per thread of the workgroup's scan */
constexpr uint32_t NBV_MAX = 4096;
constexpr uint32_t NBV_PARTS_MAX = 62; /* parts per segment (one lane each) */
constexpr uint32_t OPT_NO_NBV = 64u; /* tuning: class-3-only range verdicts through classify + parts + fold */

/* consistent's device post pass (zscrc_cpass, cpass_post_kernel): the
 * verdict's bad list classified (stale finalise commit / bad / undecided),
 * the whole raw spans' commit trailers checked. */
constexpr uint32_t CPASS_SPANS = 64;
/* cpass_post_kernel<true>'s last workgroup: one rank's digest of a consistent
 * pass as the fixed-shape
 * int64 row the ranks all-gather (zeroskip_amd/consistent.py Consistent._pack):
 * [commits, n_bad, n_stale, listed bad, listed stale, pieces, flags]
 * + listed x (file, record offset) of bad commits, ascending commit index
 * + listed x (file, record offset) of stale finalise commits
 * + pmax x (file, piece, length, raw register). */
constexpr uint32_t ROW_HEAD = 7;
constexpr uint32_t ROW_FLAG_INCOMPLETE = 1, ROW_FLAG_UNDECIDED = 2;
struct CPassRowArgs {
    const uint8_t *blk;          /* the pass's device block (cpass_post_kernel's output) */
    uint64_t off_raw, off_st, off_flags, off_bad; /* its layout */
    uint32_t list_cap;           /* entries the block lists */
    uint64_t commits;
    const uint32_t *file;        /* file id per commit */
    const int64_t *rec;          /* record offset in its file per commit */
    const int64_t *piece;        /* nspans x (file, piece code, length) */
    uint32_t nspans;
    uint32_t listed, pmax;
    int64_t checked[4];          /* piece codes of checked spans: ok, bad, tail ok, tail bad */
    int64_t *row;
};

struct CPassArgs {
    const uint8_t *base;
    uint64_t img_size;
    const uint64_t *off, *len;   /* commits */
    const uint32_t *file;        /* file id per commit */
    const unsigned long long *nbad;
    const uint64_t *bad;         /* the verdict's list (first `cap` of *nbad) */
    uint64_t cap;
    uint32_t *flags;             /* per listed entry: 0 bad, 1 stale, 2 undecided (host) */
    uint64_t *bad_out;           /* the first `out_cap` entries of bad[], beside flags, for */
    uint64_t out_cap;            /* the one copy back (flags holds out_cap entries)         */
    unsigned long long *nstale;  /* stale count over all min(*nbad, cap) entries */
    unsigned long long *ticket;  /* workgroups done (the last one publishes) */
    uint32_t nspans;
    const uint32_t *span_raw;    /* raw registers from 0 */
    const int64_t *span_commit;  /* image offset of the span's commit record, -1 = none here */
    const uint32_t *span_init;   /* shift(~0, span length): the register of ~0 after the span */
    int32_t *span_status;        /* 1 ok, 0 mismatch, 2 no commit record, -1 not checked */
    unsigned long long *next_counters; /* the next pass's [nbad, nstale, ticket]: zeroed here */
    /* host_nbad != NULL: flags / bad_out / span_status point into a pinned
     * host block, and the kernel also writes *nbad, the stale count
     * (host_nbad[1], by the last workgroup) and the span registers there
     * (host_raw) -- no copy back after it */
    uint64_t *host_nbad;
    uint32_t *host_raw;
    CPassRowArgs row;            /* row.row != NULL: build the digest row too */
};

struct RecDesc {
    uint64_t off;
    uint64_t len;
    uint32_t seed;
    uint32_t rec;         /* index in the caller's batch */
};


/* Offset of a commit descriptor whose span or commit word lies outside the
 * image (classify_kernel writes it with length 0; status 2). */
constexpr uint64_t NO_COMMIT_OFF = ~0ull;

/* How a length class is split (written by plan_kernel on the device). */
struct SplitPlan {
    uint64_t unit;   /* bytes per part (the FIRST part of a record: the rest,
                      * 1..unit bytes, so every later part is exactly unit) */
    uint32_t parts;  /* work items: parts in all, or records when direct     */
    uint32_t direct; /* 1 = enough records: no split                          */
    uint32_t K;      /* x^(8 unit) mod P: the part fold's Horner multiplier   */
    /* seg = 1 (class 3 on xteam_kernel): the class's bytes laid end to end
     * are cut into `nseg` segments of `unit` bytes, one per wave, and a part
     * is a segment's piece of one record -- every wave gets the same bytes
     * whatever the record lengths.  A record's parts: a partial first one,
     * full segments, a partial last one (part_fold_kernel shifts the Horner
     * sum by x^(8 |last part|)).  seg = nseg, 0 = parts cut per record. */
    uint32_t seg;
};

struct PlanArgs {
    const uint32_t *count; /* class sizes */
    const uint64_t *bytes; /* class byte totals */
    const struct RecDesc *desc;
    uint32_t klass;
    uint32_t target;       /* items wanted: two per team of the launch */
    uint64_t unit_min;     /* smallest part worth a team */
    uint32_t always_split; /* never direct: every record one part at least (xteam parts) */
    SplitPlan *plan;
    uint32_t *part_base;   /* per record of the class: its first part */
    uint32_t *part_rec;    /* per part: its record */
    const uint32_t *gtab;  /* operator tables (x^(8 2^k) for K) */
    /* segment plan (SplitPlan::seg) when nseg != 0 and the class's records
     * + nseg parts fit the part arrays (max_parts) */
    uint32_t nseg;
    uint32_t max_parts;
    uint64_t *rec_start;   /* per record: first byte in the class laid end to end */
    uint32_t *seg_first;   /* nseg + 1 entries: first part of each segment */
};

struct Classify {
    const uint64_t *off;
    const uint64_t *len;
    const uint32_t *seed; /* NULL -> 0 */
    uint64_t n;
    uint64_t bound[3];    /* class c holds bound[c-1] < len <= bound[c] */
    uint32_t *count;      /* [0..3] class sizes, [4..7] scatter cursors; zeroed */
    uint64_t *bytes;      /* [0..3] class byte totals; zeroed */
    RecDesc *desc;        /* n entries, class-sorted after the scatter pass */
    int pass;             /* 0 = count, 1 = scatter */
    int direct_ok;        /* the class-0 kernel reads the caller's arrays
                             (BatchDesc::direct_max): no class-0 scatter, and
                             no scatter pass at all when every record is
                             class 0 */
    int commit;           /* commit batch: spans outside img_size become
                             empty no-commit descriptors (NO_COMMIT_OFF) */
    uint64_t img_size;
    /* single = 1 (small batches, one block): both passes in one launch, the
     * counters written rather than accumulated (no zeroing needed), then the
     * split plans of classes 2 and 3 (plan[0], plan[1]; target 0 = none)
     * from the block's own counts -- one launch instead of two classify
     * passes and two plan launches */
    int single;
    PlanArgs plan[2];
    /* commit verdict batches: the bad-commit counter, zeroed by the first
     * classify launch (the class kernels run after it on the stream) */
    unsigned long long *zero_count;
    /* verdict batches whose class 0 gets no launch (the caller's length
     * range starts above it): the scatter counts every commit outside the
     * image into zero_count / bad_idx itself */
    int verdict_nocommit;
    uint64_t *bad_idx;
    uint64_t bad_cap;
    /* only3 = 1 (single, verdict_nocommit, a range above class 2 and a
     * class-3 segment plan): no count or scatter pass -- one pass writes
     * the class-3 list in record order (a commit outside the image: counted
     * into the verdict, an empty NO_COMMIT_OFF entry with no parts) with
     * each record's start, then the plan from the values in registers */
    int only3;
};

/* K fixed-stride batches of one launch (zscrc_device_fixed_multi): batch b
 * is base[b] / out[b]; stride, length, seed and count come from BatchDesc. */
constexpr int MULTI_MAX = 64;
struct MultiBatch {
    uint32_t nb;
    const uint8_t *base[MULTI_MAX];
    uint32_t *out[MULTI_MAX];
    /* a device word a store with nothing to write goes to (multi64_kernel's
     * lanes past a batch's last record): the stores stay unconditional */
    uint32_t *sink;
};

struct SpanFold {
    const uint32_t *part; /* W raw segment registers */
    uint32_t *out;
    uint32_t w;
    uint32_t k;           /* x^(8*SEG) */
    uint32_t kp2[32];     /* k^(2^b)   */
    uint32_t x_last;      /* x^(8*len of last segment) */
    uint32_t x_total;     /* x^(8*span len) */
    uint32_t r0;          /* initial register */
    uint32_t xor_out;
};

/* The folds of the spans of one zscrc_device_spans launch (blockIdx.y = span). */
struct SpanFolds {
    SpanFold f[SPANS_MAX];
};

} /* namespace zs */

#endif
