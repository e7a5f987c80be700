#!/usr/bin/env python3
"""CRC-32C throughput on device-resident batched records (BASELINE.json metric).

Default workload (BASELINE.json configs[2], the north-star roofline run): per
GPU, 65,536 chunks x 64 KiB = 4 GiB of random bytes resident in HBM; one step =
one batched CRC-32C pass over all chunks (libzscrc team kernel).  With N > 1
GPUs (one process per GPU, torchrun) every rank owns its own 4 GiB shard (weak
scaling, no data crosses xGMI) and the per-chunk digests are all-gathered over
RCCL inside the timed step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config3]

Other BASELINE configs (parity/measurement runs, same JSON shape):
  config2  1,048,576 x 64 B records (64 MiB): `value` is the cold rate (32
           rotating 64 MiB batches = 2 GiB, beyond the 256 MB L3); warm rate
           (one batch, L3-resident) alongside.
  config4  zsbench replay: 10 M pairs as byte-exact zeroskip log files
           (1,526 files, 10 M commits of 312 B spans); one step = the GPU
           verdict of every commit; per-commit arrays, the GPU writer,
           NOTBATCHED and end-to-end rates (both directions) alongside.
  config5  `consistent` full-DB re-checksum of an ~8 GiB DB (2 packed files of
           3 GiB with long commits, 1,024 finalised files, active file,
           .zsdb); strong scaling: the DB is split across ranks, digests
           all-gathered, split regions folded.

Rank 0 prints ONE JSON line.  `value` = bytes checksummed by all ranks / max
over ranks of the timed wall time, in GiB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from zeroskip_amd import device as zd  # noqa: E402,F401
from zeroskip_amd import zsfile  # noqa: E402
from zeroskip_amd._lib import check, lib  # noqa: E402

METRIC = "CRC32C GiB/s device-resident batched records, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CHUNK = 64 * 1024
NCHUNK = 65536
GIB = float(1 << 30)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def box_info(index: int | None = None) -> dict:
    """What tells one GPU box from another (read-only sysfs of the device
    this rank runs on, taken after the timed region): clock levels, power
    cap, firmware, the card's id.  Config 2 and 4's rates move 10-15 % from
    box to box while the streaming read and config 3 stay level (DESIGN_LOG.md
    1.8), so every line records the box it was measured on."""
    info = {}
    try:
        p = torch.cuda.get_device_properties(torch.cuda.current_device() if index is None else index)
        bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        info["pci"] = bdf
        base = f"/sys/bus/pci/devices/{bdf}"

        def rd(name):
            try:
                with open(os.path.join(base, name)) as f:
                    return f.read().strip()
            except OSError:
                return None
        for key in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk"):
            v = rd(key)
            if v:
                levels = [ln.split(":", 1)[1].strip().rstrip("*").strip() for ln in v.splitlines() if ":" in ln]
                info[key + "_levels"] = levels
        for key in ("power_dpm_force_performance_level", "vbios_version", "unique_id", "current_link_speed",
                    "current_link_width"):
            v = rd(key)
            if v:
                info[key] = v
        hw = os.path.join(base, "hwmon")
        if os.path.isdir(hw):
            for h in sorted(os.listdir(hw)):
                for key in ("power1_cap", "power1_cap_max"):
                    try:
                        with open(os.path.join(hw, h, key)) as f:
                            info[key + "_W"] = round(int(f.read().strip()) / 1e6, 1)
                    except (OSError, ValueError):
                        pass
    except Exception as e:  # a fingerprint never fails a bench line
        info["error"] = repr(e)[:120]
    return info


def host_cores() -> int:
    """CPU threads this process may use: the affinity mask, capped by the
    OMP_NUM_THREADS share the GPU box sets (os.cpu_count() shows the whole
    machine there)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_leg(host: np.ndarray, what: str, offs=None, lens=None, *, n=None, stride=0, fixed_len=0,
            seconds: float = 12.0, sw: bool = False) -> dict:
    """The CPU oracle (the SSE4.2 restatement of src/crc32c.c:370-453, the
    reference's crc32c_hw class) timed on a bounded sample of the workload:
    the sample's records laid end to end, dealt in byte chunks from a counter
    to persistent threads pinned one per physical core (dealt over the L3
    domains) or left to the scheduler, records cut by a chunk boundary joined
    by the zero shift
    (oracle_batch_rate) -- every usable core is the value, one core beside
    it, and a plain read of the same bytes on the same threads (the host
    memory's rate: what an all-core CRC cannot pass).  The last pass's CRCs
    are checked against the per-record oracle."""
    from oracle import oracle
    cores = host_cores()
    cpus = oracle.pick_cpus(cores)
    kw = dict(n=n, stride=stride, fixed_len=fixed_len)
    nbytes = int(lens.sum()) if lens is not None else int(n) * int(fixed_len)
    # all cores pinned (one thread per physical core) and left to the
    # scheduler: the box's other tenants share its cores, and either can be
    # the faster on a given box (profiles/r05/cpu_threads.jsonl)
    legs = [("all", "hw", cores, 0.15, True), ("all_unpinned", "hw", cores, 0.15, False), ("hw", "hw", 1, 0.15, True),
            ("all2", "hw", cores, 0.15, True), ("hw_unpinned", "hw", 1, 0.1, False), ("read", "read", cores, 0.1, True),
            ("read_unpinned", "read", cores, 0.05, False)]
    if sw:
        legs.append(("sw", "sw", 1, 0.15, True))
    res, out_all = {}, None
    for key, impl, threads, share, pin in legs:
        got, el, passes = oracle.batch_rate(host, offs, lens, impl=impl, threads=threads,
                                            cpus=cpus[:threads] if pin else None, budget=seconds * share, **kw)
        res[key] = passes * nbytes / el / GIB
        if key == "all":
            out_all = got
    pinned, unpinned = max(res["all"], res["all2"]), res["all_unpinned"]
    res["all"] = max(pinned, unpinned)
    res["hw"] = max(res["hw"], res["hw_unpinned"])   # the one core at its best too
    res["read"] = max(res["read"], res["read_unpinned"])
    want = oracle.batch(host, offs, lens, impl="hw", threads=cores, **kw)
    if not np.array_equal(out_all, want):
        raise SystemExit("cpu_baseline: the byte-split all-core pass differs from the per-record oracle")
    ideal = res["hw"] * min(cores, 8)
    d = {"value": round(res["all"], 3), "unit": "GiB/s", "cores": cores, "kind": "port",
         "value_1core": round(res["hw"], 3), "host_read_GiBs": round(res["read"], 3),
         "all_pinned": round(pinned, 3), "all_unpinned": round(unpinned, 3),
         "sample": (f"{what}: {nbytes / 2**20:.0f} MiB, repeated on {cores} threads pinned one per physical "
                    f"core ({cpus[:cores]}, two legs of ~{seconds * 0.15:.0f} s) and unpinned (~{seconds * 0.15:.0f} "
                    f"s; value = the fastest leg) and ~{seconds * 0.25:.0f} s on 1 core (pinned and unpinned, "
                    f"the faster) of {cpu_model()} ({os.cpu_count()} threads visible, {cores} usable); "
                    "persistent threads taking byte chunks from a counter, records cut by a chunk boundary "
                    "joined by the zero shift; oracle SSE4.2 crc32c_hw class (src/crc32c.c:370-453)")}
    if sw:
        d["sw_value_1core"] = round(res["sw"], 3)
    if res["all"] < ideal:
        d["scaling_note"] = (f"{res['all'] / res['hw']:.1f}x one core on {cores} threads; a plain read of the "
                             f"same bytes on the same threads runs at {res['read']:.1f} GiB/s, so the all-core "
                             "CRC is bound by host memory bandwidth"
                             if res["all"] >= 0.8 * res["read"] else
                             f"{res['all'] / res['hw']:.1f}x one core on {cores} threads (read of the same bytes "
                             f"{res['read']:.1f} GiB/s): below min(cores, 8)x, not explained by the read rate")
    return d


def spot_check(host_out: np.ndarray, data: torch.Tensor, idx: np.ndarray, stride: int, length: int) -> int:
    """Outside the timed region: the CPU oracle (the checker) recomputes the
    sampled records of the timed call; returns the number of mismatches."""
    from oracle import oracle
    bad = 0
    for i in idx.tolist():
        rec = data[i * stride:i * stride + length].cpu().numpy()
        bad += int(oracle.crc32c_hw(0, rec) != int(host_out[i]))
    return bad


def oracle_check_logs(host: np.ndarray, offs: np.ndarray, lens: np.ndarray, gpu_crc: np.ndarray,
                      stale_per_file: int) -> dict:
    """Outside the timed region, the CPU oracle (the checker,
    oracle/zs_bulk_oracle.c) over a full-size image of [nfiles, size] log
    files: (i) its own record walk of every file (zeroskip-record.c:283-331)
    re-checking every stored commit CRC with the writer's semantics
    (zeroskip-file.c:253-350); (ii) every live commit's CRC recomputed and
    compared with the GPU's per-commit crc array of the same image."""
    from oracle import oracle
    cores = host_cores()
    t0 = time.perf_counter()
    w = oracle.walk_images(list(host), threads=cores)
    commits, ok = int(w[:, 0].sum()), int(w[:, 1].sum())
    clean_walk = bool((w[:, 3] == 0).all() and (w[:, 2] == host.shape[1]).all())
    # the only stored CRCs that do not verify from seed 0: each file's stale
    # zero-length finalise commit, its last (src/mfile.c:534-546)
    stale_last = bool(((w[:, 0] - w[:, 1]) == stale_per_file).all() and
                      (stale_per_file == 0 or (w[:, 5] == w[:, 0] - 1).all()))
    live = lens > 0
    want = oracle.commit_crcs(host.reshape(-1), offs[live], lens[live], threads=cores)
    gpu_bad = int((gpu_crc[live] != want).sum())
    return {"files_walked": int(host.shape[0]), "commits_walked": commits, "commits_verified_ok": ok,
            "stale_finalise": commits - ok, "walk_clean": clean_walk and stale_last,
            "gpu_crcs_compared": int(live.sum()), "mismatches": gpu_bad + (0 if clean_walk and stale_last else 1),
            "checker": "oracle (oracle/zs_bulk_oracle.c): record walk of every file + every live commit's CRC "
                       "recomputed, compared with the GPU's per-commit crc array",
            "check_s": round(time.perf_counter() - t0, 2), "threads": cores}


def oracle_check_db(db, finalised: int) -> dict:
    """Outside the timed region, the CPU oracle over every byte of the
    config-5 DB: each header CRC (zeroskip-header.c:105-170), the .zsdb CRC
    (zeroskip-dotzsdb.c:160-235), its own walk of every active / finalised
    file with every commit re-checked, and each packed file's records region
    (hashed whole on host threads, the pieces joined by the zero shift) and
    pointer section (zeroskip-packed.c:70-131, :278-339, :442)."""
    import struct
    from oracle import oracle
    cores = host_cores()
    t0 = time.perf_counter()
    sig = 0x5A45524F534B4950
    bad_headers = 0
    logs, packed = [], []
    for f in db.files:
        im = f.image
        ver, = struct.unpack(">I", im[8:12].tobytes())
        sidx, eidx, stored = struct.unpack(">III", im[28:40].tobytes())
        bad_headers += int(oracle.header_crc(sig, ver, im[12:28].tobytes(), sidx, eidx) != stored)
        (packed if f.kind == zsfile.PACKED else logs).append(im)
    w = oracle.walk_images(logs, threads=cores)
    regions = [oracle.packed_image(im, threads=cores) for im in packed]
    dz = db.dotzsdb
    off, = struct.unpack(">Q", dz[8:16])
    cur, dstored = struct.unpack(">II", dz[53:61])
    dz_ok = oracle.dotzsdb_crc(sig, off, dz[16:53], cur) == dstored
    commits, ok = int(w[:, 0].sum()), int(w[:, 1].sum())
    region_ok = sum(int(r["records"]["status"] == 1) + int(r["pointers"]["status"] == 1) for r in regions)
    walks_clean = bool((w[:, 3] == 0).all())
    mism = bad_headers + (commits - ok - finalised) + (2 * len(regions) - region_ok) + int(not dz_ok) + \
        int(not walks_clean)
    return {"files": len(db.files), "headers_checked": len(db.files), "commits_walked": commits,
            "commits_verified_ok": ok, "stale_finalise": commits - ok,
            "regions_checked": len(regions), "region_bytes": int(sum(r["records"]["span_len"] for r in regions)),
            "pointer_sections_checked": len(regions), "dotzsdb_ok": bool(dz_ok), "mismatches": int(mism),
            "checker": "oracle (oracle/zs_bulk_oracle.c + zs_format_oracle.c): headers, .zsdb, a record walk of "
                       "every log file with every commit re-checked, every packed records region and pointer "
                       "section hashed whole on host threads",
            "check_s": round(time.perf_counter() - t0, 2), "threads": cores}


def traffic_for(config: str, kernel: str):
    """HBM bytes per launch from the PMC record of THIS kernel
    (profiles/pmc_traffic.json: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes
    of tools/prof_case.py, tools/pmc_traffic.sh + tools/traffic_summary.py),
    or None -- a record taken on another kernel is never reported for this
    one.  Returns (bytes or None, the record's provenance)."""
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        rec = json.load(open(tpath)).get(config)
    except Exception:
        rec = None
    if not rec:
        return None, "no PMC record for this config"
    if rec.get("kernel") != kernel:
        return None, f"PMC record is for {rec.get('kernel')!r}, not {kernel!r}: not reported"
    return rec["bytes_per_launch"], rec.get("record")


def read_ceiling(buf: torch.Tensor, nbytes: int, stream) -> float:
    """Same-GPU measured read ceiling: a fully coalesced non-temporal streaming
    read (libzscrc diagnostic kernel), the best median of 10 over grids of 1
    and 2 workgroups per CU, GB/s."""
    nbytes -= nbytes % 4096
    scratch = torch.zeros(4, dtype=torch.int32, device=buf.device)
    best = 0.0
    for mult in (1, 2):
        rd = []
        for i in range(13):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            check(lib().zscrc_diag_stream_read(buf.data_ptr(), nbytes, scratch.data_ptr(), mult,
                                               stream.cuda_stream), "stream read")
            b.record(stream)
            torch.cuda.synchronize()
            if i >= 3:
                rd.append(a.elapsed_time(b))
        best = max(best, nbytes / (sorted(rd)[len(rd) // 2] * 1e-3) / 1e9)
    return best


class Timer:
    """K timed steps bracketed by barrier + synchronize; max over ranks.

    The kernels' time: one timing-event pair on the kernels' stream around
    the K steps (kern_ms = its span / K: the launches' average duration, the
    gaps between them included).  A pair around every step costs 8 us a step
    on config 3 (0.6237 against 0.6154 ms, profiles/r05/event_cost.json) --
    the events themselves, not the kernel."""

    def __init__(self, world: int, dev, stream):
        self.world, self.dev, self.stream = world, dev, stream

    def run(self, step, steps: int, warmup: int, drain=None) -> float:
        for _ in range(warmup):
            step(None)
        if drain:
            drain()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record(self.stream)
        for _ in range(steps):
            step(None)
        b.record(self.stream)
        if drain:       # outstanding asynchronous work of the steps, inside the timed region
            drain()
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if self.world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = t.item()
        self.kern_ms = [a.elapsed_time(b) / steps]
        return elapsed


def line(args, world, elapsed, total_bytes, config, roofline, scaling="weak", data=None, **extra):
    d = {
        "metric": METRIC,
        "value": round(total_bytes / elapsed / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": data or "synthetic (torch.randint bytes, device-resident)",
        "config": config,
        "roofline": roofline,
    }
    d.update(extra)
    d["box"] = box_info()
    return d


def roof(nbytes: int, kern_ms: float, kernel: str, config: str, read_peak: float | None, note: str | None = None):
    achieved = nbytes / (kern_ms * 1e-3) / 1e9
    if os.environ.get("ZSCRC_OPT", "0") not in ("", "0"):
        kernel += f" [ZSCRC_OPT={os.environ['ZSCRC_OPT']}]"   # another form: no PMC record applies
    traffic, src = traffic_for(config, kernel)
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src, "kernel": kernel,
         "kernel_ms": round(kern_ms, 4), "algorithmic_bytes": nbytes}
    if note:
        r["kernel_note"] = note
    if read_peak:
        r["measured_read_peak"] = round(read_peak, 1)
        r["frac_of_measured_read_peak"] = round(achieved / read_peak, 4)
    return r


# ------------------------------------------------------------------ config 3
def run_config3(args, world, rank, dev, stream):
    g = torch.Generator(device=dev)
    g.manual_seed(0x9E3779B9 + rank)
    data = torch.randint(0, 256, (NCHUNK * CHUNK,), dtype=torch.uint8, device=dev, generator=g)
    # Every rank checksums its own 4 GiB of chunks: independent shards, so no
    # collective inside the steps (round 5 all-gathered every step's digests
    # over RCCL beside the next kernel -- an exchange the path does not have,
    # whose RCCL kernels wait for CUs the persistent kernel holds); the last
    # step's digests are gathered once, after the timed region, and checked
    outs = [torch.empty(NCHUNK, dtype=torch.int32, device=dev) for _ in range(2)]
    nstep = [0]

    def step(ev):
        i = nstep[0] % 2
        nstep[0] += 1
        if ev:
            ev[0].record(stream)
        check(lib().zscrc_device_fixed(data.data_ptr(), CHUNK, CHUNK, 0, outs[i].data_ptr(), NCHUNK,
                                       0, stream.cuda_stream), "zscrc_device_fixed")
        if ev:
            ev[1].record(stream)

    # The same-GPU read ceiling is measured first, right before the warmup:
    # config 3 runs at the package's 1400 W cap, and the power controller's
    # settling after idle (~20-30 ms, longer than 5 warmup steps) would
    # otherwise land in the timed steps (DESIGN_LOG.md 1.6,
    # profiles/r02/sustain*.jsonl); the streaming probe brings the package to
    # its loaded operating point as a sustained checksum job finds it.
    read_peak = read_ceiling(data, NCHUNK * CHUNK, stream)
    tm = Timer(world, dev, stream)
    elapsed = tm.run(step, args.steps, args.warmup)
    kern_ms = float(np.mean(tm.kern_ms))
    out = outs[(nstep[0] - 1) % 2]   # the last timed step's digests
    if world > 1:
        # every rank's digests of the last step, gathered once (untimed)
        gathered = torch.empty(NCHUNK * world, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(gathered, out)
        torch.cuda.synchronize()
        assert torch.equal(gathered[rank * NCHUNK:(rank + 1) * NCHUNK], out)
    # after the timed region, reported beside it (never the value): the
    # kernel over 200 back-to-back calls, the sustained power-capped rate
    sus = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    for a, b in sus:
        a.record(stream)
        check(lib().zscrc_device_fixed(data.data_ptr(), CHUNK, CHUNK, 0, out.data_ptr(), NCHUNK, 0,
                                       stream.cuda_stream), "zscrc_device_fixed")
        b.record(stream)
    torch.cuda.synchronize()
    sus_ms = sorted(a.elapsed_time(b) for a, b in sus)
    sustained = {"kernel_ms_median": round(sus_ms[len(sus_ms) // 2], 4),
                 "kernel_ms_mean": round(float(np.mean(sus_ms)), 4), "calls": len(sus_ms),
                 "note": "200 back-to-back calls after the timed steps (the package at its 1400 W cap; "
                         "DESIGN_LOG.md 1.6); reported only"}
    # the timed call's own outputs: 256 sampled chunks against the oracle
    torch.cuda.synchronize()
    host_out = out.cpu().numpy().view(np.uint32)
    idx = np.unique(np.concatenate([[0, NCHUNK - 1],
                                    np.random.default_rng(rank).integers(0, NCHUNK, 254)]))
    n_bad = spot_check(host_out, data, idx, CHUNK, CHUNK)
    if n_bad:
        raise SystemExit(f"config3: {n_bad} of {idx.size} sampled chunk CRCs differ from the oracle")
    kname = "zs::" + lib().zscrc_fixed_kernel(data.data_ptr(), CHUNK, CHUNK, NCHUNK).decode()
    r = roof(NCHUNK * CHUNK + NCHUNK * 4, kern_ms, kname, "config3", read_peak)
    out_line = line(args, world, elapsed, NCHUNK * CHUNK * world * args.steps,
                    {"workload": "config3: 65536 x 64 KiB chunks per GPU (4 GiB), batched CRC-32C",
                     "records_per_gpu": NCHUNK, "record_bytes": CHUNK,
                     "parallelism": f"shard{world}" + ("; digests gathered once after the timed steps "
                                                       f"({os.environ.get('BENCH_DIST', 'nccl')})" if world > 1 else "")}, r,
                    parity={"sampled_chunks": int(idx.size), "mismatches": n_bad, "checker": "oracle crc32c_hw"},
                    sustained=sustained)
    if rank == 0 and world == 1 and not args.no_cpu:
        # 8,192 of the timed chunks (512 MiB: beyond the host's L3)
        ns = 8192
        out_line["cpu_baseline"] = cpu_leg(data[:ns * CHUNK].cpu().numpy(), f"{ns} x 64 KiB chunks of the workload",
                                           n=ns, stride=CHUNK, fixed_len=CHUNK, sw=True)
    return out_line


# ------------------------------------------------------------------ config 2
def run_config2(args, world, rank, dev, stream):
    """1M x 64 B records per step (one step = one 64 MiB batch).  32 steps run
    as ONE zscrc_device_fixed_multi launch over 64 batches (ZSCRC_MULTI_MAX):
    the launch, the operator-table fill and the HBM ramp are paid once per 64
    batches, every batch is still fully checksummed.  Cold: the 64 batches are
    64 different 64 MiB buffers (4 GiB, beyond the 256 MB L3); warm: the same
    buffer 64 times (L3-resident).  The round-1 form -- single-batch launches
    in one hipGraph -- is timed alongside."""
    from zeroskip_amd import device as zd
    n, rl, rot = 1 << 20, 64, 64   # rot = ZSCRC_MULTI_MAX batches per launch
    g = torch.Generator(device=dev)
    g.manual_seed(0x64 + rank)
    bufs = torch.randint(0, 256, (rot, n * rl), dtype=torch.uint8, device=dev, generator=g)
    outs = torch.empty(rot, n, dtype=torch.int32, device=dev)
    cold_bufs, warm_bufs, out_list = list(bufs), [bufs[0]] * rot, list(outs)

    def launch(b, o, st):
        check(lib().zscrc_device_fixed(b.data_ptr(), rl, rl, 0, o.data_ptr(), n, 0, st.cuda_stream),
              "zscrc_device_fixed")

    def capture(which):
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for k in range(rot):
                launch(bufs[which(k)], outs[k], side)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            cs = torch.cuda.current_stream(dev)
            for k in range(rot):
                launch(bufs[which(k)], outs[k], cs)
        return graph

    replays = max(1, -(-max(args.steps, 100) // rot))
    steps = replays * rot
    a2 = argparse.Namespace(**{**vars(args), "steps": steps})

    def multi(batch_list):
        def step(ev):
            if ev:
                ev[0].record(stream)
            zd.crc_fixed_multi(batch_list, rl, rl, n, outs=out_list)
            if ev:
                ev[1].record(stream)
        return step

    def stepper(graph):
        def step(ev):
            if ev:
                ev[0].record(stream)
            graph.replay()
            if ev:
                ev[1].record(stream)
        return step

    read_peak = read_ceiling(bufs.view(-1), bufs.numel(), stream)   # also settles power (run_config3)
    tm = Timer(world, dev, stream)
    warm_el = tm.run(multi(warm_bufs), replays, max(1, args.warmup // rot + 1))
    warm_ms = float(np.median(tm.kern_ms)) / rot
    elapsed = tm.run(multi(cold_bufs), replays, max(1, args.warmup // rot + 1))
    cold_ms = float(np.mean(tm.kern_ms)) / rot
    # every batch of the last multi launch against plain single-batch launches
    for k in (0, rot // 2, rot - 1):
        ref = torch.empty(n, dtype=torch.int32, device=dev)
        launch(bufs[k], ref, stream)
        torch.cuda.synchronize(dev)
        assert torch.equal(ref, outs[k]), f"multi-batch result of batch {k} differs from a direct launch"
    g_cold = capture(lambda k: k)
    tm_g = Timer(world, dev, stream)
    graph_el = tm_g.run(stepper(g_cold), replays, 1)
    graph_ms = float(np.mean(tm_g.kern_ms)) / rot
    nbytes = n * rl + n * 4
    r = roof(nbytes, cold_ms, "zs::multi64_kernel", "config2", read_peak,
             f"{rot} batches of 1M x 64 B per launch; kernel_ms = launch time / {rot} batches (the algorithmic "
             "bytes and the traffic are per batch)")
    out_line = line(a2, world, elapsed, n * rl * world * steps,
                    {"workload": f"config2: 1,048,576 x 64 B records per GPU (64 MiB) per step; cold: {rot} "
                                 f"rotating batches ({rot * n * rl >> 30} GiB); {rot} steps per "
                                 "zscrc_device_fixed_multi launch",
                     "records_per_gpu": n, "record_bytes": rl, "parallelism": f"shard{world}"}, r,
                    warm={"value": round(n * rl * world * steps / warm_el / GIB, 2), "kernel_ms": round(warm_ms, 4),
                          "achieved_GBs": round(nbytes / (warm_ms * 1e-3) / 1e9, 1),
                          "note": "one batch re-read every step: L3 (Infinity Cache) resident"},
                    graph_of_launches={"value": round(n * rl * world * steps / graph_el / GIB, 2),
                                       "kernel_ms": round(graph_ms, 4),
                                       "achieved_GBs": round(nbytes / (graph_ms * 1e-3) / 1e9, 1),
                                       "note": f"round-1 form: {rot} single-batch short_kernel launches per "
                                               "hipGraph"},
                    amortized=(f"value is amortized over {rot} batches per zscrc_device_fixed_multi launch (launch "
                               "cost, LDS table fill and HBM ramp paid once per launch); the per-batch launch "
                               "form is graph_of_launches"))
    if rank == 0 and world == 1 and not args.no_cpu:
        # 8 of the cold batches (8 M records, 512 MiB: beyond the host's L3)
        h = bufs[:8].cpu().numpy().reshape(-1)
        out_line["cpu_baseline"] = cpu_leg(h, "8 batches of 1,048,576 x 64 B records", n=8 * n, stride=rl,
                                           fixed_len=rl)
    return out_line


# ------------------------------------------------------------------ config 4
def _timed(fn, reps: int, stream) -> float:
    """ms per call of fn: `reps` calls back to back between two HIP events on
    `stream` (as the timed steps of a line run), the median of three such
    blocks, one warm call first.  Back to back, the host's submission of a
    call (Python, ctypes, several launches) overlaps the previous call's
    kernels instead of being counted as idle GPU time."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return float(np.median(ts))


def _timed_ab(fns, reps: int, stream, rounds: int = 3) -> list:
    """ms per call of each fn, measured as _timed does but interleaved: each
    round times every fn once (reps calls back to back between two events);
    the median over rounds."""
    for fn in fns:
        fn()
    torch.cuda.synchronize()
    ts = [[] for _ in fns]
    for _ in range(rounds):
        for k, fn in enumerate(fns):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(reps):
                fn()
            b.record(stream)
            torch.cuda.synchronize()
            ts[k].append(a.elapsed_time(b) / reps)
    return [float(np.median(t)) for t in ts]


def run_config4(args, world, rank, dev, stream):
    """zsbench writeseqtxn replay (10 M pairs as byte-exact log files).  One
    step = the verdict of every commit on the GPU
    (zscrc_device_verify_commits_verdict: commit_kernel, spans bounded by the
    walk, no per-commit output); per-commit crc/status arrays, the writer, the
    NOTBATCHED layout and the host-memory pipelines both ways alongside."""
    from tools import zsdb_gen as zg
    pairs_total = args.pairs
    ppf = zg.pairs_per_file(True)
    nfiles = -(-pairs_total // ppf)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x5EED + rank)
    uuid = bytes(range(16))
    t0 = time.perf_counter()
    img = zg.log_files(uuid, 0, nfiles, ppf, 0, True, gen, dev)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    offs, lens = zg.log_spans(nfiles, ppf, True, True, dev)
    flat = img.view(-1)
    ncommit = offs.numel()
    span_bytes = int(lens.sum().item())
    # the longest span is known to the walk that found the commits (here: the
    # replay's layout), as in consistent.py and zscrc_zs_verify_files
    max_span = int(lens.max().item())
    vout = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(4096, dtype=torch.int64, device=dev))

    def step(ev):
        if ev:
            ev[0].record(stream)
        zsfile.verify_commits_verdict(flat, offs, lens, max_len=max_span, out=vout)
        if ev:
            ev[1].record(stream)

    read_peak = read_ceiling(flat, flat.numel(), stream)   # also settles power (run_config3)
    tm = Timer(world, dev, stream)
    elapsed = tm.run(step, args.steps, args.warmup)
    kern_ms = float(np.mean(tm.kern_ms))
    # the verdict: exactly the stale zero-length finalise commits (one per file)
    nbad = int(vout[0].item())
    stale = torch.nonzero(lens == 0).flatten()
    bad = torch.sort(vout[1][:nbad]).values
    assert nbad == nfiles and torch.equal(bad, stale), (nbad, nfiles)

    # per-commit crc + status arrays (zscrc_device_verify_commits_bounded)
    res = {}

    def arrays():
        res["crc"], res["st"] = zsfile.verify_commits(flat, offs, lens, max_len=max_span)
    arrays_ms = _timed(arrays, 10, stream)
    st = res["st"]
    n_ok = int((st == 1).sum().item())
    assert n_ok + nfiles == ncommit

    # writer side: recompute + store every commit CRC (the image is unchanged;
    # the stale finalise commits are not rewritten)
    offs_w, lens_w = offs[lens > 0].contiguous(), lens[lens > 0].contiguous()
    write_ms = _timed(lambda: zsfile.write_commits(flat, offs_w, lens_w, max_len=max_span, crc=False), 6, stream)
    write_crc_ms = _timed(lambda: zsfile.write_commits(flat, offs_w, lens_w, max_len=max_span), 6, stream)
    # the writer's CRCs out of place (commit mode 3): the kernel of the
    # host-image writer below -- 4 coalesced bytes per commit, no in-place store
    crcs_ms = _timed(lambda: zsfile.commit_crcs(flat, offs_w, lens_w, max_len=max_span), 10, stream)
    want_w = res["crc"][lens > 0]
    assert torch.equal(zsfile.commit_crcs(flat, offs_w, lens_w, max_len=max_span), want_w)

    # NOTBATCHED (zsbench writeseq): one commit per ~2 MiB file, unbounded
    # (device length classes; the spans go to xteam_kernel's parts mode)
    ppf_nb = zg.pairs_per_file(False)
    nf_nb = -(-pairs_total // ppf_nb)
    img_nb = zg.log_files(uuid, 0, nf_nb, ppf_nb, 0, False, gen, dev, batched=False)
    o_nb, l_nb = zg.log_spans(nf_nb, ppf_nb, False, False, dev)
    nbo = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(64, dtype=torch.int64, device=dev))
    # the walk knows the commits' length range: classes outside it get no
    # launch (zscrc_device_verify_commits_verdict_range)
    nb_lo, nb_hi = int(l_nb.min().item()), int(l_nb.max().item())
    nb_arr = {}

    def nb_verdict():
        zsfile.verify_commits_verdict(img_nb.view(-1), o_nb, l_nb, out=nbo, min_len=nb_lo, max_len=nb_hi)

    def nb_verdict_unranged():
        zsfile.verify_commits_verdict(img_nb.view(-1), o_nb, l_nb, out=nbo)

    def nb_arrays():
        nb_arr["crc"], nb_arr["st"] = zsfile.verify_commits(img_nb.view(-1), o_nb, l_nb)
    # interleaved, so no form sees a different power / clock state; blocks of
    # 20 calls (6 could not resolve the forms' ~13 us difference,
    # tools/probes/nb_forms.py)
    nb_ms, nb_unranged_ms, nb_arrays_ms = _timed_ab([nb_verdict, nb_verdict_unranged, nb_arrays], 20, stream,
                                                    rounds=5)
    nb_verdict()
    assert int(nbo[0].item()) == 0
    assert bool((nb_arr["st"] == 1).all())
    nb_bytes = int(l_nb.sum().item()) + 24 * nf_nb
    # the checker on the NOTBATCHED image: every ~2 MiB commit against the oracle
    nb_parity = oracle_check_logs(img_nb.cpu().numpy(), o_nb.cpu().numpy(), l_nb.cpu().numpy(),
                                  nb_arr["crc"].cpu().numpy().view(np.uint32), 0)
    assert nb_parity["mismatches"] == 0, nb_parity
    del img_nb

    # the checker at full size: every file walked and every commit CRC
    # recomputed by the CPU oracle, the GPU's crc array compared
    host = img.cpu()
    parity = oracle_check_logs(host.numpy(), offs.cpu().numpy(), lens.cpu().numpy(),
                               res["crc"].cpu().numpy().view(np.uint32), 1)
    parity["notbatched"] = nb_parity
    if parity["mismatches"] or parity["commits_walked"] != ncommit:
        raise SystemExit(f"config4: the oracle disagrees with the GPU: {parity}")

    # end to end from host memory, both directions
    e2e = {}
    if rank == 0 and not args.no_e2e:
        pinned = torch.empty(host.shape, dtype=torch.uint8, pin_memory=True)
        pinned.copy_(host)
        for kind, src in (("pageable", host), ("pinned", pinned)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            img.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            e2e[f"h2d_{kind}_GBs"] = round(img.numel() / (time.perf_counter() - t0) / 1e9, 2)
        # verify: zscrc_zs_verify_files over the host file images (threaded
        # walks + pinned staging + overlapped H2D + one verify)
        images = list(host.numpy().reshape(nfiles, -1))
        kinds = [zsfile.FINALISED] * nfiles
        zsfile.verify_files(images, kinds)                 # warm: pinned slots, device buffers
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            rep = zsfile.verify_files(images, kinds)
            dt = time.perf_counter() - t0
            best = dt if best is None or dt < best else best
        assert rep["commits"] == ncommit and rep["bad_commits"] == 0, rep
        e2e["verify_files_s"] = round(best, 4)
        e2e["verify_files_GBs"] = round(host.numel() / best / 1e9, 2)
        e2e["verify_files_phases_s"] = {"copy": round(rep["copy_s"], 4), "verify_tail": round(rep["verify_tail_s"], 4),
                                        "total_in_library": round(rep["total_s"], 4)}
        # write: host images -> H2D -> write_commits -> D2H of the images
        back = torch.empty(host.shape, dtype=torch.uint8, pin_memory=True)
        for kind, src, dst in (("pinned", pinned, back), ("pageable", host, torch.empty_like(host))):
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                img.copy_(src, non_blocking=True)
                zsfile.write_commits(flat, offs_w, lens_w, max_len=max_span, crc=False)
                dst.copy_(img, non_blocking=True)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            e2e[f"write_{kind}_s"] = round(min(ts), 4)
            e2e[f"write_{kind}_GBs"] = round(host.numel() / min(ts) / 1e9, 2)
        assert torch.equal(back, pinned)
        # the write pipelined: file-aligned chunks, H2D / writer / D2H each on
        # its own stream, so the two copy directions (PCIe is full duplex)
        # and the kernel overlap chunk by chunk
        fsz = flat.numel() // nfiles
        per = 64
        ow_h, lw_h = offs_w.cpu(), lens_w.cpu()
        chunks = []
        for f0 in range(0, nfiles, per):
            c0, c1 = f0 * fsz, min(nfiles, f0 + per) * fsz
            sel = (ow_h >= c0) & (ow_h < c1)
            chunks.append((c0, c1, (ow_h[sel] - c0).to(dev), lw_h[sel].to(dev)))
        assert sum(int(c[2].numel()) for c in chunks) == int(offs_w.numel())
        s_in, s_k, s_out = (torch.cuda.Stream(dev) for _ in range(3))
        src_f, dst_f = pinned.view(-1), back.view(-1)

        def pipelined():
            for c0, c1, o, ln in chunks:
                with torch.cuda.stream(s_in):
                    flat[c0:c1].copy_(src_f[c0:c1], non_blocking=True)
                    e_in = torch.cuda.Event()
                    e_in.record(s_in)
                s_k.wait_event(e_in)
                with torch.cuda.stream(s_k):
                    zsfile.write_commits(flat[c0:c1], o, ln, max_len=max_span, crc=False)
                    e_k = torch.cuda.Event()
                    e_k.record(s_k)
                s_out.wait_event(e_k)
                with torch.cuda.stream(s_out):
                    dst_f[c0:c1].copy_(flat[c0:c1], non_blocking=True)
            torch.cuda.synchronize()
        back.zero_()
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipelined()
            ts.append(time.perf_counter() - t0)
        assert torch.equal(back, pinned)
        e2e["write_pipelined_s"] = round(min(ts), 4)
        e2e["write_pipelined_GBs"] = round(host.numel() / min(ts) / 1e9, 2)
        # the writer for a host image, CRCs back (zscrc_zs_fill_commits):
        # image H2D in chunks, commit mode 3, 4 B per commit D2H, host threads
        # patch the CRC fields -- the reference writer builds its commit
        # records on the host (src/zeroskip-file.c:315-331).  The fields are
        # zeroed first, so the first call is checked byte for byte.
        ow_np = offs_w.cpu().numpy().astype(np.uint64)
        lw_np = lens_w.cpu().numpy().astype(np.uint64)
        fields = (ow_np + lw_np + 4).astype(np.int64)[:, None] + np.arange(4, dtype=np.int64)
        for kind, buf in (("pinned", pinned.view(-1)), ("pageable", host.view(-1).clone())):
            arr = buf.numpy()
            arr[fields] = 0
            zsfile.fill_commits(buf, ow_np, lw_np, max_len=max_span)
            assert torch.equal(buf, host.view(-1)), f"fill_commits ({kind}) differs from the GPU-written image"
            ts, rep_f = [], None
            for _ in range(3):
                t0 = time.perf_counter()
                rep_f = zsfile.fill_commits(buf, ow_np, lw_np, max_len=max_span)
                ts.append(time.perf_counter() - t0)
            e2e[f"write_crcs_{kind}_s"] = round(min(ts), 4)
            e2e[f"write_crcs_{kind}_GBs"] = round(host.numel() / min(ts) / 1e9, 2)
            e2e[f"write_crcs_{kind}_phases_s"] = {"setup": round(rep_f["setup_s"], 5), "h2d": round(rep_f["h2d_s"], 4),
                                                  "total": round(rep_f["total_s"], 4),
                                                  "chunks": rep_f["chunks"], "threads": rep_f["threads"]}
            del buf, arr
        e2e["write_crcs_pipelined_GBs"] = e2e["write_crcs_pinned_GBs"]
        e2e["note"] = ("verify: host file images -> verdicts, walks included (zscrc_zs_verify_files, "
                       f"{rep['threads']} host threads); write: host images -> H2D -> GPU commit writer -> "
                       "D2H of the images (image bytes / wall time), whole image at once or pipelined in "
                       f"{len(chunks)} file-aligned chunks on three streams; write_crcs: host image -> H2D chunks "
                       "-> commit CRCs out of place -> 4 B per commit D2H -> host threads patch the image "
                       "(zscrc_zs_fill_commits); PCIe-bound, never the line's value")
        del images, pinned, back

    nbytes = span_bytes + 8 * ncommit + 16 * ncommit   # spans + commit trailers + descriptors
    r = roof(nbytes, kern_ms, "zs::commit_kernel<false, true, 1024>", "config4", read_peak,
             "verdict, the run-only form at 16 waves per CU: run rounds of 64 back-to-back spans as coalesced "
             "1 KiB loads, other rounds in one-piece quad bursts")
    out_line = line(args, world, elapsed, span_bytes * world * args.steps,
                    {"workload": f"config4: zsbench writeseqtxn replay, {pairs_total} pairs per GPU, "
                                 f"{nfiles} log files, {ncommit} commits (312 B spans + stale finalise "
                                 "commits), GPU verdict of every commit", "pairs": pairs_total,
                     "files": nfiles, "commits": ncommit, "parallelism": f"replica{world}"},
                    r, data="synthetic zsbench records (key %016d, 255 charset chars + NUL, fixed seed), "
                            "byte-exact zeroskip log images in HBM",
                    verdict={"bad_commits": nbad, "stale_finalise_commits": nfiles}, parity=parity,
                    per_commit_arrays={"ms": round(arrays_ms, 4),
                                       "GBs": round((nbytes + 8 * ncommit) / (arrays_ms * 1e-3) / 1e9, 1),
                                       "note": "zscrc_device_verify_commits_bounded: crc + status per commit "
                                               "(8 B of HBM writes per commit)"},
                    write={"ms": round(write_ms, 4), "GBs": round((span_bytes + 8 * ncommit) / (write_ms * 1e-3) / 1e9, 1),
                           "ms_with_crc_array": round(write_crc_ms, 4),
                           "crc_array_ms": round(crcs_ms, 4),
                           "crc_array_GBs": round((span_bytes + 8 * ncommit + 16 * ncommit + 4 * ncommit) /
                                                  (crcs_ms * 1e-3) / 1e9, 1),
                           "note": "ms: zscrc_device_write_commits_bounded, CRCs into the image (d_crc NULL); "
                                   "crc_array_ms: zscrc_device_commit_crcs_bounded, the writer's CRCs to a "
                                   "coalesced 4 B array, image untouched (the kernel of write_crcs in e2e)"},
                    notbatched={"files": nf_nb, "commits": nf_nb, "verify_ms": round(nb_ms, 4),
                                "GBs": round(nb_bytes / (nb_ms * 1e-3) / 1e9, 1),
                                "frac": round(nb_bytes / (nb_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                "verify_unranged_ms": round(nb_unranged_ms, 4),
                                "arrays_ms": round(nb_arrays_ms, 4),
                                "note": "verify_ms: the verdict with the walk's length range (min/max span), "
                                        "unranged: without it, arrays: per-commit crc + status; the three "
                                        "timed interleaved"},
                    e2e=e2e, gen_s=round(t_gen, 2))
    if rank == 0 and world == 1 and not args.no_cpu:
        # the first quarter of the replay's files (~2.5 M commit spans, ~0.8 GB)
        nf = nfiles // 4
        k = int((offs < nf * (flat.numel() // nfiles)).sum().item())
        h = img[:nf].cpu().numpy().reshape(-1)
        o, l_ = offs[:k].cpu().numpy(), lens[:k].cpu().numpy()
        out_line["cpu_baseline"] = cpu_leg(h, f"the commit spans of the first {nf} files ({k} spans)", o, l_)
    return out_line


# ------------------------------------------------------------------ config 5
def run_config5(args, world, rank, dev, stream):
    from tools import zsdb_gen as zg
    from zeroskip_amd import consistent as cs
    t0 = time.perf_counter()
    db = zg.make_db(device=dev, packed=2, packed_region_bytes=args.packed_mib << 20,
                    finalised=args.finalised)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    job = cs.Consistent(cs.open_db(db), rank, world)
    t_open = time.perf_counter() - t0
    job.prepare()

    # the native pass pipelined (zscrc_cpass_submit / _collect): step k
    # enqueues pass k and reads pass k - 1's block while the device runs pass
    # k, so the host's reading and the next launches stay off the device's
    # critical path; every pass is collected and checked inside the timed
    # region (drain).  BENCH_C5_SYNC=1: one synchronous pass per step.
    pipelined = os.environ.get("BENCH_C5_SYNC") != "1"
    reports = []

    def step(ev):
        if not pipelined or not job.submit(ev):
            reports.append(job.run(events=ev))
            return
        if job.pending() > 1:
            reports.append(job.collect())

    def drain():
        while job.pending():
            reports.append(job.collect())

    probe = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
    read_peak = read_ceiling(probe, probe.numel(), stream)   # also settles power (run_config3)
    del probe
    tm = Timer(world, dev, stream)
    elapsed = tm.run(step, args.steps, args.warmup, drain=drain)
    assert len(reports) == args.steps + args.warmup, (len(reports), args.steps, args.warmup)
    for rep in reports:
        assert rep.ok and rep.n_stale == args.finalised, (rep.ok, rep.n_bad, rep.n_stale, rep.walk_errors[:5])
    rep = reports[-1]
    # the checker over the whole DB (rank 0; every rank holds the same images)
    parity = oracle_check_db(job.db, args.finalised) if rank == 0 else None
    if parity and parity["mismatches"]:
        raise SystemExit(f"config5: the oracle disagrees: {parity}")
    kern_ms = float(np.mean(tm.kern_ms))
    ncommit = len(job.c_off)
    local_bytes = job.local.bytes_checked
    nbytes = local_bytes + 16 * ncommit + 16 * len(job.pieces)   # bytes + commit / span descriptors
    r = roof(nbytes, kern_ms, "zscrc_cpass_run", "config5", read_peak,
             "commit_kernel verdict over the short commit spans + one xteam_kernel<1> launch over the records "
             "regions / pointer sections + span fold + post kernel + one small copy back, this rank")
    out_line = line(args, world, elapsed, job.plan.weight * args.steps,
                    {"workload": f"config5: consistent over a {job.plan.weight / GIB:.2f} GiB DB "
                                 f"(2 packed x {args.packed_mib} MiB, {args.finalised} finalised, 1 active, "
                                 f".zsdb), {rep.commits} commits", "db_bytes": job.plan.weight,
                     "files": rep.files, "commits": rep.commits,
                     "parallelism": f"split{world}" + ("+allgather_digests" if world > 1 else "")},
                    r, scaling="strong", parity=parity,
                    data="synthetic zeroskip DB generated on the GPU (tools/zsdb_gen.py), device-resident",
                    prepare={k: round(v, 4) if isinstance(v, float) else v for k, v in job.prepare_times.items()},
                    device_pass={"verified_spans": len(job.c_off), "longest_verified_span": job.c_max,
                                 "raw_spans": [q[3] - q[2] for q in job.pieces][:16]},
                    run_timing={k: round(v, 5) for k, v in rep.timing.items()},
                    passes={"checked": len(reports), "pipelined": bool(pipelined and job._cpass is not None),
                            "note": "every pass's report collected and checked inside the timed region; "
                                    "pipelined: pass k's copy back read while pass k + 1 runs"},
                    gen_s=round(t_gen, 2), open_s=round(t_open, 2))
    if rank == 0 and world == 1 and not args.no_cpu:
        # 64 finalised files' commit spans + 768 MiB of a packed records region
        fin = [f for f in job.db.files if f.kind == zsfile.FINALISED][:64]
        so = [zsfile.walk(f.image)[:2] for f in fin]
        region = 768 << 20
        host = np.concatenate([f.image for f in fin] + [job.db.files[0].image[40:40 + region]])
        bases = np.cumsum([0] + [f.size for f in fin])
        offs = np.concatenate([s[0].astype(np.int64) + b for s, b in zip(so, bases)] + [np.array([bases[-1]])])
        lens = np.concatenate([s[1].astype(np.int64) for s in so] + [np.array([region])])
        out_line["cpu_baseline"] = cpu_leg(host, "64 finalised files' commit spans + 768 MiB of a packed region",
                                           offs, lens)
    return out_line


def torchrun_cmd(n: int) -> list:
    """The launch the driver uses for N > 1 (one rank per GPU, 127.0.0.1)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]


def launch_ranks(n: int) -> int:
    import subprocess
    cmd = torchrun_cmd(n)
    print("bench.py: --gpus %d without WORLD_SIZE: launching %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    if os.environ.get("BENCH_LAUNCH_DRYRUN") == "1":
        print(json.dumps({"launch": cmd}), flush=True)
        return 0
    return subprocess.call(cmd)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="config3", choices=["config2", "config3", "config4", "config5"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-e2e", action="store_true", help="config4: skip the end-to-end leg")
    ap.add_argument("--pairs", type=int, default=10_000_000, help="config4 pairs per GPU")
    ap.add_argument("--packed-mib", type=int, default=3072, help="config5 packed records region size")
    ap.add_argument("--finalised", type=int, default=1024, help="config5 finalised files")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # --gpus N without a launcher: one process per GPU is the contract, so
        # start torchrun as a child (before anything touches the GPU) and
        # exit with its status -- never a silent one-GPU measurement
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        # the file-image APIs of rank r use its own GPU only (zscrc_set_devices)
        os.environ.setdefault("ZSCRC_DEVICES", str(local))
    # BENCH_SHARE_GPU=1: rehearsal of the N-rank path on a box with fewer GPUs
    # (ranks share devices round-robin; RCCL, or gloo with BENCH_DIST=gloo)
    if os.environ.get("BENCH_SHARE_GPU") == "1":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("BENCH_DIST", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if lib().zscrc_device_count() < 1:
        raise SystemExit("libzscrc: no gfx950 device")
    stream = torch.cuda.current_stream(dev)
    run = {"config2": run_config2, "config3": run_config3, "config4": run_config4,
           "config5": run_config5}[args.workload]
    out = run(args, world, rank, dev, stream)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
