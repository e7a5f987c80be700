"""Per-wave timing of commit_kernel (zscrc_diag_wave_times) on config 4's
verdict: 10 M commits of 312-byte spans in 1,526 log files.  Splits the
launch into table fill, run rounds and quad-burst rounds (file boundaries,
stale finalise commits), and the tail (the spread of per-wave end times),
with and without the per-record trailer + verdict (tuning bit 8192) and the
chains (4096), so the gap between the verdict and the bare load + hash of
tools/probes/run_probe.hip can be named.  The run-only form (default) runs 16 waves
per workgroup, 12 with bit 1 << 31; commit_kernel alone (1 << 29) 8; the
listed form (16384) is not timed here (its second launch reuses the wave slots).
usage (GPU box): python tools/probes/commit_waves.py [base|all]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402
from zeroskip_amd._lib import check, lib  # noqa: E402

def block_waves(opt):
    if opt & (1 << 29):
        return 8    # commit_kernel: 512-thread workgroups
    return 12 if opt & (1 << 31) else 16


def waves(name, fn, nwaves, opt=0):
    buf = torch.zeros(nwaves * 4, dtype=torch.int64, device="cuda")
    lib().zscrc_set_opt(opt)
    try:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(10):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / 10
        check(lib().zscrc_diag_wave_times(buf.data_ptr()), "wave times")
        fn()
        torch.cuda.synchronize()
        check(lib().zscrc_diag_wave_times(None), "wave times off")
    finally:
        lib().zscrc_set_opt(0)
    a = buf.view(-1, 4).cpu().numpy().astype(np.int64)
    live = a[:, 0] > 0
    a = a[live]
    t0 = a[:, 0].min()
    ent, fill, end = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, (a[:, 2] - t0) / 100.0
    rounds, runs = a[:, 3] & 0xFFFFFFFF, a[:, 3] >> 32
    quads = rounds - runs
    work = end - fill
    # per-wave least squares: work_us ~ x * run rounds + y * quad rounds
    A = np.stack([runs, quads], 1).astype(np.float64)
    coef, *_ = np.linalg.lstsq(A, work, rcond=None)
    # where the spread lives: inside a workgroup (its 8 waves) or between
    # workgroups (CUs), and between XCDs (blockIdx.x % 8)
    wid = np.nonzero(live)[0]
    blk = wid // block_waves(opt)
    ub = np.unique(blk)
    bmax = np.array([end[blk == b].max() for b in ub])
    bmin = np.array([end[blk == b].min() for b in ub])
    xcd = ub % 8
    spread = {"within_block_range_us_p50": round(float(np.median(bmax - bmin)), 1),
              "block_end_us_p10_p50_max": [round(float(np.percentile(bmax, q)), 1) for q in (10, 50, 100)],
              "xcd_block_end_us_median": [round(float(np.median(bmax[xcd == x])), 1) for x in range(8)]}
    row = {"case": name, "opt": opt, "spread": spread, "ms_per_call_back_to_back": round(ms, 4), "waves": int(live.sum()),
           "kernel_us": round(float(end.max()), 1), "entry_us_max": round(float(ent.max()), 1),
           "fill_us_p50_max": [round(float(np.median(fill - ent)), 2), round(float((fill - ent).max()), 2)],
           "end_us_p10_p50_p90_max": [round(float(np.percentile(end, q)), 1) for q in (10, 50, 90, 100)],
           "rounds_total": int(rounds.sum()), "run_rounds_total": int(runs.sum()),
           "rounds_per_wave_min_max": [int(rounds.min()), int(rounds.max())],
           "quad_rounds_per_wave_min_max": [int(quads.min()), int(quads.max())],
           "us_per_run_round": round(float(coef[0]), 4), "us_per_quad_round": round(float(coef[1]), 4),
           "tail_us_p50_to_max": round(float(end.max() - np.median(end)), 1)}
    print(json.dumps(row), flush=True)


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nw = ncu * 16
    ppf = zg.pairs_per_file(True)
    nfiles = -(-10_000_000 // ppf)
    img = zg.log_files(bytes(range(16)), 0, nfiles, ppf, 0, True, g, dev).view(-1)
    offs, lens = zg.log_spans(nfiles, ppf, True, True, dev)
    mx = int(lens.max().item())
    vout = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(4096, dtype=torch.int64, device=dev))
    fn = lambda: zsfile.verify_commits_verdict(img, offs, lens, max_len=mx, out=vout)  # noqa: E731
    waves("config4 verdict (run-only kernel, other rounds in quad bursts)", fn, nw)
    waves("config4 verdict, commit_kernel alone (1 << 29)", fn, nw, 1 << 29)
    waves("config4 verdict, run-only at 12 waves (1 << 31)", fn, nw, 1 << 31)
    if sys.argv[1:] == ["base"]:
        return
    waves("config4 verdict, static rounds (1 << 22)", fn, nw, 1 << 22)
    waves("config4 verdict, no trailer / stores (diag 8192)", fn, nw, 8192)
    waves("config4 verdict, no chains (diag 4096)", fn, nw, 4096)
    waves("config4 verdict, no run rounds (2048)", fn, nw, 2048)
    # the same spans without the stale finalise commits or file ends inside a
    # round: one contiguous run of 10 M spans (the run-round shape alone)
    live = lens > 0
    ol, ll = offs[live].contiguous(), lens[live].contiguous()
    waves("config4 live commits only (no stale finalise)", lambda: zsfile.verify_commits_verdict(
        img, ol, ll, max_len=mx, out=vout), nw)


if __name__ == "__main__":
    main()
