"""Profiling target: exactly REPS device passes of one BASELINE config and
nothing else on the GPU after setup, so rocprofv3 per-dispatch counters sum to
REPS passes (traffic per pass = sum over the zs:: dispatches / REPS).

usage: python tools/prof_case.py config2|config3|config4|config5 [REPS]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402


def main():
    cfg = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    if cfg == "config3":
        data = torch.randint(0, 256, (65536 * 65536,), dtype=torch.uint8, device=dev, generator=g)
        out = torch.empty(65536, dtype=torch.int32, device=dev)
        run = lambda k: zd.crc_fixed(data, 65536, 65536, 65536, out=out)  # noqa: E731
    elif cfg == "config2":
        # one pass = one zscrc_device_fixed_multi launch over 64 batches of
        # 1M x 64 B (bench.py's step unit is one batch: summarize divides by 64)
        bufs = torch.randint(0, 256, (64, 64 << 20), dtype=torch.uint8, device=dev, generator=g)
        blist = list(bufs)
        outs = [torch.empty(1 << 20, dtype=torch.int32, device=dev) for _ in range(64)]
        run = lambda k: zd.crc_fixed_multi(blist, 64, 64, 1 << 20, outs=outs)  # noqa: E731
    elif cfg == "config4":
        from tools import zsdb_gen as zg
        ppf = zg.pairs_per_file(True)
        nfiles = -(-10_000_000 // ppf)
        img = zg.log_files(bytes(range(16)), 0, nfiles, ppf, 0, True, g, dev)
        offs, lens = zg.log_spans(nfiles, ppf, True, True, dev)
        mx = int(lens.max().item())
        vout = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(4096, dtype=torch.int64, device=dev))
        if os.environ.get("C4_ARRAYS"):     # per-commit crc + status arrays
            run = lambda k: zsfile.verify_commits(img.view(-1), offs, lens, max_len=mx)  # noqa: E731
        else:                               # the bench line's verdict
            run = lambda k: zsfile.verify_commits_verdict(img.view(-1), offs, lens, max_len=mx, out=vout)  # noqa: E731
    elif cfg == "config4nb":
        # NOTBATCHED: one ~2 MiB commit per log file, unbounded verdict (bench.py's notbatched leg)
        from tools import zsdb_gen as zg
        ppf = zg.pairs_per_file(False)
        nfiles = -(-10_000_000 // ppf)
        img = zg.log_files(bytes(range(16)), 0, nfiles, ppf, 0, False, g, dev, batched=False)
        offs, lens = zg.log_spans(nfiles, ppf, False, False, dev)
        vout = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(64, dtype=torch.int64, device=dev))
        lo, hi = int(lens.min().item()), int(lens.max().item())
        mode = os.environ.get("C4NB_MODE", "range")
        forms = [lambda k: zsfile.verify_commits_verdict(img.view(-1), offs, lens, out=vout, min_len=lo,  # noqa: E731
                                                         max_len=hi),
                 lambda k: zsfile.verify_commits_verdict(img.view(-1), offs, lens, out=vout),  # noqa: E731
                 lambda k: zsfile.verify_commits(img.view(-1), offs, lens)]  # noqa: E731
        if mode == "mixed":                 # pass k: form k % 3 (ranged verdict, verdict, arrays), one process
            run = lambda k: forms[k % 3](k)  # noqa: E731
        elif mode == "arrays":              # per-commit crc + status arrays
            run = lambda k: zsfile.verify_commits(img.view(-1), offs, lens)  # noqa: E731
        elif mode == "unranged":
            run = lambda k: zsfile.verify_commits_verdict(img.view(-1), offs, lens, out=vout)  # noqa: E731
        else:                               # the bench line's verdict: the walk's length range
            run = lambda k: zsfile.verify_commits_verdict(img.view(-1), offs, lens, out=vout,  # noqa: E731
                                                          min_len=lo, max_len=hi)
    elif cfg == "config4w":
        # the writer side of config 4: every live commit's CRC recomputed and stored
        from tools import zsdb_gen as zg
        ppf = zg.pairs_per_file(True)
        nfiles = -(-10_000_000 // ppf)
        img = zg.log_files(bytes(range(16)), 0, nfiles, ppf, 0, True, g, dev)
        offs, lens = zg.log_spans(nfiles, ppf, True, True, dev)
        live = lens > 0
        ow, lw = offs[live].contiguous(), lens[live].contiguous()
        if os.environ.get("C4_CRCS"):       # the writer's CRCs out of place (commit mode 3)
            crc = torch.empty(ow.numel(), dtype=torch.int32, device=dev)
            from zeroskip_amd._lib import check as _ck, lib as _lb
            run = lambda k: _ck(_lb().zscrc_device_commit_crcs_bounded(  # noqa: E731
                img.data_ptr(), img.numel(), ow.data_ptr(), lw.data_ptr(), ow.numel(), 312, crc.data_ptr(), None,
                torch.cuda.current_stream().cuda_stream), "crcs")
        else:
            run = lambda k: zsfile.write_commits(img.view(-1), ow, lw, max_len=312, crc=False)  # noqa: E731
    elif cfg == "config5":
        from tools import zsdb_gen as zg
        from zeroskip_amd import consistent as cs
        db = zg.make_db(device=dev)
        job = cs.Consistent(cs.open_db(db), 0, 1)
        job.prepare()
        run = lambda k: job.run()  # noqa: E731
    elif cfg.startswith("fixed"):
        # fixedSTRIDE_LEN_SHIFT: 10M records of LEN bytes every STRIDE bytes, record 0 at SHIFT
        stride, ln, shift = (int(x) for x in cfg[5:].split("_"))
        n = 10_000_000
        data = torch.randint(0, 256, (shift + stride * n,), dtype=torch.uint8, device=dev, generator=g)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        run = lambda k: zd.crc_fixed(data[shift:], stride, ln, n, out=out)  # noqa: E731
    else:
        raise SystemExit(f"unknown config {cfg}")
    if "ZS_DEPTH" in os.environ:
        from zeroskip_amd._lib import lib as _l
        _l().zscrc_set_prefetch(1, int(os.environ["ZS_DEPTH"]))
    torch.cuda.synchronize()
    # marker dispatch: the passes are the zs:: dispatches after this one
    from zeroskip_amd._lib import check, lib
    scratch = torch.zeros(4096, dtype=torch.int32, device=dev)
    check(lib().zscrc_diag_stream_read(scratch.data_ptr(), 8192, scratch.data_ptr(), 1,
                                       torch.cuda.current_stream().cuda_stream), "marker")
    if os.environ.get("PC_TIME"):  # sustained-rate probe: ms per pass per block of 50 passes
        import json
        import time
        blocks = []
        for k0 in range(0, reps, 50):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(k0, min(reps, k0 + 50)):
                run(k)
            torch.cuda.synchronize()
            blocks.append(round((time.perf_counter() - t0) * 1e3 / (min(reps, k0 + 50) - k0), 4))
        print(json.dumps({"case": cfg, "reps": reps, "ms_per_pass_by_block50": blocks}), flush=True)
        return
    for k in range(reps):
        run(k)
    torch.cuda.synchronize()
    print("done", cfg, reps)


if __name__ == "__main__":
    main()
