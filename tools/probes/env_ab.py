"""Interleaved A/B of an environment switch the library reads per call, on
config 4's bench batch: verdict, per-commit arrays, CRC array, writer.
Median of 15 calls per value (each call's own launches, a fill launch
included, inside its event pair), values alternating call by call; the
outputs of every value are compared with the first's.
usage: python tools/probes/env_ab.py VAR value [value ...]
e.g.   python tools/probes/env_ab.py ZSCRC_VERDICT_MEMSET 0 1"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402


def main():
    var, modes = sys.argv[1], sys.argv[2:]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    ppf = zg.pairs_per_file(True)
    nfiles = -(-10_000_000 // ppf)
    img = zg.log_files(bytes(range(16)), 0, nfiles, ppf, 0, True, g, dev).view(-1)
    offs, lens = zg.log_spans(nfiles, ppf, True, True, dev)
    mx = int(lens.max().item())
    live = lens > 0
    ow, lw = offs[live].contiguous(), lens[live].contiguous()
    vout = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(4096, dtype=torch.int64, device=dev))
    cases = {"config4_verdict": lambda: zsfile.verify_commits_verdict(img, offs, lens, max_len=mx, out=vout)[0].clone(),
             "config4_verify": lambda: zsfile.verify_commits(img, offs, lens, max_len=mx),
             "config4_crcs": lambda: zsfile.commit_crcs(img, ow, lw, max_len=mx),
             "config4_write": lambda: zsfile.write_commits(img, ow, lw, max_len=mx)}
    only = os.environ.get("AB_CASES")
    st = torch.cuda.current_stream()
    for name, fn in cases.items():
        if only and name not in only.split(","):
            continue
        ts = {m: [] for m in modes}
        outs = {}
        for i in range(17):
            for m in modes:
                os.environ[var] = m
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                r = fn()
                b.record(st)
                torch.cuda.synchronize()
                if i >= 2:
                    ts[m].append(a.elapsed_time(b))
                outs[m] = r
        os.environ.pop(var, None)
        row = {"case": name}
        for m in modes:
            v = sorted(ts[m])
            row[f"{m}_ms"] = round(v[len(v) // 2], 4)
            row[f"{m}_min"] = round(v[0], 4)
            o, o0 = outs[m], outs[modes[0]]
            o = o if isinstance(o, torch.Tensor) else torch.cat([x.view(-1).to(torch.int64) for x in o])
            o0 = o0 if isinstance(o0, torch.Tensor) else torch.cat([x.view(-1).to(torch.int64) for x in o0])
            if not torch.equal(o, o0):
                row[f"{m}_MISMATCH"] = True
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
