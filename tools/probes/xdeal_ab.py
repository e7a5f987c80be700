"""Interleaved A/B of xteam_kernel's span segments per wave (zscrc_set_xdeal:
0 = the static walk's two contiguous segments per wave, else that many per
wave dealt per workgroup) on a 3 GiB span and on config 5's multi-span
shape (two 3 GiB records regions + two pointer sections in one launch).
Median of 15 calls each, the settings alternating call by call; every
setting's results compared with the static walk's.
usage (GPU box): python tools/probes/xdeal_ab.py [per_wave ...]   (default 0 4 8 16)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd._lib import lib  # noqa: E402


def main():
    vals = [int(x) for x in sys.argv[1:]] or [0, 4, 8, 16]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    if os.environ.get("XD_NB"):
        return notbatched(vals, dev, g)
    buf = torch.randint(0, 256, ((6 << 30) + (16 << 20),), dtype=torch.uint8, device=dev, generator=g)
    r3 = 3221222000  # config 5's records region
    cases = {"span_3GiB": lambda: zd.crc_span(buf[:3 << 30]),
             "spans_config5": lambda: zd.crc_spans(buf, [0, r3 + 7, 2 * r3 + 64, 2 * r3 + 64 + 6254808],
                                                   [r3, r3, 6254808, 6254808])}
    st = torch.cuda.current_stream()
    old = lib().zscrc_set_xdeal(16)
    try:
        for name, fn in cases.items():
            ts = {v: [] for v in vals}
            outs = {}
            for i in range(17):
                for v in vals:
                    lib().zscrc_set_xdeal(v)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    r = fn()
                    b.record(st)
                    torch.cuda.synchronize()
                    if i >= 2:
                        ts[v].append(a.elapsed_time(b))
                    outs[v] = r.clone()
            row = {"case": name}
            for v in vals:
                row[f"xdeal{v}_ms"] = round(sorted(ts[v])[len(ts[v]) // 2], 4)
                if not torch.equal(outs[v], outs[vals[0]]):
                    row[f"xdeal{v}_MISMATCH"] = True
            print(json.dumps(row), flush=True)
    finally:
        lib().zscrc_set_xdeal(old)


def notbatched(vals, dev, g):
    """config 4 NOTBATCHED (1,488 commits of ~2 MiB), the ranged verdict with
    class-3 segment plans dealt (tuning bit 1 << 27) at per_wave segments per
    wave, or one segment per wave (0)."""
    from tools import zsdb_gen as zg
    from zeroskip_amd import zsfile
    ppf = zg.pairs_per_file(False)
    nf = -(-10_000_000 // ppf)
    img = zg.log_files(bytes(range(16)), 0, nf, ppf, 0, False, g, dev, batched=False).view(-1)
    offs, lens = zg.log_spans(nf, ppf, False, False, dev)
    lo, hi = int(lens.min().item()), int(lens.max().item())
    out = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(64, dtype=torch.int64, device=dev))
    st = torch.cuda.current_stream()
    ts = {v: [] for v in vals}
    old = lib().zscrc_set_xdeal(16)
    try:
        for i in range(17):
            for v in vals:
                lib().zscrc_set_xdeal(v)
                lib().zscrc_set_opt((1 << 27) if v else 0)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                crc, stat = zsfile.verify_commits(img, offs, lens)
                zsfile.verify_commits_verdict(img, offs, lens, out=out, min_len=lo, max_len=hi)
                b.record(st)
                torch.cuda.synchronize()
                assert int(out[0].item()) == 0 and bool((stat == 1).all()), v
                if i >= 2:
                    ts[v].append(a.elapsed_time(b) / 2)
    finally:
        lib().zscrc_set_opt(0)
        lib().zscrc_set_xdeal(old)
    print(json.dumps({"case": "config4_nb (arrays + ranged verdict, per call)",
                      **{f"xdeal{v}_ms": round(sorted(ts[v])[len(ts[v]) // 2], 4) for v in vals}}), flush=True)


if __name__ == "__main__":
    main()
