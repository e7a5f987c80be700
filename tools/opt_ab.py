"""Interleaved A/B of zscrc_set_opt bits on the config-4 verify and a
fixed-stride 320-byte batch and config 2's 32 x 64 MiB multi-batch launch
(median of 15 launches each, modes alternating
launch by launch).  usage: python tools/opt_ab.py [bits ...] (default 0 1)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402
from zeroskip_amd._lib import lib  # noqa: E402


def main():
    modes = [int(x) for x in sys.argv[1:]] or [0, 1]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    ppf = zg.pairs_per_file(True)
    nfiles = -(-10_000_000 // ppf)
    img = zg.log_files(bytes(range(16)), 0, nfiles, ppf, 0, True, g, dev).view(-1)
    offs, lens = zg.log_spans(nfiles, ppf, True, True, dev)
    mx = int(lens.max().item())
    live = lens > 0
    vout = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(4096, dtype=torch.int64, device=dev))
    ow, lw = offs[live].contiguous(), lens[live].contiguous()
    nb_files = -(-10_000_000 // zg.pairs_per_file(False))
    img_nb = zg.log_files(bytes(range(16)), 0, nb_files, zg.pairs_per_file(False), 0, False, g, dev,
                          batched=False).view(-1) if "config4_nb" in (os.environ.get("AB_CASES") or "") else None
    o_nb, l_nb = zg.log_spans(nb_files, zg.pairs_per_file(False), False, False, dev)
    nb_lo, nb_hi = int(l_nb.min().item()), int(l_nb.max().item())
    vout_nb = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(64, dtype=torch.int64, device=dev))
    fx = torch.randint(0, 256, (320 * 10_000_000,), dtype=torch.uint8, device=dev, generator=g)
    only = os.environ.get("AB_CASES")
    bufs = torch.randint(0, 256, (32, 64 << 20), dtype=torch.uint8, device=dev, generator=g)
    blist = list(bufs)
    c3 = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev, generator=g)
    cases = {"config3": lambda: zd.crc_fixed(c3, 65536, 65536, 65536),
             "fixed_16KiB": lambda: zd.crc_fixed(c3, 16384, 16384, 262144),
             "fixed_4KiB": lambda: zd.crc_fixed(c3, 4096, 4096, 1 << 20),
             "fixed_1MiB": lambda: zd.crc_fixed(c3, 1 << 20, 1 << 20, 4096),
             "span_3GiB": lambda: zd.crc_span(c3[:3 << 30]),
             # config 5's multi-span launch shape: two ~3 GiB records regions
             # and their pointer sections in one xteam launch + one fold
             "spans_config5": lambda: zd.crc_spans(c3, [0, 1 << 30, 3 << 30, (3 << 30) + (200 << 20)],
                                                   [3 << 30, 3 << 30, 200 << 20, 180 << 20]),
             "config4_verify": lambda: zsfile.verify_commits(img, offs, lens, max_len=mx),
             "config4_write": lambda: zsfile.write_commits(img, ow, lw, max_len=mx),
             "config4_write_nocrc": lambda: zsfile.write_commits(img, ow, lw, max_len=mx, crc=False),
             "config4_crcs": lambda: zsfile.commit_crcs(img, ow, lw, max_len=mx),
             "config4_verdict": lambda: zsfile.verify_commits_verdict(img, offs, lens, max_len=mx, out=vout),
             "config4_nb": lambda: zsfile.verify_commits(img_nb, o_nb, l_nb)[1],
             # the bench's NOTBATCHED verdict: the walk's length range given
             "config4_nb_verdict": lambda: zsfile.verify_commits_verdict(img_nb, o_nb, l_nb, out=vout_nb,
                                                                         min_len=nb_lo, max_len=nb_hi)[0],
             "fixed_320x312": lambda: zd.crc_fixed(fx, 320, 312, 10_000_000),
             "config2_multi32": lambda: torch.stack(zd.crc_fixed_multi(blist, 64, 64, 1 << 20)),
             "config2_warm32": lambda: torch.stack(zd.crc_fixed_multi([blist[0]] * 32, 64, 64, 1 << 20))}
    st = torch.cuda.current_stream()
    for name, fn in cases.items():
        if only and name not in only.split(","):
            continue
        ts = {m: [] for m in modes}
        outs = {}
        for i in range(17):
            for m in modes:
                lib().zscrc_set_opt(m)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                r = fn()
                b.record(st)
                torch.cuda.synchronize()
                if i >= 2:
                    ts[m].append(a.elapsed_time(b))
                outs[m] = r
        lib().zscrc_set_opt(0)
        row = {"case": name}
        for m in modes:
            row[f"opt{m}_ms"] = round(sorted(ts[m])[len(ts[m]) // 2], 4)
            o = outs[m] if isinstance(outs[m], torch.Tensor) or outs[m] is None else outs[m][0]
            o0 = outs[modes[0]] if isinstance(outs[modes[0]], torch.Tensor) or outs[modes[0]] is None else outs[modes[0]][0]
            if o is not None and o0 is not None and not torch.equal(o, o0):
                row[f"opt{m}_MISMATCH"] = True
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
