"""One-lane-per-record (G = 1) walks A/B on one GPU: team ring walks
(depth 1, 2) vs the short-record kernel (3, 4).  Fixed-stride shapes,
a variable zsbench batch and config-4 commit verification.  JSON lines."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tools.probes.crc_sweep import timeit  # noqa: E402
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402
from zeroskip_amd._lib import lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    big = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
    out = torch.empty(1 << 24, dtype=torch.int32, device=dev)
    cases = [("64B x1M (cfg2)", 64, 64, 1 << 20, 0), ("64B x16M", 64, 64, 1 << 24, 0),
             ("312B/320 x10M", 320, 312, 10_000_000, 0), ("312B/320 x10M +3", 320, 312, 10_000_000, 3),
             ("1KiB x4M", 1024, 1024, 1 << 22, 0), ("200B/200 x16M", 200, 200, 1 << 24, 0)]
    cases += [("320B/320 aligned", 320, 320, 10_000_000, 0), ("320B/320 +8", 320, 320, 10_000_000, 8),
              ("312B/320 +8 (pieces 64B-aligned)", 320, 312, 10_000_000, 8),
              ("312B/320 +40 (zeroskip layout)", 320, 312, 10_000_000, 40),
              ("256B/256 aligned", 256, 256, 10_000_000, 0), ("256B/256 +4", 256, 256, 10_000_000, 4)]
    depths = (3, 9, 10)
    for name, stride, length, n, shift in cases:
        for dp in depths:
            lib().zscrc_set_prefetch(1, dp)
            ms = timeit(lambda: zd.crc_fixed(big[shift:], stride, length, n, out=out[:n]))
            print(json.dumps({"case": name, "depth": dp, "ms": round(ms, 4),
                              "GBs": round(n * length / ms / 1e6, 1)}), flush=True)
    # variable batch: zsbench spans through descriptors (classify + class 0)
    n = 10_000_000
    offs = torch.arange(n, dtype=torch.int64, device=dev) * 320 + 40
    lens = torch.full((n,), 312, dtype=torch.int64, device=dev)
    for dp in (3, 9, 10):
        lib().zscrc_set_prefetch(1, dp)
        ms = timeit(lambda: zd.crc_batch(big, offs, lens, out=out[:n]))
        print(json.dumps({"case": "variable 312B x10M", "depth": dp, "ms": round(ms, 4),
                          "GBs": round(n * 312 / ms / 1e6, 1)}), flush=True)
    # config-4 commit verification on generated log files
    from tools import zsdb_gen as zg
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    ppf = zg.pairs_per_file(True)
    del big
    img = zg.log_files(bytes(16), 0, 1526, ppf, 0, True, g, dev)
    o, ln = zg.log_spans(1526, ppf, True, True, dev)
    for dp in (3, 9, 10):
        lib().zscrc_set_prefetch(1, dp)
        ms = timeit(lambda: zsfile.verify_commits(img.view(-1), o, ln))
        _, st = zsfile.verify_commits(img.view(-1), o, ln)
        ok = int((st == 1).sum().item())
        print(json.dumps({"case": "config4 verify", "depth": dp, "ms": round(ms, 4), "ok": ok,
                          "GBs": round((int(ln.sum().item()) + 8 * o.numel()) / ms / 1e6, 1)}), flush=True)
    lib().zscrc_set_prefetch(1, -1)


if __name__ == "__main__":
    main()
