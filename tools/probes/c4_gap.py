"""Where config 4's verify time goes beyond the fixed-stride rate (diagnostic):
fixed 312 B / 320 B +40, the same records as a bounded variable batch, the
same with seeds, and commit verification of config-4 log images."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tools.probes.crc_sweep import timeit  # noqa: E402
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402

dev = torch.device("cuda:0")
n = 10_000_000
big = torch.randint(0, 256, (n * 320 + 4096,), dtype=torch.uint8, device=dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
offs = torch.arange(n, dtype=torch.int64, device=dev) * 320 + 40
lens = torch.full((n,), 312, dtype=torch.int64, device=dev)
seeds = torch.zeros(n, dtype=torch.int32, device=dev)


def rep(name, f, nbytes=n * 312):
    ms = timeit(f)
    print(json.dumps({"case": name, "ms": round(ms, 4), "GBs": round(nbytes / ms / 1e6, 1)}), flush=True)


rep("fixed 312/320 +40", lambda: zd.crc_fixed(big[40:], 320, 312, n, out=out))
rep("variable bounded", lambda: zd.crc_batch(big, offs, lens, out=out, max_len=312))
rep("variable bounded + seeds", lambda: zd.crc_batch(big, offs, lens, seeds, out=out, max_len=312))
rep("variable unbounded", lambda: zd.crc_batch(big, offs, lens, out=out))
del big
g = torch.Generator(device=dev)
g.manual_seed(1)
ppf = zg.pairs_per_file(True)
img = zg.log_files(bytes(16), 0, 1526, ppf, 0, True, g, dev)
o, ln = zg.log_spans(1526, ppf, True, True, dev)
m = o.numel()
sb = int(ln.sum().item())
rep("config4 crc only (bounded batch over the spans)", lambda: zd.crc_batch(img.view(-1), o, ln, max_len=312), sb)
rep("config4 verify bounded", lambda: zsfile.verify_commits(img.view(-1), o, ln, max_len=312), sb)
