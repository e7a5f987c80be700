"""One-lane records of 321-1024 bytes (fixed stride): piece walk (walk 3) vs
quad-cooperative bursts (walk 10) vs 16-lane teams.  JSON lines (diagnostic)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tools.probes.crc_sweep import timeit  # noqa: E402
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd._lib import DEFAULT_TEAMS, lib  # noqa: E402

dev = torch.device("cuda:0")
big = torch.randint(0, 256, (3 << 30,), dtype=torch.uint8, device=dev)
out = torch.empty(1 << 24, dtype=torch.int32, device=dev)
lib().zscrc_set_small_team(1)
for ln, stride, shift in [(352, 360, 40), (400, 400, 0), (448, 456, 40), (520, 520, 0), (600, 608, 40),
                          (640, 648, 40), (312, 320, 40), (700, 704, 40), (800, 808, 40), (900, 904, 40),
                          (1000, 1000, 0)]:
    n = min(1 << 24, (2 << 30) // stride)
    row = {"len": ln, "stride": stride, "shift": shift}
    lib().zscrc_set_teams(1 << 20, 1 << 20)
    for w in (3, 10):
        lib().zscrc_set_prefetch(1, w)
        ms = timeit(lambda: zd.crc_fixed(big[shift:], stride, ln, n, out=out[:n]))
        row[f"w{w}"] = round(n * ln / ms / 1e6, 1)
    lib().zscrc_set_teams(0, 1 << 20)
    ms = timeit(lambda: zd.crc_fixed(big[shift:], stride, ln, n, out=out[:n]))
    row["g16"] = round(n * ln / ms / 1e6, 1)
    print(json.dumps(row), flush=True)
lib().zscrc_set_prefetch(1, -1)
lib().zscrc_set_small_team(0)
lib().zscrc_set_teams(*DEFAULT_TEAMS)
