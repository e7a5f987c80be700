"""Run one fixed-stride batch case repeatedly (profiling target).
usage: python tools/probes/crc_case.py STRIDE LEN N [G1_MAX G16_MAX] [REPS]
env: ZS_DEPTH = G1 walk override (zscrc_set_prefetch(1, depth)), ZS_SHIFT = byte
offset of record 0 in the buffer"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd._lib import lib  # noqa: E402

stride, length, n = (int(x) for x in sys.argv[1:4])
if len(sys.argv) > 5:
    lib().zscrc_set_teams(int(sys.argv[4]), int(sys.argv[5]))
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
if "ZS_DEPTH" in os.environ:
    lib().zscrc_set_prefetch(1, int(os.environ["ZS_DEPTH"]))
shift = int(os.environ.get("ZS_SHIFT", "0"))
d = torch.randint(0, 256, (shift + stride * (n - 1) + length,), dtype=torch.uint8, device="cuda")[shift:]
out = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(reps):
    zd.crc_fixed(d, stride, length, n, out=out)
torch.cuda.synchronize()
print("done", stride, length, n)
