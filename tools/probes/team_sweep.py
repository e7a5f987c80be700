"""Fixed-stride rate by record length for the current team-size policy (set
ZSCRC_SMALL_TEAM / ZSCRC_G1_MAX in the environment to A/B policies).  Packed
(stride = length) and 64-byte-padded strides.  JSON lines."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tools.probes.crc_sweep import timeit  # noqa: E402
from zeroskip_amd import device as zd  # noqa: E402

LENS = (128, 192, 200, 256, 312, 320, 384, 448, 512, 520, 640, 700, 768, 896, 1000, 1024)


def main():
    dev = torch.device("cuda:0")
    big = torch.randint(0, 256, (3 << 30,), dtype=torch.uint8, device=dev)
    out = torch.empty(1 << 24, dtype=torch.int32, device=dev)
    tag = os.environ.get("TAG", "")
    for rl in LENS:
        for stride in sorted({rl, (rl + 63) // 64 * 64}):
            n = min(1 << 24, (2 << 30) // stride)
            ms = timeit(lambda: zd.crc_fixed(big, stride, rl, n, out=out[:n]), reps=20)
            print(json.dumps({"tag": tag, "len": rl, "stride": stride, "n": n,
                              "GBs": round(n * rl / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
