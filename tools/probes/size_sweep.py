"""Fixed overhead vs streaming rate of the one-lane-per-record kernel: 64-byte
records, n = 2^14 .. 2^24, plus the empty-batch launch.  JSON lines."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tools.probes.crc_sweep import timeit  # noqa: E402
from zeroskip_amd import device as zd  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    big = torch.randint(0, 256, (1 << 30,), dtype=torch.uint8, device=dev)
    out = torch.empty(1 << 24, dtype=torch.int32, device=dev)
    for rl in (64, 312):
        for lg in range(14, 25):
            n = 1 << lg
            if n * rl > big.numel():
                break
            ms = timeit(lambda: zd.crc_fixed(big, rl, rl, n, out=out[:n]), reps=20)
            print(json.dumps({"rec": rl, "n": n, "us": round(ms * 1e3, 2),
                              "GBs": round(n * rl / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
