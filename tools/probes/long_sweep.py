"""Long records on one GPU: one span (segments + fold) vs the split path of
variable batches (1-3 long records, parts + part fold), 8 GiB buffer.  JSON lines."""
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
    big = torch.randint(0, 256, (8 << 30,), dtype=torch.uint8, device=dev)
    G = 1 << 30
    for gib in (1, 3):
        ms = timeit(lambda: zd.crc_span(big, length=gib * G))
        print(json.dumps({"case": f"span {gib} GiB", "ms": round(ms, 4), "GBs": round(gib * G / ms / 1e6, 1)}), flush=True)
    for lens in ([3 * G], [3 * G, 3 * G], [3 * G + 40, 3 * G - 8, 1 << 20], [1 << 20, 3 * G, 3 * G - 8],
                 [2 * G] * 3, [G] * 6, [G] * 5, [64 << 20] * 96):
        offs = [0]
        for ln in lens[:-1]:
            offs.append(offs[-1] + ln + 8)
        o = torch.tensor(offs, dtype=torch.int64, device=dev)
        ln = torch.tensor(lens, dtype=torch.int64, device=dev)
        ms = timeit(lambda: zd.crc_batch(big, o, ln))
        tot = sum(lens)
        print(json.dumps({"case": f"batch {len(lens)} x ~{lens[0] >> 20} MiB", "ms": round(ms, 4),
                          "GBs": round(tot / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
