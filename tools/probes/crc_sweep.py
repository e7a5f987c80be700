"""Kernel-variant sweep on one GPU (tuning aid; prints one JSON line per case)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd._lib import DEFAULT_TEAMS, lib  # noqa: E402


def timeit(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    big = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
    out = torch.empty(1 << 24, dtype=torch.int32, device=dev)
    cases = [
        ("cfg3 64KiB g64", 65536, 65536, 65536, (0, 0)),
        ("cfg3 64KiB g16", 65536, 65536, 65536, (0, 1 << 40)),
        ("cfg3 64KiB g1", 65536, 65536, 65536, (1 << 40, 1 << 40)),
        ("cfg2 64B g1", 64, 64, 1 << 20, DEFAULT_TEAMS),
        ("cfg2 64B g1 x16 (1 GiB)", 64, 64, 1 << 24, DEFAULT_TEAMS),
        ("zsbench 312B g1", 320, 312, 10_000_000, DEFAULT_TEAMS),
        ("zsbench 312B g16", 320, 312, 10_000_000, (0, 1 << 40)),
        ("4KiB g1", 4096, 4096, 1 << 20, (1 << 40, 1 << 40)),
        ("4KiB g16", 4096, 4096, 1 << 20, (0, 1 << 40)),
        ("4KiB g64", 4096, 4096, 1 << 20, (0, 0)),
        ("zsbench 312B default", 320, 312, 10_000_000, DEFAULT_TEAMS),
        ("1KiB g1", 1024, 1024, 1 << 22, (1 << 40, 1 << 40)),
        ("1KiB g16", 1024, 1024, 1 << 22, (0, 1 << 40)),
        ("256KiB g16", 262144, 262144, 16384, (0, 1 << 40)),
        ("256KiB g64", 262144, 262144, 16384, (0, 0)),
        ("1MiB g64 (4096 recs)", 1 << 20, 1 << 20, 4096, (0, 0)),
    ]
    scratch = torch.zeros(4, dtype=torch.int32, device=dev)
    for mult in (1, 2, 4):
        ms = timeit(lambda: lib().zscrc_diag_stream_read(big.data_ptr(), 4 << 30, scratch.data_ptr(),
                                                          mult, torch.cuda.current_stream().cuda_stream))
        print(json.dumps({"case": f"stream_read grid x{mult}", "ms": round(ms, 4),
                          "GBs": round((4 << 30) / ms / 1e6, 1)}), flush=True)
    for name, stride, length, n, teams in cases:
        lib().zscrc_set_teams(*teams)
        g = 1 if teams[0] >= length else (16 if teams[1] >= length else 64)
        for depth in (-1, 0, 1, 2, -1):
            lib().zscrc_set_prefetch(g, depth)
            ms = timeit(lambda: zd.crc_fixed(big, stride, length, n, out=out[:n]))
            byt = n * length
            print(json.dumps({"case": name, "depth": depth, "ms": round(ms, 4),
                              "GBs": round(byt / ms / 1e6, 1),
                              "GiBs": round(byt / ms / 1e6 * 1e9 / (1 << 30), 1)}), flush=True)
    for g in (1, 16, 64):
        lib().zscrc_set_prefetch(g, -1)
    lib().zscrc_set_teams(*DEFAULT_TEAMS)
    ms = timeit(lambda: zd.crc_span(big))
    print(json.dumps({"case": "span 4 GiB", "ms": round(ms, 4), "GBs": round((4 << 30) / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
