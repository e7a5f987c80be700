#!/usr/bin/env python3
"""repack's records-region CRC (one crc32_end over the whole
region, src/zeroskip-packed.c:442 -> src/mfile.c:534-546) on the GPU.

Times, over the same host bytes (anonymous memory and a file-backed mmap):
  cpu      libzscrc's CPU path (crc32c_hw below the offload threshold, 1 thread)
  stream   zscrc_stream copy mode (pinned staging, the caller may reuse its buffer)
  nocopy   zscrc_stream NOCOPY (DMA straight from the caller's memory)
  scalar   crc32c_hw with ZSCRC_GPU_MIN set (the unchanged reference symbol)
All results are checked equal.  Prints one JSON line per source.
usage: python tools/repack_bench.py [--mib 4096] [--file /tmp/x]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zeroskip_amd import crc32c as zc  # noqa: E402
from zeroskip_amd._lib import lib  # noqa: E402
from zeroskip_amd.stream import CrcStream  # noqa: E402


def timed(fn, reps=3):
    best, val = None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        v = fn()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
        assert val is None or v == val
        val = v
    return best, val


def run(buf: np.ndarray, what: str, chunk: int) -> dict:
    n = buf.nbytes
    lib().zscrc_set_gpu_min(0)
    t_cpu, c0 = timed(lambda: zc.crc32c_hw(0, buf), 2)

    def stream(nocopy):
        with CrcStream(0, chunk_bytes=chunk, nocopy=nocopy) as s:
            for i in range(0, n, 16 << 20):          # mfile_write-sized appends
                s.update(buf[i:i + (16 << 20)])
        return s.crc

    t_s, c1 = timed(lambda: stream(False))
    t_n, c2 = timed(lambda: stream(True))
    lib().zscrc_set_gpu_min(1 << 20)
    t_x, c3 = timed(lambda: zc.crc32c_hw(0, buf))
    lib().zscrc_set_gpu_min(0)
    assert c0 == c1 == c2 == c3, (c0, c1, c2, c3)
    g = lambda t: round(n / t / 1e9, 2)  # noqa: E731
    return {"source": what, "bytes": n, "chunk": chunk, "cpu_GBs": g(t_cpu), "stream_copy_GBs": g(t_s),
            "stream_nocopy_GBs": g(t_n), "scalar_offload_GBs": g(t_x), "crc": f"{c0:08x}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=4096)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--file", default=None)
    a = ap.parse_args()
    n = a.mib << 20
    buf = np.random.default_rng(3).integers(0, 256, n, dtype=np.uint8)
    print(json.dumps(run(buf, "anonymous", a.chunk_mib << 20)), flush=True)
    if a.file:
        buf.tofile(a.file)
        mm = np.memmap(a.file, dtype=np.uint8, mode="r")
        _ = int(mm[::4096].sum())                  # page cache warm
        print(json.dumps(run(mm, "mmap", a.chunk_mib << 20)), flush=True)
        del mm
        os.unlink(a.file)


if __name__ == "__main__":
    main()
