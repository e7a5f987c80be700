#!/usr/bin/env python3
"""Where the drop-in crc32c_hw (include/zscrc.h Part 1, zscrc_api.cpp) should
start offloading: one pageable host buffer of S bytes, 1 MiB .. 4 GiB, hashed
by the library's CPU path on one core (the reference's crc32c_hw class,
src/crc32c.c:370-453) and by the GPU offload (zscrc_stream from the caller's
memory, ZSCRC_STREAM_NOCOPY) -- warm (device initialised by an earlier call)
and cold (the first call of a fresh process: HIP init, operator tables,
staging included).  One JSON line per size to stdout.

    python tools/probes/crossover.py [--max-mib 4096] [--cold-mib 64,1024,4096]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _buf(nbytes: int) -> np.ndarray:
    return np.random.default_rng(nbytes).integers(0, 256, nbytes, dtype=np.uint8)


def cold(mib: int) -> dict:
    """Fresh process: the first offloaded call, device init included."""
    os.environ["ZSCRC_GPU_MIN"] = "1"
    from zeroskip_amd._lib import lib, stats
    a = _buf(mib << 20)
    L = lib()
    s0 = stats()[1]
    t0 = time.perf_counter()
    crc = L.crc32c_hw(0, a.ctypes.data, a.nbytes)
    dt = time.perf_counter() - t0
    assert stats()[1] == s0 + 1, "the call did not run on the GPU"
    return {"mib": mib, "cold_gpu_s": dt, "crc": crc}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=4096)
    ap.add_argument("--cold-mib", default="64,1024,4096")
    ap.add_argument("--cold-child", type=int, default=0)
    a = ap.parse_args()
    if a.cold_child:
        print(json.dumps(cold(a.cold_child)), flush=True)
        return
    # cold first, each in its own process, before this one touches the GPU
    colds = {}
    for m in [int(x) for x in a.cold_mib.split(",") if x]:
        if m > a.max_mib:
            continue
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cold-child", str(m)],
                             capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            raise SystemExit(f"cold child {m} MiB failed: {out.stderr[-2000:]}")
        colds[m] = json.loads(out.stdout.strip().splitlines()[-1])
    from zeroskip_amd._lib import lib, stats
    L = lib()
    L.zscrc_set_gpu_min(1)
    w = _buf(1 << 20)
    L.crc32c_hw(0, w.ctypes.data, w.nbytes)          # device init outside the timings
    m = 1
    while m <= a.max_mib:
        buf = _buf(m << 20)
        reps = 5 if m <= 256 else 3

        def best(gpu: bool) -> tuple[float, int]:
            L.zscrc_set_gpu_min(1 if gpu else 0)
            ts, crc = [], 0
            for _ in range(reps):
                s0 = stats()[1]
                t0 = time.perf_counter()
                crc = L.crc32c_hw(0, buf.ctypes.data, buf.nbytes)
                ts.append(time.perf_counter() - t0)
                assert (stats()[1] - s0 == 1) == gpu
            return min(ts), crc
        t_cpu, c_cpu = best(False)
        t_gpu, c_gpu = best(True)
        assert c_cpu == c_gpu, (m, c_cpu, c_gpu)
        row = {"mib": m, "cpu_1core_s": round(t_cpu, 6), "gpu_warm_s": round(t_gpu, 6),
               "cpu_GBs": round(buf.nbytes / t_cpu / 1e9, 2), "gpu_warm_GBs": round(buf.nbytes / t_gpu / 1e9, 2),
               "gpu_wins_warm": t_gpu < t_cpu}
        if m in colds:
            assert colds[m]["crc"] == c_cpu
            row["gpu_cold_s"] = round(colds[m]["cold_gpu_s"], 4)
            row["gpu_wins_cold"] = colds[m]["cold_gpu_s"] < t_cpu
        print(json.dumps(row), flush=True)
        del buf
        m *= 2
    L.zscrc_set_gpu_min(0)


if __name__ == "__main__":
    main()
