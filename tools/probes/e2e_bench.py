#!/usr/bin/env python3
"""End-to-end (host memory -> GPU -> verdict) rates of zscrc_zs_verify_files on
the BASELINE config-4 replay (zsbench BATCHED / NOTBATCHED log files) and a
config-5-shaped DB directory on disk (zscrc_zs_consistent), beside the CPU
oracle's crc32c_hw class over the same spans on 1 core and on every usable
host core.  Prints one JSON line per case.

usage: python tools/probes/e2e_bench.py [--pairs 10000000] [--reps 5] [--dbdir /tmp/zsdb]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from zeroskip_amd import consistent as cs  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402


def cores() -> int:
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


def cpu_rate(images, seconds=4.0):
    """oracle crc32c_hw over every commit span of the images (+ 8-byte
    trailer words excluded), 1 thread and all threads: GB/s of file bytes."""
    from oracle import oracle
    host = np.concatenate(images)
    base = np.cumsum([0] + [im.nbytes for im in images])[:-1]
    offs, lens = [], []
    for b, im in zip(base, images):
        o, ln, _, _ = zsfile.walk(im)
        offs.append(o.astype(np.uint64) + np.uint64(b))
        lens.append(ln.astype(np.uint64))
    offs, lens = np.concatenate(offs), np.concatenate(lens)
    out = {}
    for t in (1, cores()):
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds / 2:
            oracle.batch(host, offs, lens, impl="hw", threads=t)
            done += 1
        out[t] = host.nbytes * done / (time.perf_counter() - t0) / 1e9
    return out


def gpu_rate(images, kinds, reps, threads=0):
    zsfile.verify_files(images, kinds, threads)          # warm: pinned / device caches
    best, rep = None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        rep = zsfile.verify_files(images, kinds, threads)
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    return best, rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dbdir", default=None)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    from tools import zsdb_gen as zg
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x5EED)
    uuid = bytes(range(16))
    for batched in (True, False):
        ppf = zg.pairs_per_file(batched)
        nf = -(-a.pairs // ppf)
        img = zg.log_files(uuid, 0, nf, ppf, 0, True, gen, dev, batched=batched)
        host = img.cpu().numpy()
        del img
        images = list(host)
        kinds = [zsfile.FINALISED] * len(images)
        total = host.nbytes
        c = None if a.no_cpu else cpu_rate(images)
        for stage in ("0", "1"):
            os.environ["ZSCRC_FILES_STAGE"] = stage
            dt, rep = gpu_rate(images, kinds, a.reps)
            line = {"case": f"config4 {'BATCHED' if batched else 'NOTBATCHED'}",
                    "copies": "pinned staging" if rep["staged"] else "pageable H2D from the images",
                    "files": len(images), "bytes": total, "commits": rep["commits"], "bad": rep["bad_commits"],
                    "stale": rep["stale_empty_commits"], "e2e_s": round(dt, 4),
                    "e2e_GBs": round(total / dt / 1e9, 2), "threads": rep["threads"],
                    "copy_s": round(rep["copy_s"], 4), "verify_tail_s": round(rep["verify_tail_s"], 5)}
            if c:
                line["cpu_1core_GBs"] = round(c[1], 2)
                line[f"cpu_{cores()}core_GBs"] = round(c[cores()], 2)
            print(json.dumps(line), flush=True)
        os.environ.pop("ZSCRC_FILES_STAGE")
        del host, images
    if a.dbdir:
        db = zg.make_db(device=dev, packed=2, packed_region_bytes=3072 << 20, finalised=1024)
        zg.write_dir(db, a.dbdir)
        del db
        torch.cuda.empty_cache()
        for stage in ("0", "1"):
            os.environ["ZSCRC_FILES_STAGE"] = stage
            cs.consistent_native(a.dbdir)                  # warm (page cache, pinned, device buffers)
            best = None
            for _ in range(a.reps):
                t0 = time.perf_counter()
                r = cs.consistent_native(a.dbdir)
                dt = time.perf_counter() - t0
                best = dt if best is None or dt < best else best
            print(json.dumps({"case": "config5 DB directory (zscrc_zs_consistent)",
                              "copies": "pinned staging" if stage == "1" else "pageable H2D from the mmaps",
                              "bytes": r["bytes"], "files": r["files"], "commits": r["commits"],
                              "consistent": r["consistent"], "stale": r["stale_empty_commits"],
                              "e2e_s": round(best, 4), "e2e_GBs": round(r["bytes"] / best / 1e9, 2)}), flush=True)
        os.environ.pop("ZSCRC_FILES_STAGE")


if __name__ == "__main__":
    main()
