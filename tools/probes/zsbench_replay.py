#!/usr/bin/env python3
"""BASELINE config 4: zsbench write + verify replay on the GPU.

Replays `zsbench writeseqtxn` / `writeseq` (benchmark/zsbench.c:159-217) as a
byte-exact zeroskip log image: N pairs, key "%016d" (16 B -> 40 B key record),
value = 255 charset chars + NUL (256 B -> 272 B value record), files finalised
at 2 MiB (src/zeroskip.c:914-925).
  BATCHED   one transaction per pair: [key][value][8 B commit] = 320 B,
            span 312 B (10 M commits for 10 M pairs)
  NOTBATCHED one transaction: every file is one ~2 MiB span closed by the
            finalise commit.
(The reference's finalise commit after an already-committed transaction hashes
a stale register, src/mfile.c:534-546 + zeroskip-active.c:122; files here end
at their last real commit.)

write  = the GPU computes every commit CRC (span + host-order trailer word) and
         stores it big-endian into the commit record;
verify = the GPU recomputes every commit CRC and compares with the stored one.
Timed device-resident (kernel only) and end-to-end (host image -> H2D, pinned
and pageable; the host record walk; D2H of the results).  The image written by
the GPU is spot-checked against the CPU oracle.

usage: python tools/probes/zsbench_replay.py [--pairs N] [--mode batched|notbatched|both]
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

from oracle import oracle  # noqa: E402  (spot checks + CPU baseline only)
from oracle import zs_format as zf  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402

TWOMB = 2 << 20
KEYREC, VALREC = 40, 272
CHARSET = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
                        b"0123456789!@#$%^&*()-=_+|{}[];<>,./?:", dtype=np.uint8)
UUID = bytes(range(16))


def be64_bytes(v: int) -> np.ndarray:
    return np.frombuffer(int(v).to_bytes(8, "big"), dtype=np.uint8)


def build(pairs: int, mode: str, seed: int = 0x5EED):
    """Image (uint8) + commit span descriptors, commit CRC fields zero."""
    pair = KEYREC + VALREC + (8 if mode == "batched" else 0)
    per_file = -(-(TWOMB - zf.HDR_SIZE) // pair)          # adds until size >= 2 MiB
    nfiles = -(-pairs // per_file)
    sizes = []
    for f in range(nfiles):
        k = min(per_file, pairs - f * per_file)
        sizes.append(zf.HDR_SIZE + k * pair + (8 if mode == "notbatched" else 0))
    img = np.zeros(sum(sizes), dtype=np.uint8)
    key_w = be64_bytes((zf.REC_KEY << 56) | (16 << 40) | KEYREC)
    val_w = be64_bytes((zf.REC_VALUE << 56) | (256 << 32))
    rng = np.random.default_rng(seed)
    span_off, span_len = [], []
    base = 0
    digits = 10 ** np.arange(15, -1, -1, dtype=np.int64)
    for f in range(nfiles):
        k = min(per_file, pairs - f * per_file)
        img[base:base + zf.HDR_SIZE] = np.frombuffer(zf.header_bytes(UUID, f, f), dtype=np.uint8)
        body = img[base + zf.HDR_SIZE: base + zf.HDR_SIZE + k * pair].reshape(k, pair)
        body[:, 0:8] = key_w
        ids = np.arange(f * per_file, f * per_file + k, dtype=np.int64)
        body[:, 24:40] = (48 + (ids[:, None] // digits[None, :]) % 10).astype(np.uint8)
        body[:, 40:48] = val_w
        body[:, 56:311] = CHARSET[rng.integers(0, len(CHARSET), (k, 255), dtype=np.uint8)]
        body[:, 311] = 0
        first = base + zf.HDR_SIZE
        if mode == "batched":
            body[:, 312:320] = be64_bytes((zf.REC_COMMIT << 56) | (312 << 32))
            span_off.append(first + np.arange(k, dtype=np.int64) * pair)
            span_len.append(np.full(k, 312, dtype=np.int64))
        else:
            n = k * pair
            img[first + n: first + n + 8] = be64_bytes((zf.REC_COMMIT << 56) | (n << 32))
            span_off.append(np.array([first], dtype=np.int64))
            span_len.append(np.array([n], dtype=np.int64))
        base += sizes[f]
    return img, np.concatenate(span_off), np.concatenate(span_len), np.array(sizes, dtype=np.int64)


def ev_time(fn, reps=5):
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


def run(pairs: int, mode: str) -> dict:
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    img, soff, slen, sizes = build(pairs, mode)
    t_build = time.perf_counter() - t0
    n = len(soff)
    span_bytes = int(slen.sum())
    trailer = 8 * n

    # ---- end-to-end H2D (pageable numpy, then pinned) -------------------------
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d_img = torch.from_numpy(img).to(dev)
    torch.cuda.synchronize()
    t_h2d_pageable = time.perf_counter() - t0
    pinned = torch.empty(img.nbytes, dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = img
    t0 = time.perf_counter()
    d_img.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize()
    t_h2d_pinned = time.perf_counter() - t0

    d_off = torch.from_numpy(soff).to(dev)
    d_len = torch.from_numpy(slen).to(dev)
    # ---- write pass: compute + store every commit CRC on the GPU ---------------
    def write():
        zsfile.write_commits(d_img, d_off, d_len)

    write()
    torch.cuda.synchronize()
    t_write = ev_time(write)

    # ---- verify pass ------------------------------------------------------------
    out = {}

    def verify():
        out["crc"], out["st"] = zsfile.verify_commits(d_img, d_off, d_len)

    t_verify = ev_time(verify)
    st = out["st"].cpu().numpy()
    ok_all = bool((st == 1).all())

    # ---- host walk (what verify-on-open does before the GPU pass) --------------
    host_img = d_img.cpu().numpy()
    t0 = time.perf_counter()
    base, walked = 0, 0
    for sz in sizes.tolist():
        o, l, rc, end = zsfile.walk(host_img[base:base + sz])
        assert rc == zsfile.END and end == sz, (rc, end, sz)
        walked += len(o)
        base += sz
    t_walk = time.perf_counter() - t0
    assert walked == n

    # ---- oracle spot check of the GPU-written image -----------------------------
    rng = np.random.default_rng(1)
    sample = rng.choice(n, size=min(n, 2000), replace=False)
    for i in sample.tolist():
        o, L = int(soff[i]), int(slen[i])
        w0 = int.from_bytes(host_img[o + L:o + L + 8].tobytes(), "big")
        want = oracle.crc32c_hw(oracle.crc32c_hw(0, host_img[o:o + L]),
                                (w0 & 0xFFFFFFFF00000000).to_bytes(8, "little"))
        assert want == (w0 & 0xFFFFFFFF), i

    # ---- CPU baseline: the same verify on one core (oracle hw path) -------------
    cpu_n = min(n, 200_000 if mode == "batched" else 200)
    t0 = oracle.now()
    oracle.batch(host_img, soff[:cpu_n].astype(np.uint64), slen[:cpu_n].astype(np.uint64),
                 impl="hw", threads=1)
    cpu_s = oracle.now() - t0
    cpu_gbs = int(slen[:cpu_n].sum()) / cpu_s / 1e9

    GB = 1e9
    return {
        "config": "config4 zsbench replay", "mode": mode, "pairs": pairs, "commits": n,
        "files": len(sizes), "image_bytes": int(img.nbytes), "span_bytes": span_bytes,
        "all_commits_verified": ok_all, "oracle_spot_checks": int(len(sample)),
        "write_ms": round(t_write, 3), "verify_ms": round(t_verify, 3),
        "verify_GBs_device": round((span_bytes + trailer) / (t_verify * 1e-3) / GB, 1),
        "write_GBs_device": round((span_bytes + trailer) / (t_write * 1e-3) / GB, 1),
        "h2d_pageable_GBs": round(img.nbytes / t_h2d_pageable / GB, 2),
        "h2d_pinned_GBs": round(img.nbytes / t_h2d_pinned / GB, 2),
        "host_walk_s": round(t_walk, 3),
        "e2e_verify_pinned_GBs": round(img.nbytes / (t_h2d_pinned + t_verify * 1e-3) / GB, 2),
        "e2e_verify_pinned_with_walk_GBs": round(img.nbytes / (t_h2d_pinned + t_walk + t_verify * 1e-3) / GB, 2),
        "cpu_1core_verify_GBs": round(cpu_gbs, 2),
        "build_s": round(t_build, 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=10_000_000)
    ap.add_argument("--mode", default="both")
    a = ap.parse_args()
    for m in (["batched", "notbatched"] if a.mode == "both" else [a.mode]):
        print(json.dumps(run(a.pairs, m)), flush=True)


if __name__ == "__main__":
    main()
