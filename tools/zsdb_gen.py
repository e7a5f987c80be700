#!/usr/bin/env python3
"""Synthetic zeroskip DB directories for BASELINE config 5,
generated on the GPU.

Layout, oldest first (file names as zeroskip-filename.c:18-67 makes them):
  packed     zeroskip-<uuid>-<s>-<e>   [Header][records][commit][count][ptrs][final]
             (zeroskip-packed.c:384-473; records regions > 16 MiB get LONG commits)
  finalised  zeroskip-<uuid>-<i>-<i>   zsbench writeseqtxn pairs (key "%016d",
             255-char value + NUL, one commit per pair) up to >= 2 MiB, closed by
             the zero-length commit zs_active_file_finalise writes after a
             committed transaction (stale CRC: zeroskip-active.c:122 +
             mfile.c:534-546)
  active     zeroskip-<uuid>-<n>       the same pairs, no finalise
  .zsdb      offset = active size, curidx = n (zeroskip-dotzsdb.c)

By default every CRC is written by the engine itself -- the commit CRCs by
the GPU writer (zscrc_device_write_commits), header / .zsdb / stale-commit
words by libzscrc's host functions -- so this is the engine acting as
zeroskip's writer.  tests/test_gpu_consistent.py re-checks generated DBs with
the independent oracle walker (oracle/zs_format.py).

writer="cpu" (CLI --cpu-writer; test infrastructure) writes every commit CRC
with the CPU oracle instead (oracle/zs_bulk_oracle.c oracle_write_commits,
the writer of src/zeroskip-file.c:253-350, on host threads): images the GPU
verifier then checks without the GPU writer ever having touched them, so
writer and verifier are never each other's only witness.
"""
from __future__ import annotations

import os
import struct
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from zeroskip_amd import zsfile  # noqa: E402
from zeroskip_amd.crc32c import crc32c_hw  # noqa: E402

SIG = 0x5A45524F534B4950
HDR = 40
TWOMB = 2 << 20
T_KEY, T_VALUE, T_COMMIT, T_2ND, T_FINAL, T_LONG_COMMIT, T_LONG_FINAL = 1, 2, 4, 8, 16, 36, 48
MAX_SHORT = 16777215
KEYREC, VALREC, PAIR = 40, 272, 320          # zsbench: 16 B key, 256 B value
CHARSET = (b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
           b"0123456789!@#$%^&*()-=_+|{}[];<>,./?:")     # zsbench.c:125-129


def _be64(v: int) -> torch.Tensor:
    return torch.tensor(list(int(v).to_bytes(8, "big")), dtype=torch.uint8)


def header(uuid: bytes, s: int, e: int) -> bytes:
    h = bytearray(struct.pack("<Q", SIG) + struct.pack(">I", 1) + uuid + struct.pack(">III", s, e, 0))
    _, _, c = zsfile.header_crc(bytes(h))
    h[36:40] = struct.pack(">I", c)
    return bytes(h)


def dotzsdb(offset: int, uuidstr: bytes, curidx: int) -> bytes:
    d = bytearray(struct.pack("<Q", SIG) + struct.pack(">Q", offset) + uuidstr + struct.pack(">II", curidx, 0))
    _, _, c = zsfile.dotzsdb_crc(bytes(d))
    d[57:61] = struct.pack(">I", c)
    return bytes(d)


def _digits(ids: torch.Tensor) -> torch.Tensor:
    """"%016d" of each id as [n, 16] uint8."""
    p = torch.tensor([10 ** k for k in range(15, -1, -1)], dtype=torch.int64, device=ids.device)
    return (48 + (ids[:, None] // p[None, :]) % 10).to(torch.uint8)


def _charset_values(n: int, vlen: int, gen: torch.Generator, device) -> torch.Tensor:
    cs = torch.tensor(list(CHARSET), dtype=torch.uint8, device=device)
    v = cs[torch.randint(0, len(CHARSET), (n, vlen), generator=gen, device=device)]
    v[:, -1] = 0
    return v


def _cpu_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n)


def write_commits(flat: torch.Tensor, offs: torch.Tensor, lens: torch.Tensor, writer: str = "gpu") -> None:
    """Commit CRCs of the spans [offs, +lens) of `flat` into their records:
    the GPU writer, or (writer="cpu") the CPU oracle's writer on host threads
    (the image goes to the host and back)."""
    if writer == "gpu":
        zsfile.write_commits(flat, offs, lens)
        return
    assert writer == "cpu", writer
    from oracle import oracle     # test infrastructure: the checker acting as the writer
    host = flat.cpu().numpy()
    oracle.write_commits(host, offs.cpu().numpy(), lens.cpu().numpy(), threads=_cpu_threads())
    flat.copy_(torch.from_numpy(host))


def _span_crcs(flat: torch.Tensor, offs: torch.Tensor, lens: torch.Tensor, writer: str) -> list:
    if writer == "gpu":
        from zeroskip_amd.device import crc_batch
        return [c & 0xFFFFFFFF for c in crc_batch(flat, offs, lens).cpu().tolist()]
    from oracle import oracle
    host = flat.cpu().numpy()
    return [int(c) for c in oracle.batch(host, offs.cpu().numpy(), lens.cpu().numpy(), threads=_cpu_threads())]


def log_files(uuid: bytes, first_idx: int, nfiles: int, pairs: int, first_pair: int,
              finalise: bool, gen, device, batched: bool = True, writer: str = "gpu") -> torch.Tensor:
    """[nfiles, size] uint8 zsbench log files (zsbench.c:159-217), commit
    CRCs written by the GPU (writer="cpu": by the CPU oracle).  batched: one
    commit per pair (writeseqtxn); else one commit closing each file
    (writeseq: the finalise at 2 MiB commits the open transaction).
    `finalise` (batched only) appends the stale zero-length commit of
    zs_active_file_finalise."""
    pair = PAIR if batched else KEYREC + VALREC
    tail = 8 if (finalise or not batched) else 0
    size = HDR + pairs * pair + tail
    img = torch.zeros(nfiles, size, dtype=torch.uint8, device=device)
    body = img[:, HDR:HDR + pairs * pair].view(nfiles, pairs, pair)
    body[:, :, 0:8] = _be64((T_KEY << 56) | (16 << 40) | KEYREC).to(device)
    ids = torch.arange(first_pair, first_pair + nfiles * pairs, dtype=torch.int64, device=device)
    body[:, :, 24:40] = _digits(ids).view(nfiles, pairs, 16)
    body[:, :, 40:48] = _be64((T_VALUE << 56) | (256 << 32)).to(device)
    body[:, :, 56:312] = _charset_values(nfiles * pairs, 256, gen, device).view(nfiles, pairs, 256)
    for f in range(nfiles):
        img[f, :HDR] = torch.tensor(list(header(uuid, first_idx + f, first_idx + f)), dtype=torch.uint8)
    flat = img.view(-1)
    base = torch.arange(nfiles, dtype=torch.int64, device=device)[:, None] * size
    if not batched:
        n = pairs * pair
        img[:, size - 8:] = _be64((T_COMMIT << 56) | (n << 32)).to(device)
        offs = (base[:, 0] + HDR).contiguous()
        write_commits(flat, offs, torch.full_like(offs, n), writer)
        return img
    body[:, :, 312:320] = _be64((T_COMMIT << 56) | (312 << 32)).to(device)
    offs = (base + HDR + torch.arange(pairs, dtype=torch.int64, device=device)[None, :] * PAIR).reshape(-1)
    write_commits(flat, offs, torch.full_like(offs, 312), writer)
    if finalise:
        # mf->crc32 still holds crc32c(0, last span): the finalise commit hashes it
        last = (base[:, 0] + HDR + (pairs - 1) * PAIR).contiguous()
        span_crc = _span_crcs(flat, last, torch.full_like(last, 312), writer)
        w = T_COMMIT << 56
        if writer == "gpu":
            tail = [w | crc32c_hw(c, struct.pack("<Q", w)) for c in span_crc]
        else:
            from oracle import oracle
            tail = [w | oracle.commit_crc(c, 0) for c in span_crc]
        img[:, size - 8:] = torch.tensor([list(t.to_bytes(8, "big")) for t in tail],
                                         dtype=torch.uint8, device=device)
    return img


def log_spans(nfiles: int, pairs: int, batched: bool, finalise: bool, device):
    """(span_off, span_len) int64 device tensors of every commit of
    log_files(...) laid out back to back (the stale finalise commits included)."""
    pair = PAIR if batched else KEYREC + VALREC
    tail = 8 if (finalise or not batched) else 0
    size = HDR + pairs * pair + tail
    base = torch.arange(nfiles, dtype=torch.int64, device=device)[:, None] * size
    if not batched:
        offs = base[:, 0] + HDR
        return offs.contiguous(), torch.full_like(offs, pairs * pair)
    offs = base + HDR + torch.arange(pairs, dtype=torch.int64, device=device)[None, :] * PAIR
    lens = torch.full_like(offs, 312)
    if finalise:
        offs = torch.cat([offs, base + size - 8], 1)
        lens = torch.cat([lens, torch.zeros_like(base)], 1)
    return offs.reshape(-1).contiguous(), lens.reshape(-1).contiguous()


def pairs_per_file(batched: bool = True) -> int:
    """Pairs added before the active file reaches 2 MiB (zeroskip.c:914-925)."""
    return -(-(TWOMB - HDR) // (PAIR if batched else KEYREC + VALREC))


def packed_file(uuid: bytes, s: int, e: int, region_bytes: int, vlen: int, first_key: int,
                gen, device, writer: str = "gpu") -> tuple[torch.Tensor, int]:
    """One packed file with ~region_bytes of key/value records in key order
    (and its record count)."""
    vrec = 16 + ((vlen + 7) & ~7)
    pair = KEYREC + vrec
    n = max(1, region_bytes // pair)
    rlen = n * pair
    rcommit = 24 if rlen > MAX_SHORT else 8
    plen = 8 + 8 * n
    fcommit = 24 if plen > MAX_SHORT else 8
    size = HDR + rlen + rcommit + plen + fcommit
    img = torch.randint(0, 256, (size,), dtype=torch.uint8, generator=gen, device=device)
    img[:HDR] = torch.tensor(list(header(uuid, s, e)), dtype=torch.uint8)
    recs = img[HDR:HDR + rlen].view(n, pair)
    recs[:, 0:8] = _be64((T_KEY << 56) | (16 << 40) | KEYREC).to(device)
    recs[:, 8:24] = 0
    recs[:, 24:40] = _digits(torch.arange(first_key, first_key + n, dtype=torch.int64, device=device))
    recs[:, 40:48] = _be64((T_VALUE << 56) | (vlen << 32)).to(device)
    recs[:, 48:56] = 0
    if vrec - 16 > vlen:
        recs[:, 56 + vlen:] = 0
    r = HDR + rlen
    if rcommit == 24:
        img[r:r + 8] = _be64(T_LONG_COMMIT << 56).to(device)
        img[r + 8:r + 16] = _be64(rlen).to(device)
        img[r + 16:r + 24] = _be64(T_2ND << 56).to(device)
    else:
        img[r:r + 8] = _be64((T_COMMIT << 56) | (rlen << 32)).to(device)
    p = r + rcommit
    ptrs = torch.empty(n + 1, dtype=torch.int64, device=device)
    ptrs[0] = n
    ptrs[1:] = HDR + torch.arange(n, dtype=torch.int64, device=device) * pair
    img[p:p + plen] = ptrs.view(torch.uint8).view(-1, 8).flip(1).reshape(-1)   # big-endian
    fo = p + plen
    if fcommit == 24:
        img[fo:fo + 8] = _be64(T_LONG_FINAL << 56).to(device)
        img[fo + 8:fo + 16] = _be64(plen).to(device)
        img[fo + 16:fo + 24] = _be64(T_2ND << 56).to(device)
    else:
        img[fo:fo + 8] = _be64((T_FINAL << 56) | (plen << 32)).to(device)
    write_commits(img, torch.tensor([HDR, p], dtype=torch.int64, device=device),
                  torch.tensor([rlen, plen], dtype=torch.int64, device=device), writer)
    return img, n


def make_db(device="cuda", packed: int = 2, packed_region_bytes: int = 3 << 30, packed_vlen: int = 4064,
            finalised: int = 1024, active_pairs: int = 1000, seed: int = 0x5EED,
            uuid: bytes = bytes(range(16)), writer: str = "gpu") -> dict:
    """{file name: device uint8 tensor} + {".zsdb": bytes}; all on `device`.
    writer: "gpu" (the engine) or "cpu" (the CPU oracle) writes the commit CRCs."""
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    u = uuid.hex()
    uuidstr = f"{u[:8]}-{u[8:12]}-{u[12:16]}-{u[16:20]}-{u[20:]}"
    name = lambda *ix: "zeroskip-" + uuidstr + "".join(f"-{i}" for i in ix)  # noqa: E731
    db, idx, key = {}, 0, 0
    span = 8
    for k in range(packed):
        img, n = packed_file(uuid, idx, idx + span - 1, packed_region_bytes, packed_vlen, key, gen, device,
                             writer)
        db[name(idx, idx + span - 1)] = img
        key += n
        idx += span
    pairs = pairs_per_file()
    if finalised:
        logs = log_files(uuid, idx, finalised, pairs, key, True, gen, device, writer=writer)
        for f in range(finalised):
            db[name(idx + f, idx + f)] = logs[f]
        idx += finalised
        key += finalised * pairs
    act = log_files(uuid, idx, 1, active_pairs, key, False, gen, device, writer=writer)[0]
    db[name(idx)] = act
    db[".zsdb"] = dotzsdb(act.numel(), uuidstr.encode() + b"\0", idx)
    return db


def write_dir(db: dict, path: str) -> int:
    os.makedirs(path, exist_ok=True)
    total = 0
    for n, v in db.items():
        data = v if isinstance(v, (bytes, bytearray)) else v.cpu().numpy().tobytes()
        with open(os.path.join(path, n), "wb") as fh:
            fh.write(data)
        total += len(data)
    return total


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--packed", type=int, default=2)
    ap.add_argument("--packed-mib", type=int, default=3072)
    ap.add_argument("--finalised", type=int, default=1024)
    ap.add_argument("--cpu-writer", action="store_true",
                    help="commit CRCs written by the CPU oracle instead of the GPU writer (test infrastructure)")
    a = ap.parse_args()
    d = make_db(packed=a.packed, packed_region_bytes=a.packed_mib << 20, finalised=a.finalised,
                writer="cpu" if a.cpu_writer else "gpu")
    print(write_dir(d, a.out), "bytes written to", a.out)
