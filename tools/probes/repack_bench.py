#!/usr/bin/env python3
"""repack's records-region CRC (one crc32_end over the whole
region, src/zeroskip-packed.c:442 -> src/mfile.c:534-546) on the GPU.

Times, over the same host bytes (anonymous memory and a file-backed mmap):
  cpu      libzscrc's CPU path (crc32c_hw below the offload threshold, 1 thread)
  stream   zscrc_stream copy mode (pinned staging, the caller may reuse its buffer)
  nocopy   zscrc_stream NOCOPY (DMA straight from the caller's memory)
  scalar   crc32c_hw with ZSCRC_GPU_MIN set (the unchanged reference symbol)
All results are checked equal.  Prints one JSON line per source.

--pack N additionally writes a packed file of N records (16-byte keys, values
of --value-bytes) through the packed-file writer (zscrc_pack_*, records and
pointer CRCs on the GPU while the host writes the file), and times the CPU
crc32_end the reference would run over the same records region afterwards
(src/zeroskip-packed.c:442, one core).
--repack-dir N runs zsdb_repack (src/zeroskip.c:1419-1571) through
zscrc_zs_repack over a generated DB directory, branch 1 (finalised zsbench
log files holding N pairs) and branch 2 (two packed files of N/2 records
each), and reports the library's own list / merge / write split against the
wall time of the Python call (the Python share).
usage: python tools/probes/repack_bench.py [--mib 4096] [--file /tmp/x] [--pack N --out /tmp/p] [--repack-dir N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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


def pack(nrec: int, vbytes: int, out: str, chunk: int) -> dict:
    from zeroskip_amd import repack
    rng = np.random.default_rng(7)
    vals = rng.integers(0, 256, (64, vbytes), dtype=np.uint8)     # 64 distinct values, reused
    keys = [b"%016d" % i for i in range(nrec)]
    kblob = np.frombuffer(b"".join(keys), dtype=np.uint8)
    koff = np.arange(nrec, dtype=np.uint64) * 16
    klen = np.full(nrec, 16, dtype=np.uint64)
    voff = (np.arange(nrec, dtype=np.uint64) & np.uint64(63)) * np.uint64(vbytes)
    vlen = np.full(nrec, vbytes, dtype=np.uint64)
    t0 = time.perf_counter()
    with repack.Packer(out, bytes(range(16)), 1, 2, chunk_bytes=chunk) as p:
        if os.environ.get("PACK_PER_RECORD"):
            for i, k in enumerate(keys):
                p.add(k, vals[i & 63])
        else:   # one zscrc_pack_add_batch per 65,536 records
            for i in range(0, nrec, 65536):
                p.add_arrays(kblob, koff[i:i + 65536], klen[i:i + 65536], vals, voff[i:i + 65536],
                             vlen[i:i + 65536])
    t_pack = time.perf_counter() - t0
    rep = p.report
    mm = np.memmap(out, dtype=np.uint8, mode="r")
    region = mm[40:40 + rep["region_bytes"]]
    lib().zscrc_set_gpu_min(0)
    t_crc, c = timed(lambda: zc.crc32c_hw(0, region), 2)
    assert c == rep["region_crc"], (hex(c), hex(rep["region_crc"]))
    del region, mm
    os.unlink(out)
    return {"source": "packed-file writer", "records": nrec, "value_bytes": vbytes,
            "file_bytes": rep["file_bytes"], "pack_s": round(t_pack, 3),
            "pack_GBs": round(rep["file_bytes"] / t_pack / 1e9, 2),
            "cpu_region_crc_s": round(t_crc, 3), "cpu_region_crc_GBs": round(rep["region_bytes"] / t_crc / 1e9, 2),
            "api": "per-record zscrc_pack_add" if os.environ.get("PACK_PER_RECORD") else
                   "zscrc_pack_add_batch, 65,536 records per call",
            "note": "pack_s includes serialising every record, the GPU CRCs and the "
                    "file writes; cpu_region_crc_s is the reference's extra one-core crc32_end over the "
                    "written region (what the GPU pipeline removes)"}


def repack_dirs(nrec: int, tmp: str) -> list:
    import shutil
    import tempfile
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import zsdb_gen
    from zeroskip_amd import repack
    out = []
    per = zsdb_gen.pairs_per_file()
    cases = (("finalised", dict(packed=0, finalised=-(-nrec // per), active_pairs=100)),
             ("packed", dict(packed=2, packed_region_bytes=(nrec // 2) * 120, packed_vlen=64, finalised=0,
                             active_pairs=100)))
    for name, kw in cases:
        d = tempfile.mkdtemp(prefix="zsrepack_", dir=tmp)
        try:
            db = zsdb_gen.make_db("cuda", **kw)
            nbytes = zsdb_gen.write_dir(db, d)
            del db
            t0 = time.perf_counter()
            rep = repack.repack_dir(d)
            wall = time.perf_counter() - t0
            out.append({"source": "zscrc_zs_repack", "branch": rep["branch"], "input": name,
                        "db_bytes": nbytes, "records_in": rep["records_in"], "records_out": rep["records_out"],
                        "files_merged": rep["files_merged"], "out_bytes": rep["pack"]["file_bytes"],
                        "list_s": round(rep["list_s"], 3), "merge_s": round(rep["merge_s"], 3),
                        "write_s": round(rep["write_s"], 3), "total_s": round(rep["total_s"], 3),
                        "wall_s": round(wall, 3), "python_share": round(max(0.0, wall - rep["total_s"]) / wall, 4),
                        "records_per_s": round(rep["records_in"] / wall), "note": "page-cache files, no fsync"})
        finally:
            shutil.rmtree(d, ignore_errors=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=4096)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--file", default=None)
    ap.add_argument("--pack", type=int, default=0, help="records for the packed-file writer leg")
    ap.add_argument("--value-bytes", type=int, default=16384)
    ap.add_argument("--out", default="/tmp/zscrc_pack_bench")
    ap.add_argument("--repack-dir", type=int, default=0, help="pairs for the zscrc_zs_repack leg")
    ap.add_argument("--tmp", default="/tmp")
    a = ap.parse_args()
    if a.repack_dir:
        for r in repack_dirs(a.repack_dir, a.tmp):
            print(json.dumps(r), flush=True)
        return
    if a.pack:
        print(json.dumps(pack(a.pack, a.value_bytes, a.out, a.chunk_mib << 20)), flush=True)
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
