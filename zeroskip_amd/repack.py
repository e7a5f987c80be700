"""Repack output on the GPU: packed zeroskip files written through
libzscrc's packed-file writer (include/zscrc.h, zscrc_pack_*).

The writer mirrors the reference's repack output path
(zs_packed_file_new_from_memtree, src/zeroskip-packed.c:384-473, and
zs_packed_file_new_from_packed_files, :617-742): header, records in key order,
records-region commit, pointer section, final commit.  Every byte of the
records region and of the pointer section is checksummed on the GPU while the
host writes the file.  ``repack_dir`` is the driver of zsdb_repack
(src/zeroskip.c:1419-1571) for the checksum-relevant part: it merges the
finalised files of a DB directory (newest record of a key wins, deletes kept
as delete records, as the memtree of finalised records holds them) into one
packed file.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

from ._lib import check, lib

FSYNC = 1  # ZSCRC_PACK_FSYNC


class PackReport(ctypes.Structure):
    _fields_ = [("records", ctypes.c_uint64), ("region_bytes", ctypes.c_uint64),
                ("file_bytes", ctypes.c_uint64), ("region_crc", ctypes.c_uint32),
                ("pointers_crc", ctypes.c_uint32), ("commit_crc", ctypes.c_uint32),
                ("final_crc", ctypes.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Packer:
    """with Packer(path, uuid, startidx, endidx) as p: p.add(key, value); ...
    Keys must be added in key order; value None writes a delete record."""

    def __init__(self, path: str, uuid: bytes, startidx: int = 0, endidx: int = 0,
                 chunk_bytes: int = 0, fsync: bool = False):
        assert len(uuid) == 16
        self._h = ctypes.c_void_p()
        check(lib().zscrc_pack_open(ctypes.byref(self._h), os.fsencode(path), bytes(uuid), startidx, endidx,
                                    chunk_bytes, FSYNC if fsync else 0), "zscrc_pack_open")
        self.report: dict | None = None

    def add(self, key, value=None) -> None:
        k = np.frombuffer(key, dtype=np.uint8) if isinstance(key, (bytes, bytearray, memoryview)) else key
        if value is None:
            check(lib().zscrc_pack_add(self._h, k.ctypes.data, k.nbytes, None, 0), "zscrc_pack_add")
            return
        v = np.frombuffer(value, dtype=np.uint8) if isinstance(value, (bytes, bytearray, memoryview)) else value
        # a zero-length value still needs a non-NULL pointer (NULL = delete)
        vp = v.ctypes.data if v.nbytes else ctypes.addressof(_EMPTY)
        check(lib().zscrc_pack_add(self._h, k.ctypes.data, k.nbytes, vp, v.nbytes), "zscrc_pack_add")

    def add_many(self, records) -> None:
        """(key, value-or-None) pairs in key order, one library call
        (zscrc_pack_add_batch): keys and values packed into two blobs."""
        records = list(records)
        if not records:
            return
        klen = np.fromiter((len(k) for k, _ in records), dtype=np.uint64, count=len(records))
        koff = np.zeros(len(records), dtype=np.uint64)
        np.cumsum(klen[:-1], out=koff[1:])
        kblob = np.frombuffer(b"".join(k for k, _ in records) or b"\0", dtype=np.uint8)
        vlen = np.fromiter((0 if v is None else len(v) for _, v in records), dtype=np.uint64, count=len(records))
        voff = np.zeros(len(records), dtype=np.uint64)
        np.cumsum(vlen[:-1], out=voff[1:])
        voff[[i for i, (_, v) in enumerate(records) if v is None]] = ~np.uint64(0)
        vblob = np.frombuffer(b"".join(v for _, v in records if v is not None) or b"\0", dtype=np.uint8)
        self.add_arrays(kblob, koff, klen, vblob, voff, vlen)

    def add_arrays(self, kblob, koff, klen, vblob, voff, vlen) -> None:
        """Records i = kblob[koff[i]:+klen[i]] -> vblob[voff[i]:+vlen[i]]
        (voff[i] == 2**64-1: a delete; vblob None: all deletes), numpy arrays,
        no copies (values may share bytes)."""
        n = len(koff)
        koff, klen = np.ascontiguousarray(koff, np.uint64), np.ascontiguousarray(klen, np.uint64)
        kblob = np.ascontiguousarray(kblob).view(np.uint8)
        assert len(klen) == n and (n == 0 or int((koff + klen).max()) <= kblob.nbytes)
        vp = op = lp = None
        if vblob is not None:
            vblob = np.ascontiguousarray(vblob).view(np.uint8)
            voff, vlen = np.ascontiguousarray(voff, np.uint64), np.ascontiguousarray(vlen, np.uint64)
            live = voff != ~np.uint64(0)
            assert len(voff) == n and len(vlen) == n
            assert not live.any() or int((voff[live] + vlen[live]).max()) <= vblob.nbytes
            vp, op, lp = vblob.ctypes.data, voff.ctypes.data, vlen.ctypes.data
        check(lib().zscrc_pack_add_batch(self._h, kblob.ctypes.data, koff.ctypes.data, klen.ctypes.data,
                                         vp, op, lp, n), "zscrc_pack_add_batch")

    def close(self) -> dict:
        if self._h:
            rep = PackReport()
            h, self._h = self._h, ctypes.c_void_p()
            check(lib().zscrc_pack_close(h, ctypes.byref(rep)), "zscrc_pack_close")
            self.report = rep.as_dict()
        return self.report

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        if et is None:
            self.close()
        elif self._h:
            h, self._h = self._h, ctypes.c_void_p()
            lib().zscrc_pack_close(h, None)   # frees the writer (file kept as written)


_EMPTY = ctypes.c_uint8(0)


def _records_of(image) -> list[tuple[bytes, bytes | None]]:
    """(key, value-or-None) of every record of an active/finalised file, in
    file order, by the reference walk (src/zeroskip-record.c:283-331)."""
    buf = memoryview(image)
    out, off, n = [], 40, len(buf)
    while off + 8 <= n:
        w, = struct.unpack_from(">Q", buf, off)
        t = w >> 56
        if t in (1, 33):                              # KEY / LONG_KEY
            if t == 1:
                klen, voff = (w >> 40) & 0xFFFF, w & 0xFFFFFFFF
            else:
                klen, voff = struct.unpack_from(">QQ", buf, off + 8)
            key = bytes(buf[off + 24:off + 24 + klen])
            v = off + voff
            vw, = struct.unpack_from(">Q", buf, v)
            vlen = (vw >> 32) & 0xFFFFFF if (vw >> 56) == 2 else struct.unpack_from(">Q", buf, v + 8)[0]
            out.append((key, bytes(buf[v + 16:v + 16 + vlen])))
            off = v + 16 + ((vlen + 7) & ~7)
        elif t in (64, 32):                           # DELETED / LONG_DELETED
            klen = (w >> 40) & 0xFFFF if t == 64 else struct.unpack_from(">Q", buf, off + 8)[0]
            out.append((bytes(buf[off + 24:off + 24 + klen]), None))
            off += 24 + ((klen + 7) & ~7)
        elif t in (4, 36):                            # COMMIT / LONG_COMMIT
            off += 8 if t == 4 else 24
        else:
            break
    return out


def repack_dir(dbdir: str, out_path: str, uuid: bytes, startidx: int, endidx: int,
               chunk_bytes: int = 0) -> dict:
    """Merge the finalised files `zeroskip-<uuid>-<idx>-<idx>` of dbdir (in
    index order; the newest record of a key wins) into one packed file at
    out_path, CRCs on the GPU.  Returns the writer's report."""
    from . import consistent, zsfile
    db = consistent.open_db(dbdir)
    merged: dict[bytes, bytes | None] = {}
    for f in db.files:                     # sorted by index: newer files last
        if f.kind == zsfile.FINALISED:
            for k, v in _records_of(f.image):
                merged[k] = v
    keys = sorted(merged)
    with Packer(out_path, uuid, startidx, endidx, chunk_bytes=chunk_bytes) as p:
        for i in range(0, len(keys), 65536):
            p.add_many((k, merged[k]) for k in keys[i:i + 65536])
    return p.report
