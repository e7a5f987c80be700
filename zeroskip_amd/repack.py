"""Repack output on the GPU: packed zeroskip files written through
libzscrc's packed-file writer (include/zscrc.h, zscrc_pack_*).

The writer mirrors the reference's repack output path
(zs_packed_file_new_from_memtree, src/zeroskip-packed.c:384-473, and
zs_packed_file_new_from_packed_files, :617-742): header, records in key order,
records-region commit, pointer section, final commit.  Every byte of the
records region and of the pointer section is checksummed on the GPU while the
host writes the file.  ``repack_dir`` runs zsdb_repack (src/zeroskip.c:
1419-1571) over a DB directory in ONE call into the library
(zscrc_zs_repack, zeroskip_amd/csrc/zscrc_repack.cpp): record listing, the
key merge (finalised files, or the reference's two packed files), the
writer, the unlinks and the .zsdb rewrite are all C++.
"""
from __future__ import annotations

import ctypes
import os

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
            # an exception mid-packing: no commits, the partial file removed
            h, self._h = self._h, ctypes.c_void_p()
            lib().zscrc_pack_abort(h)


_EMPTY = ctypes.c_uint8(0)


class RepackReport(ctypes.Structure):
    """zscrc_repack_report (include/zscrc.h)."""
    _fields_ = [("branch", ctypes.c_int32), ("startidx", ctypes.c_uint32), ("endidx", ctypes.c_uint32),
                ("files_merged", ctypes.c_uint64), ("records_in", ctypes.c_uint64),
                ("records_out", ctypes.c_uint64), ("dotzsdb_crc", ctypes.c_uint32), ("pack", PackReport),
                ("list_s", ctypes.c_double), ("merge_s", ctypes.c_double), ("write_s", ctypes.c_double),
                ("total_s", ctypes.c_double), ("path", ctypes.c_char * 4096)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("pack", "path")}
        d["pack"] = self.pack.as_dict()
        d["path"] = self.path.decode()
        return d


REFERENCE_COMPAT = 2  # ZSCRC_REPACK_REFERENCE_COMPAT


def repack_dir(dbdir: str, threads: int = 0, fsync: bool = False, reference_compat: bool = False) -> dict:
    """zsdb_repack over a DB directory (zscrc_zs_repack): branch 1 merges the
    finalised files, branch 2 the reference's two packed files; returns the
    report (branch 0: nothing to pack).  reference_compat: branch 2 writes the
    reference's bytes including its loss of records after a delete
    (src/zeroskip-iterator.c:258-259; include/zscrc.h)."""
    rep = RepackReport()
    flags = (FSYNC if fsync else 0) | (REFERENCE_COMPAT if reference_compat else 0)
    check(lib().zscrc_zs_repack(os.fsencode(dbdir), flags, threads, ctypes.byref(rep)), "zscrc_zs_repack")
    return rep.as_dict()


def records(image, kind: int):
    """(key_off, key_len, val_off, val_len) uint64 arrays of a file image's
    records (zscrc_zs_records); val_off == 2**64-1 marks a delete."""
    a = np.ascontiguousarray(np.frombuffer(image, dtype=np.uint8) if isinstance(image, (bytes, bytearray))
                             else image)
    cap = a.nbytes // 32 + 16
    while True:
        out = np.empty((cap, 4), np.uint64)
        n = ctypes.c_size_t()
        rc = lib().zscrc_zs_records(a.ctypes.data, a.nbytes, kind, out.ctypes.data, cap, ctypes.byref(n))
        if rc == 3:                              # ZSCRC_ZS_OVERFLOW
            cap = n.value
            continue
        if rc < 0:
            check(rc, "zscrc_zs_records")
        return out[:n.value].T.copy(), rc
