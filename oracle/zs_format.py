"""zeroskip on-disk format: writer + CRC verifier (TEST INFRASTRUCTURE ONLY).

Restates, for the checksummed parts, the reference's
  - header          src/zeroskip-header.c:30-94 (write), :105-170 (validate)
  - key/value/delete records  src/zeroskip-file.c:23-183
  - commit records  src/zeroskip-file.c:253-350 (WRITER semantics; the long
                    verifier in zeroskip-record.c:234-266 is broken)
  - record walk     src/zeroskip-record.c:283-331 (+ the key/value skip :156-181)
  - packed files    src/zeroskip-packed.c:384-473 (layout), :70-131 + :278-339
                    (pointer-section verify)
  - transaction CRC span semantics  src/zeroskip.c:863-951 (crc32_begin on the
                    first add of a txn), :953-1004 (remove: crc32_begin always),
                    src/mfile.c:526-546 (crc32_begin / crc32_end)
All CRCs come from oracle.crc32c_hw.  Numbers on disk are big-endian; the
CRC trailers are hashed as host (little-endian) 64-bit words.
"""
from __future__ import annotations

import struct

import numpy as np

from . import oracle

ZS_SIGNATURE = 0x5A45524F534B4950
ZS_VERSION = 1
HDR_SIZE = 40
REC_UNUSED, REC_KEY, REC_VALUE, REC_COMMIT, REC_2ND_HALF, REC_FINAL, REC_LONG, REC_DELETED = \
    0, 1, 2, 4, 8, 16, 32, 64
REC_LONG_KEY, REC_LONG_VALUE = REC_KEY | REC_LONG, REC_VALUE | REC_LONG
REC_LONG_COMMIT, REC_LONG_FINAL = REC_COMMIT | REC_LONG, REC_FINAL | REC_LONG
REC_LONG_DELETED = REC_LONG | REC_LONG  # == 32, as written in zeroskip-priv.h:119
MAX_SHORT_KEY_LEN = 65535
MAX_SHORT_VAL_LEN = 16777215
M64 = (1 << 64) - 1


def be64(v: int) -> bytes:
    return struct.pack(">Q", v & M64)


def le64(v: int) -> bytes:
    return struct.pack("<Q", v & M64)


def rup8(n: int) -> int:
    return (n + 7) & ~7


# ------------------------------------------------------------------ header
def header_crc(version: int, uuid: bytes, startidx: int, endidx: int) -> int:
    c = oracle.crc32c_hw(0, b"")
    c = oracle.crc32c_hw(c, struct.pack("<Q", ZS_SIGNATURE))
    c = oracle.crc32c_hw(c, struct.pack("<I", version))
    c = oracle.crc32c_hw(c, uuid)
    c = oracle.crc32c_hw(c, struct.pack("<I", startidx))
    return oracle.crc32c_hw(c, struct.pack("<I", endidx))


def header_bytes(uuid: bytes, startidx: int = 0, endidx: int = 0, version: int = ZS_VERSION) -> bytes:
    assert len(uuid) == 16
    crc = header_crc(version, uuid, startidx, endidx)
    return (struct.pack("<Q", ZS_SIGNATURE) + struct.pack(">I", version) + uuid +
            struct.pack(">III", startidx, endidx, crc))


def header_check(img: bytes) -> tuple[bool, int, int]:
    sig, = struct.unpack_from("<Q", img, 0)
    version, = struct.unpack_from(">I", img, 8)
    uuid = bytes(img[12:28])
    sidx, eidx, stored = struct.unpack_from(">III", img, 28)
    computed = header_crc(version, uuid, sidx, eidx)
    return sig == ZS_SIGNATURE and computed == stored, stored, computed


# ------------------------------------------------------------------ .zsdb
def dotzsdb_bytes(offset: int, uuidstr: bytes, curidx: int) -> bytes:
    """61-byte .zsdb (zeroskip-dotzsdb.c:70-150): native signature, BE64
    offset, 37-byte uuid string, BE32 index, BE32 CRC over host-order fields."""
    assert len(uuidstr) == 37
    crc = oracle.dotzsdb_crc(ZS_SIGNATURE, offset, uuidstr, curidx)
    return struct.pack("<Q", ZS_SIGNATURE) + struct.pack(">Q", offset) + uuidstr + \
        struct.pack(">II", curidx, crc)


# ------------------------------------------------------------------ records
def key_record(key: bytes) -> bytes:
    kbuflen = 24 + rup8(len(key))
    if len(key) > MAX_SHORT_KEY_LEN:
        head = be64(REC_LONG_KEY << 56) + be64(len(key)) + be64(kbuflen)
    else:
        head = be64((REC_KEY << 56) | (len(key) << 40) | kbuflen) + be64(0) + be64(0)
    return head + key + bytes(kbuflen - 24 - len(key))


def value_record(val: bytes) -> bytes:
    vbuflen = 16 + rup8(len(val))
    if len(val) > MAX_SHORT_VAL_LEN:
        head = be64(REC_LONG_VALUE << 56) + be64(len(val))
    else:
        head = be64((REC_VALUE << 56) | (len(val) << 32)) + be64(0)
    return head + val + bytes(vbuflen - 16 - len(val))


def delete_record(key: bytes) -> bytes:
    assert len(key) <= MAX_SHORT_KEY_LEN, "long delete records are never walkable (SURVEY App. A)"
    kbuflen = 24 + rup8(len(key))
    return be64((REC_DELETED << 56) | (len(key) << 40)) + be64(0) + be64(0) + key + \
        bytes(kbuflen - 24 - len(key))


def commit_record(span_crc: int, span_len: int, final: bool = False) -> bytes:
    """The 8- or 24-byte commit record closing a span whose crc32c(0, span) is
    span_crc (zeroskip-file.c:253-350)."""
    if span_len > MAX_SHORT_VAL_LEN:
        t1 = (REC_LONG_FINAL if final else REC_LONG_COMMIT) << 56
        t2 = REC_2ND_HALF << 56
        c = oracle.crc32c_hw(span_crc, le64(t1))
        c = oracle.crc32c_hw(c, le64(span_len))
        c = oracle.crc32c_hw(c, le64(t2))
        return be64(t1) + be64(span_len) + be64(t2 | c)
    w = ((REC_FINAL if final else REC_COMMIT) << 56) | (span_len << 32)
    c = oracle.crc32c_hw(span_crc, le64(w))
    return be64(w | c)


class FileWriter:
    """An active/finalised zeroskip file built the way zsdb_add / zsdb_remove /
    zsdb_commit build it (CRC span = bytes since crc32_begin)."""

    def __init__(self, uuid: bytes, idx: int = 0):
        self.buf = bytearray(header_bytes(uuid, idx, idx))
        self.begin = None  # crc32_begin offset, None = not computing
        self.mf_crc32 = 0  # struct mfile.crc32: xcalloc'd (mfile.c:50), then the last span CRC

    def add(self, key: bytes, val: bytes):
        if self.begin is None:       # zeroskip.c:930-931
            self.begin = len(self.buf)
        self.buf += key_record(key) + value_record(val)

    def remove(self, key: bytes):
        self.begin = len(self.buf)   # zeroskip.c:985 (unconditional crc32_begin)
        self.buf += delete_record(key)

    def commit(self, final: bool = False):
        begin = len(self.buf) if self.begin is None else self.begin
        span = bytes(self.buf[begin:])
        self.mf_crc32 = oracle.crc32c_hw(0, span)
        self.buf += commit_record(self.mf_crc32, len(span), final)
        self.begin = None

    def finalise(self):
        """zs_active_file_finalise (zeroskip-active.c:105-144) writes a commit
        unconditionally.  After an already-committed transaction
        crc32_data_len is 0 and crc32_end returns the STALE register of the
        previous span (mfile.c:534-546), so the record is a zero-length commit
        hashed from the previous span's CRC -- which the reference verifier
        (zeroskip-record.c:204-232, from 0) rejects unless there was no
        previous span."""
        if self.begin is not None:
            return self.commit()
        w = REC_COMMIT << 56
        self.buf += be64(w | oracle.crc32c_hw(self.mf_crc32, le64(w)))

    def image(self) -> bytes:
        return bytes(self.buf)


def packed_file(records, uuid: bytes, startidx: int, endidx: int) -> bytes:
    """[Header][records in key order][commit][count][ptrs][final commit]
    (zeroskip-packed.c:384-473).  records: [(key, value-or-None)] sorted."""
    buf = bytearray(header_bytes(uuid, startidx, endidx))
    ptrs = []
    for key, val in records:
        ptrs.append(len(buf))
        buf += delete_record(key) if val is None else key_record(key) + value_record(val)
    span = bytes(buf[HDR_SIZE:])
    buf += commit_record(oracle.crc32c_hw(0, span), len(span))
    pstart = len(buf)
    buf += be64(len(ptrs)) + b"".join(be64(p) for p in ptrs)
    pspan = bytes(buf[pstart:])
    buf += commit_record(oracle.crc32c_hw(0, pspan), len(pspan), final=True)
    return bytes(buf)


# ------------------------------------------------------------------ verify
def _commit_check(img, off: int, seed: int = 0):
    """Decode the commit record at `off`; return (span_off, span_len, rec_len,
    stored, computed) with the writer's trailer semantics.  `seed`: the CRC
    the span continues from (crc32_begin stores crc32c(0,0,0) = 0,
    mfile.c:526-532; a finalise without crc32_begin continues from the
    previous span's CRC, mfile.c:534-546)."""
    w0, = struct.unpack_from(">Q", img, off)
    t = w0 >> 56
    if t in (REC_COMMIT, REC_FINAL):
        n = (w0 >> 32) & 0xFFFFFF
        c = oracle.crc32c_hw(seed, bytes(img[off - n:off]))
        c = oracle.crc32c_hw(c, le64(w0 & 0xFFFFFFFF00000000))
        return off - n, n, 8, w0 & 0xFFFFFFFF, c
    if t in (REC_LONG_COMMIT, REC_LONG_FINAL):
        n, w2 = struct.unpack_from(">QQ", img, off + 8)
        c = oracle.crc32c_hw(seed, bytes(img[off - n:off]))
        c = oracle.crc32c_hw(c, le64(w0))
        c = oracle.crc32c_hw(c, le64(n))
        c = oracle.crc32c_hw(c, le64(w2 & 0xFF00000000000000))
        return off - n, n, 24, w2 & 0xFFFFFFFF, c
    raise ValueError(f"not a commit record at {off} (type {t})")


def walk(img) -> tuple[list[dict], int, str]:
    """Walk an active/finalised file from the header like
    zs_record_read_from_file (record.c:283-331).  Returns (commits, end offset,
    stop reason)."""
    commits, off, n = [], HDR_SIZE, len(img)
    while off < n:
        if off + 8 > n:
            return commits, off, "truncated"
        w0, = struct.unpack_from(">Q", img, off)
        t = w0 >> 56
        if t in (REC_KEY, REC_LONG_KEY):
            if t == REC_KEY:
                voff = w0 & 0xFFFFFFFF
            else:
                voff, = struct.unpack_from(">Q", img, off + 16)
            off += voff
            v0, = struct.unpack_from(">Q", img, off)
            vlen = (v0 >> 32) & 0xFFFFFF if (v0 >> 56) == REC_VALUE else \
                struct.unpack_from(">Q", img, off + 8)[0]
            off += 16 + rup8(vlen)
        elif t in (REC_DELETED, REC_LONG_DELETED):
            # zs_key_base.slen is a uint16_t (zeroskip-priv.h:124): the 24-bit
            # mask of record.c:87 is truncated to the key length by the store
            klen = (w0 >> 40) & 0xFFFF if t == REC_DELETED else struct.unpack_from(">Q", img, off + 8)[0]
            off += 24 + rup8(klen)
        elif t in (REC_COMMIT, REC_LONG_COMMIT):
            so, sl, rl, stored, computed = _commit_check(img, off)
            commits.append(dict(commit_off=off, span_off=so, span_len=sl, stored=stored,
                                computed=computed, ok=stored == computed))
            off += rl
        else:  # FINAL / 2ND_HALF / UNUSED / VALUE: the reference does not advance
            return commits, off, f"stop at type {t}"
    return commits, off, "end"


def packed_check(img) -> list[dict]:
    """The two commits of a packed file: records region and pointer section
    (zeroskip-packed.c:278-339, plus the records commit it never checks)."""
    n = len(img)
    w, = struct.unpack_from(">Q", img, n - 8)
    foff = n - 24 if (w >> 56) == REC_2ND_HALF else n - 8
    out = []
    so, sl, rl, stored, computed = _commit_check(img, foff)
    out.append(dict(kind="pointers", commit_off=foff, span_off=so, span_len=sl, stored=stored,
                    computed=computed, ok=stored == computed))
    w, = struct.unpack_from(">Q", img, so - 8)
    roff = so - 24 if (w >> 56) == REC_2ND_HALF else so - 8
    so2, sl2, rl2, st2, cp2 = _commit_check(img, roff)
    out.append(dict(kind="records", commit_off=roff, span_off=so2, span_len=sl2, stored=st2,
                    computed=cp2, ok=st2 == cp2))
    return out


# ------------------------------------------------------------------ records (repack)
def _record(img, off: int):
    """(key, value-or-None, next offset) of the key / delete record at off
    (zeroskip-record.c:38-181 read paths)."""
    w0, = struct.unpack_from(">Q", img, off)
    t = w0 >> 56
    if t in (REC_KEY, REC_LONG_KEY):
        if t == REC_KEY:
            klen, voff = (w0 >> 40) & 0xFFFF, w0 & 0xFFFFFFFF
        else:
            klen, voff = struct.unpack_from(">QQ", img, off + 8)
        v = off + voff
        vw, = struct.unpack_from(">Q", img, v)
        vlen = (vw >> 32) & 0xFFFFFF if (vw >> 56) == REC_VALUE else struct.unpack_from(">Q", img, v + 8)[0]
        return bytes(img[off + 24:off + 24 + klen]), bytes(img[v + 16:v + 16 + vlen]), v + 16 + rup8(vlen)
    if t in (REC_DELETED, REC_LONG_DELETED):
        klen = (w0 >> 40) & 0xFFFF if t == REC_DELETED else struct.unpack_from(">Q", img, off + 8)[0]
        return bytes(img[off + 24:off + 24 + klen]), None, off + 24 + rup8(klen)
    return None


def file_records(img) -> list:
    """[(key, value-or-None)] of an active / finalised file in file order:
    the record walk of zeroskip-record.c:283-331, commits skipped."""
    out, off, n = [], HDR_SIZE, len(img)
    while off + 8 <= n:
        t = img[off]
        if t in (REC_COMMIT, REC_LONG_COMMIT):
            off += 8 if t == REC_COMMIT else 24
            continue
        r = _record(img, off)
        if r is None:
            break
        out.append(r[:2])
        off = r[2]
    return out


def packed_records(img) -> list:
    """[(key, value-or-None)] of a packed file in pointer order
    (zeroskip-packed.c:70-131: the pointer section after the records commit)."""
    pc = packed_check(img)[0]
    poff = pc["span_off"]
    count, = struct.unpack_from(">Q", img, poff)
    ptrs = struct.unpack_from(">%dQ" % count, img, poff + 8)
    return [_record(img, p)[:2] for p in ptrs]


def repack_finalised(images) -> list:
    """Branch 1 of zsdb_repack (src/zeroskip.c:1460-1505): finalised files
    loaded oldest first into the memtree (a later record of a key replaces an
    earlier one, deletes kept), walked in key order."""
    merged = {}
    for img in images:
        for k, v in file_records(img):
            merged[k] = v
    return sorted(merged.items())


def repack_packed(older, newer) -> list:
    """Branch 2 (src/zeroskip.c:1510-1565, zeroskip-packed.c:617-742) on the
    two files it takes: on a key in both, the older file's record (its
    iterator priority is the larger, zeroskip.c:520-526); a winning delete
    drops the key."""
    merged = dict(packed_records(newer))
    merged.update(packed_records(older))
    return sorted((k, v) for k, v in merged.items() if v is not None)


# ------------------------------------------------------------------ bulk (zsbench replay)
def zsbench_key(i: int) -> bytes:
    return b"%016d" % i  # benchmark/zsbench.c:183


def zsbench_values(n: int, vallen: int, seed: int) -> np.ndarray:
    """vallen-1 chars of the zsbench charset + NUL (zsbench.c:123-143) per
    value, from a fixed-seed PRNG (the reference seeds from time())."""
    charset = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
                            b"0123456789!@#$%^&*()-=_+|{}[];<>,./?:", dtype=np.uint8)
    rng = np.random.default_rng(seed)
    v = charset[rng.integers(0, len(charset), (n, vallen), dtype=np.int64)]
    v[:, -1] = 0
    return v
