"""zsdb_consistent on the GPU(s): a full re-checksum of a zeroskip DB directory.

The reference declares the operation and implements nothing:
``zsdb_consistent`` returns ZS_NOTIMPLEMENTED (src/zeroskip.c:1399-1407) and
``zeroskip consistent`` parses its options and exits 0
(tool/cmd-consistent.c:23-49).  SURVEY.md §8f-2 defines it for this engine as
"every CRC the format carries, recomputed":

* ``.zsdb``: signature + CRC over its host-order fields
  (src/zeroskip-dotzsdb.c:105-119, struct zeroskip-priv.h:83-91);
* every ``zeroskip-<uuid>-<idx>[-<idx>]`` file (names interpreted like
  interpret_db_filename, src/zeroskip.c:200-235): header signature + CRC
  (src/zeroskip-header.c:105-170), header indices against the file name;
* active / finalised files: the record walk of src/zeroskip-record.c:283-331
  and every commit CRC (writer semantics, src/zeroskip-file.c:253-350);
* packed files: the pointer-section commit the reference checks
  (src/zeroskip-packed.c:278-339) AND the records-region commit it never
  checks (written by zeroskip-packed.c:442 through one crc32_end).

Zero-length commits whose CRC is the previous span's register hashed with the
trailer -- what zs_active_file_finalise writes after an already-committed
transaction (src/zeroskip-active.c:122 + src/mfile.c:534-546) -- are reported
apart, as ``stale_empty_commits``, because the reference's own verifier
(zeroskip-record.c:204-232) rejects them although nothing is corrupt.

Work split (one process per GPU, launched by torchrun): the byte weight of the
DB is cut into `world` equal ranges.  Active / finalised files and packed tails
(records commit + pointer section + final commit) go whole to the rank holding
their midpoint; a packed records region crossing a cut is split there.  Every
rank stages its ranges into one device buffer, walks its files on the host
(threads; the ctypes calls release the GIL), verifies all its commits in ONE
device launch and computes RAW registers of its split pieces in another.  The
per-rank digests are all-gathered as one fixed-shape int64 tensor per rank
(tens of kilobytes; no pickling in the timed pass); split regions are folded with
the zero-shift operator (``shard.fold``) and their commit trailers applied on
the host.  Input bytes never cross xGMI.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import re
import struct
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np
import torch

from . import zsfile
from .shard import fold

PREFIX = "zeroskip-"
DOTZSDB = ".zsdb"
HDR = 40
M32 = 0xFFFFFFFF
T_COMMIT, T_2ND, T_FINAL, T_LONG_COMMIT, T_LONG_FINAL = 4, 8, 16, 36, 48
_NAME = re.compile(r"zeroskip-(.{36})-(\d+)(?:-(\d+))?$")
SPLIT_ALIGN = 64 << 10
SLOT_ALIGN = 256


# --------------------------------------------------------------------- the DB
@dataclass
class DbFile:
    name: str
    kind: int                 # zsfile.ACTIVE / FINALISED / PACKED
    uuid: str
    startidx: int
    endidx: int
    image: np.ndarray         # the file bytes (np.memmap for a directory)
    dev: torch.Tensor | None = None   # optional device-resident copy

    @property
    def size(self) -> int:
        return int(self.image.nbytes)


def parse_name(name: str):
    """(kind, uuidstr, startidx, endidx) or None, like interpret_db_filename
    (src/zeroskip.c:200-235): one index = active, two equal = finalised,
    two different = packed."""
    m = _NAME.search(name)
    if not m or not name.startswith(PREFIX):
        return None
    s = int(m.group(2))
    if m.group(3) is None:
        return zsfile.ACTIVE, m.group(1), s, s
    e = int(m.group(3))
    return (zsfile.FINALISED if e == s else zsfile.PACKED), m.group(1), s, e


def _as_u8(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy().view(np.uint8).reshape(-1)
    if isinstance(x, np.ndarray):
        return x.view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(x), dtype=np.uint8)


@dataclass
class Db:
    dotzsdb: bytes | None
    files: list[DbFile]


def open_db(src) -> Db:
    """A DB from a directory (files memory-mapped, nothing read yet) or from a
    mapping {file name: bytes | np.ndarray | torch.Tensor} (in-memory images;
    a CUDA tensor is used in place as the device-resident copy)."""
    files, dot = [], None
    if isinstance(src, (str, os.PathLike)):
        names = sorted(os.listdir(src))
        get = {}
        for n in names:
            p = os.path.join(src, n)
            if not os.path.isfile(p):
                continue
            if n == DOTZSDB:
                with open(p, "rb") as fh:
                    dot = fh.read()
            elif parse_name(n):
                sz = os.path.getsize(p)
                get[n] = (np.memmap(p, dtype=np.uint8, mode="r") if sz else np.zeros(0, np.uint8), None)
    else:
        get = {}
        for n, v in src.items():
            if n == DOTZSDB:
                dot = bytes(_as_u8(v))
            elif parse_name(n):
                dev = v if isinstance(v, torch.Tensor) and v.is_cuda else None
                get[n] = (_as_u8(v), dev)
    for n, (img, dev) in get.items():
        kind, uuid, s, e = parse_name(n)
        files.append(DbFile(n, kind, uuid, s, e, img, dev))
    files.sort(key=lambda f: (f.startidx, f.endidx, f.name))
    return Db(dot, files)


# ------------------------------------------------------- the native pass
CPASS_SPANS, CPASS_LIST = 64, 1000   # include/zscrc.h


class CPassSpec(ctypes.Structure):
    """zscrc_cpass_spec (include/zscrc.h)."""
    _fields_ = [("d_image", ctypes.c_void_p), ("image_size", ctypes.c_uint64), ("n", ctypes.c_size_t),
                ("d_off", ctypes.c_void_p), ("d_len", ctypes.c_void_p), ("d_file", ctypes.c_void_p),
                ("max_len", ctypes.c_uint64), ("nspans", ctypes.c_size_t), ("span_off", ctypes.c_void_p),
                ("span_len", ctypes.c_void_p), ("span_commit", ctypes.c_void_p)]


class CPassRowSpec(ctypes.Structure):
    """zscrc_cpass_row_spec (include/zscrc.h)."""
    _fields_ = [("d_rec", ctypes.c_void_p), ("piece_fid", ctypes.c_void_p), ("piece_code", ctypes.c_void_p),
                ("listed", ctypes.c_uint32), ("pmax", ctypes.c_uint32), ("checked", ctypes.c_int64 * 4)]


class CPassResult(ctypes.Structure):
    """zscrc_cpass_result (include/zscrc.h)."""
    _fields_ = [("n_bad", ctypes.c_uint64), ("n_stale", ctypes.c_uint64), ("n_undecided", ctypes.c_uint64),
                ("complete", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("n_listed_bad", ctypes.c_uint64), ("n_listed_stale", ctypes.c_uint64),
                ("bad", ctypes.c_uint64 * CPASS_LIST), ("stale", ctypes.c_uint64 * CPASS_LIST),
                ("undecided", ctypes.c_uint64 * CPASS_SPANS), ("span_raw", ctypes.c_uint32 * CPASS_SPANS),
                ("span_status", ctypes.c_int32 * CPASS_SPANS)]


# span pieces checked on the device travel in the digest with these piece
# indices (the host folds only the split ones: index >= 0, or -1 for a
# pointer section whose commit is not in this rank's buffer)
CHECKED_OK, CHECKED_BAD, CHECKED_TAIL_OK, CHECKED_TAIL_BAD = -2, -3, -4, -5


# ------------------------------------------------------------------ the plan
@dataclass
class Unit:
    fid: int
    what: str                 # "file" | "tail" (packed: commit + pointers + final) | "piece" (of a records region)
    lo: int                   # byte range of the file this unit checksums
    hi: int
    rank: int = 0
    piece: int = 0            # for "piece": its index within the region


@dataclass
class Plan:
    world: int
    units: list[Unit]
    packed: dict              # fid -> dict(roff, rlen, poff, plen, rc)
    weight: int


def _packed_layout(img: np.ndarray):
    off, ln, rc = zsfile.packed_spans(img)
    return dict(roff=int(off[0]), rlen=int(ln[0]), poff=int(off[1]), plen=int(ln[1]), rc=int(rc))


def make_plan(db: Db, world: int) -> Plan:
    """Deterministic cut of the DB into `world` ranges of equal byte weight
    (the same on every rank; only packed tails are read to build it)."""
    seq, packed = [], {}
    for fid, f in enumerate(db.files):
        if f.kind == zsfile.PACKED:
            lay = _packed_layout(f.image)
            packed[fid] = lay
            if lay["rc"] == 0:
                rend = lay["roff"] + lay["rlen"]
                seq.append((Unit(fid, "region", lay["roff"], rend), True))
                seq.append((Unit(fid, "tail", rend, f.size), False))
                continue
        seq.append((Unit(fid, "file", 0, f.size), False))
    W = sum(u.hi - u.lo for u, _ in seq)
    bounds = [(W * r) // world for r in range(world + 1)]

    def rank_of(x):
        r = 0
        while r + 1 < world and bounds[r + 1] <= x:
            r += 1
        return r

    units, cur = [], 0
    for u, splittable in seq:
        w = u.hi - u.lo
        if not splittable:
            u.rank = rank_of(cur + w // 2)
            units.append(u)
        else:
            cuts = [u.lo]
            for r in range(1, world):
                if cur < bounds[r] < cur + w:
                    c = u.lo + bounds[r] - cur
                    c = u.lo + ((c - u.lo) // SPLIT_ALIGN) * SPLIT_ALIGN
                    if cuts[-1] < c < u.hi:
                        cuts.append(c)
            cuts.append(u.hi)
            # a records region is always checksummed as raw pieces (one span
            # each, zscrc_device_span) and its commit trailer checked on the
            # host -- also whole, on one rank
            for i in range(len(cuts) - 1):
                a, b = cuts[i], cuts[i + 1]
                units.append(Unit(u.fid, "piece", a, b, rank_of(cur + (a - u.lo) + (b - a) // 2), i))
        cur += w
    return Plan(world, units, packed, W)


# ---------------------------------------------------------------- device side
class GpuBackend:
    """The product path: libzscrc kernels on the staged device buffer."""

    native_pass = True    # the whole device pass as one C call (zscrc_cpass)

    def __init__(self, device: torch.device):
        self.device = device

    def empty(self, n: int) -> torch.Tensor:
        return torch.empty(max(n, 1), dtype=torch.uint8, device=self.device)

    def verify(self, buf, off, ln, seed=None, max_len=None):
        return zsfile.verify_commits(buf, off, ln, seed, max_len)

    def raw(self, buf, off, ln):
        from .device import crc_batch
        return crc_batch(buf, off, ln, raw=True)

    def raw_spans(self, buf, off: list, ln: list, d_off, d_ln):
        """raw registers of a few long spans (records-region pieces, pointer
        sections; host offsets): up to 8 in one zscrc_device_spans call (one
        segment launch of the coalesced whole-wave teams over every CU, one
        fold launch), else one zscrc_device_span each; many: one variable
        batch."""
        from .device import crc_span, crc_spans
        if len(off) > 64:
            return self.raw(buf, d_off, d_ln)
        if len(off) <= 8 and os.environ.get("ZS_SPANS_MULTI", "1") != "0":
            return crc_spans(buf, off, ln, raw=True)
        out = torch.empty(len(off), dtype=torch.int32, device=buf.device)
        for i, (o, n) in enumerate(zip(off, ln)):
            crc_span(buf, offset=o, length=n, out=out[i:i + 1], raw=True)
        return out

    def crc(self, buf, off, ln, max_len=None):
        from .device import crc_batch
        return crc_batch(buf, off, ln, max_len=max_len)

    ROWS_CAP, RAW_CAP = 4096, 64

    def mismatch_rows(self, st, crc, d_end, buf, raw):
        """(rows, raw registers) of the commits with status != 1 in one
        device->host copy (zscrc_device_mismatch_rows); None if they do not
        fit the buffer."""
        from ._lib import check, lib
        if raw is not None and raw.numel() > self.RAW_CAP:
            return None
        dev = buf.device
        key = (dev, self.ROWS_CAP)
        if getattr(self, "_post_key", None) != key:
            self._post = torch.empty(1 + self.RAW_CAP + 18 * self.ROWS_CAP, dtype=torch.int64, device=dev)
            self._post_key = key
        post = self._post
        with torch.cuda.device(dev):
            check(lib().zscrc_device_mismatch_rows(st.data_ptr(), crc.data_ptr(), d_end.data_ptr(), buf.data_ptr(),
                                                   buf.numel(), st.numel(), post.data_ptr(),
                                                   post[1 + self.RAW_CAP:].data_ptr(), self.ROWS_CAP,
                                                   torch.cuda.current_stream(dev).cuda_stream),
                  "zscrc_device_mismatch_rows")
        k = 0 if raw is None else raw.numel()
        if k:
            post[1:1 + k] = raw.to(torch.int64) & M32
        h = post.cpu().numpy()
        cnt = int(h[0])
        if cnt > self.ROWS_CAP:
            return None
        rows = h[1 + self.RAW_CAP:1 + self.RAW_CAP + 18 * cnt].reshape(-1, 18)
        rows = rows[np.argsort(rows[:, 0], kind="stable")]
        return rows, h[1:1 + k].tolist()

    def sync(self):
        torch.cuda.synchronize(self.device)


_RAW8 = None


def _raw8(x: np.ndarray) -> np.ndarray:
    """raw CRC-32C register (from 0, no conditioning) of the 8 little-endian
    bytes of each uint64 in x: XOR of per-byte tables (CRC linearity)."""
    global _RAW8
    if _RAW8 is None:
        from .crc32c import crc32c_hw
        t = np.zeros((8, 256), np.uint32)
        for k in range(8):
            for v in range(256):
                t[k, v] = crc32c_hw(M32, bytes(k) + bytes([v]) + bytes(7 - k)) ^ M32
        _RAW8 = t
    r = np.zeros(x.shape, np.uint32)
    for k in range(8):
        r ^= _RAW8[k][((x >> np.uint64(8 * k)) & np.uint64(255)).astype(np.intp)]
    return r


def _commit_rec(img: np.ndarray, off: int):
    """(type, span_len, rec_len, stored, trailer words) of the commit at off."""
    w0 = int.from_bytes(img[off:off + 8].tobytes(), "big")
    t = w0 >> 56
    if t in (T_COMMIT, T_FINAL):
        return t, (w0 >> 32) & 0xFFFFFF, 8, w0 & M32, [w0 & 0xFFFFFFFF00000000]
    if t in (T_LONG_COMMIT, T_LONG_FINAL) and off + 24 <= img.nbytes:
        n = int.from_bytes(img[off + 8:off + 16].tobytes(), "big")
        w2 = int.from_bytes(img[off + 16:off + 24].tobytes(), "big")
        return t, n, 24, w2 & M32, [w0, n, w2 & 0xFF00000000000000]
    return t, None, 0, None, None


def _trailer_crc(span_crc: int, words) -> int:
    from .crc32c import crc32c_hw
    return crc32c_hw(span_crc, b"".join(struct.pack("<Q", w) for w in words))


@dataclass
class Report:
    ok: bool = True
    files: int = 0
    commits: int = 0
    bytes_checked: int = 0
    dotzsdb: dict = field(default_factory=dict)
    n_bad: int = 0            # counts (the lists hold at most MAX_LISTED per rank)
    n_stale: int = 0
    header_errors: list = field(default_factory=list)
    walk_errors: list = field(default_factory=list)
    issues: list = field(default_factory=list)
    timing: dict = field(default_factory=dict)
    # (file id, commit offset) rows; named and sorted only when read, so the
    # timed pass does no per-commit Python work
    names: object = None
    bad_rows: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.int64))
    stale_rows: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.int64))
    extra_bad: list = field(default_factory=list)           # (file name, commit offset)

    def _named(self, rows) -> list:
        return [(self.names[int(f)], int(x)) for f, x in rows]

    @property
    def bad_commits(self) -> list:
        """(file, commit offset) of every listed bad commit, sorted."""
        return sorted(self._named(self.bad_rows) + list(self.extra_bad))

    @property
    def stale_empty_commits(self) -> list:
        """(file, commit offset) of every listed stale empty commit, sorted."""
        return sorted(self._named(self.stale_rows))

    def as_dict(self):
        d = {k: v for k, v in self.__dict__.items() if k not in ("names", "bad_rows", "stale_rows", "extra_bad")}
        d["bad_commits"] = self.bad_commits
        d["stale_empty_commits"] = self.stale_empty_commits
        return d


class Consistent:
    """One rank's share of a consistency check.  ``prepare()`` stages the
    rank's bytes on its device and walks its files (host); ``run()`` is the
    device pass + exchange + fold and can be repeated (device-resident)."""

    MAX_LISTED = 1000

    def __init__(self, db: Db, rank: int = 0, world: int = 1, backend=None, group=None,
                 threads: int = 8):
        self.db, self.rank, self.world, self.group = db, rank, world, group
        self.backend = backend or GpuBackend(torch.device("cuda", torch.cuda.current_device()))
        self.threads = threads
        self.plan = make_plan(db, world)
        self.mine = [u for u in self.plan.units if u.rank == rank]
        self._names = None   # file names by id, for the bad / stale lists
        self._pmax = 0
        self._host_all = None

    # ---------------------------------------------------------------- prepare
    def prepare(self):
        t0 = time.perf_counter()
        db, be = self.db, self.backend
        # device layout: one slot per unit; a whole span also needs its commit record
        slots, pos = [], 0
        for u in self.mine:
            hi = u.hi
            slots.append((u, u.lo, hi, pos))
            pos += -(-(hi - u.lo) // SLOT_ALIGN) * SLOT_ALIGN
        self.buf = be.empty(pos)
        self._slots = slots
        pinned = None
        if any(db.files[u.fid].dev is None for u, *_ in slots) and self.buf.is_cuda:
            pinned = torch.empty(max(pos, 1), dtype=torch.uint8, pin_memory=True)
        host = pinned.numpy() if pinned is not None else (self.buf.numpy() if not self.buf.is_cuda else None)
        for u, lo, hi, p in slots:
            f = db.files[u.fid]
            if f.dev is not None:
                self.buf[p:p + hi - lo].copy_(f.dev.view(torch.uint8).reshape(-1)[lo:hi], non_blocking=True)
            else:
                host[p:p + hi - lo] = f.image[lo:hi]
        t_read = time.perf_counter()
        if pinned is not None:
            self.buf.copy_(pinned[:self.buf.numel()], non_blocking=True)

        # host side: headers, walks, commit descriptors (while the copy runs)
        self.local = Report()
        c_off, c_len, c_file, c_rec = [], [], [], []
        pieces = []           # (fid, piece, lo, hi, slot offset)
        header_of = set()

        def walk(item):
            u, lo, hi, p = item
            return zsfile.walk(db.files[u.fid].image)

        file_units = [s for s in slots if s[0].what == "file" and db.files[s[0].fid].kind != zsfile.PACKED]
        with ThreadPoolExecutor(max_workers=max(1, self.threads)) as ex:
            walks = dict(zip([s[0].fid for s in file_units], ex.map(walk, file_units)))
        for u, lo, hi, p in slots:
            f = db.files[u.fid]
            if u.what in ("file", "tail") and u.fid not in header_of:
                header_of.add(u.fid)
                self._check_header(f)
            if u.what == "file" and f.kind == zsfile.PACKED:
                self.local.walk_errors.append((f.name, self.plan.packed[u.fid]["rc"], 0))
            elif u.what == "file":
                so, sl, rc, end = walks[u.fid]
                self._check_walk(f, so, sl, rc, end)
                c_off.append(so.astype(np.int64) + (p - lo))
                c_len.append(sl.astype(np.int64))
                c_file.append(np.full(len(so), u.fid, np.int64))
                c_rec.append(so.astype(np.int64) + sl.astype(np.int64))
            elif u.what == "tail":
                # the pointer section: a raw span, its commit checked on the host
                lay = self.plan.packed[u.fid]
                pieces.append((u.fid, -1, lay["poff"], lay["poff"] + lay["plen"], lay["poff"] - lo + p))
            else:
                pieces.append((u.fid, u.piece, u.lo, u.hi, p))
        cat = (lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.int64))
        self.c_off, self.c_len, self.c_file, self.c_rec = map(cat, (c_off, c_len, c_file, c_rec))
        # longest span, for zscrc_device_verify_commits_bounded (the host walk knows it)
        self.c_max = int(self.c_len.max()) if len(self.c_len) else 0
        self.pieces = pieces
        dev = self.buf.device
        self.d_off = torch.from_numpy(self.c_off).to(dev)
        self.d_len = torch.from_numpy(self.c_len).to(dev)
        self.d_end = self.d_off + self.d_len
        self._ar8 = torch.arange(8, device=dev)
        self.d_poff = torch.tensor([q[4] for q in pieces], dtype=torch.int64, device=dev)
        self.d_plen = torch.tensor([q[3] - q[2] for q in pieces], dtype=torch.int64, device=dev)
        self.local.files = len(header_of)
        self.local.bytes_checked = int(sum(u.hi - u.lo for u in self.mine))
        be.sync()
        t1 = time.perf_counter()
        self.prepare_times = dict(stage_s=t_read - t0, walk_and_copy_s=t1 - t_read, total_s=t1 - t0,
                                  staged_bytes=pos)
        # split pieces per rank are fixed by the plan: the exchange row's size
        self._pmax = max([sum(1 for u in self.plan.units if u.rank == r and u.what in ("piece", "tail"))
                          for r in range(self.world)] + [0])
        # host-side findings do not change between runs: exchanged once, here
        native_ok = bool(getattr(be, "native_pass", False) and os.environ.get("ZS_POSTPASS", "native") == "native"
                         and len(pieces) <= CPASS_SPANS)
        host = dict(files=self.local.files, bytes=self.local.bytes_checked,
                    header_errors=self.local.header_errors, walk_errors=self.local.walk_errors,
                    issues=self.local.issues, native_ok=native_ok)
        if self.world == 1:
            self._host_all = [host]
        else:
            import torch.distributed as dist
            self._host_all = [None] * self.world
            dist.all_gather_object(self._host_all, host, group=self.group)
        self._dotzsdb = self._check_dotzsdb()    # the .zsdb does not change between passes
        self._cpass = None
        # every rank takes the same path, so their collectives pair up
        if all(h.get("native_ok", False) for h in self._host_all):
            self._make_cpass(slots)
        return self

    def dev_offset(self, fid: int, off: int) -> int:
        """Where byte `off` of file `fid` sits in this rank's device buffer
        (KeyError: not in this rank's share)."""
        for u, lo, hi, p in self._slots:
            if u.fid == fid and lo <= off < hi:
                return p + off - lo
        raise KeyError((fid, off))

    def _make_cpass(self, slots):
        """The device pass as one C call (zscrc_cpass): verdict batch, raw
        spans, post kernel, one small copy back."""
        from ._lib import check, lib
        dev = self.buf.device
        self.d_file = torch.from_numpy(self.c_file.astype(np.int32)).to(dev)
        tail_at = {u.fid: p for u, lo, hi, p in slots if u.what == "tail"}
        so, sl, sc = [], [], []
        for fid, k, lo, hi, p in self.pieces:
            lay = self.plan.packed[fid]
            so.append(p)
            sl.append(hi - lo)
            if k < 0:                                   # pointer section: its final commit follows
                sc.append(p + (hi - lo))
            elif lo == lay["roff"] and hi == lay["roff"] + lay["rlen"] and fid in tail_at:
                sc.append(tail_at[fid])                 # whole region, its commit record staged here
            else:
                sc.append(-1)                           # a split piece: folded on the host
        self._span_off = np.array(so, np.uint64)
        self._span_len = np.array(sl, np.uint64)
        self._span_commit = np.array(sc, np.int64)
        spec = CPassSpec(self.buf.data_ptr(), self.buf.numel(), len(self.c_off), self.d_off.data_ptr(),
                         self.d_len.data_ptr(), self.d_file.data_ptr(), self.c_max, len(so),
                         self._span_off.ctypes.data, self._span_len.ctypes.data, self._span_commit.ctypes.data)
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            check(lib().zscrc_cpass_create(ctypes.byref(h), ctypes.byref(spec)), "zscrc_cpass_create")
        self._cpass = h
        self._cres = CPassResult()
        # the digest row on the device (zscrc_cpass_submit_row): the exchange
        # of world > 1 all-gathers it without a host round trip
        self.d_rec = torch.from_numpy(self.c_rec.astype(np.int64)).to(dev)
        self._piece_fid = np.array([q[0] for q in self.pieces], np.int64)
        self._piece_code = np.array([q[1] for q in self.pieces], np.int64)
        rs = CPassRowSpec(self.d_rec.data_ptr(), self._piece_fid.ctypes.data, self._piece_code.ctypes.data,
                          self.MAX_LISTED, max(self._pmax, len(self.pieces)),
                          (ctypes.c_int64 * 4)(CHECKED_OK, CHECKED_BAD, CHECKED_TAIL_OK, CHECKED_TAIL_BAD))
        with torch.cuda.device(dev):
            check(lib().zscrc_cpass_set_row(h, ctypes.byref(rs)), "zscrc_cpass_set_row")
        self._row_len = self.HEAD + 4 * self.MAX_LISTED + 4 * max(self._pmax, len(self.pieces))
        self._row = torch.zeros(self._row_len, dtype=torch.int64, device=dev)
        self._rows = None

    def __del__(self):
        h = getattr(self, "_cpass", None)
        if h:
            try:
                from ._lib import lib
                lib().zscrc_cpass_destroy(h)
            except Exception:
                pass

    def _check_header(self, f: DbFile):
        rc, st, cp = zsfile.header_crc(f.image)
        if rc != 0 or st != cp:
            self.local.header_errors.append((f.name, "signature" if rc else "crc", st, cp))
            return
        sidx = int.from_bytes(f.image[28:32].tobytes(), "big")
        eidx = int.from_bytes(f.image[32:36].tobytes(), "big")
        if (sidx, eidx) != (f.startidx, f.endidx):
            self.local.issues.append(f"{f.name}: header indices {sidx}-{eidx} do not match the name")

    def _check_walk(self, f: DbFile, so, sl, rc, end):
        if rc != zsfile.END:
            self.local.walk_errors.append((f.name, int(rc), int(end)))
            return
        last = HDR
        if len(so):
            e = int(so[-1] + sl[-1])
            _, _, rl, _, _ = _commit_rec(f.image, e)
            last = e + rl
        if last != f.size:
            self.local.issues.append(f"{f.name}: {f.size - last} bytes after the last commit")

    # -------------------------------------------------------------------- run
    def run(self, events=None) -> Report:
        """events: optional (start, end) device events recorded around the
        device pass (bench.py's kernel timing)."""
        if self._cpass is not None:
            rep = self._run_native_rows(events) if self.world > 1 else self._run_native(events)
            if rep is not None:
                return rep
        return self._run_torch(events)

    def device_row(self, events=None) -> torch.Tensor:
        """Enqueue one native pass whose digest row (include/zscrc.h,
        zscrc_cpass_submit_row) lands in a device tensor; nothing waits."""
        from ._lib import check, lib
        dev = self.buf.device
        stream = torch.cuda.current_stream(dev)
        with torch.cuda.device(dev):
            ev = self._c_events(events, stream)
            check(lib().zscrc_cpass_submit_row(self._cpass, ctypes.c_void_p(stream.cuda_stream), ev[0], ev[1],
                                               ctypes.c_void_p(self._row.data_ptr())), "zscrc_cpass_submit_row")
        return self._row

    def _row_buffers(self, nccl: bool, slot: int):
        """Per host slot: the device row, the gathered rows (device under nccl,
        host under gloo) and pinned host rows."""
        if getattr(self, "_rowbuf", None) is None:
            dev = self.buf.device
            n = self.world * self._row_len
            self._rowbuf = [dict(row=torch.zeros(self._row_len, dtype=torch.int64, device=dev),
                                 rows=torch.empty(n, dtype=torch.int64, device=dev if nccl else "cpu"),
                                 host=torch.empty(n, dtype=torch.int64, pin_memory=True))
                            for _ in range(2)]
        return self._rowbuf[slot]

    def _submit_rows(self, events, slot: int) -> bool:
        """world > 1, pipelined: pass k's row on the device, its all-gather
        queued (async) and the gathered rows' copy into pinned host memory
        queued behind it; collect() waits for the copy and merges -- while pass
        k + 1 already runs."""
        import torch.distributed as dist
        from ._lib import check, lib
        nccl = dist.get_backend(self.group) == "nccl"
        b = self._row_buffers(nccl, slot)
        dev = self.buf.device
        stream = torch.cuda.current_stream(dev)
        with torch.cuda.device(dev):
            ev = self._c_events(events, stream)
            check(lib().zscrc_cpass_submit_row(self._cpass, ctypes.c_void_p(stream.cuda_stream), ev[0], ev[1],
                                               ctypes.c_void_p(b["row"].data_ptr())), "zscrc_cpass_submit_row")
        t0 = time.perf_counter()
        if nccl:
            # the gather (RCCL's own stream) and the copy to the host (a side
            # stream waiting for it) run beside the next pass's kernels: the
            # compute stream never waits for the exchange
            work = dist.all_gather_into_tensor(b["rows"], b["row"], group=self.group, async_op=True)
            if getattr(self, "_xstream", None) is None:
                self._xstream = torch.cuda.Stream(dev)
            with torch.cuda.stream(self._xstream):
                work.wait()   # the side stream waits for the collective (the host does not)
                b["host"].copy_(b["rows"], non_blocking=True)
                done = torch.cuda.Event()
                done.record(self._xstream)
        else:
            dist.all_gather_into_tensor(b["rows"], b["row"].cpu(), group=self.group)
            b["host"].copy_(b["rows"])
            done = None
        self._inflight.append((slot, t0, done))
        self._next_slot ^= 1
        return True

    def _collect_rows(self) -> Report:
        slot, t0, done = self._inflight.pop(0)
        if done is not None:
            done.synchronize()
        rows = self._rowbuf[slot]["host"].numpy().reshape(self.world, -1)
        t_x = time.perf_counter()
        if (rows[:, self.HEAD - 1] != 0).any():
            return self._run_torch()
        rep = self._merge([self._unpack(r, rows[r]) for r in range(self.world)])
        t1 = time.perf_counter()
        rep.timing = dict(device_s=0.0, exchange_s=t_x - t0, fold_s=t1 - t_x, total_s=t1 - t0, host_round_trips=1)
        return rep

    def _run_native_rows(self, events):
        """world > 1: the pass and its digest row on the device, one
        all-gather of the rows (RCCL under nccl: device to device), one copy of
        all rows to the host -- the step's only host round trip.  None (every
        rank takes the torch path, the same rows tell each the same) when a
        rank's pass left commits undecided or listed only part of them."""
        import torch.distributed as dist
        t0 = time.perf_counter()
        row = self.device_row(events)
        nccl = dist.get_backend(self.group) == "nccl"
        if self._rows is None:
            self._rows = torch.empty(self.world * self._row_len, dtype=torch.int64,
                                     device=row.device if nccl else "cpu")
            self._rows_h = torch.empty(self.world * self._row_len, dtype=torch.int64, pin_memory=True)
        dist.all_gather_into_tensor(self._rows, row if nccl else row.cpu(), group=self.group)
        self._rows_h.copy_(self._rows, non_blocking=True)
        torch.cuda.current_stream(row.device).synchronize()
        rows = self._rows_h.numpy().reshape(self.world, -1)
        t_x = time.perf_counter()
        if (rows[:, self.HEAD - 1] != 0).any():
            return None
        allsum = [self._unpack(r, rows[r]) for r in range(self.world)]
        rep = self._merge(allsum)
        t1 = time.perf_counter()
        rep.timing = dict(device_s=0.0, exchange_s=t_x - t0, fold_s=t1 - t_x, total_s=t1 - t0,
                          host_round_trips=1)
        return rep

    def _run_native(self, events):
        """One C call: the verdict batch, the raw spans, the post kernel and
        one small copy back; the digest is built from that block alone.  None
        (the torch path decides) when the pass left commits undecided or
        listed only part of its mismatches."""
        from ._lib import check, lib
        t0 = time.perf_counter()
        res = self._cres
        dev = self.buf.device
        stream = torch.cuda.current_stream(dev)
        # the C pass switches to the device it was created on; the stream and
        # the events are that device's (zscrc_cpass_run_timed records the end
        # event before its host-side wait)
        with torch.cuda.device(dev):
            ev = self._c_events(events, stream)
            check(lib().zscrc_cpass_run_timed(self._cpass, ctypes.c_void_p(stream.cuda_stream), ev[0], ev[1],
                                              ctypes.byref(res)), "zscrc_cpass_run_timed")
        return self._native_report(res, t0)

    @staticmethod
    def _c_events(events, stream):
        if not events:
            return (None, None)
        for e in events:          # torch creates its events lazily, on the first record
            e.record(stream)
        return (ctypes.c_void_p(events[0].cuda_event), ctypes.c_void_p(events[1].cuda_event))

    # ------------------------------------------------ pipelined native passes
    def submit(self, events=None) -> bool:
        """Enqueue one native pass (zscrc_cpass_submit) into the next of two
        host slots and return at once, so the host reads pass k while the
        device runs pass k + 1; collect() returns the passes' reports in
        submission order.  False (nothing enqueued): no native pass here."""
        from ._lib import check, lib
        if self._cpass is None:
            return False
        if not hasattr(self, "_inflight"):
            self._inflight, self._next_slot = [], 0
            self._cres_slot = (CPassResult(), CPassResult())
        slot = self._next_slot
        if slot in [q[0] for q in self._inflight]:
            raise RuntimeError("both host slots hold uncollected passes")
        if self.world > 1:
            return self._submit_rows(events, slot)
        dev = self.buf.device
        stream = torch.cuda.current_stream(dev)
        with torch.cuda.device(dev):
            ev = self._c_events(events, stream)
            check(lib().zscrc_cpass_submit(self._cpass, ctypes.c_void_p(stream.cuda_stream), ev[0], ev[1], slot),
                  "zscrc_cpass_submit")
        self._inflight.append((slot, time.perf_counter(), None))
        self._next_slot ^= 1
        return True

    def pending(self) -> int:
        return len(getattr(self, "_inflight", []))

    def collect(self) -> Report:
        """The report of the oldest submitted pass (waits for its copy back).
        A pass that left commits undecided is decided by the torch path (a
        synchronous pass of its own)."""
        from ._lib import check, lib
        if self.world > 1:
            return self._collect_rows()
        slot, t0, _ = self._inflight.pop(0)
        res = self._cres_slot[slot]
        with torch.cuda.device(self.buf.device):
            check(lib().zscrc_cpass_collect(self._cpass, slot, ctypes.byref(res)), "zscrc_cpass_collect")
        rep = self._native_report(res, t0)
        return rep if rep is not None else self._run_torch()

    def _native_report(self, res, t0):
        if res.n_undecided or not res.complete:
            return None
        t_dev = time.perf_counter()
        digest = self._native_digest(res)
        allsum = self._gather(digest)
        t_x = time.perf_counter()
        rep = self._merge(allsum)
        t1 = time.perf_counter()
        rep.timing = dict(device_s=t_dev - t0, exchange_s=t_x - t_dev, fold_s=t1 - t_x, total_s=t1 - t0)
        return rep

    def _native_digest(self, res) -> dict:
        """A native pass's host block (zscrc_cpass_result) as this rank's digest."""
        L = self.MAX_LISTED
        bad_i = np.ctypeslib.as_array(res.bad)[:res.n_listed_bad].astype(np.int64)
        stale_i = np.ctypeslib.as_array(res.stale)[:res.n_listed_stale].astype(np.int64)
        pieces = []
        n_bad = int(res.n_bad)
        for k, (fid, pc, lo, hi, p) in enumerate(self.pieces):
            st = res.span_status[k]
            if st < 0:
                pieces.append((fid, pc, hi - lo, res.span_raw[k]))
            else:
                pieces.append((fid, (CHECKED_TAIL_OK if st == 1 else CHECKED_TAIL_BAD) if pc < 0 else
                               (CHECKED_OK if st == 1 else CHECKED_BAD), hi - lo, 0))
        return dict(commits=len(self.c_off), n_bad=n_bad, n_stale=int(res.n_stale),
                    bad=np.stack([self.c_file[bad_i[:L]], self.c_rec[bad_i[:L]]], 1),
                    stale=np.stack([self.c_file[stale_i[:L]], self.c_rec[stale_i[:L]]], 1),
                    pieces=np.array(pieces, np.int64).reshape(-1, 4))

    def _run_torch(self, events=None) -> Report:
        be = self.backend
        t0 = time.perf_counter()
        n = len(self.c_off)
        loc = self.local
        bad_idx = np.zeros(0, np.int64)
        if events:
            events[0].record()
        if n:
            # the host walk knows the longest span: short-span batches skip
            # the device-side length classes (zscrc_device_verify_commits_bounded)
            crc, st = be.verify(self.buf, self.d_off, self.d_len, max_len=self.c_max)
        raw = None
        if self.pieces:
            if hasattr(be, "raw_spans"):
                raw = be.raw_spans(self.buf, [q[4] for q in self.pieces], [q[3] - q[2] for q in self.pieces],
                                   self.d_poff, self.d_plen)
            else:
                raw = be.raw(self.buf, self.d_poff, self.d_plen)
        if events:
            events[1].record()
        pack = np.zeros((0, 18), np.int64)
        raw_h = []
        done = False
        if n and hasattr(be, "mismatch_rows") and os.environ.get("ZS_POSTPASS", "native") == "native":
            # one kernel writes the mismatch rows, one copy brings them (and
            # the raw span registers) back; more mismatches than the buffer
            # holds: the torch path below
            got = be.mismatch_rows(st, crc, self.d_end, self.buf, raw)
            if got is not None:
                pack, raw_h = got
                bad_idx = pack[:, 0]
                done = True
        if n and not done:
            # one round trip: the mismatches, their predecessors' computed
            # commit CRCs, the commit words after both spans (and the raw
            # registers of the long spans)
            bad = torch.nonzero(st != 1).reshape(-1)
            both = torch.stack([bad, (bad - 1).clamp(min=0)])
            at = (self.d_end[both][:, :, None] + self._ar8).clamp(max=self.buf.numel() - 1)
            w = self.buf[at].to(torch.int64)
            cols = [bad[:, None], crc[both[1]].to(torch.int64)[:, None] & M32, w[0], w[1]]
            pack = torch.cat(cols, 1)
            if raw is not None:
                flat = torch.cat([pack.reshape(-1), raw.to(torch.int64) & M32]).cpu().numpy()
                raw_h = flat[pack.numel():].tolist()
                pack = flat[:pack.numel()].reshape(-1, 18)
            else:
                pack = pack.cpu().numpy()
            bad_idx = pack[:, 0]
        elif raw is not None and not done:
            raw_h = [v & M32 for v in raw.cpu().tolist()]
        t_dev = time.perf_counter()

        # zero-length mismatches right after a span of the same file: the
        # finalise quirk if the stored CRC chains from the previous span's CRC
        # S: stored = crc32c(S, T).  The device computed crc32c(S, T_prev) for
        # the previous commit, and with 8-byte trailers
        #   crc32c(S, T) = crc32c(S, T_prev) ^ raw(T ^ T_prev)
        # (CRC linearity: same register before both trailers), so the check is
        # a host-side 8-byte correction -- no second device pass.  Long (24-byte)
        # trailers, rare, are re-verified on the device with S as the seed.
        qm = (self.c_len[bad_idx] == 0) & (bad_idx > 0)
        qm[qm] = self.c_file[bad_idx[qm] - 1] == self.c_file[bad_idx[qm]]
        q = bad_idx[qm]
        stale_i = np.zeros(0, np.int64)
        if len(q):
            k = pack[qm]
            w = k[:, 2:18].astype(np.uint8)
            w_i = np.ascontiguousarray(w[:, :8]).view(">u8").ravel().astype(np.uint64)
            w_p = np.ascontiguousarray(w[:, 8:]).view(">u8").ravel().astype(np.uint64)
            short = np.isin(w_i >> np.uint64(56), (T_COMMIT, T_FINAL)) & \
                np.isin(w_p >> np.uint64(56), (T_COMMIT, T_FINAL))
            x = (w_i ^ w_p) & np.uint64(0xFFFFFFFF00000000)
            expect = k[:, 1].astype(np.uint32) ^ _raw8(x)
            good = short & (expect == (w_i & np.uint64(M32)).astype(np.uint32))
            stale_i = q[good]
            ql = q[~short]
            if len(ql):
                dq = torch.from_numpy(ql).to(self.d_off.device)
                prev = be.crc(self.buf, self.d_off[dq - 1], self.d_len[dq - 1],
                              max_len=int(self.c_len[ql - 1].max()))
                _, st2 = be.verify(self.buf, self.d_off[dq], self.d_len[dq], prev, max_len=0)
                stale_i = np.sort(np.concatenate([stale_i, ql[(st2 == 1).cpu().numpy()]]))
        bad_i = np.setdiff1d(bad_idx, stale_i, assume_unique=True)

        L = self.MAX_LISTED
        digest = dict(commits=n, n_bad=len(bad_i), n_stale=len(stale_i),
                      bad=np.stack([self.c_file[bad_i[:L]], self.c_rec[bad_i[:L]]], 1),
                      stale=np.stack([self.c_file[stale_i[:L]], self.c_rec[stale_i[:L]]], 1),
                      pieces=np.array([(q[0], q[1], q[3] - q[2], r) for q, r in zip(self.pieces, raw_h)],
                                      np.int64).reshape(-1, 4))
        allsum = self._gather(digest)
        t_x = time.perf_counter()
        rep = self._merge(allsum)
        t1 = time.perf_counter()
        rep.timing = dict(device_s=t_dev - t0, exchange_s=t_x - t_dev, fold_s=t1 - t_x, total_s=t1 - t0)
        return rep

    # ------------------------------------------------------------- exchange
    HEAD = 7   # commits, n_bad, n_stale, listed bad, listed stale, pieces, flags (include/zscrc.h row)

    def _pack(self, d) -> np.ndarray:
        """One rank's digest as a fixed-shape int64 row: the head, then
        MAX_LISTED (file, offset) pairs of bad and of stale commits, then the
        rank's split pieces (file, piece, length, raw register), padded to the
        plan's largest per-rank piece count (the same on every rank)."""
        L = self.MAX_LISTED
        row = np.zeros(self.HEAD + 4 * L + 4 * self._pmax, np.int64)
        row[:self.HEAD] = (d["commits"], d["n_bad"], d["n_stale"], len(d["bad"]), len(d["stale"]),
                           len(d["pieces"]), 0)
        o = self.HEAD
        row[o:o + 2 * len(d["bad"])] = d["bad"].reshape(-1)
        o += 2 * L
        row[o:o + 2 * len(d["stale"])] = d["stale"].reshape(-1)
        o += 2 * L
        row[o:o + 4 * len(d["pieces"])] = d["pieces"].reshape(-1)
        return row

    def _unpack(self, r: int, row: np.ndarray) -> dict:
        L = self.MAX_LISTED
        commits, n_bad, n_stale, nb, ns, npc, _flags = (int(v) for v in row[:self.HEAD])
        o = self.HEAD
        bad = row[o:o + 2 * nb].reshape(-1, 2)
        o += 2 * L
        stale = row[o:o + 2 * ns].reshape(-1, 2)
        o += 2 * L
        pieces = [tuple(int(v) for v in p) for p in row[o:o + 4 * npc].reshape(-1, 4)]
        h = self._host_all[r]
        return dict(rank=r, commits=commits, n_bad=n_bad, n_stale=n_stale, bad=bad, stale=stale, pieces=pieces,
                    files=h["files"], bytes=h["bytes"], header_errors=h["header_errors"],
                    walk_errors=h["walk_errors"], issues=h["issues"])

    def _gather(self, digest):
        """Per-rank digests to every rank: one fixed-shape all-gather of int64
        rows (RCCL under nccl: a device tensor; gloo: host), no pickling.  The
        host-side findings (headers, walks) were exchanged once in prepare()."""
        if self.world == 1:
            h = self._host_all[0]
            return [dict(rank=0, commits=digest["commits"], n_bad=digest["n_bad"], n_stale=digest["n_stale"],
                         bad=digest["bad"], stale=digest["stale"],
                         pieces=[tuple(int(v) for v in p) for p in digest["pieces"]],
                         files=h["files"], bytes=h["bytes"], header_errors=h["header_errors"],
                         walk_errors=h["walk_errors"], issues=h["issues"])]
        row = self._pack(digest)
        import torch.distributed as dist
        dev = torch.device("cpu")
        if dist.get_backend(self.group) == "nccl":
            dev = torch.device("cuda", torch.cuda.current_device())
        mine = torch.from_numpy(row).to(dev)
        out = torch.empty(self.world * row.size, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, mine, group=self.group)
        rows = out.cpu().numpy().reshape(self.world, -1)
        return [self._unpack(r, rows[r]) for r in range(self.world)]

    def _merge(self, allsum) -> Report:
        if self._names is None:
            self._names = [f.name for f in self.db.files]
        rep = Report(names=self._names)
        rep.dotzsdb = getattr(self, "_dotzsdb", None) or self._check_dotzsdb()
        pieces = {}
        bads, stales = [], []
        for s in allsum:
            rep.commits += s["commits"]
            rep.files += s["files"]
            rep.bytes_checked += s["bytes"]
            bads.append(s["bad"])
            stales.append(s["stale"])
            rep.n_bad += s["n_bad"]
            rep.n_stale += s["n_stale"]
            rep.header_errors += [tuple(h) for h in s["header_errors"]]
            rep.walk_errors += [tuple(w) for w in s["walk_errors"]]
            rep.issues += s["issues"]
            for fid, k, ln, r in s["pieces"]:
                if k <= CHECKED_OK:             # checked on the device, trailer included
                    rep.commits += 1
                    if k in (CHECKED_BAD, CHECKED_TAIL_BAD):
                        lay = self.plan.packed[fid]
                        at = lay["poff"] + lay["plen"] if k == CHECKED_TAIL_BAD else lay["roff"] + lay["rlen"]
                        rep.extra_bad.append((self.db.files[fid].name, at))
                        rep.n_bad += 1
                    continue
                pieces.setdefault((fid, k < 0), []).append((k, r, ln))
            if s["n_bad"] > len(s["bad"]):
                rep.issues.append(f"rank {s['rank']}: {s['n_bad'] - len(s['bad'])} more bad commits not listed")
        # records regions (folded from their pieces) and pointer sections:
        # the span register, then the commit trailer after it
        for (fid, tail), ps in sorted(pieces.items()):
            ps.sort()
            f, lay = self.db.files[fid], self.plan.packed[fid]
            span = fold([(r, ln) for _, r, ln in ps])
            rep.commits += 1
            at = lay["poff"] + lay["plen"] if tail else lay["roff"] + lay["rlen"]
            _, _, _, stored, words = _commit_rec(f.image, at)
            if stored is None or _trailer_crc(span, words) != stored:
                rep.extra_bad.append((f.name, at))
                rep.n_bad += 1
        rep.bad_rows = np.concatenate(bads) if bads else rep.bad_rows
        rep.stale_rows = np.concatenate(stales) if stales else rep.stale_rows
        dz = rep.dotzsdb
        rep.issues += self._dotzsdb_issues(dz)
        rep.ok = (not rep.n_bad and not rep.header_errors and not rep.walk_errors
                  and dz.get("ok", False))
        return rep

    def _dotzsdb_issues(self, dz) -> list:
        """.zsdb against the file set (uuids, the active file's index and
        size): host metadata only, fixed for an opened DB, so built once (a
        walk over every file object per run was most of a run's host tail)."""
        if getattr(self, "_dz_issues", None) is not None and self._dz_key is dz:
            return self._dz_issues
        out = []
        if dz.get("present"):
            uu = {f.uuid for f in self.db.files}
            if uu - {dz["uuid"]}:
                out.append(f"files with a uuid other than .zsdb's: {sorted(uu - {dz['uuid']})}")
            act = [f for f in self.db.files if f.kind == zsfile.ACTIVE]
            if len(act) > 1:
                out.append(f"{len(act)} active files")
            for f in act:
                if f.startidx != dz["curidx"]:
                    out.append(f"{f.name}: active index {f.startidx} != .zsdb curidx {dz['curidx']}")
                elif f.size != dz["offset"]:
                    out.append(f"{f.name}: size {f.size} != .zsdb offset {dz['offset']}")
        self._dz_issues, self._dz_key = out, dz
        return out

    def _check_dotzsdb(self) -> dict:
        d = self.db.dotzsdb
        if d is None:
            return dict(present=False, ok=False)
        rc, st, cp = zsfile.dotzsdb_crc(d)
        if rc != 0 and len(d) < 61:
            return dict(present=True, ok=False, rc=rc)
        return dict(present=True, ok=rc == 0 and st == cp, rc=rc, stored=st, computed=cp,
                    offset=int.from_bytes(d[8:16], "big"),
                    uuid=d[16:52].decode("latin-1"), curidx=int.from_bytes(d[53:57], "big"))


class NativeReport(ctypes.Structure):
    """zscrc_consistent_report (include/zscrc.h)."""
    _fields_ = [("files", ctypes.c_uint64), ("commits", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("bad_commits", ctypes.c_uint64), ("stale_empty_commits", ctypes.c_uint64),
                ("header_errors", ctypes.c_uint64), ("walk_errors", ctypes.c_uint64),
                ("dotzsdb", ctypes.c_int), ("consistent", ctypes.c_int), ("first_bad", ctypes.c_char * 512)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["first_bad"] = self.first_bad.decode(errors="replace")
        return d


def consistent_native(dbdir: str) -> dict:
    """The C entry point (one process, current GPU): zscrc_zs_consistent."""
    from ._lib import check, lib
    rep = NativeReport()
    check(lib().zscrc_zs_consistent(os.fsencode(dbdir), ctypes.byref(rep)), "zscrc_zs_consistent")
    return rep.as_dict()


def consistent(src, rank: int = 0, world: int = 1, group=None, backend=None) -> Report:
    """Check a DB (directory or in-memory mapping); every rank returns the
    same merged report."""
    return Consistent(open_db(src), rank, world, backend, group).prepare().run()


def main(argv=None) -> int:
    """``python -m zeroskip_amd.consistent DBDIR`` (cmd-consistent's slot):
    exit 0 if consistent, 1 if not.  Under torchrun every rank takes a share."""
    ap = argparse.ArgumentParser(prog="zeroskip consistent")
    ap.add_argument("dbdir")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    rep = consistent(a.dbdir, rank, world)
    if rank == 0:
        if a.json:
            print(json.dumps(rep.as_dict(), default=str))
        else:
            print(f"{a.dbdir}: {'consistent' if rep.ok else 'NOT consistent'} -- {rep.files} files, "
                  f"{rep.commits} commits, {rep.bytes_checked} bytes; bad commits {rep.n_bad}, "
                  f"header errors {len(rep.header_errors)}, walk errors {len(rep.walk_errors)}, "
                  f"stale empty commits {rep.n_stale}, .zsdb ok {rep.dotzsdb.get('ok')}")
            for b in rep.bad_commits[:20]:
                print(f"  bad commit: {b[0]} at offset {b[1]}")
            for w in rep.walk_errors[:20]:
                print(f"  walk stopped: {w[0]} rc {w[1]} at offset {w[2]}")
            for line in rep.issues:
                print("  " + line)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if rep.ok else 1


if __name__ == "__main__":
    sys.exit(main())
