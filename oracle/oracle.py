"""ctypes view of the CPU checker (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this module.  It restates /root/reference/src/crc32c.c (see
oracle/zs_oracle.c for the file:line map) and is never used by the product
package ``zeroskip_amd``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libzsoracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_SO):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_SO)
        u32, u64, vp, sz = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t
        for name in ("oracle_crc32c_sw", "oracle_crc32c_hw", "oracle_crc32c",
                     "oracle_crc32c_bitwise"):
            f = getattr(L, name)
            f.argtypes = [u32, vp, sz]
            f.restype = u32
        L.oracle_crc32c_init.argtypes = []
        L.oracle_crc32c_init.restype = None
        L.oracle_have_sse42.restype = ctypes.c_int
        L.oracle_shift.argtypes = [u32, u64]
        L.oracle_shift.restype = u32
        L.oracle_combine.argtypes = [u32, u32, u64]
        L.oracle_combine.restype = u32
        L.oracle_batch.argtypes = [vp, vp, vp, vp, vp, u64, u64, u64, ctypes.c_int, ctypes.c_int]
        L.oracle_batch.restype = ctypes.c_int
        L.oracle_now.restype = ctypes.c_double
        L.oracle_batch_rate.argtypes = [vp, vp, vp, vp, vp, u64, u64, u64, ctypes.c_int, ctypes.c_int, vp,
                                        ctypes.c_double, ctypes.POINTER(u64)]
        L.oracle_batch_rate.restype = ctypes.c_double
        L.oracle_commit_crc.argtypes = [u32, u64, ctypes.c_int]
        L.oracle_commit_crc.restype = u32
        L.oracle_header_crc.argtypes = [u64, u32, ctypes.c_char_p, u32, u32]
        L.oracle_header_crc.restype = u32
        L.oracle_dotzsdb_crc.argtypes = [u64, u64, ctypes.c_char_p, u32]
        L.oracle_dotzsdb_crc.restype = u32
        L.oracle_get_sb4.argtypes = [vp]
        # zs_bulk_oracle.c
        L.oracle_walk_images.argtypes = [vp, vp, u64, vp, ctypes.c_int]
        L.oracle_walk_images.restype = ctypes.c_int
        L.oracle_span_crc.argtypes = [vp, u64, ctypes.c_int]
        L.oracle_span_crc.restype = u32
        L.oracle_packed_image.argtypes = [vp, u64, ctypes.c_int, vp]
        L.oracle_packed_image.restype = None
        L.oracle_write_commits.argtypes = [vp, vp, vp, u64, ctypes.c_int]
        L.oracle_write_commits.restype = ctypes.c_int
        L.oracle_commit_crcs.argtypes = [vp, vp, vp, u64, vp, ctypes.c_int]
        L.oracle_commit_crcs.restype = ctypes.c_int
        _lib = L
    return _lib


def _buf(data):
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8)
        return a, a.ctypes.data, a.nbytes
    b = bytes(data)
    cb = ctypes.create_string_buffer(b, len(b))
    return cb, ctypes.addressof(cb), len(b)


def crc32c_sw(crc: int, data) -> int:
    keep, ptr, n = _buf(data)
    return lib().oracle_crc32c_sw(crc, ptr, n)


def crc32c_hw(crc: int, data) -> int:
    keep, ptr, n = _buf(data)
    return lib().oracle_crc32c_hw(crc, ptr, n)


def crc32c_bitwise(crc: int, data) -> int:
    keep, ptr, n = _buf(data)
    return lib().oracle_crc32c_bitwise(crc, ptr, n)


def shift(reg: int, nbytes: int) -> int:
    return lib().oracle_shift(reg, nbytes)


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return lib().oracle_combine(crc_a, crc_b, len_b)


def batch(base: np.ndarray, offs=None, lens=None, seeds=None, *, n=None, stride=0,
          fixed_len=0, impl: str = "hw", threads: int = 1) -> np.ndarray:
    """CRC32C of records inside ``base`` (uint8 array)."""
    base = np.ascontiguousarray(base).view(np.uint8)
    if n is None:
        n = len(offs) if offs is not None else len(lens)
    out = np.zeros(n, dtype=np.uint32)
    o = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
    ln = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint64)
    s = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    rc = lib().oracle_batch(base.ctypes.data,
                            None if o is None else o.ctypes.data,
                            None if ln is None else ln.ctypes.data,
                            None if s is None else s.ctypes.data,
                            out.ctypes.data, n, stride, fixed_len,
                            {"sw": 0, "hw": 1, "bitwise": 2}[impl], threads)
    assert rc == 0
    return out


def now() -> float:
    return lib().oracle_now()


def pick_cpus(n: int) -> list:
    """n logical CPUs of this process's affinity mask for the timing leg: one
    per physical core, dealt round robin over the L3 domains (CCDs), so the
    threads neither share a core's SMT siblings nor crowd one CCD's link to
    memory.  Fewer physical cores than n: SMT siblings fill in."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        return []

    def rd(path, default):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return default
    doms, seen = {}, set()
    spill = []
    for c in allowed:
        base = f"/sys/devices/system/cpu/cpu{c}"
        core = (rd(base + "/topology/physical_package_id", "0"), rd(base + "/topology/core_id", str(c)))
        l3 = rd(base + "/cache/index3/id", "0")
        if core in seen:
            spill.append(c)
            continue
        seen.add(core)
        doms.setdefault((core[0], l3), []).append(c)
    order, lists = [], [doms[k] for k in sorted(doms)]
    while any(lists) and len(order) < n:
        for li in lists:
            if li and len(order) < n:
                order.append(li.pop(0))
    return (order + spill)[:n]


def batch_rate(base: np.ndarray, offs=None, lens=None, seeds=None, *, n=None, stride=0, fixed_len=0,
               impl: str = "hw", threads: int = 1, cpus=None, budget: float = 5.0):
    """The bench's CPU timing leg (oracle_batch_rate): the batch's records laid
    end to end and dealt in byte chunks (~16 per thread, >= 256 KiB) from a
    counter to persistent threads (pinned to `cpus` if given), records cut by
    a chunk boundary joined by the zero shift; passes repeated for `budget`
    seconds.  impl "read" times a plain
    read of the same bytes (the host memory bound).  Returns (crcs of the
    last pass, seconds, passes)."""
    base = np.ascontiguousarray(base).view(np.uint8)
    if n is None:
        n = len(offs) if offs is not None else len(lens)
    out = np.zeros(n, dtype=np.uint32)
    o = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
    ln = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint64)
    s = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    cp = None
    if cpus:
        cp = np.full(threads, -1, dtype=np.int32)
        cp[:min(threads, len(cpus))] = cpus[:threads]
    passes = ctypes.c_uint64(0)
    el = lib().oracle_batch_rate(base.ctypes.data,
                                 None if o is None else o.ctypes.data,
                                 None if ln is None else ln.ctypes.data,
                                 None if s is None else s.ctypes.data,
                                 out.ctypes.data, n, stride, fixed_len,
                                 {"sw": 0, "hw": 1, "bitwise": 2, "read": 3}[impl], threads,
                                 None if cp is None else cp.ctypes.data, budget, ctypes.byref(passes))
    assert el >= 0, "oracle_batch_rate failed"
    return out, el, int(passes.value)


def commit_crc(span_crc: int, span_len: int, final: bool = False) -> int:
    return lib().oracle_commit_crc(span_crc, span_len, int(final))


def header_crc(signature: int, version: int, uuid: bytes, startidx: int, endidx: int) -> int:
    return lib().oracle_header_crc(signature, version, uuid, startidx, endidx)


def dotzsdb_crc(signature: int, offset: int, uuidstr: bytes, curidx: int) -> int:
    assert len(uuidstr) == 37
    return lib().oracle_dotzsdb_crc(signature, offset, uuidstr, curidx)


def slice4_tables() -> np.ndarray:
    t = np.zeros((4, 256), dtype=np.uint32)
    lib().oracle_get_sb4(t.ctypes.data)
    return t


def crc32c_py(crc: int, data: bytes) -> int:
    """Independent pure-Python bit-at-a-time CRC-32C (small inputs only)."""
    r = crc ^ 0xFFFFFFFF
    for b in bytes(data):
        r ^= b
        for _ in range(8):
            r = (r >> 1) ^ (0x82F63B78 if r & 1 else 0)
    return r ^ 0xFFFFFFFF


# ------------------------------------------------------------------ bulk (zs_bulk_oracle.c)
WALK_FIELDS = ("commits", "ok", "end", "stop", "first_bad_off", "first_bad_idx")


def walk_images(images, threads: int = 1) -> np.ndarray:
    """[n, 6] uint64: the record walk of every active / finalised image
    (zeroskip-record.c:283-331), each commit re-checked from seed 0 with the
    writer's trailer semantics; columns as WALK_FIELDS (stop: 0 end of image,
    1 truncated, 2 a type the walk does not advance over, 3 a commit record
    that does not fit).  images: uint8 numpy arrays."""
    arrs = [np.ascontiguousarray(a).view(np.uint8).reshape(-1) for a in images]
    addr = np.array([a.ctypes.data for a in arrs], dtype=np.uint64)
    size = np.array([a.nbytes for a in arrs], dtype=np.uint64)
    out = np.zeros((len(arrs), 6), dtype=np.uint64)
    assert lib().oracle_walk_images(addr.ctypes.data, size.ctypes.data, len(arrs), out.ctypes.data, threads) == 0
    return out


def span_crc(data: np.ndarray, threads: int = 1) -> int:
    """crc32c(0, data) on `threads` threads (pieces joined by the zero shift)."""
    a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return lib().oracle_span_crc(a.ctypes.data, a.nbytes, threads)


def packed_image(img: np.ndarray, threads: int = 1) -> dict:
    """A packed file's two commits (zeroskip-packed.c:70-131, :278-339, :442):
    status 1 ok / 0 bad / 2 layout, span offset and length of each."""
    a = np.ascontiguousarray(img).view(np.uint8).reshape(-1)
    out = np.zeros(6, dtype=np.uint64)
    lib().oracle_packed_image(a.ctypes.data, a.nbytes, threads, out.ctypes.data)
    o = [int(x) for x in out]
    return {"pointers": {"status": o[0], "span_off": o[1], "span_len": o[2]},
            "records": {"status": o[3], "span_off": o[4], "span_len": o[5]}}


def write_commits(base: np.ndarray, offs, lens, threads: int = 1) -> None:
    """The commit writer (zeroskip-file.c:253-350) in place: the record after
    each span, whose type byte is already there, is written whole."""
    assert base.flags.c_contiguous and base.dtype == np.uint8
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    assert lib().oracle_write_commits(base.ctypes.data, o.ctypes.data, ln.ctypes.data, len(o), threads) == 0


def commit_crcs(base: np.ndarray, offs, lens, threads: int = 1) -> np.ndarray:
    """The CRC the writer stores for each span (nothing written)."""
    b = np.ascontiguousarray(base).view(np.uint8).reshape(-1)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    out = np.zeros(len(o), dtype=np.uint32)
    assert lib().oracle_commit_crcs(b.ctypes.data, o.ctypes.data, ln.ctypes.data, len(o), out.ctypes.data,
                                    threads) == 0
    return out
