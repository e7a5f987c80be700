"""Python mirror of zeroskip's checksum API (reference include/libzeroskip/crc32c.h:15-24).

Same names, argument meaning and results as ``/root/reference/src/crc32c.c``;
every call goes through libzscrc.so.  ``crc`` chains exactly like the C API:
``crc32c(crc32c(0, a), b) == crc32c(0, a + b)``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import lib


def _ptr(data):
    """(keepalive, address, nbytes) for bytes / bytearray / memoryview / ndarray."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data)
        return a, a.ctypes.data, a.nbytes
    mv = memoryview(data).cast("B")
    if mv.readonly:
        b = ctypes.create_string_buffer(mv.tobytes(), mv.nbytes)
        return b, ctypes.addressof(b), mv.nbytes
    arr = (ctypes.c_char * mv.nbytes).from_buffer(mv)
    return arr, ctypes.addressof(arr), mv.nbytes


def crc32c_init() -> None:
    """src/crc32c.c:668-673."""
    lib().crc32c_init()


def crc32c_hw(crc: int, data) -> int:
    """src/crc32c.c:370-453 (the symbol zeroskip's library code calls)."""
    keep, p, n = _ptr(data)
    return lib().crc32c_hw(crc, p, n)


def crc32c_sw(crc: int, data) -> int:
    """src/crc32c.c:613-645."""
    keep, p, n = _ptr(data)
    return lib().crc32c_sw(crc, p, n)


def crc32c(crc: int, data) -> int:
    """src/crc32c.c:675-684."""
    keep, p, n = _ptr(data)
    return lib().crc32c(crc, p, n)


def crc32c_map(data, length: int | None = None) -> int:
    """src/crc32c.c:686-689 (length truncated to unsigned, as in the reference)."""
    b = bytes(data)
    n = len(b) if length is None else length
    return lib().crc32c_map(b, n & 0xFFFFFFFF)


def crc32c_buf(s: bytes) -> int:
    """src/crc32c.c:708-711 (NUL-terminated string)."""
    return lib().crc32c_buf(bytes(s))


class _cstring(ctypes.Structure):
    _fields_ = [("len", ctypes.c_size_t), ("alloc", ctypes.c_size_t), ("buf", ctypes.c_char_p)]


def crc32c_cstring(s: bytes) -> int:
    """src/crc32c.c:703-706 over a zeroskip cstring (cstring.h:23-29)."""
    b = bytes(s)
    cs = _cstring(len(b), len(b) + 1, b)
    return lib().crc32c_cstring(ctypes.byref(cs))


class _iovec(ctypes.Structure):
    _fields_ = [("iov_base", ctypes.c_void_p), ("iov_len", ctypes.c_size_t)]


def crc32c_iovec(parts) -> int:
    """src/crc32c.c:691-701: chain over the parts, skipping empty ones."""
    keeps, vec = [], (_iovec * max(1, len(parts)))()
    for i, part in enumerate(parts):
        keep, p, n = _ptr(part)
        keeps.append(keep)
        vec[i].iov_base, vec[i].iov_len = (p if n else None), n
    return lib().crc32c_iovec(vec, len(parts))


def crc32c_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """crc(A||B) from crc(A), crc(B), |B| (generalises src/crc32c.c:363-367)."""
    return lib().crc32c_combine(crc_a, crc_b, len_b)


def shift(reg: int, nbytes: int) -> int:
    """Raw register after ``nbytes`` zero bytes."""
    return lib().zscrc_shift(reg, nbytes)
