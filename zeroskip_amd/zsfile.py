"""zeroskip file images: walk, span descriptors and GPU commit verification.

Python view of include/zscrc.h Part 3 (zeroskip_amd/csrc/zscrc_zs.cpp).  The
walk follows the reference (src/zeroskip-record.c:283-331); each commit's CRC
(span + host-order trailer words, src/zeroskip-file.c:253-350) is recomputed
and compared on the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import LEN_UNBOUNDED, check, lib

END, STOPPED, TRUNCATED, OVERFLOW, BADSIG = 0, 1, 2, 3, 4
ACTIVE, FINALISED, PACKED = 0, 1, 2


class Report(ctypes.Structure):
    _fields_ = [("header_rc", ctypes.c_int), ("header_stored", ctypes.c_uint32),
                ("header_computed", ctypes.c_uint32), ("walk_rc", ctypes.c_int),
                ("end_off", ctypes.c_uint64), ("n_commits", ctypes.c_uint64),
                ("n_bad", ctypes.c_uint64), ("first_bad", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def _host(image):
    a = np.ascontiguousarray(np.frombuffer(image, dtype=np.uint8) if isinstance(image, (bytes, bytearray, memoryview)) else image)
    return a, a.ctypes.data, a.nbytes


def walk(image):
    """(span_off, span_len, rc, end_off) of every commit of an active or
    finalised file image."""
    a, p, n = _host(image)
    cap = n // 8 + 1
    off = np.empty(cap, np.uint64)
    ln = np.empty(cap, np.uint64)
    nc = ctypes.c_size_t()
    end = ctypes.c_uint64()
    rc = lib().zscrc_zs_walk(p, n, off.ctypes.data, ln.ctypes.data, cap, ctypes.byref(nc),
                             ctypes.byref(end))
    if rc < 0:
        check(rc, "zscrc_zs_walk")
    return off[:nc.value], ln[:nc.value], rc, end.value


def packed_spans(image):
    a, p, n = _host(image)
    off = np.empty(2, np.uint64)
    ln = np.empty(2, np.uint64)
    rc = lib().zscrc_zs_packed_spans(p, n, off.ctypes.data, ln.ctypes.data)
    return off, ln, rc


def header_crc(image):
    a, p, n = _host(image)
    st, cp = ctypes.c_uint32(), ctypes.c_uint32()
    rc = lib().zscrc_zs_header_crc(p, n, ctypes.byref(st), ctypes.byref(cp))
    return rc, st.value, cp.value


def dotzsdb_crc(image):
    a, p, n = _host(image)
    st, cp = ctypes.c_uint32(), ctypes.c_uint32()
    rc = lib().zscrc_zs_dotzsdb_crc(p, n, ctypes.byref(st), ctypes.byref(cp))
    return rc, st.value, cp.value


def verify_image(image, kind: int = ACTIVE) -> dict:
    """Header on the CPU, every commit on the current GPU (synchronous)."""
    a, p, n = _host(image)
    rep = Report()
    check(lib().zscrc_zs_verify_image(p, n, kind, ctypes.byref(rep)), "zscrc_zs_verify_image")
    return rep.as_dict()


def verify_commits(d_image: torch.Tensor, span_off: torch.Tensor, span_len: torch.Tensor,
                   seed: torch.Tensor | None = None, max_len: int | None = None):
    """Device-resident commit verification: (crc, status) int32 tensors;
    status 1 = stored CRC matches, 0 = mismatch, 2 = no commit record.
    seed (int32, optional): span i's CRC continues from seed[i]
    (zscrc_device_verify_commits_seeded) -- the reference's zero-length
    finalise commit chains from the previous span's CRC.
    max_len (optional): a known bound on the span lengths, e.g. from the host
    walk (zscrc_device_verify_commits_bounded); results never depend on it."""
    n = span_off.numel()
    size = d_image.numel() * d_image.element_size()
    crc = torch.empty(n, dtype=torch.int32, device=d_image.device)
    st = torch.empty(n, dtype=torch.int32, device=d_image.device)
    with torch.cuda.device(d_image.device):
        stream = torch.cuda.current_stream(d_image.device).cuda_stream
        if max_len is not None:
            assert seed is None or (seed.numel() == n and seed.dtype == torch.int32)
            check(lib().zscrc_device_verify_commits_bounded(
                d_image.data_ptr(), size, span_off.data_ptr(), span_len.data_ptr(),
                None if seed is None else seed.data_ptr(), n, max_len, crc.data_ptr(), st.data_ptr(),
                stream), "zscrc_device_verify_commits_bounded")
        elif seed is None:
            check(lib().zscrc_device_verify_commits(
                d_image.data_ptr(), size, span_off.data_ptr(), span_len.data_ptr(), n, crc.data_ptr(),
                st.data_ptr(), stream), "zscrc_device_verify_commits")
        else:
            assert seed.numel() == n and seed.dtype == torch.int32 and seed.device == d_image.device
            check(lib().zscrc_device_verify_commits_seeded(
                d_image.data_ptr(), size, span_off.data_ptr(), span_len.data_ptr(), seed.data_ptr(), n,
                crc.data_ptr(), st.data_ptr(), stream), "zscrc_device_verify_commits_seeded")
    return crc, st


def verify_commits_verdict(d_image: torch.Tensor, span_off: torch.Tensor, span_len: torch.Tensor,
                           seed: torch.Tensor | None = None, max_len: int | None = None, cap: int = 4096,
                           out: tuple | None = None, min_len: int = 0):
    """Device verdict (zscrc_device_verify_commits_verdict): (nbad, bad)
    int64 device tensors -- nbad[0] = commits that do not verify, bad[:min(
    nbad, cap)] their indices in no particular order.  No per-commit output.
    `out`: preallocated (nbad, bad) tensors to reuse.  max_len alone: a bound
    the results never depend on (zscrc_device_verify_commits_verdict); with
    min_len > 0, [min_len, max_len] is a range every span length must lie in
    (zscrc_device_verify_commits_verdict_range: classes outside it get no
    launch)."""
    n = span_off.numel()
    size = d_image.numel() * d_image.element_size()
    dev = d_image.device
    if out is None:
        out = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(max(cap, 1), dtype=torch.int64, device=dev))
    nbad, bad = out
    assert seed is None or (seed.numel() == n and seed.dtype == torch.int32)
    mx = LEN_UNBOUNDED if max_len is None else max_len
    stream = torch.cuda.current_stream(dev).cuda_stream
    sp = None if seed is None else seed.data_ptr()
    with torch.cuda.device(dev):
        if min_len > 0:
            check(lib().zscrc_device_verify_commits_verdict_range(
                d_image.data_ptr(), size, span_off.data_ptr(), span_len.data_ptr(), sp, n, min_len, mx,
                nbad.data_ptr(), bad.data_ptr(), min(cap, bad.numel()), stream),
                "zscrc_device_verify_commits_verdict_range")
        else:
            check(lib().zscrc_device_verify_commits_verdict(
                d_image.data_ptr(), size, span_off.data_ptr(), span_len.data_ptr(), sp, n, mx,
                nbad.data_ptr(), bad.data_ptr(), min(cap, bad.numel()), stream),
                "zscrc_device_verify_commits_verdict")
    return nbad, bad


def write_commits(d_image: torch.Tensor, span_off: torch.Tensor, span_len: torch.Tensor,
                  max_len: int | None = None, status: bool = False, crc: bool = True):
    """Writer side on the GPU: compute every commit CRC and store it
    big-endian into its commit record in `d_image` (in place).  max_len: a
    known bound on the span lengths (zscrc_device_write_commits_bounded).
    crc=False: the CRCs only go into the image (returns None).
    Returns the CRCs, or (crc, status) with status=True: 1 written, 2 no
    commit record there (nothing written)."""
    n = span_off.numel()
    size = d_image.numel() * d_image.element_size()
    want_crc = crc
    crc = torch.empty(n, dtype=torch.int32, device=d_image.device) if want_crc else None
    st = torch.empty(n, dtype=torch.int32, device=d_image.device) if status else None
    with torch.cuda.device(d_image.device):
        check(lib().zscrc_device_write_commits_bounded(
            d_image.data_ptr(), size, span_off.data_ptr(), span_len.data_ptr(), n,
            LEN_UNBOUNDED if max_len is None else max_len, None if crc is None else crc.data_ptr(),
            None if st is None else st.data_ptr(),
            torch.cuda.current_stream(d_image.device).cuda_stream), "zscrc_device_write_commits_bounded")
    return (crc, st) if status else crc


def commit_crcs(d_image: torch.Tensor, span_off: torch.Tensor, span_len: torch.Tensor,
                max_len: int | None = None, status: bool = False):
    """The writer's commit CRCs out of place (zscrc_device_commit_crcs_bounded):
    an int32 tensor, crc[i] = what zscrc_device_write_commits would store for
    span i; the image is only read.  status=True: (crc, status), 1 a commit
    record is there, 2 none."""
    n = span_off.numel()
    size = d_image.numel() * d_image.element_size()
    crc = torch.empty(n, dtype=torch.int32, device=d_image.device)
    st = torch.empty(n, dtype=torch.int32, device=d_image.device) if status else None
    with torch.cuda.device(d_image.device):
        check(lib().zscrc_device_commit_crcs_bounded(
            d_image.data_ptr(), size, span_off.data_ptr(), span_len.data_ptr(), n,
            LEN_UNBOUNDED if max_len is None else max_len, crc.data_ptr(), None if st is None else st.data_ptr(),
            torch.cuda.current_stream(d_image.device).cuda_stream), "zscrc_device_commit_crcs_bounded")
    return (crc, st) if status else crc


class FillReport(ctypes.Structure):
    """zscrc_fill_report (include/zscrc.h)."""
    _fields_ = [("commits", ctypes.c_uint64), ("no_record", ctypes.c_uint64), ("long_commits", ctypes.c_uint64),
                ("bytes", ctypes.c_uint64), ("desc_bytes", ctypes.c_uint64), ("chunks", ctypes.c_uint64),
                ("staged", ctypes.c_int32), ("threads", ctypes.c_int32), ("h2d_s", ctypes.c_double),
                ("total_s", ctypes.c_double), ("setup_s", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def fill_commits(image, span_off, span_len, max_len: int | None = None, threads: int = 0) -> dict:
    """The commit writer for a HOST image (zscrc_zs_fill_commits): every
    commit CRC computed on the current GPU and stored into `image` in place
    (a writable uint8 numpy array or CPU tensor; pinned memory is copied
    directly, pageable memory through pinned staging).  span_off / span_len:
    sorted, disjoint spans (uint64 numpy arrays or CPU tensors)."""
    if isinstance(image, torch.Tensor):
        assert not image.is_cuda and image.is_contiguous()
        ptr, size = image.data_ptr(), image.numel() * image.element_size()
    else:
        assert image.flags.c_contiguous and image.flags.writeable
        ptr, size = image.ctypes.data, image.nbytes
    o = np.ascontiguousarray(span_off.numpy() if isinstance(span_off, torch.Tensor) else span_off, dtype=np.uint64)
    ln = np.ascontiguousarray(span_len.numpy() if isinstance(span_len, torch.Tensor) else span_len, dtype=np.uint64)
    assert o.shape == ln.shape
    rep = FillReport()
    check(lib().zscrc_zs_fill_commits(ptr, size, o.ctypes.data, ln.ctypes.data, len(o),
                                      LEN_UNBOUNDED if max_len is None else max_len, threads, ctypes.byref(rep)),
          "zscrc_zs_fill_commits")
    return rep.as_dict()


class FilesReport(ctypes.Structure):
    """zscrc_files_report (include/zscrc.h)."""
    _fields_ = [("files", ctypes.c_uint64), ("commits", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("bad_commits", ctypes.c_uint64), ("stale_empty_commits", ctypes.c_uint64),
                ("header_errors", ctypes.c_uint64), ("walk_errors", ctypes.c_uint64),
                ("first_bad_file", ctypes.c_uint64), ("first_bad_off", ctypes.c_uint64),
                ("first_bad_what", ctypes.c_int32), ("threads", ctypes.c_int32), ("staged", ctypes.c_int32),
                ("copy_s", ctypes.c_double), ("verify_tail_s", ctypes.c_double), ("total_s", ctypes.c_double),
                ("devices", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def set_devices(ids) -> None:
    """Device slots of verify_files / consistent (zscrc_set_devices): a list
    of device ids, repeats allowed; None or [] = the default (env
    ZSCRC_DEVICES, else every visible gfx950 device)."""
    ids = list(ids or [])
    arr = (ctypes.c_int * max(1, len(ids)))(*ids)
    check(lib().zscrc_set_devices(arr, len(ids)), "zscrc_set_devices")


def devices() -> list:
    """The device slots a verify_files call would use now."""
    arr = (ctypes.c_int * 64)()
    n = lib().zscrc_files_devices(arr, 64)
    if n < 0:
        check(n, "zscrc_files_devices")
    return list(arr[:n])


def verify_files(images, kinds=None, threads: int = 0) -> dict:
    """End to end from host memory (zscrc_zs_verify_files): every header,
    walk and commit CRC of the given file images (numpy uint8 arrays, bytes
    or memmaps; kinds default ACTIVE), on the current GPU.  Synchronous."""
    arrs = [_host(im)[0] for im in images]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data if a.nbytes else None for a in arrs])
    sizes = np.array([a.nbytes for a in arrs], np.uint64)
    kk = np.array([ACTIVE] * n if kinds is None else list(kinds), np.int32)
    rep = FilesReport()
    check(lib().zscrc_zs_verify_files(ptrs, sizes.ctypes.data, kk.ctypes.data, n, threads, ctypes.byref(rep)),
          "zscrc_zs_verify_files")
    return rep.as_dict()
