"""Device-resident batches on torch tensors (ROCm build of PyTorch).

Torch supplies device memory and the stream; the work is done by libzscrc's
gfx950 kernels, launched on the tensor's current stream.  Nothing here falls
back to the CPU: a missing library or a non-gfx950 device raises.
"""
from __future__ import annotations

import torch

from ._lib import LEN_UNBOUNDED, ZSCRC_RAW, check, lib


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _dev(t: torch.Tensor) -> torch.device:
    if not t.is_cuda:
        raise ValueError("expected a device tensor")
    return t.device


def crc_fixed(data: torch.Tensor, stride: int, length: int, n: int, seed: int = 0,
              out: torch.Tensor | None = None, raw: bool = False) -> torch.Tensor:
    """out[i] = crc32c(seed, data[i*stride : i*stride+length]) for i < n.

    ``data`` is any contiguous device tensor (viewed as bytes)."""
    dev = _dev(data)
    nbytes = data.numel() * data.element_size()
    if n and (n - 1) * stride + length > nbytes:
        raise ValueError("records extend past the end of the buffer")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(lib().zscrc_device_fixed(data.data_ptr(), stride, length, seed & 0xFFFFFFFF,
                                       out.data_ptr(), n, ZSCRC_RAW if raw else 0,
                                       _stream(dev)), "zscrc_device_fixed")
    return out


def crc_fixed_multi(batches: list[torch.Tensor], stride: int, length: int, n: int, seed: int = 0,
                    outs: list[torch.Tensor] | None = None, raw: bool = False) -> list[torch.Tensor]:
    """crc_fixed over each of the device buffers in `batches` (same stride,
    length and count), in one call (zscrc_device_fixed_multi): one persistent
    launch for records of <= 64 bytes."""
    import ctypes
    k = len(batches)
    dev = _dev(batches[0])
    for b in batches:
        if n and (n - 1) * stride + length > b.numel() * b.element_size():
            raise ValueError("records extend past the end of a batch buffer")
    if outs is None:
        outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(k)]
    bases = (ctypes.c_void_p * k)(*[b.data_ptr() for b in batches])
    optrs = (ctypes.c_void_p * k)(*[o.data_ptr() for o in outs])
    with torch.cuda.device(dev):
        check(lib().zscrc_device_fixed_multi(bases, optrs, k, stride, length, seed & 0xFFFFFFFF, n,
                                             ZSCRC_RAW if raw else 0, _stream(dev)), "zscrc_device_fixed_multi")
    return outs


def crc_batch(data: torch.Tensor, offs: torch.Tensor, lens: torch.Tensor,
              seeds: torch.Tensor | None = None, out: torch.Tensor | None = None,
              raw: bool = False, max_len: int | None = None) -> torch.Tensor:
    """out[i] = crc32c(seeds[i], data[offs[i] : offs[i]+lens[i]]) (int64 offs/lens).
    max_len: a known bound on every lens[i] (zscrc_device_batch_bounded);
    results never depend on it."""
    dev = _dev(data)
    n = offs.numel()
    if offs.dtype != torch.int64 or lens.dtype != torch.int64:
        raise TypeError("offs and lens must be int64 device tensors")
    if seeds is not None and seeds.dtype != torch.int32:
        raise TypeError("seeds must be an int32 device tensor")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(lib().zscrc_device_batch_bounded(data.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                               None if seeds is None else seeds.data_ptr(),
                                               out.data_ptr(), n, ZSCRC_RAW if raw else 0,
                                               LEN_UNBOUNDED if max_len is None else max_len,
                                               _stream(dev)), "zscrc_device_batch_bounded")
    return out


def crc_span(data: torch.Tensor, seed: int = 0, length: int | None = None,
             offset: int = 0, out: torch.Tensor | None = None, raw: bool = False) -> torch.Tensor:
    """One CRC over ``length`` bytes of ``data`` starting at byte ``offset``
    (whole tensor by default), spread over every CU.  Returns a 1-element
    int32 device tensor."""
    dev = _dev(data)
    nbytes = data.numel() * data.element_size()
    if length is None:
        length = nbytes - offset
    if offset < 0 or offset + length > nbytes:
        raise ValueError("span outside the buffer")
    if out is None:
        out = torch.empty(1, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(lib().zscrc_device_span(data.data_ptr() + offset, length, seed & 0xFFFFFFFF,
                                      out.data_ptr(), None, ZSCRC_RAW if raw else 0,
                                      _stream(dev)), "zscrc_device_span")
    return out


def crc_spans(data: torch.Tensor, offsets, lengths, seeds=None, out: torch.Tensor | None = None,
              raw: bool = False) -> torch.Tensor:
    """CRC of each span data[offsets[i] : +lengths[i]] in one call
    (zscrc_device_spans: one segment launch and one fold launch for up to 8
    spans of >= 16 KiB).  Returns an int32 device tensor."""
    import ctypes
    dev = _dev(data)
    nbytes = data.numel() * data.element_size()
    k = len(offsets)
    assert len(lengths) == k
    for o, n in zip(offsets, lengths):
        if o < 0 or o + n > nbytes:
            raise ValueError("span outside the buffer")
    if out is None:
        out = torch.empty(k, dtype=torch.int32, device=dev)
    bufs = (ctypes.c_void_p * max(k, 1))(*[data.data_ptr() + int(o) for o in offsets])
    lens = (ctypes.c_uint64 * max(k, 1))(*[int(n) for n in lengths])
    sds = (ctypes.c_uint32 * max(k, 1))(*[int(v) & 0xFFFFFFFF for v in seeds]) if seeds is not None else None
    with torch.cuda.device(dev):
        check(lib().zscrc_device_spans(bufs, lens, sds, out.data_ptr(), k, ZSCRC_RAW if raw else 0,
                                       _stream(dev)), "zscrc_device_spans")
    return out


def as_u32(t: torch.Tensor) -> list[int]:
    """int32 device tensor of CRCs -> python ints (unsigned)."""
    return [v & 0xFFFFFFFF for v in t.cpu().tolist()]
