"""Incremental CRC-32C of a host byte stream on the GPU (include/zscrc.h
``zscrc_stream_*``): the crc32_begin / mfile_write / crc32_end shape of
zeroskip's commit and repack paths (/root/reference/src/mfile.c:270-290,
:526-546; the records-region CRC of src/zeroskip-packed.c:442).

    with CrcStream(seed=0) as s:
        for block in blocks:
            s.update(block)
    crc = s.crc

No CPU fallback: without a gfx950 device open() raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import ZSCRC_STREAM_NOCOPY, check, lib


class CrcStream:
    def __init__(self, seed: int = 0, chunk_bytes: int = 0, nocopy: bool = False):
        self._h = ctypes.c_void_p()
        self._keep = []
        self.nocopy = nocopy
        self.crc = None
        check(lib().zscrc_stream_open(ctypes.byref(self._h), seed & 0xFFFFFFFF, chunk_bytes,
                                      ZSCRC_STREAM_NOCOPY if nocopy else 0), "zscrc_stream_open")

    def update(self, data) -> None:
        a = data if isinstance(data, np.ndarray) else np.frombuffer(memoryview(data), dtype=np.uint8)
        a = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        if self.nocopy:
            self._keep.append(a)  # must stay alive and unchanged until final()
        check(lib().zscrc_stream_update(self._h, a.ctypes.data, a.nbytes), "zscrc_stream_update")

    def final(self) -> int:
        if self.crc is None:
            out = ctypes.c_uint32()
            h, self._h = self._h, None
            check(lib().zscrc_stream_final(h, ctypes.byref(out)), "zscrc_stream_final")
            self._keep.clear()
            self.crc = out.value
        return self.crc

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.final()
        return False
