"""zeroskip_amd -- MI355X-native CRC-32C engine for zeroskip.

The product is the C-ABI library ``libzscrc.so`` built in this directory from
``csrc/`` (gfx950 HIP kernels + host API).  This package is its Python view:

* :mod:`zeroskip_amd.crc32c` mirrors the reference checksum API
  (``/root/reference/include/libzeroskip/crc32c.h:15-24``);
* :mod:`zeroskip_amd.device` runs batches on device-resident torch tensors;
* :mod:`zeroskip_amd.shard` shards a span over ranks (one process per GPU) and
  folds the per-rank digests gathered with ``torch.distributed``.

There is no fallback: if ``libzscrc.so`` is missing the import fails.
"""
from ._lib import lib, build_library, LIB_PATH, ZscrcError, check  # noqa: F401

__all__ = ["lib", "build_library", "LIB_PATH", "ZscrcError", "check"]
