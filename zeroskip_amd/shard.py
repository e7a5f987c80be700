"""Multi-GPU CRC-32C of one logical byte stream: one process per GPU.

The repack / consistency path checksums spans that can be gigabytes long
(zeroskip's whole packed records region goes through ONE crc32_end,
/root/reference/src/mfile.c:534-546 via zeroskip-packed.c:442).  Here the span
is cut into contiguous byte ranges, one per rank; every rank computes the RAW
register of its own range on its own GPU (no data crosses xGMI), the tiny
(register, length) digests are all-gathered over RCCL, and every rank folds
them with the zero-shift operator:

    reg = shift(R0, L) ^ XOR_r shift(raw_r, bytes after range r)

XOR is not an NCCL reduction op, so the exchange is a gather, not an
all-reduce.  The fold is the reference's crc32c_shift (src/crc32c.c:363-367)
generalised to any distance (libzscrc ``zscrc_shift``).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from ._lib import lib

M32 = 0xFFFFFFFF


def shard_ranges(total: int, world: int, align: int = 4096) -> list[tuple[int, int]]:
    """Contiguous [start, end) byte ranges, one per rank, cut on `align`."""
    per = -(-total // world)
    per = -(-per // align) * align if total >= align * world else per
    out, start = [], 0
    for _ in range(world):
        end = min(total, start + per)
        out.append((start, end))
        start = end
    return out


def fold(digests: list[tuple[int, int]], seed: int = 0, raw_seed: bool = False) -> int:
    """Fold per-range (raw register, length) digests, in stream order, into
    crc32c(seed, stream).  With raw_seed the seed is the initial register and
    the raw final register is returned."""
    L = lib()
    total = sum(n for _, n in digests)
    reg = (seed if raw_seed else seed ^ M32) & M32
    reg = L.zscrc_shift(reg, total)
    after = total
    for r, n in digests:
        after -= n
        reg ^= L.zscrc_shift(r & M32, after)
    return reg if raw_seed else reg ^ M32


def gpu_raw_partial(local: torch.Tensor) -> int:
    """Raw register (from 0) of this rank's bytes, on this rank's GPU."""
    from .device import crc_span
    if local.numel() == 0:
        return 0
    out = crc_span(local, seed=0, raw=True)
    return int(out.item()) & M32


def sharded_crc(local: torch.Tensor, seed: int = 0, group=None,
                partial_fn: Callable[[torch.Tensor], int] | None = None) -> int:
    """crc32c(seed, concat of every rank's `local` bytes in rank order).

    Every rank passes its own range (a uint8 tensor on its GPU); the result is
    returned on every rank.  `partial_fn` replaces the GPU partial (CPU tests)."""
    partial = (partial_fn or gpu_raw_partial)(local)
    n = local.numel() * local.element_size()
    dev = local.device if (local.is_cuda and dist.get_backend(group) == "nccl") else torch.device("cpu")
    mine = torch.tensor([partial, n], dtype=torch.int64, device=dev)
    world = dist.get_world_size(group)
    allv = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allv, mine, group=group)
    v = allv.cpu().tolist()
    return fold([(v[2 * i], v[2 * i + 1]) for i in range(world)], seed)


def gather_digests(local_out: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather every rank's per-record CRC vector (int32, same length on
    every rank) -- the per-range digest exchange of a sharded verify."""
    world = dist.get_world_size(group)
    allv = torch.empty(world * local_out.numel(), dtype=local_out.dtype, device=local_out.device)
    dist.all_gather_into_tensor(allv, local_out.contiguous(), group=group)
    return allv
