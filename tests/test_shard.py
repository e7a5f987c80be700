"""Sharded CRC over ranks (gloo, world size 2 and 3, CPU): the digest exchange
and the fold reproduce the oracle CRC of the whole stream.  The per-rank raw
partial is computed by the oracle here (no GPU); on the GPU box the same fold
runs over libzscrc partials (tests/test_gpu_parity.py::test_sharded_*)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle
from zeroskip_amd import shard

M32 = 0xFFFFFFFF


def cpu_partial(t: torch.Tensor) -> int:
    # raw register from 0: crc with init ~0 -> xor both ends
    b = t.numpy().tobytes()
    return (~oracle.crc32c_hw(M32, b)) & M32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, seed, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = np.random.default_rng(123).integers(0, 256, total, dtype=np.uint8)
    ranges = shard.shard_ranges(total, world, align=64)
    lo, hi = ranges[rank]
    local = torch.from_numpy(data[lo:hi].copy())
    crc = shard.sharded_crc(local, seed=seed, partial_fn=cpu_partial)
    digs = shard.gather_digests(torch.tensor([rank * 10 + 1, rank * 10 + 2], dtype=torch.int32))
    q.put((rank, crc, digs.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 100_003), (3, 4096 * 3 + 7), (2, 5)])
def test_sharded_crc_gloo(world, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, 0x5EED, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = np.random.default_rng(123).integers(0, 256, total, dtype=np.uint8)
    want = oracle.crc32c_hw(0x5EED, data)
    for rank, crc, digs in res:
        assert crc == want, rank
        assert digs == [v for r in range(world) for v in (r * 10 + 1, r * 10 + 2)]


def test_shard_ranges_cover_stream():
    for total in (0, 1, 4095, 4096, 10**7 + 3):
        for world in (1, 2, 3, 8):
            r = shard.shard_ranges(total, world)
            assert len(r) == world and r[0][0] == 0 and r[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))


def test_fold_matches_oracle_any_split():
    rng = np.random.default_rng(9)
    d = rng.integers(0, 256, 20000, dtype=np.uint8)
    cuts = sorted(rng.integers(0, 20000, 6).tolist())
    bounds = [0] + cuts + [20000]
    digs = [(cpu_partial(torch.from_numpy(d[a:b].copy())), b - a) for a, b in zip(bounds, bounds[1:])]
    assert shard.fold(digs, 0xABCDEF) == oracle.crc32c_hw(0xABCDEF, d)


def test_fold_random_splits():
    """The GF(2) fold of per-piece raw registers over random cuts -- empty
    pieces, one-byte pieces, a single piece -- and random seeds equals the
    oracle CRC of the whole stream (200 trials)."""
    rng = np.random.default_rng(19)
    for _ in range(200):
        n = int(rng.integers(0, 5000))
        d = rng.integers(0, 256, n, dtype=np.uint8)
        k = int(rng.integers(0, 9))
        bounds = [0] + sorted(rng.integers(0, n + 1, k).tolist()) + [n]
        digs = [(cpu_partial(torch.from_numpy(d[a:b].copy())), b - a) for a, b in zip(bounds, bounds[1:])]
        seed = int(rng.integers(0, 1 << 32))
        assert shard.fold(digs, seed) == oracle.crc32c_hw(seed, d), (n, bounds, seed)


def test_sharded_crc_gloo_four_ranks():
    test_sharded_crc_gloo(4, 3 * 4096 + 65 * 17)
