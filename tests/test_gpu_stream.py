"""zscrc_stream_* (host byte streams checksummed on the GPU) against the
oracle: irregular update sizes across chunk boundaries, both copy modes,
seeds, many chunks (register-array growth), empty streams."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle
from zeroskip_amd.stream import CrcStream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nocopy", [False, True])
@pytest.mark.parametrize("seed", [0, 0xDEADBEEF])
def test_irregular_updates(gpu, nocopy, seed):
    rng = np.random.default_rng(5 + nocopy)
    data = rng.integers(0, 256, (24 << 20) + 12345, dtype=np.uint8)
    cuts = [0, 1, 8, 15, 4096, (1 << 20) - 3, (1 << 20) + 5, 7 << 20, (7 << 20) + 1, 19 << 20, len(data)]
    with CrcStream(seed, chunk_bytes=1 << 20, nocopy=nocopy) as s:
        for a, b in zip(cuts, cuts[1:]):
            s.update(data[a:b])
    assert s.crc == oracle.crc32c_hw(seed, data)


def test_many_chunks(gpu):
    data = np.random.default_rng(9).integers(0, 256, (20 << 20) + 77, dtype=np.uint8)
    s = CrcStream(7, chunk_bytes=4096)        # > 4096 chunks: the register array grows
    for i in range(0, len(data), 3 << 20):
        s.update(data[i:i + (3 << 20)])
    assert s.final() == oracle.crc32c_hw(7, data)


def test_empty_and_tiny(gpu):
    assert CrcStream(0x1234).final() == 0x1234
    s = CrcStream(0)
    s.update(b"")
    s.update(b"lorem")
    s.update(b" ipsum")
    assert s.final() == 0xdfb4e6c9          # tests/unit-crc32c.c:36


def test_default_chunk_large(gpu):
    data = np.random.default_rng(11).integers(0, 256, (200 << 20) + 3, dtype=np.uint8)
    with CrcStream(0, nocopy=True) as s:
        s.update(data)
    assert s.crc == oracle.crc32c_hw(0, data)


@pytest.mark.parametrize("per_wave", [16, 0], ids=["dealt", "static"])
@pytest.mark.parametrize("shape", ["mixed", "equal", "fallback_short", "fallback_many"])
def test_device_spans(gpu, shape, per_wave):
    """zscrc_device_spans (one segment launch + one fold launch for up to 8
    spans) against the oracle: spans of very different lengths, unaligned
    offsets, seeds, standard and raw registers; short or many spans take
    the per-span path.  The segments dealt per workgroup (16 per wave) or
    on the static walk (two per wave)."""
    import torch
    from oracle import oracle
    from zeroskip_amd import device as zd
    from zeroskip_amd._lib import lib
    old = lib().zscrc_set_xdeal(per_wave)
    try:
        _device_spans(gpu, shape, torch, oracle, zd)
    finally:
        lib().zscrc_set_xdeal(old)


def _device_spans(gpu, shape, torch, oracle, zd):
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, (300 << 20) + 4096, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    if shape == "mixed":
        spans = [(3, 200 << 20), (1, 16 << 10), ((200 << 20) + 17, 40 << 20), ((250 << 20) + 2, 1000003),
                 ((260 << 20) + 5, 33 << 10)]
    elif shape == "equal":
        spans = [(i * (32 << 20), 32 << 20) for i in range(8)]
    elif shape == "fallback_short":
        spans = [(0, 100), (7, 64 << 20), (5, 1 << 10)]
    else:
        spans = [(i * (1 << 20) + i, (1 << 20) + 3 * i) for i in range(11)]
    offs, lens = [o for o, _ in spans], [n for _, n in spans]
    seeds = [int(v) for v in rng.integers(0, 2**32, len(spans), dtype=np.uint64)]
    got = zd.crc_spans(d, offs, lens, seeds).cpu().numpy().view(np.uint32)
    want = [oracle.crc32c_hw(s, host[o:o + n]) for (o, n), s in zip(spans, seeds)]
    assert [int(v) for v in got] == want, shape
    raw = zd.crc_spans(d, offs, lens, raw=True).cpu().numpy().view(np.uint32)
    want_raw = [(~oracle.crc32c_hw(0xFFFFFFFF, host[o:o + n])) & 0xFFFFFFFF for o, n in spans]
    assert [int(v) for v in raw] == want_raw, shape
