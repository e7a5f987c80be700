"""Parity of the gfx950 kernels (through the C ABI) with the CPU oracle.

Bit-exact equality on every record; the oracle (oracle/zs_oracle.c) is the
checker, the golden fixtures pin it to the reference's known answers."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from tests.golden.datagen import xorshift64_bytes
from zeroskip_amd import device as zd
from zeroskip_amd import crc32c as zc
from zeroskip_amd._lib import DEFAULT_TEAMS, QTEAM_DEFAULT, lib, stats

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "crc32c_golden.json")))
M32 = 0xFFFFFFFF


def to_dev(a: np.ndarray, dev) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def u32(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


@pytest.fixture(params=[DEFAULT_TEAMS, (0, 0), (1 << 40, 1 << 40), (0, 1 << 40)],
                ids=["default", "all-g64", "all-g1", "all-g16"])
def teams(request, gpu):
    lib().zscrc_set_teams(*request.param)
    yield request.param
    lib().zscrc_set_teams(*DEFAULT_TEAMS)


@pytest.fixture(params=[-1, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10],
                ids=["g1-auto", "g1-ring1", "g1-ring2", "g1-short", "g1-short-pf", "g1-short-pf2",
                     "g1-burst2", "g1-burst3", "g1-burst4", "g1-record-burst", "g1-record-burst-quad"])
def g1_walk(request, gpu):
    lib().zscrc_set_prefetch(1, request.param)
    yield request.param
    lib().zscrc_set_prefetch(1, -1)


def test_golden_cases_g1_walks(gpu, g1_walk):
    """Every one-lane-per-record walk (team ring / short kernel) on the golden
    cases, the fixed-stride shapes and a commit batch."""
    lib().zscrc_set_teams(1 << 40, 1 << 40)
    try:
        data = xorshift64_bytes(GOLDEN["data"]["bytes"])
        rows = np.array(GOLDEN["cases"], dtype=np.uint64)
        d = to_dev(data, gpu)
        offs = to_dev(rows[:, 0].astype(np.int64), gpu)
        lens = to_dev(rows[:, 1].astype(np.int64), gpu)
        seeds = to_dev(rows[:, 2].astype(np.uint32).view(np.int32), gpu)
        assert np.array_equal(u32(zd.crc_batch(d, offs, lens, seeds)), rows[:, 3].astype(np.uint32))
        for stride, length, n in [(64, 64, 70000), (320, 312, 20000), (1040, 1037, 3000), (7, 7, 500)]:
            data = rand_bytes(stride * (n - 1) + length, stride * 7 + length)
            out = u32(zd.crc_fixed(to_dev(data, gpu), stride, length, n, seed=0x77))
            assert np.array_equal(out, _oracle_seeded(data, stride, length, n, 0x77)), (stride, length)
            raw = u32(zd.crc_fixed(to_dev(data[3:], gpu), stride, length - 3, n - 1, raw=True))
            ref = oracle.batch(data[3:], n=n - 1, stride=stride, fixed_len=length - 3, impl="hw",
                               seeds=np.full(n - 1, M32, np.uint32)) ^ np.uint32(M32)
            assert np.array_equal(raw, ref), (stride, length, "raw")
    finally:
        lib().zscrc_set_teams(*DEFAULT_TEAMS)


def test_golden_cases_variable_batch(gpu, teams):
    data = xorshift64_bytes(GOLDEN["data"]["bytes"])
    rows = np.array(GOLDEN["cases"], dtype=np.uint64)
    d = to_dev(data, gpu)
    offs = to_dev(rows[:, 0].astype(np.int64), gpu)
    lens = to_dev(rows[:, 1].astype(np.int64), gpu)
    seeds = to_dev(rows[:, 2].astype(np.uint32).view(np.int32), gpu)
    out = u32(zd.crc_batch(d, offs, lens, seeds))
    assert np.array_equal(out, rows[:, 3].astype(np.uint32))


def test_kats_on_device(gpu):
    for k in GOLDEN["kats"] + [dict(hex=GOLDEN["crc32bench"]["text"].encode().hex(), seed=0,
                                    crc=GOLDEN["crc32bench"]["crc"])]:
        raw = np.frombuffer(bytes.fromhex(k["hex"]), dtype=np.uint8)
        buf = to_dev(np.concatenate([raw, np.zeros(8, np.uint8)]), gpu)
        offs = torch.zeros(1, dtype=torch.int64, device=gpu)
        lens = torch.full((1,), len(raw), dtype=torch.int64, device=gpu)
        seeds = torch.tensor([np.uint32(k["seed"]).view(np.int32)], device=gpu)
        assert u32(zd.crc_batch(buf, offs, lens, seeds))[0] == k["crc"]


@pytest.mark.parametrize("stride,length,n", [
    (64, 64, 1 << 20),          # BASELINE config 2, full size: 1M x 64 B
    (320, 312, 20000),          # zsbench BATCHED span (key 40 B + value 272 B)
    (65536, 65536, 512),        # config 3 shape (64 KiB chunks), 32 MiB
    (4096, 4000, 3000),
    (1040, 1037, 5000),         # unaligned starts, ragged tails
    (100000, 99999, 300),
    (8, 8, 100000),
    (5, 5, 1000),               # < 8 bytes: serial path
])
def test_fixed_stride(gpu, stride, length, n):
    data = rand_bytes(stride * (n - 1) + length, stride + length)
    out = u32(zd.crc_fixed(to_dev(data, gpu), stride, length, n, seed=0x1234))
    ref = _oracle_seeded(data, stride, length, n, 0x1234)
    bad = np.nonzero(out != ref)[0]
    assert bad.size == 0, bad[:10]


@pytest.mark.parametrize("mode,shapes", [
    (0, [(128, 128, 50000), (256, 256, 30000), (1024, 1024, 5000), (768, 640, 8000)]),
    (2, [(64, 64, 70000), (320, 312, 20000), (1040, 1000, 3000), (200, 200, 9000),
         (130, 129, 5000), (7, 7, 500), (1, 1, 100), (256, 256, 3000)]),
], ids=["auto-aligned", "forced-ragged"])
def test_two_lane_teams(gpu, mode, shapes):
    """2-lane teams (zscrc_set_small_team): chosen automatically on 128-byte
    aligned records, forced onto ragged lengths, odd strides and a base 3 bytes
    off alignment."""
    lib().zscrc_set_small_team(mode)
    lib().zscrc_set_teams(1024, 1 << 20)
    try:
        if mode == 0:
            assert lib().zscrc_team_for(256, 1 << 20) == 2
            assert lib().zscrc_team_for(312, 1 << 20) == 1
        for stride, length, n in shapes:
            data = rand_bytes(stride * (n - 1) + length + 3, stride * 3 + length)
            out = u32(zd.crc_fixed(to_dev(data, gpu), stride, length, n, seed=0x5a5a))
            assert np.array_equal(out, _oracle_seeded(data, stride, length, n, 0x5a5a)), (stride, length)
            out = u32(zd.crc_fixed(to_dev(data[3:], gpu), stride, length, n, seed=7))
            assert np.array_equal(out, _oracle_seeded(data[3:], stride, length, n, 7)), (stride, length, "+3")
    finally:
        lib().zscrc_set_small_team(0)
        lib().zscrc_set_teams(*DEFAULT_TEAMS)


@pytest.mark.parametrize("bound", ["exact", "loose", "wrong", "none"])
def test_bounded_batch(gpu, bound):
    """zscrc_device_batch_bounded: a length bound of short records takes one
    kernel over the caller's arrays; results never depend on the bound (a
    wrong one included)."""
    rng = np.random.default_rng(11)
    n = 40000
    lens = rng.integers(0, 400, n).astype(np.uint64)
    lens[::97] = rng.integers(401, 5000, lens[::97].size)   # a few longer ones
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 9, n - 1).astype(np.uint64))
    data = rand_bytes(int(offs[-1] + lens[-1]) + 8, 5)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ref = oracle.batch(data, offs, lens, seeds, impl="hw", threads=8)
    mx = {"exact": int(lens.max()), "loose": 640, "wrong": 300, "none": None}[bound]
    if bound == "exact":
        lens = np.minimum(lens, 600).astype(np.uint64)      # all short: the one-kernel path
        ref = oracle.batch(data, offs, lens, seeds, impl="hw", threads=8)
        mx = int(lens.max())
    d = to_dev(data, gpu)
    out = u32(zd.crc_batch(d, to_dev(offs.astype(np.int64), gpu), to_dev(lens.astype(np.int64), gpu),
                           to_dev(seeds.view(np.int32), gpu), max_len=mx))
    assert np.array_equal(out, ref), np.nonzero(out != ref)[0][:10]


def _oracle_seeded(data, stride, length, n, seed):
    offs = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, length, dtype=np.uint64)
    seeds = np.full(n, seed, dtype=np.uint32)
    return oracle.batch(data, offs, lens, seeds, impl="hw", threads=8)


def test_variable_random_batch(gpu, teams):
    rng = np.random.default_rng(42)
    n = 4000
    lens = np.exp(rng.uniform(0, np.log(300000), n)).astype(np.int64)
    lens[rng.integers(0, n, 200)] = rng.integers(0, 9, 200)  # tiny records
    total = int(lens.sum()) + 64 * n
    data = rand_bytes(total, 99)
    gaps = rng.integers(0, 64, n)
    offs = np.cumsum(np.concatenate([[0], lens[:-1] + gaps[:-1]])).astype(np.int64)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = u32(zd.crc_batch(to_dev(data, gpu), to_dev(offs, gpu), to_dev(lens, gpu),
                           to_dev(seeds.view(np.int32), gpu)))
    ref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), seeds, impl="hw",
                       threads=8)
    bad = np.nonzero(out != ref)[0]
    assert bad.size == 0, [(int(i), int(offs[i]), int(lens[i])) for i in bad[:10]]


@pytest.mark.parametrize("lens", [[(1 << 20) + 1], [3 * (1 << 20) + 13], [(64 << 20) + 5],
                                  [(1 << 20) + 7, 100, (5 << 20) + 3, 8, (2 << 20)]],
                         ids=["1MiB+1", "3MiB+13", "64MiB+5", "mixed"])
def test_few_long_records_split(gpu, lens):
    """A handful of long records: each is split into up to 8192 parts (every
    CU busy) and the parts are folded per record by a block-parallel fold."""
    lens = np.array(lens, np.int64)
    offs = np.cumsum(np.concatenate([[3], lens[:-1] + 5])).astype(np.int64)
    data = rand_bytes(int(offs[-1] + lens[-1]) + 8, 2024)
    seeds = (np.arange(len(lens), dtype=np.uint32) * 0x9E3779B9).astype(np.uint32)
    out = u32(zd.crc_batch(to_dev(data, gpu), to_dev(offs, gpu), to_dev(lens, gpu),
                           to_dev(seeds.view(np.int32), gpu)))
    ref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), seeds, impl="hw", threads=8)
    assert np.array_equal(out, ref), (out, ref)


def test_raw_registers(gpu):
    data = rand_bytes(64 * 4096, 5)
    reg_in = 0x0BADF00D
    out = u32(zd.crc_fixed(to_dev(data, gpu), 4096, 4096, 64, seed=reg_in, raw=True))
    for i in range(64):
        want = (~oracle.crc32c_hw(~reg_in & M32, data[i * 4096:(i + 1) * 4096])) & M32
        assert out[i] == want


@pytest.mark.parametrize("length,offset", [
    (0, 0), (5, 3), (1000, 1), ((1 << 20) - 1, 0), (1 << 20, 0), ((3 << 20) + 7, 5),
    ((64 << 20) + 13, 2), (256 << 20, 0),
])
def test_span(gpu, length, offset):
    data = rand_bytes(length + offset + 16, length)
    out = u32(zd.crc_span(to_dev(data, gpu), seed=0xC0FFEE, length=length, offset=offset))
    assert out[0] == oracle.crc32c_hw(0xC0FFEE, data[offset:offset + length])


@pytest.mark.parametrize("per_wave", [16, 4, 0], ids=["dealt16", "dealt4", "static"])
def test_span_xteam_dealt(gpu, per_wave):
    """Spans on xteam_kernel (forced down to 16 KiB spans with a 4 KiB
    threshold): per_wave segments per wave dealt per workgroup by the LDS
    counter, or the static walk's two -- unaligned offsets, ragged last
    segments, seeds, and SEG_MIN-sized segments (more segments than the
    grid's waves x per_wave would give)."""
    old = lib().zscrc_set_xdeal(per_wave)
    lib().zscrc_set_xteam(1, 4096)
    try:
        for length, offset in [(16 << 10, 0), ((16 << 10) + 3, 1), ((1 << 20) - 1, 2), ((64 << 20) + 13, 2),
                               ((300 << 20) + 5, 1), (513 << 20, 0)]:
            data = rand_bytes(length + offset + 16, length + per_wave)
            out = u32(zd.crc_span(to_dev(data, gpu), seed=0xC0FFEE, length=length, offset=offset))
            assert out[0] == oracle.crc32c_hw(0xC0FFEE, data[offset:offset + length]), (length, offset)
    finally:
        lib().zscrc_set_xteam(1, 256 << 10)
        lib().zscrc_set_xdeal(old)


def test_span_3gib_dealt_vs_static(gpu):
    """A 3 GiB span at an odd offset (xteam_kernel by default: 64 Ki segments
    dealt per workgroup) against the threaded oracle (seed 0) and, seeded,
    against the static walk."""
    n = (3 << 30) + 12345
    g = torch.Generator(device=gpu)
    g.manual_seed(31)
    d = torch.randint(0, 256, (n + 3,), dtype=torch.uint8, device=gpu, generator=g)
    dealt0 = u32(zd.crc_span(d, length=n, offset=3))[0]
    dealt7 = u32(zd.crc_span(d, seed=7, length=n, offset=3))[0]
    old = lib().zscrc_set_xdeal(0)
    try:
        static7 = u32(zd.crc_span(d, seed=7, length=n, offset=3))[0]
    finally:
        lib().zscrc_set_xdeal(old)
    host = d[3:].cpu().numpy()
    del d
    assert dealt7 == static7
    assert dealt0 == oracle.span_crc(host, threads=min(16, os.cpu_count() or 1))


def test_span_equals_fold_of_records(gpu):
    # size-independent property at BASELINE config-3 record size: one span CRC
    # over N chunks == combine-chain of the N per-chunk CRCs
    n, L = 2048, 65536
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=gpu)
    per = u32(zd.crc_fixed(d, L, L, n))
    whole = u32(zd.crc_span(d))[0]
    acc = 0
    for c in per:
        acc = zc.crc32c_combine(acc, int(c), L)
    assert acc == whole
    # and a sample of chunks against the oracle
    host = d.cpu().numpy()
    for i in (0, 1, 777, n - 1):
        assert per[i] == oracle.crc32c_hw(0, host[i * L:(i + 1) * L])


def test_host_batch(gpu):
    import ctypes
    rng = np.random.default_rng(8)
    n = 500
    lens = rng.integers(0, 50000, n).astype(np.uint64)
    offs = np.cumsum(np.concatenate([[0], lens[:-1] + 3])).astype(np.uint64)
    data = rand_bytes(int(offs[-1] + lens[-1]) + 8, 1)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    rc = lib().zscrc_host_batch(data.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                seeds.ctypes.data, out.ctypes.data, n)
    assert rc == 0, lib().zscrc_last_error()
    assert np.array_equal(out, oracle.batch(data, offs, lens, seeds, impl="hw", threads=8))


def test_scalar_offload(gpu):
    saved = (lib().zscrc_gpu_min(0), lib().zscrc_gpu_min(1))
    before = stats()
    lib().zscrc_set_gpu_min(1 << 20)
    try:
        d = rand_bytes((5 << 20) + 3, 77)
        assert zc.crc32c_hw(0x42, d) == oracle.crc32c_hw(0x42, d)
        assert zc.crc32c(0, d[1:]) == oracle.crc32c_hw(0, d[1:])
        small = d[:37]
        assert zc.crc32c_hw(0, small) == oracle.crc32c_hw(0, small)
    finally:
        lib().zscrc_set_gpu_min_pair(*saved)
    after = stats()
    assert after[1] - before[1] == 2   # both large calls ran on the GPU
    assert after[0] - before[0] == 1   # the 37-byte call stayed on the CPU


def test_scalar_offload_cached_and_pieces(gpu):
    """The cached per-device offload stream (no allocation per call) over
    sizes that take one piece, several pieces and a ragged last piece, with
    seeds; each call on the GPU and equal to the oracle."""
    saved = (lib().zscrc_gpu_min(0), lib().zscrc_gpu_min(1))
    lib().zscrc_set_gpu_min(1)
    try:
        for n in (1, 4095, (4 << 20) + 17, (33 << 20) + 5, (97 << 20) + 1):
            d = rand_bytes(n, n)
            before = stats()
            assert zc.crc32c_hw(0xA5A5A5A5, d) == oracle.crc32c_hw(0xA5A5A5A5, d), n
            assert stats()[1] - before[1] == 1, n
    finally:
        lib().zscrc_set_gpu_min_pair(*saved)


@pytest.mark.parametrize("mode", ["team16", "xteam", "qteam-static", "qteam-qfold", "qteam"])
def test_config3_headline_dispatch(gpu, mode):
    """BASELINE config 3 at full size through the exact call bench.py times:
    zscrc_device_fixed on 65,536 x 64 KiB chunks (4 GiB), seed 0, flags 0 --
    by default the 16-lane team walk (team_kernel<16>) with xor_io = ~0; also
    the coalesced whole-wave teams (xteam_kernel) forced on -- every CRC
    against the oracle."""
    n, L = 65536, 65536
    g = torch.Generator(device=gpu)
    g.manual_seed(0x9E3779B9)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=gpu, generator=g)
    lib().zscrc_set_xteam(1, 32768 if mode == "xteam" else 256 << 10)
    lib().zscrc_set_qteam(1 if mode.startswith("qteam") else 0)
    lib().zscrc_set_opt(QSTATIC if mode == "qteam-static" else QFOLD if mode == "qteam-qfold" else 0)
    try:
        name = lib().zscrc_fixed_kernel(d.data_ptr(), L, L, n).decode()
        assert name == {"team16": "team_kernel<16>", "xteam": "xteam_kernel",
                        "qteam": "qteam_dyn_kernel", "qteam-qfold": "qteam_dyn_kernel+qfold_kernel",
                        "qteam-static": "qteam_kernel"}[mode]
        out = torch.empty(n, dtype=torch.int32, device=gpu)
        from zeroskip_amd._lib import check
        check(lib().zscrc_device_fixed(d.data_ptr(), L, L, 0, out.data_ptr(), n, 0,
                                       torch.cuda.current_stream(gpu).cuda_stream), "zscrc_device_fixed")
        got = u32(out)
        host = d.cpu().numpy()
        del d
    finally:
        lib().zscrc_set_xteam(1, 256 << 10)
        lib().zscrc_set_qteam(QTEAM_DEFAULT)
        lib().zscrc_set_opt(0)
    ref = oracle.batch(host, n=n, stride=L, fixed_len=L, impl="hw", threads=min(16, os.cpu_count() or 1))
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, bad[:10]


def test_xteam_shapes(gpu):
    """xteam_kernel (coalesced whole-wave teams) on ragged shapes: unaligned
    bases and strides, front-padded first steps at the buffer start, records
    shorter than one step, < 8-byte records, gaps between records, fewer
    records than waves -- forced on with a 1-byte threshold."""
    lib().zscrc_set_xteam(1, 1)
    lib().zscrc_set_teams(0, 1 << 20)   # no one-lane records: xteam down to 1 byte
    try:
        for stride, length, n, off in [(65536, 65536, 300, 0), (4096, 4096, 3000, 0), (100000, 99999, 300, 1),
                                       (5200, 5199, 700, 3), (8192, 4096, 1000, 2), (4097, 4097, 333, 3),
                                       (64, 64, 10000, 0), (320, 312, 5000, 1), (8, 8, 1000, 0),
                                       (5, 5, 100, 1), (12345, 12000, 7, 1)]:
            data = rand_bytes(stride * (n - 1) + length + off, stride + length + n)
            assert lib().zscrc_xteam_for(length, n) == 1
            out = u32(zd.crc_fixed(to_dev(data[off:], gpu), stride, length, n, seed=0xA5A5))
            ref = _oracle_seeded(data[off:], stride, length, n, 0xA5A5)
            bad = np.nonzero(out != ref)[0]
            assert bad.size == 0, (stride, length, n, off, bad[:10])
            raw = u32(zd.crc_fixed(to_dev(data[off:], gpu), stride, length, n, seed=0x1234, raw=True))
            want = (~oracle.crc32c_hw(~0x1234 & M32, data[off:off + length])) & M32
            assert raw[0] == want, (stride, length, "raw")
    finally:
        lib().zscrc_set_xteam(1, 256 << 10)
        lib().zscrc_set_teams(*DEFAULT_TEAMS)


QDEAL = 1 << 25    # zs::BatchDesc::opt: qteam records cut into parts dealt per workgroup, at any size
QSTATIC = 1 << 24  # qteam's static walk at any size
QFOLD = 32         # qteam_dyn's part fold as a second launch (qfold_kernel), not in LDS


@pytest.mark.parametrize("opt,P", [(0, "3"), (QDEAL, "3"), (QDEAL, "1"), (QDEAL | QFOLD, "3")],
                         ids=["static", "dealt-parts", "dealt-parts-P1", "dealt-parts-qfold"])
def test_qteam_shapes(gpu, opt, P, monkeypatch):
    """qteam_kernel (coalesced 16-lane column-quad teams) on ragged shapes of
    equal-length records: a partial last group of four, unaligned bases (the
    first record's front-padded step clamped at the buffer start), ragged
    tails, gaps between records, seeds and raw registers -- every CRC against
    the oracle; shapes it must not take (a different last length, stride
    not a multiple of 4) go to team_kernel<16>."""
    lib().zscrc_set_qteam(1)
    lib().zscrc_set_opt(opt)
    if opt:
        # parts of 3 KiB (1 KiB): ragged first parts, many per record; the
        # part registers fit LDS (the in-kernel fold) on some shapes, not on
        # others (qfold_kernel)
        monkeypatch.setenv("ZSCRC_QDYN_P", P)
    names = set()
    try:
        for stride, length, n, off in [(8192, 8192, 16385, 0), (8200, 8195, 16390, 1), (16384, 12000, 16387, 3),
                                       (65540, 65537, 16385, 2), (12288, 9000, 16400, 0), (2048, 2048, 16387, 0),
                                       (4100, 4097, 16390, 1), (3000, 2050, 16384, 2),
                                       (4096, 8192, 16384, 0), (0, 9000, 16386, 1)]:   # overlapping, stride 0
            data = rand_bytes(stride * (n - 1) + length + off, stride + length + n)
            dd = to_dev(data[off:], gpu)
            name = lib().zscrc_fixed_kernel(dd.data_ptr(), stride, length, n).decode()
            names.add(name)
            assert name == ("qteam_kernel" if not opt else "qteam_dyn_kernel+qfold_kernel" if opt & QFOLD
                            else name if name in ("qteam_dyn_kernel", "qteam_dyn_kernel+qfold_kernel") else None)
            out = u32(zd.crc_fixed(dd, stride, length, n, seed=0xA5A5))
            ref = _oracle_seeded(data[off:], stride, length, n, 0xA5A5)
            bad = np.nonzero(out != ref)[0]
            assert bad.size == 0, (stride, length, n, off, bad[:10])
            raw = u32(zd.crc_fixed(dd, stride, length, n, seed=0x1234, raw=True))
            want = (~oracle.crc32c_hw(~0x1234 & M32, data[off:off + length])) & M32
            assert raw[0] == want, (stride, length, "raw")
            del dd
        if opt == QDEAL and P == "1":
            assert names == {"qteam_dyn_kernel", "qteam_dyn_kernel+qfold_kernel"}, names
        d = torch.zeros(16, dtype=torch.uint8, device=gpu)
        assert lib().zscrc_fixed_kernel(d.data_ptr(), 8194, 8192, 16384).decode() == "team_kernel<16>"
    finally:
        lib().zscrc_set_qteam(QTEAM_DEFAULT)
        lib().zscrc_set_opt(0)


@pytest.mark.parametrize("qteam,opt", [(1, 4), (1, 8), (0, 16)], ids=["qteam-xor3-1", "qteam-xor3-2", "team16-xor3"])
def test_xor3_variants(gpu, qteam, opt):
    """The A/B variants of the 16-lane walks (zscrc_set_opt bits 4 / 8: qteam
    XOR3 groupings; 16: team_kernel<16>'s two-level walk with XOR3) on
    16,384 equal 8 KiB records and an unaligned ragged shape, every CRC
    against the oracle."""
    lib().zscrc_set_qteam(qteam)
    lib().zscrc_set_opt(opt)
    try:
        for stride, length, n, off in [(8192, 8192, 16384, 0), (12292, 12290, 16390, 3)]:
            data = rand_bytes(stride * (n - 1) + length + off, stride + n + opt)
            dd = to_dev(data[off:], gpu)
            name = lib().zscrc_fixed_kernel(dd.data_ptr(), stride, length, n).decode()
            assert name == ("qteam_kernel" if qteam else "team_kernel<16>")
            out = u32(zd.crc_fixed(dd, stride, length, n, seed=0x5A5A))
            ref = _oracle_seeded(data[off:], stride, length, n, 0x5A5A)
            bad = np.nonzero(out != ref)[0]
            assert bad.size == 0, (stride, length, n, off, bad[:10])
            del dd
    finally:
        lib().zscrc_set_opt(0)
        lib().zscrc_set_qteam(QTEAM_DEFAULT)


def test_config2_full_size_vs_oracle(gpu):
    # BASELINE config 2 at full size: 1,048,576 x 64 B records, every CRC checked
    n = 1 << 20
    d = torch.randint(0, 256, (n * 64,), dtype=torch.uint8, device=gpu)
    out = u32(zd.crc_fixed(d, 64, 64, n))
    ref = oracle.batch(d.cpu().numpy(), n=n, stride=64, fixed_len=64, impl="hw", threads=8)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("n,rl,stride", [(3 << 20, 64, 64), (2_500_000, 312, 320)])
def test_short_records_beyond_stash(gpu, n, rl, stride):
    """More records than the short kernel keeps in LDS (8 per thread): results
    stored per record; zeroskip-like 312/320 layout too."""
    d = torch.randint(0, 256, (stride * (n - 1) + rl + 40,), dtype=torch.uint8, device=gpu)
    out = u32(zd.crc_fixed(d[40:], stride, rl, n, seed=0xabc))
    ref = oracle.batch(d[40:].cpu().numpy(), n=n, stride=stride, fixed_len=rl, impl="hw", threads=8,
                       seeds=np.full(n, 0xabc, np.uint32))
    assert np.array_equal(out, ref)


def _sharded_worker(rank, world, port, total, q):
    import os
    import torch.distributed as dist
    from zeroskip_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = np.random.default_rng(321).integers(0, 256, total, dtype=np.uint8)
    lo, hi = shard.shard_ranges(total, world)[rank]
    local = torch.from_numpy(data[lo:hi].copy()).to("cuda:0")
    q.put((rank, shard.sharded_crc(local, seed=0x77)))   # GPU raw partials, gloo exchange
    dist.destroy_process_group()


def test_sharded_span_gpu_partials(gpu):
    # two ranks on the one GPU of this box (gloo for the digest exchange; the
    # 8-GPU run uses RCCL): per-rank libzscrc raw partials folded == oracle
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    total, world = (24 << 20) + 12345, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.crc32c_hw(0x77, np.random.default_rng(321).integers(0, 256, total, dtype=np.uint8))
    assert all(c == want for _, c in res)


def test_beyond_4gib(gpu):
    """64-bit offsets and lengths: a 4.5 GiB buffer -- the whole-buffer span,
    one record longer than 4 GiB (split plan), records straddling and past the
    4 GiB offset (one-lane and team kernels), bounded and unbounded."""
    total = (4 << 30) + (512 << 20) + 77
    g = torch.Generator(device=gpu)
    g.manual_seed(4242)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu, generator=g)
    h = d.cpu().numpy()
    four = 1 << 32
    rng = np.random.default_rng(3)
    offs = [0, four - 100, four - 3, four + 5, four + 1000, total - 5000, 7]
    lens = [four + 77, 300, 70, 64, 20000, 5000, 1 << 20]
    so = rng.integers(four, total - 700, 20000).astype(np.uint64)   # short records past 4 GiB
    offs = np.concatenate([np.array(offs, np.uint64), so])
    lens = np.concatenate([np.array(lens, np.uint64), rng.integers(0, 640, so.size).astype(np.uint64)])
    ref = oracle.batch(h, offs, lens, impl="hw", threads=8)
    d_off = to_dev(offs.astype(np.int64), gpu)
    d_len = to_dev(lens.astype(np.int64), gpu)
    assert np.array_equal(u32(zd.crc_batch(d, d_off, d_len)), ref)
    short = slice(7, None)
    assert np.array_equal(u32(zd.crc_batch(d, d_off[short], d_len[short], max_len=640)), ref[short])
    whole = oracle.batch(h, np.array([0], np.uint64), np.array([total], np.uint64), impl="hw", threads=1)[0]
    assert u32(zd.crc_span(d))[0] == whole
    # fixed stride with record i at i * 600 MiB: offsets past 4 GiB in the fixed path
    stride, ln = 600 << 20, 1 << 20
    n = (total - ln) // stride + 1
    ref_f = oracle.batch(h, n=n, stride=stride, fixed_len=ln, impl="hw", threads=8)
    assert np.array_equal(u32(zd.crc_fixed(d, stride, ln, n)), ref_f)


def test_two_streams_share_scratch(gpu):
    """Variable batches and spans enqueued alternately on two streams without
    host synchronisation: the device's shared class lists / part registers
    must be ordered across the streams (scratch_acquire/release)."""
    rng = np.random.default_rng(21)
    cases = []
    for k in range(2):
        n = 3000
        lens = rng.integers(0, 3000, n).astype(np.uint64)
        lens[:3] = [5 << 20, 3 << 20, 70000]                  # split classes too
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1])
        data = rand_bytes(int(offs[-1] + lens[-1]), 50 + k)
        cases.append((to_dev(data, gpu), to_dev(offs.astype(np.int64), gpu), to_dev(lens.astype(np.int64), gpu),
                      oracle.batch(data, offs, lens, impl="hw", threads=8),
                      oracle.batch(data, np.array([0], np.uint64), np.array([data.size], np.uint64),
                                   impl="hw")[0]))
    streams = [torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)]
    outs = []
    for rep in range(6):
        for k, st in enumerate(streams):
            d, o, ln, _, _ = cases[k]
            with torch.cuda.stream(st):
                outs.append((k, zd.crc_batch(d, o, ln), zd.crc_span(d)))
    torch.cuda.synchronize()
    for k, b, sp in outs:
        assert np.array_equal(b.cpu().numpy().view(np.uint32), cases[k][3])
        assert (sp.cpu().numpy().view(np.uint32)[0]) == cases[k][4]


@pytest.mark.parametrize("stride,length,n,k", [
    (64, 64, 1 << 20, 8),        # BASELINE config 2 records, 8 batches in one launch
    (64, 64, 1000, 64),          # ZSCRC_MULTI_MAX batches, fewer records than threads
    (48, 40, 30001, 5),          # front padding inside the piece, ragged count
    (13, 11, 20000, 3),          # unaligned starts, tail bytes
    (7, 5, 5000, 4),             # < 8 bytes: byte path
    (4096, 1000, 300, 3),        # > 64 bytes: one launch per batch
])
def test_fixed_multi(gpu, stride, length, n, k):
    """zscrc_device_fixed_multi (one persistent launch over k batches) equals
    the oracle on every record of every batch, plain and raw."""
    bufs, hosts = [], []
    for b in range(k):
        h = rand_bytes(stride * (n - 1) + length + b, 1000 * b + length)[b:]
        hosts.append(h)
        bufs.append(to_dev(h, gpu))
    before = stats()
    outs = zd.crc_fixed_multi(bufs, stride, length, n, seed=0x31337)
    if length <= 64:
        assert stats()[2] - before[2] == 1          # one launch for all k batches
    for b in range(k):
        assert np.array_equal(u32(outs[b]), _oracle_seeded(hosts[b], stride, length, n, 0x31337)), b
    raws = zd.crc_fixed_multi(bufs[:2], stride, length, n, seed=7, raw=True)
    for b in range(min(k, 2)):
        ref = oracle.batch(hosts[b], n=n, stride=stride, fixed_len=length, impl="hw",
                           seeds=np.full(n, ~7 & M32, np.uint32)) ^ np.uint32(M32)
        assert np.array_equal(u32(raws[b]), ref)


@pytest.mark.parametrize("shift,n", [(0, 4099), (16, 1000), (48, 128), (3, 777), (0, 1), (0, 1 << 20),
                                     (0, 128 * 4 * 37 + 129)])
def test_fixed_multi_64_offsets(gpu, shift, n):
    """64-byte record batches at base offsets: 16-byte aligned bases take the
    coalesced chunk kernel (multi64_kernel; ragged last chunks), others the
    per-lane piece walk -- both against the oracle."""
    k = 3
    big = to_dev(rand_bytes(k * (64 * n + 64) + 64, n + shift), gpu)
    bufs = [big[shift + b * (64 * n + 64):] for b in range(k)]
    hosts = [b.cpu().numpy() for b in bufs]
    for opt in (0, 2, 1 << 21, 1 << 23):   # multi64 (chunks dealt), the piece walk, multi64d, multi64's static walk
        lib().zscrc_set_opt(opt)
        try:
            outs = zd.crc_fixed_multi(bufs, 64, 64, n, seed=0xC0C0)
        finally:
            lib().zscrc_set_opt(0)
        for b in range(k):
            assert np.array_equal(u32(outs[b]), _oracle_seeded(hosts[b], 64, 64, n, 0xC0C0)), (opt, b)
