"""The CPU oracle against the reference's known answers and golden vectors."""
import json
import os

import numpy as np
import pytest

from oracle import oracle
from tests.golden.datagen import xorshift64_bytes

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "crc32c_golden.json")))


@pytest.mark.parametrize("kat", GOLDEN["kats"], ids=lambda k: k["name"])
def test_kats(kat):
    d = bytes.fromhex(kat["hex"])
    for f in (oracle.crc32c_hw, oracle.crc32c_sw, oracle.crc32c_bitwise):
        assert f(kat["seed"], d) == kat["crc"]
    assert oracle.crc32c_py(kat["seed"], d) == kat["crc"]


def test_reference_unit_test_chained():
    # tests/unit-crc32c.c:28-49: crc32c("lorem") then " ipsum" == crc32c("lorem ipsum")
    oracle.lib().oracle_crc32c_init()
    c1 = oracle.crc32c_hw(oracle.crc32c_hw(0, b"lorem"), b" ipsum")
    c2 = oracle.crc32c_sw(oracle.crc32c_sw(0, b"lorem"), b" ipsum")
    assert c1 == c2 == 0xDFB4E6C9


def test_golden_cases():
    data = xorshift64_bytes(GOLDEN["data"]["bytes"])
    for align, n, seed, crc in GOLDEN["cases"]:
        d = data[align:align + n]
        assert oracle.crc32c_hw(seed, d) == crc
        assert oracle.crc32c_sw(seed, d) == crc


def test_crc32bench_string():
    b = GOLDEN["crc32bench"]
    assert len(b["text"]) == 574
    assert oracle.crc32c_sw(0, b["text"].encode()) == b["crc"]


def test_hw_sw_agree_long_blocks():
    # exercises the 3x8192 and 3x256 interleave of crc32c.c:393-429 at odd alignments
    rng = np.random.default_rng(7)
    d = rng.integers(0, 256, 3 * 8192 * 3 + 4000, dtype=np.uint8)
    for align in range(8):
        for n in (3 * 8192 - 1, 3 * 8192, 3 * 8192 + 13, 2 * 3 * 8192 + 3 * 256 + 5):
            x = d[align:align + n]
            assert oracle.crc32c_hw(0x55, x) == oracle.crc32c_sw(0x55, x) == \
                oracle.crc32c_bitwise(0x55, x)


def test_combine_identity():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, 1000, dtype=np.uint8)
    b = rng.integers(0, 256, 777, dtype=np.uint8)
    ab = np.concatenate([a, b])
    assert oracle.combine(oracle.crc32c_hw(0, a), oracle.crc32c_hw(0, b), len(b)) == \
        oracle.crc32c_hw(0, ab)


def test_batch_threads_match():
    d = xorshift64_bytes(64 * 1024)
    ref = oracle.batch(d, n=1024, stride=64, fixed_len=64, impl="bitwise")
    for impl in ("hw", "sw"):
        for th in (1, 4):
            assert np.array_equal(oracle.batch(d, n=1024, stride=64, fixed_len=64, impl=impl,
                                               threads=th), ref)


def test_format_crcs_follow_writer():
    # short commit (zeroskip-file.c:303-328): crc32c(span_crc, LE64(type<<56|len<<32))
    span = b"k" * 40 + b"v" * 272
    sc = oracle.crc32c_hw(0, span)
    word = ((4 << 56) | (len(span) << 32)).to_bytes(8, "little")
    assert oracle.commit_crc(sc, len(span)) == oracle.crc32c_hw(sc, word)
    # long commit (zeroskip-file.c:266-302): type1, length, type2 words chained
    n = 16777216
    w1 = (36 << 56).to_bytes(8, "little")
    w2 = n.to_bytes(8, "little")
    w3 = (8 << 56).to_bytes(8, "little")
    assert oracle.commit_crc(sc, n) == oracle.crc32c_hw(oracle.crc32c_hw(oracle.crc32c_hw(sc, w1), w2), w3)


def test_batch_rate_byte_split_matches_per_record():
    """bench.py's all-core timing leg (oracle_batch_rate): records cut by the
    threads' byte ranges -- long spans, zero-length records at range bounds,
    seeds -- joined by the zero shift equal the per-record oracle."""
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 1 << 23, dtype=np.uint8)
    lens = np.array([0, 5, 1 << 21, 0, 0, 17, 3000, 1 << 20, 0, 64] + list(rng.integers(0, 5000, 300)),
                    dtype=np.uint64)
    offs = rng.integers(0, len(data) - (1 << 21) - 1, len(lens)).astype(np.uint64)
    seeds = rng.integers(0, 1 << 32, len(lens), dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(data, offs, lens, seeds, impl="hw")
    for t in (1, 2, 3, 7, 16, 33):
        got, el, passes = oracle.batch_rate(data, offs, lens, seeds, impl="hw", threads=t, budget=0.01,
                                            cpus=oracle.pick_cpus(t))
        assert passes >= 1 and el > 0
        assert np.array_equal(got, want), t
    got, _, _ = oracle.batch_rate(data, n=2000, stride=4096, fixed_len=4093, impl="sw", threads=5, budget=0.01)
    assert np.array_equal(got, oracle.batch(data, n=2000, stride=4096, fixed_len=4093, impl="sw"))
    # the caller's own CPU mask is left as it was
    import os
    before = os.sched_getaffinity(0)
    oracle.batch_rate(data, n=1, fixed_len=1 << 20, impl="read", threads=2, budget=0.01, cpus=oracle.pick_cpus(2))
    assert os.sched_getaffinity(0) == before


def test_bench_cpu_leg_small():
    import bench
    rng = np.random.default_rng(6)
    data = rng.integers(0, 256, 1 << 22, dtype=np.uint8)
    d = bench.cpu_leg(data, "test", n=64, stride=1 << 16, fixed_len=1 << 16, seconds=0.3, sw=True)
    assert d["kind"] == "port" and d["value"] > 0 and d["value_1core"] > 0 and d["host_read_GiBs"] > 0
    lens = np.array([1 << 21, 100, 0, 1 << 20], dtype=np.int64)
    offs = np.array([0, 5, 9, 1 << 21], dtype=np.int64)
    d = bench.cpu_leg(data, "spans", offs, lens, seconds=0.3)
    assert d["cores"] >= 1 and "sw_value_1core" not in d
