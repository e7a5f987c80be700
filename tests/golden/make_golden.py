"""Regenerate tests/golden/crc32c_golden.json.

Known answers come from the reference's own test (tests/unit-crc32c.c:36), the
CRC catalogue check value of CRC-32/ISCSI, and RFC 3720 appendix B.4.  The
seeded cases are computed by the CPU oracle (oracle/zs_oracle.c) and every one
of them is cross-checked against the oracle's slice-by-4, SSE4.2 and bit-wise
paths, and against an independent pure-Python bit-wise CRC for len <= 2048.

usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from datagen import SEED, xorshift64_bytes  # noqa: E402
from oracle import oracle  # noqa: E402

# benchmark/crc32bench.c:22 -- the string crc32bench hashes 65536 times
CRC32BENCH_STR = (
    "Lorem Ipsum is simply dummy text of the printing and typesetting industry. Lorem Ipsum "
    "has been the industry's standard dummy text ever since the 1500s, when an unknown printer "
    "took a galley of type and scrambled it to make a type specimen book. It has survived not "
    "only five centuries, but also the leap into electronic typesetting, remaining essentially "
    "unchanged. It was popularised in the 1960s with the release of Letraset sheets containing "
    "Lorem Ipsum passages, and more recently with desktop publishing software like Aldus "
    "PageMaker including versions of Lorem Ipsum.")


def kats():
    k = [
        ("reference unit test", "tests/unit-crc32c.c:36", b"lorem ipsum", 0, 0xDFB4E6C9),
        ("CRC-32/ISCSI check", "CRC catalogue", b"123456789", 0, 0xE3069283),
        ("32 zero bytes", "RFC 3720 B.4", bytes(32), 0, 0x8A9136AA),
        ("32 0xFF bytes", "RFC 3720 B.4", b"\xff" * 32, 0, 0x62A8AB43),
        ("32 incrementing", "RFC 3720 B.4", bytes(range(32)), 0, 0x46DD794E),
        ("32 decrementing", "RFC 3720 B.4", bytes(range(31, -1, -1)), 0, 0x113FDB5C),
        ("empty", "crc32c.c:691-694 crc32c(0,0,0)", b"", 0, 0),
    ]
    out = [dict(name=n, source=s, hex=d.hex(), seed=seed, crc=c) for n, s, d, seed, c in k]
    # chained form of the reference unit test (tests/unit-crc32c.c:37-43)
    out.append(dict(name="reference unit test, chained", source="tests/unit-crc32c.c:37-43",
                    hex=b" ipsum".hex(), seed=oracle.crc32c_hw(0, b"lorem"), crc=0xDFB4E6C9))
    return out


def main():
    data = xorshift64_bytes(70016)
    cases = []
    lens = list(range(0, 301)) + [511, 512, 513, 767, 768, 769, 1023, 1024, 1025, 2047, 2048,
                                   4095, 4096, 4097, 16383, 16384, 16385, 24575, 24576, 24577,
                                   65535, 65536, 65537, 69999]
    for n in lens:
        for seed in (0, 0x1234, 0xFFFFFFFF):
            cases.append((0, n, seed))
    for align in range(1, 16):
        for n in (1, 3, 4, 7, 8, 9, 15, 16, 17, 63, 64, 65, 255, 256, 257, 1000, 4097, 65536):
            cases.append((align, n, 0x1234))
    rows = []
    for align, n, seed in cases:
        d = data[align:align + n]
        c = oracle.crc32c_hw(seed, d)
        assert c == oracle.crc32c_sw(seed, d) == oracle.crc32c_bitwise(seed, d), (align, n)
        if n <= 2048:
            assert c == oracle.crc32c_py(seed, d.tobytes()), (align, n)
        rows.append([align, n, seed, c])
    for k in kats():
        d = bytes.fromhex(k["hex"])
        assert oracle.crc32c_hw(k["seed"], d) == k["crc"], k["name"]
        assert oracle.crc32c_py(k["seed"], d) == k["crc"], k["name"]
    bench = dict(source="benchmark/crc32bench.c:22", text=CRC32BENCH_STR,
                 len=len(CRC32BENCH_STR),
                 crc=oracle.crc32c_hw(0, CRC32BENCH_STR.encode()))
    assert bench["crc"] == oracle.crc32c_py(0, CRC32BENCH_STR.encode())
    doc = dict(
        description="CRC-32C golden vectors for zeroskip_amd parity tests",
        data=dict(generator="tests/golden/datagen.py xorshift64_bytes", seed=hex(SEED), bytes=70016),
        columns=["align", "len", "seed", "crc"], cases=rows, kats=kats(), crc32bench=bench)
    with open(os.path.join(HERE, "crc32c_golden.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print(f"{len(rows)} seeded cases, {len(doc['kats'])} KATs")


if __name__ == "__main__":
    main()
