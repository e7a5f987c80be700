"""Mutations of zeroskip file images for the parser / verifier fuzz tests
(tests/test_parse_fuzz.py, tests/test_gpu_fuzz.py): the same kinds as
tests/c/parse_fuzz.c -- truncation, trailing bytes, bit flips, an 8-byte
word (record headers, lengths, offsets) set to an extreme value."""
import struct

EXTREME = [0, (1 << 64) - 1, (1 << 63) - 1, 0x01FFFFFFFFFFFFFF, 0x04FFFFFFFFFFFFFF, 0x20FFFFFF00000000,
           0x40FFFF0000000000, 0x0100FFFFFFFFFFFF]


def mutate(rng, image: bytes) -> bytes:
    b = bytearray(image)
    how = rng.randrange(6)
    if how == 0:
        b = b[:rng.randrange(len(b))]
    elif how == 1:
        b += bytes(rng.randrange(256) for _ in range(rng.randrange(64)))
    for _ in range(rng.randrange(8)):
        if b:
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
    if how >= 2 and len(b) >= 8:
        at = rng.randrange(len(b) // 8) * 8
        b[at:at + 8] = struct.pack(">Q", EXTREME[rng.randrange(len(EXTREME))] ^ rng.randrange(256))
    return bytes(b)


def oracle_walk(image: bytes):
    """The format oracle's walk, or None where it cannot read the mutated
    image (an access past its end)."""
    from oracle import zs_format as zf
    try:
        return zf.walk(image)
    except (struct.error, IndexError, ValueError):
        return None
