"""The kernel's work decomposition (tests/kernel_model.py mirrors
zscrc_kernels.hip team_register) reproduces the oracle on the CPU, for every
team size, alignment and length class: front-padded grids, the initial
register spilling across steps, ragged tails, < 8-byte records."""
import numpy as np
import pytest

from oracle import oracle
from tests import kernel_model as km
from tests.golden.datagen import xorshift64_bytes

DATA = xorshift64_bytes(9000)
MEM = bytes(256) + DATA.tobytes() + bytes(64)


@pytest.mark.parametrize("G", [1, 16, 64])
def test_model_matches_oracle(G):
    lens = list(range(0, 72)) + [127, 128, 129, 255, 256, 257, 1023, 1024, 1025, 1027, 4095,
                                 4097, 4099, 8192 + 64 * 3 + 1]
    for align in range(0, 16, 1 if G == 1 else 3):
        for n in lens:
            for seed in (0, 0xFFFFFFFF, 0x1234):
                want = oracle.crc32c_hw(seed, DATA[align:align + n])
                assert km.crc32c(MEM, 256 + align, n, seed, G) == want, (G, align, n, seed)


def test_operator_tables_are_slice_by_4():
    # shift(b<<8j, 4) is the reference's slice-by-4 table crc32c_lookup[3-j]
    # (src/crc32c.c:459-596, used as lookup[0][w>>24] ... lookup[3][w&0xff])
    t = oracle.slice4_tables()
    S4 = km.shift_table(4)
    for j in range(4):
        assert list(t[3 - j]) == S4[j]
