"""libzscrc.so loads and exports every symbol include/zscrc.h declares; host-side
logic (GF(2) shift/combine, the scalar CPU path) matches the oracle.  No GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import oracle
from zeroskip_amd import LIB_PATH, lib
from zeroskip_amd import crc32c as zc
from zeroskip_amd._lib import SIGNATURES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zscrc.h")

REFERENCE_SYMBOLS = ["crc32c_init", "crc32c_sw", "crc32c_hw", "crc32c", "crc32c_map",
                     "crc32c_cstring", "crc32c_buf", "crc32c_iovec"]  # libzeroskip.symbols:113-120


def header_functions():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b([a-z_0-9]+)\s*\([^;{]*\)\s*;", txt)))


def test_header_declares_reference_api():
    fns = header_functions()
    for s in REFERENCE_SYMBOLS:
        assert s in fns


def test_every_declared_symbol_is_exported():
    L = ctypes.CDLL(LIB_PATH)
    fns = header_functions()
    assert len(fns) >= 18
    for name in fns:
        assert hasattr(L, name), name
        assert name in SIGNATURES, f"python binding lacks {name}"


def test_exports_are_dynamic_symbols():
    import subprocess
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB_PATH], text=True)
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for name in header_functions():
        assert name in syms, name


def test_gf2_shift_and_combine_match_oracle():
    rng = np.random.default_rng(11)
    for _ in range(200):
        reg = int(rng.integers(0, 2**32))
        n = int(rng.integers(0, 2**40))
        assert lib().zscrc_shift(reg, n) == oracle.shift(reg, n)
    a, b = rng.integers(0, 256, 333, dtype=np.uint8), rng.integers(0, 256, 4097, dtype=np.uint8)
    assert zc.crc32c_combine(oracle.crc32c_hw(7, a), oracle.crc32c_hw(0, b), len(b)) == \
        oracle.crc32c_hw(7, np.concatenate([a, b]))


@pytest.mark.parametrize("fn", ["crc32c_hw", "crc32c_sw", "crc32c"])
def test_scalar_cpu_path_matches_oracle(fn):
    # host-side scalar path (no offload configured): the drop-in for <=37-byte fields
    f = getattr(zc, fn)
    rng = np.random.default_rng(5)
    d = rng.integers(0, 256, 3 * 4096 * 3 + 999, dtype=np.uint8)
    for align in range(8):
        for n in (0, 1, 5, 8, 37, 57, 511, 1536, 1537, 3 * 4096, 3 * 4096 * 3 + 5):
            x = d[align:align + n]
            assert f(0xABCD, x) == oracle.crc32c_hw(0xABCD, x)


def test_scalar_wrappers_reference_semantics():
    assert zc.crc32c_hw(zc.crc32c_hw(0, b"lorem"), b" ipsum") == 0xDFB4E6C9
    assert zc.crc32c_map(b"lorem ipsum") == 0xDFB4E6C9
    assert zc.crc32c_buf(b"lorem ipsum") == 0xDFB4E6C9
    assert zc.crc32c_cstring(b"lorem ipsum") == 0xDFB4E6C9
    assert zc.crc32c_iovec([b"lo", b"", b"rem ", b"ipsum"]) == 0xDFB4E6C9
    assert zc.crc32c_iovec([]) == 0
    assert zc.crc32c(0, b"") == 0


def test_scalar_cpu_path_random():
    """The host path (SSE4.2 3-stream / slice-by-8) on random lengths,
    alignments and seeds, chained in random pieces; crc32c_combine over
    random splits -- each equal to the oracle."""
    rng = np.random.default_rng(23)
    d = rng.integers(0, 256, 300_000, dtype=np.uint8)
    for _ in range(300):
        n = int(rng.integers(0, 120_000))
        a = int(rng.integers(0, d.size - n + 1))
        seed = int(rng.integers(0, 2**32))
        x = d[a:a + n]
        want = oracle.crc32c_hw(seed, x)
        fn = (zc.crc32c_hw, zc.crc32c_sw, zc.crc32c)[int(rng.integers(0, 3))]
        assert fn(seed, x) == want, (fn.__name__, n, a)
        cut = int(rng.integers(0, n + 1))
        assert zc.crc32c_hw(zc.crc32c_hw(seed, x[:cut]), x[cut:]) == want
        assert zc.crc32c_combine(oracle.crc32c_hw(seed, x[:cut]), oracle.crc32c_hw(0, x[cut:]), n - cut) == want
