"""Deterministic test data shared by the golden-fixture generator and the tests.

xorshift64 (Marsaglia, shifts 13/7/17) seeded with 0x9E3779B97F4A7C15, as
SURVEY.md sec 8d / BASELINE.md specify for the synthetic inputs; each 64-bit
state is emitted as 8 little-endian bytes.
"""
import numpy as np

SEED = 0x9E3779B97F4A7C15
MASK = (1 << 64) - 1


def xorshift64_bytes(n: int, seed: int = SEED) -> np.ndarray:
    words = (n + 7) // 8
    out = np.empty(words, dtype=np.uint64)
    x = seed & MASK
    for i in range(words):
        x ^= (x << 13) & MASK
        x ^= x >> 7
        x ^= (x << 17) & MASK
        out[i] = x
    return out.view(np.uint8)[:n].copy()
