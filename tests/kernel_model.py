"""Pure-Python model of the team decomposition in zscrc_kernels.hip.

Mirrors team_register<G>() step by step (front-padded step grid, masked first
step carrying the initial register, fused "word then skip" operator, log-tree
fold, byte tail) using the same operator tables, so the decomposition can be
checked against the oracle on the CPU.  Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

POLY = 0x82F63B78
M32 = 0xFFFFFFFF


def gf2_mul(a: int, b: int) -> int:
    acc = 0
    while a:
        if a & 0x80000000:
            acc ^= b
        a = (a << 1) & M32
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return acc


def xpow8n(n: int) -> int:
    r, sq = 0x80000000, 0x00800000
    while n:
        if n & 1:
            r = gf2_mul(r, sq)
        sq = gf2_mul(sq, sq)
        n >>= 1
    return r


_tabs: dict[int, list[list[int]]] = {}


def shift_table(n: int):
    if n not in _tabs:
        m = xpow8n(n)
        _tabs[n] = [[gf2_mul(m, b << (8 * j)) for b in range(256)] for j in range(4)]
    return _tabs[n]


def op(n: int, x: int) -> int:
    t = shift_table(n)
    return t[0][x & 0xFF] ^ t[1][(x >> 8) & 0xFF] ^ t[2][(x >> 16) & 0xFF] ^ t[3][x >> 24]


def byte_step(r: int, b: int) -> int:
    return op(4, ((r ^ b) & 0xFF) << 24) ^ (r >> 8)


def team_register(mem: bytes, A: int, length: int, R0: int, G: int) -> int:
    """Register after [A, A+length) of `mem` from register R0, team of G lanes."""
    if length < 8:
        r = R0
        for i in range(length):
            r = byte_step(r, mem[A + i])
        return r
    STEP = G * 64
    E = (A + length) & ~3
    nb = E - A
    S = (nb + STEP - 1) // STEP
    V0 = E - S * STEP

    def word(q):
        return int.from_bytes(mem[q:q + 4], "little")

    accs = []
    for j in range(G):
        acc = 0
        for s in range(S):
            p = V0 + s * STEP + 64 * j
            w = []
            for k in range(16):
                q = p + 4 * k
                if s == 0 and V0 != A:
                    v = 0
                    if q + 4 > A:
                        v = word(q)
                        if q < A:
                            v &= (M32 << (8 * (A - q))) & M32
                    d = A - q
                    if 0 <= d < 4:
                        v ^= (R0 << (8 * d)) & M32
                    elif -4 < d < 0:
                        v ^= R0 >> (8 * -d)
                else:
                    v = word(q)
                    if s == 0 and j == 0 and k == 0:
                        v ^= R0
                    if s == 1 and j == 0 and k == 0 and A + 4 > V0 + STEP:
                        v ^= R0 >> (8 * (V0 + STEP - A))
                w.append(v)
            for k in range(15):
                acc = op(4, acc ^ w[k])
            skip = (G - 1) * 64 if (G != 1 and s + 1 < S) else 0
            acc = op(4 + skip, acc ^ w[15])
        accs.append(acc)
    k = 0
    while (1 << k) < G:
        sh = [op(64 << k, a) for a in accs]
        accs = [accs[j] ^ sh[j - (1 << k)] if j & (1 << k) else accs[j] for j in range(G)]
        k += 1
    acc = accs[G - 1]
    for i in range(A + length - E):
        acc = byte_step(acc, mem[E + i])
    return acc


def crc32c(mem: bytes, A: int, length: int, seed: int, G: int) -> int:
    return team_register(mem, A, length, seed ^ M32, G) ^ M32
