"""Randomised parity soak of the device batch entry points against the CPU
oracle (oracle/zs_oracle.c), on shapes the structured tests do not build:
records in random order, overlapping and duplicated, lengths straddling
every dispatch boundary (the one-lane / 2-lane / 16-lane / wavefront /
split-record classes and the 8-byte serial path), the last record ending
at the buffer's last byte, random seeds, raw registers, correct / loose /
wrong length bounds, and the fixed-stride and multi-batch forms at random
strides and base offsets, and single / multi-span calls at random
lengths, offsets and seeds.  Every CRC is compared, bit for bit."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from zeroskip_amd import device as zd
from zeroskip_amd._lib import DEFAULT_TEAMS

pytestmark = pytest.mark.gpu

M32 = np.uint32(0xFFFFFFFF)
EDGES = [0, 1, 7, 8, 9, 15, 16, 63, 64, 65, 127, 128, 129, 639, 640, 641, 1023, 1024, 1025, 4095, 4096,
         16383, 16384, 65535, 65536, 65537, (1 << 20) - 1, 1 << 20, (1 << 20) + 1]


def _lengths(rng, n, kind):
    if kind == "edges":
        return rng.choice(np.array(EDGES, np.int64), n)
    if kind == "short":
        return rng.integers(0, 700, n).astype(np.int64)
    if kind == "loguniform":
        return np.exp(rng.uniform(0, np.log(3 << 20), n)).astype(np.int64)
    # mixed: mostly short, a few long
    lens = rng.integers(0, 400, n).astype(np.int64)
    k = max(1, n // 200)
    lens[rng.integers(0, n, k)] = rng.integers(1 << 16, 5 << 20, k)
    return lens


def _case(seed):
    rng = np.random.default_rng(seed)
    kind = ["edges", "short", "loguniform", "mixed"][seed % 4]
    n = int(rng.integers(1, [6000, 60000, 600, 20000][seed % 4]))
    lens = _lengths(rng, n, kind)
    size = int(max(int(lens.max()) + 1, lens.sum() // 2 + 4096))
    offs = (rng.integers(0, 1 << 62, n) % (size - lens + 1)).astype(np.int64)  # overlapping, any order
    if n > 4:
        dup = rng.integers(0, n, n // 5)
        offs[dup[1:]], lens[dup[1:]] = offs[dup[0]], lens[dup[0]]             # duplicates
    j = int(rng.integers(0, n))
    offs[j] = size - lens[j]                                                  # ends at the last byte
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    return rng, data, offs, lens, seeds


def _dev(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


# env ZSCRC_SOAK_SEEDS: batches per block (default 25; longer soaks on request);
# ZSCRC_SOAK_BASE: first seed of every randomised test here and in
# test_gpu_consistent.py (default 0; another base explores new cases)
SEEDS = int(os.environ.get("ZSCRC_SOAK_SEEDS", "25"))
BASE = int(os.environ.get("ZSCRC_SOAK_BASE", "0"))


@pytest.mark.parametrize("block", range(4))
def test_random_batches(gpu, block):
    for seed in range(BASE + SEEDS * block, BASE + SEEDS * block + SEEDS):
        rng, data, offs, lens, seeds = _case(seed)
        ref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), seeds, impl="hw", threads=8)
        d, o, l = _dev(data, gpu), _dev(offs, gpu), _dev(lens, gpu)
        s = _dev(seeds.view(np.int32), gpu)
        bound = [None, int(lens.max()), int(lens.max()) * 2 + 1, max(1, int(lens.max()) // 2)][seed % 4]
        out = _u32(zd.crc_batch(d, o, l, s, max_len=bound))
        bad = np.nonzero(out != ref)[0]
        assert bad.size == 0, (seed, [(int(i), int(offs[i]), int(lens[i])) for i in bad[:5]])
        # raw registers: raw(s) = ~crc32c(~s)
        raw = _u32(zd.crc_batch(d, o, l, s, raw=True))
        rref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), seeds ^ M32, impl="hw",
                            threads=8) ^ M32
        assert np.array_equal(raw, rref), seed


@pytest.mark.parametrize("teams", [(0, 0), (1 << 40, 1 << 40), (0, 1 << 40)], ids=["g64", "g1", "g16"])
def test_random_batches_forced_teams(gpu, teams):
    from zeroskip_amd._lib import lib
    lib().zscrc_set_teams(*teams)
    try:
        for seed in (101, 102, 103, 104):
            _, data, offs, lens, seeds = _case(seed)
            lens = np.minimum(lens, 1 << 18)
            offs = np.minimum(offs, data.size - lens)
            ref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), seeds, impl="hw", threads=8)
            out = _u32(zd.crc_batch(_dev(data, gpu), _dev(offs, gpu), _dev(lens, gpu),
                                    _dev(seeds.view(np.int32), gpu)))
            assert np.array_equal(out, ref), (teams, seed)
    finally:
        lib().zscrc_set_teams(*DEFAULT_TEAMS)


def test_random_fixed_and_multi(gpu):
    rng = np.random.default_rng(7)
    for it in range(24):
        length = int(rng.choice([1, 5, 8, 31, 63, 64, 65, 129, 312, 640, 641, 4000, 65536]))
        stride = length + int(rng.choice([0, 0, 1, 8, 13, 64]))
        n = int(rng.integers(1, max(2, min(200000, (48 << 20) // stride))))
        shift = int(rng.integers(0, 64))
        seed = int(rng.integers(0, 1 << 32))
        data = rng.integers(0, 256, shift + stride * (n - 1) + length, dtype=np.uint8)
        offs = (np.arange(n, dtype=np.uint64) * stride + shift)
        lens = np.full(n, length, np.uint64)
        ref = oracle.batch(data, offs, lens, np.full(n, seed, np.uint32), impl="hw", threads=8)
        d = _dev(data, gpu)
        out = _u32(zd.crc_fixed(d[shift:], stride, length, n, seed=seed))
        assert np.array_equal(out, ref), (it, stride, length, n, shift)
        if length <= 64 and it % 2 == 0:
            k = int(rng.integers(1, 5))
            bufs = [d[shift:]] + [_dev(rng.integers(0, 256, data.size - shift, dtype=np.uint8), gpu)
                                  for _ in range(k - 1)]
            outs = zd.crc_fixed_multi(bufs, stride, length, n, seed=seed)
            for b, (buf, o) in enumerate(zip(bufs, outs)):
                h = buf.cpu().numpy()
                r = oracle.batch(h, offs - np.uint64(shift), lens, np.full(n, seed, np.uint32), impl="hw",
                                 threads=8)
                assert np.array_equal(_u32(o), r), (it, b, stride, length, n, shift)


def test_random_spans(gpu):
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, 96 << 20, dtype=np.uint8)
    d = _dev(data, gpu)
    for it in range(16):
        length = int(np.exp(rng.uniform(np.log(1), np.log(90 << 20))))
        off = int(rng.integers(0, data.size - length + 1))
        seed = int(rng.integers(0, 1 << 32))
        ref = oracle.batch(data, np.array([off], np.uint64), np.array([length], np.uint64),
                           np.array([seed], np.uint32), impl="hw", threads=8)
        got = _u32(zd.crc_span(d, seed=seed, length=length, offset=off))
        assert got[0] == ref[0], (it, off, length)
        k = int(rng.integers(1, 9))
        lens = np.exp(rng.uniform(np.log(16 << 10), np.log(24 << 20), k)).astype(np.int64)
        offs = (rng.integers(0, 1 << 62, k) % (data.size - lens + 1)).astype(np.int64)
        seeds = rng.integers(0, 1 << 32, k, dtype=np.uint64).astype(np.uint32)
        ref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), seeds, impl="hw", threads=8)
        got = _u32(zd.crc_spans(d, offs.tolist(), lens.tolist(), seeds.tolist()))
        assert np.array_equal(got, ref), (it, k)


# ---------------------------------------------------------------- wrong bounds
G1, G16 = 640, 1 << 20


def test_wrong_bounds_batches(gpu):
    """zscrc_device_batch_bounded: a bound below some lengths never changes a
    result (the header's contract) -- at or below the one-lane bound (one
    kernel over the caller's arrays) and between the classes (every class
    still launched).  Includes the soak case that found the class pruning:
    one 2 MiB record beside 466 short ones, bound 1 MiB."""
    cases = [_case(339)]
    rng = np.random.default_rng(17)
    n = 3000
    lens = rng.choice(np.array([0, 5, 64, 300, 640, 641, 5000, 8191, 8192, 70000, G16, G16 + 1, 3 << 20], np.int64), n)
    size = int(lens.sum() // 3 + (4 << 20))
    offs = (rng.integers(0, 1 << 62, n) % (size - lens + 1)).astype(np.int64)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    cases.append((rng, rng.integers(0, 256, size, dtype=np.uint8), offs, lens, seeds))
    for _, data, offs, lens, seeds in cases:
        ref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), seeds, impl="hw", threads=8)
        d, o, l = _dev(data, gpu), _dev(offs, gpu), _dev(lens, gpu)
        s = _dev(seeds.view(np.int32), gpu)
        for bound in (1, 300, G1, G1 + 1, 5000, 8192, 9000, G16 // 2, G16, G16 + 1):
            out = _u32(zd.crc_batch(d, o, l, s, max_len=bound))
            bad = np.nonzero(out != ref)[0]
            assert bad.size == 0, (bound, [(int(i), int(lens[i])) for i in bad[:5]])


def test_wrong_bounds_commits(gpu):
    """The commit entry points with a bound below some span lengths (the
    _bounded / verdict contract: results never depend on it): per-commit
    arrays, the verdict (a corruption in a long span still found), the
    writer's CRC array and the in-place writer, each equal to the unbounded
    call's; spans of 0-640 bytes with some of 5,000 / 100,000 / 2.1 M."""
    from zeroskip_amd import zsfile
    rng = np.random.default_rng(23)
    n = 20000
    lens = rng.integers(0, G1 + 1, n)
    lens[rng.integers(0, n, 40)] = rng.choice([5000, 100000, 2_100_000], 40)
    offs = np.zeros(n, np.int64)
    offs[0] = 43
    offs[1:] = 43 + np.cumsum(lens + 8 + rng.integers(0, 8, n))[:-1]
    size = int(offs[-1] + lens[-1] + 8 + 64)
    host = rng.integers(0, 256, size, dtype=np.uint8)
    host[offs + lens] = 4                                   # COMMIT records
    oracle.write_commits(host, offs.astype(np.uint64), lens.astype(np.uint64), threads=8)
    img = _dev(host, gpu)
    o, ln = _dev(offs, gpu), _dev(lens.astype(np.int64), gpu)
    crc0, st0 = zsfile.verify_commits(img, o, ln)
    assert bool((st0 == 1).all())
    long_i = int(np.nonzero(lens == lens.max())[0][0])
    bad_img = img.clone()
    bad_img[int(offs[long_i]) + 12345] ^= 1
    fields = (o + ln + 4).view(-1, 1) + torch.arange(4, device=o.device).view(1, -1)
    for bound in (300, G1, 1000, 50000, G16):
        crc, st = zsfile.verify_commits(img, o, ln, max_len=bound)
        assert torch.equal(crc, crc0) and torch.equal(st, st0), bound
        nbad, _ = zsfile.verify_commits_verdict(img, o, ln, max_len=bound)
        assert int(nbad.item()) == 0, bound
        nbad, badi = zsfile.verify_commits_verdict(bad_img, o, ln, max_len=bound)
        assert int(nbad.item()) == 1 and int(badi[0].item()) == long_i, bound
        assert torch.equal(zsfile.commit_crcs(img, o, ln, max_len=bound), crc0), bound
        z = img.clone()
        z[fields.view(-1)] = 0
        zsfile.write_commits(z, o, ln, max_len=bound, crc=False)
        assert torch.equal(z, img), bound


# ------------------------------------------------------------ random commits
T_KEY, T_COMMIT, T_FINAL = 1, 4, 16


def _commit_case(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([37, 2000, 30000, 250_000]))
    kind = seed % 3
    if kind == 0:                                   # 0-640 uniform, edges weighted
        lens = rng.integers(0, G1 + 1, n)
        lens[rng.random(n) < 0.05] = rng.integers(0, 9)
    elif kind == 1:                                 # zsbench-like: mostly 312, some others
        lens = np.full(n, 312)
        odd = rng.random(n) < 0.03
        lens[odd] = rng.integers(0, 2000, int(odd.sum()))
    else:                                           # short with long ones among them
        lens = rng.integers(0, 400, n)
        k = max(1, n // 500)
        lens[rng.integers(0, n, k)] = rng.choice([641, 5000, 70000, 1_100_000, 2_500_000], k)
    lens = lens.astype(np.int64)
    gaps = rng.integers(0, 8, n) * int(rng.integers(0, 2))       # back to back, or gaps
    offs = np.zeros(n, np.int64)
    offs[0] = 40 + int(rng.integers(0, 8))
    offs[1:] = offs[0] + np.cumsum(lens + 8 + gaps)[:-1]
    size = int(offs[-1] + lens[-1] + 8 + 64)
    host = rng.integers(0, 256, size, dtype=np.uint8)
    u = rng.random(n)
    has_rec = u >= 0.03
    final = has_rec & (u < 0.08)
    at = offs + lens
    host[at[~has_rec]] = T_KEY
    host[at[has_rec & ~final]] = T_COMMIT
    host[at[final]] = T_FINAL
    oracle.write_commits(host, offs[has_rec].astype(np.uint64), lens[has_rec].astype(np.uint64), threads=8)
    clean = host.copy()
    rec = np.nonzero(has_rec)[0]
    hit = rng.choice(rec, min(rec.size, 1 + n // 2000), replace=False)
    for j, i in enumerate(hit):
        o, ln = int(offs[i]), int(lens[i])
        if ln and j % 2 == 0:
            host[o + int(rng.integers(0, ln))] ^= 0x40
        else:
            host[o + ln + 4 + j % 4] ^= 0x02
    bound = [None, int(lens.max()), max(1, int(lens.max()) // 3), 300][seed % 4]
    # verification seeds (the chained finalise commit): a few record spans
    # verified from a nonzero seed, expected CRC recomputed from it
    sd = np.zeros(n, np.uint32)
    pick = has_rec & (rng.random(n) < 0.05)
    sd[pick] = rng.integers(1, 1 << 32, int(pick.sum()), dtype=np.uint64).astype(np.uint32)
    return host, clean, offs, lens, has_rec, hit, bound, sd


@pytest.mark.parametrize("seed", range(BASE, BASE + int(os.environ.get("ZSCRC_SOAK_COMMITS", "12"))))
def test_random_commit_batches(gpu, seed):
    """Random commit images -- lengths short / zsbench-like / with long spans,
    back to back or with gaps, 3 % without a commit record, FINAL records,
    a few corruptions in spans and stored CRCs, batches below and above the
    run-only split, bounds none / exact / wrong -- through the per-commit
    arrays, the verdict, the writer's CRC array and the in-place writer,
    each against the oracle's writer (src/zeroskip-file.c:253-350)."""
    from zeroskip_amd import zsfile
    host, clean, offs, lens, has_rec, hit, bound, sd = _commit_case(seed)
    n = offs.size
    img, o, ln = _dev(host, gpu), _dev(offs, gpu), _dev(lens, gpu)
    want = oracle.commit_crcs(host, offs[has_rec].astype(np.uint64), lens[has_rec].astype(np.uint64), threads=8)
    crc, st = zsfile.verify_commits(img, o, ln, max_len=bound)
    crc, st = crc.cpu().numpy().view(np.uint32), st.cpu().numpy()
    assert np.array_equal(crc[has_rec], want), seed
    want_st = np.where(has_rec, 1, 2)
    want_st[hit] = 0
    assert np.array_equal(st, want_st), (seed, np.nonzero(st != want_st)[0][:5])
    bad = set(np.nonzero(want_st != 1)[0].tolist())
    nbad, badi = zsfile.verify_commits_verdict(img, o, ln, max_len=bound, cap=max(4096, len(bad)))
    k = int(nbad.item())
    assert k == len(bad) and set(badi[:k].cpu().tolist()) == bad, seed
    # seeded: span i's CRC continues from sd[i] (0 = from scratch)
    seeded = np.nonzero(sd)[0]
    if seeded.size:
        crc_s, st_s = zsfile.verify_commits(img, o, ln, seed=_dev(sd.view(np.int32), gpu), max_len=bound)
        crc_s = crc_s.cpu().numpy().view(np.uint32)
        for i in seeded[:200]:
            oi, li = int(offs[i]), int(lens[i])
            fin = host[oi + li] == T_FINAL
            w = oracle.commit_crc(oracle.crc32c_hw(int(sd[i]), host[oi:oi + li]), li, bool(fin))
            assert crc_s[i] == w, (seed, int(i))
        rest = np.nonzero(has_rec & (sd == 0))[0]
        assert np.array_equal(crc_s[rest], crc[rest]), seed
    # the writer on the clean image: its CRC array, then in place over zeroed fields
    sel = np.nonzero(has_rec)[0]
    os_, ls_ = _dev(offs[sel], gpu), _dev(lens[sel], gpu)
    cimg = _dev(clean, gpu)
    wc = oracle.commit_crcs(clean, offs[sel].astype(np.uint64), lens[sel].astype(np.uint64), threads=8)
    assert np.array_equal(_u32(zsfile.commit_crcs(cimg, os_, ls_, max_len=bound)), wc), seed
    fields = (os_ + ls_ + 4).view(-1, 1) + torch.arange(4, device=os_.device).view(1, -1)
    z = cimg.clone()
    z[fields.view(-1)] = 0
    zsfile.write_commits(z, os_, ls_, max_len=bound, crc=False)
    assert torch.equal(z, cimg), seed


# ------------------------------------------------- host-memory entry points
def test_random_streams(gpu):
    """zscrc_stream_*: random totals cut into random updates (empty, 1 byte,
    unaligned, larger than a chunk), random chunk sizes and seeds, copied or
    NOCOPY -- the final CRC equals the oracle's over the concatenation."""
    from zeroskip_amd.stream import CrcStream
    rng = np.random.default_rng(31)
    pool = rng.integers(0, 256, 96 << 20, dtype=np.uint8)
    for it in range(24):
        total = int(np.exp(rng.uniform(0, np.log(90 << 20))))
        start = int(rng.integers(0, pool.size - total + 1))
        buf = pool[start:start + total]
        cuts = np.sort(rng.integers(0, total + 1, int(rng.integers(0, 40))))
        cuts = np.concatenate([[0], cuts, [total]])
        seed = int(rng.integers(0, 1 << 32))
        chunk = int(rng.choice([0, 4096, 1 << 20, 3 << 20, 64 << 20]))
        nocopy = bool(it % 3 == 0)
        s = CrcStream(seed=seed, chunk_bytes=chunk, nocopy=nocopy)
        for a, b in zip(cuts[:-1], cuts[1:]):
            s.update(buf[a:b])
        want = oracle.batch(buf, np.array([0], np.uint64), np.array([total], np.uint64),
                            np.array([seed], np.uint32), impl="hw")[0]
        assert s.final() == want, (it, total, chunk, nocopy, len(cuts))


def test_random_dropin_offload(gpu):
    """The drop-in symbols with the offload threshold lowered to 4 KiB, so
    random lengths around it and far above it go to the GPU: crc32c_hw /
    crc32c / crc32c_iovec chained from random seeds at random alignments
    equal the oracle's; the counters show the GPU ran."""
    from zeroskip_amd import crc32c as zc
    from zeroskip_amd._lib import lib, stats
    rng = np.random.default_rng(37)
    pool = rng.integers(0, 256, 40 << 20, dtype=np.uint8)
    warm, cold = lib().zscrc_gpu_min(0), lib().zscrc_gpu_min(1)
    lib().zscrc_set_gpu_min(4096)
    try:
        before = stats()[1]
        for it in range(40):
            n = int(rng.choice([4095, 4096, 4097, 65537, int(rng.integers(0, 40 << 20))]))
            a = int(rng.integers(0, pool.size - n + 1))
            seed = int(rng.integers(0, 1 << 32))
            want = oracle.batch(pool[a:a + n], np.array([0], np.uint64), np.array([n], np.uint64),
                                np.array([seed], np.uint32), impl="hw")[0]
            assert zc.crc32c_hw(seed, pool[a:a + n]) == want, (it, n, a)
            assert zc.crc32c(seed, pool[a:a + n]) == want, (it, n, a)
            k = int(rng.integers(1, 6))
            cuts = np.sort(rng.integers(0, n + 1, k - 1))
            parts = [pool[a + x:a + y] for x, y in zip(np.concatenate([[0], cuts]), np.concatenate([cuts, [n]]))]
            want0 = oracle.batch(pool[a:a + n], np.array([0], np.uint64), np.array([n], np.uint64),
                                 np.array([0], np.uint32), impl="hw")[0]
            assert zc.crc32c_iovec(parts) == want0, (it, n, k)
        assert stats()[1] > before
    finally:
        lib().zscrc_set_gpu_min_pair(warm, cold)


def test_random_host_batches(gpu):
    """zscrc_host_batch (host arrays in, results back): random records in
    any order over a host buffer equal the oracle's."""
    from zeroskip_amd._lib import lib
    import ctypes
    for seed in (3, 7, 11, 19):
        _, data, offs, lens, seeds = _case(seed)
        o = np.ascontiguousarray(offs.astype(np.uint64))
        l = np.ascontiguousarray(lens.astype(np.uint64))
        out = np.zeros(o.size, np.uint32)
        rc = lib().zscrc_host_batch(data.ctypes.data, o.ctypes.data, l.ctypes.data, seeds.ctypes.data,
                                    out.ctypes.data, o.size)
        assert rc == 0
        ref = oracle.batch(data, o, l, seeds, impl="hw", threads=8)
        assert np.array_equal(out, ref), seed


def test_random_spans_any_shape(gpu):
    """zscrc_device_spans past its one-launch shape (more than 8 spans, spans
    under 16 KiB, empty ones: one span call each) and zscrc_device_span at 0
    and tiny lengths, seeds and raw registers -- every result the oracle's."""
    rng = np.random.default_rng(41)
    data = rng.integers(0, 256, 24 << 20, dtype=np.uint8)
    d = _dev(data, gpu)
    for it in range(20):
        k = int(rng.integers(1, 13))
        lens = np.where(rng.random(k) < 0.5, rng.integers(0, 16 << 10, k), rng.integers(16 << 10, 6 << 20, k))
        offs = (rng.integers(0, 1 << 62, k) % (data.size - lens + 1)).astype(np.int64)
        seeds = rng.integers(0, 1 << 32, k, dtype=np.uint64).astype(np.uint32)
        raw = bool(it % 2)
        got = _u32(zd.crc_spans(d, offs.tolist(), lens.tolist(), seeds.tolist(), raw=raw))
        s = seeds ^ M32 if raw else seeds
        ref = oracle.batch(data, offs.astype(np.uint64), lens.astype(np.uint64), s, impl="hw", threads=8)
        assert np.array_equal(got, ref ^ M32 if raw else ref), (it, k, lens.tolist())
    for n in (0, 1, 3, 7, 8, 9, 63, 64, 65, 1023):
        off = int(rng.integers(0, 4096))
        seed = int(rng.integers(0, 1 << 32))
        got = _u32(zd.crc_span(d, seed=seed, length=n, offset=off))[0]
        ref = oracle.batch(data, np.array([off], np.uint64), np.array([n], np.uint64), np.array([seed], np.uint32),
                           impl="hw")[0]
        assert got == ref, (n, off)


@pytest.mark.parametrize("seed", range(8))
def test_random_fill(gpu, seed):
    """zscrc_zs_fill_commits (the writer for host images) on the random
    commit images with their CRC fields blanked, at random chunk sizes (spans
    straddling chunk ends, spans longer than a chunk streamed apart), staging
    threads and bounds: the image comes back byte for byte as the oracle's
    writer left it; spans without a commit record untouched and counted."""
    from zeroskip_amd import zsfile
    _, clean, offs, lens, has_rec, _, bound, _ = _commit_case(seed)
    rng = np.random.default_rng(77 + seed)
    blank = clean.copy()
    rec = np.nonzero(has_rec)[0]
    blank[(offs[rec] + lens[rec] + 4)[:, None] + np.arange(4)] = 0
    chunk = [64 << 10, 1 << 20, 3 << 20, 0][seed % 4]
    old = os.environ.get("ZSCRC_FILL_CHUNK")
    if chunk:
        os.environ["ZSCRC_FILL_CHUNK"] = str(chunk)
    try:
        rep = zsfile.fill_commits(blank, offs.astype(np.uint64), lens.astype(np.uint64), max_len=bound,
                                  threads=int(rng.integers(0, 5)))
    finally:
        if old is None:
            os.environ.pop("ZSCRC_FILL_CHUNK", None)
        else:
            os.environ["ZSCRC_FILL_CHUNK"] = old
    assert rep["commits"] == rec.size and rep["no_record"] == offs.size - rec.size, rep
    assert np.array_equal(blank, clean), (seed, np.nonzero(blank != clean)[0][:5])


def _random_file(rng, idx):
    from oracle import zs_format as zf
    w = zf.FileWriter(bytes(rng.integers(0, 256, 16, dtype=np.uint8)), idx)
    for _ in range(int(rng.integers(0, 300))):
        u = rng.random()
        if u < 0.75:
            key = bytes(rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8))
            val = bytes(rng.integers(0, 256, int(rng.choice([0, 5, 100, 4000, 70000])), dtype=np.uint8))
            w.add(key, val)
        elif u < 0.85:
            w.remove(bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)))
        else:
            w.commit(final=bool(rng.random() < 0.1))
    if rng.random() < 0.5:
        w.finalise()
    else:
        w.commit()
    img = bytearray(w.image())
    for _ in range(int(rng.integers(0, 3))):       # corruptions past the header
        if len(img) > 48:
            img[int(rng.integers(40, len(img)))] ^= 1 << int(rng.integers(0, 8))
    return bytes(img)


def test_random_files(gpu):
    """zscrc_zs_verify_image / zscrc_zs_verify_files on random active files
    written the way zsdb_add / zsdb_remove / zsdb_commit write them (the
    format oracle's FileWriter: short and 70 KB values, deletes, FINAL
    commits, the finalise quirk), some bytes flipped: the verdicts equal the
    format oracle's walk of each image (the fuzz test's semantics)."""
    from tests import fuzzlib
    from zeroskip_amd import zsfile
    rng = np.random.default_rng(53)
    imgs, bads, ncommits = [], [], []
    for i in range(40):
        img = _random_file(rng, i)
        o = fuzzlib.oracle_walk(img)
        if o is None:
            continue
        off, ln, rc, wend = zsfile.walk(img)
        bad = [not c["ok"] for c in o[0][:len(off)]]
        rep = zsfile.verify_image(img)
        assert rep["n_commits"] == len(off) and rep["n_bad"] == sum(bad), (i, rep, sum(bad))
        imgs.append(img)
        bads.append(sum(bad))
        ncommits.append(len(off))
    assert len(imgs) > 25
    rep = zsfile.verify_files(imgs)
    assert rep["files"] == len(imgs) and rep["commits"] == sum(ncommits)
    assert rep["bad_commits"] + rep["stale_empty_commits"] == sum(bads), rep
    # the same files over three device slots (one GPU repeated): the same verdicts
    zsfile.set_devices([0, 0, 0])
    try:
        rep3 = zsfile.verify_files(imgs)
    finally:
        zsfile.set_devices([])
    keys = ("files", "commits", "bytes", "bad_commits", "stale_empty_commits", "header_errors", "walk_errors",
            "first_bad_file", "first_bad_off", "first_bad_what")
    assert {k: rep3[k] for k in keys} == {k: rep[k] for k in keys} and rep3["devices"] == 3, (rep, rep3)


def test_random_fixed_large(gpu):
    """Big fixed-stride batches on the 16-lane coalesced teams (qteam: records
    of 2 KiB and up; parts dealt per workgroup and folded in LDS or by the
    fold launch on big batches): random lengths 2 KiB-1 MiB (not multiples of
    the 1 KiB step), strides, misaligned bases and totals up to ~1.2 GB, every
    CRC against the oracle."""
    g = torch.Generator(device=gpu)
    g.manual_seed(61)
    total = 1_300_000_000
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu, generator=g)
    host = d.cpu().numpy()
    rng = np.random.default_rng(61)
    for it in range(12):
        length = int(np.exp(rng.uniform(np.log(2048), np.log(1 << 20))))
        if it % 3 == 0:
            length = int(rng.choice([2048, 4096, 16384, 65536, 65536 + 8, 1 << 20]))
        stride = length + int(rng.choice([0, 0, 8, 13, 1024]))
        shift = int(rng.choice([0, 0, 4, 16, 37]))
        budget = int(rng.choice([64 << 20, 300 << 20, total - 64]))
        n = max(1, (budget - shift - length) // stride + 1)
        seed = int(rng.integers(0, 1 << 32))
        out = _u32(zd.crc_fixed(d[shift:], stride, length, n, seed=seed))
        offs = np.arange(n, dtype=np.uint64) * stride + shift
        ref = oracle.batch(host, offs, np.full(n, length, np.uint64), np.full(n, seed, np.uint32), impl="hw",
                           threads=16)
        bad = np.nonzero(out != ref)[0]
        assert bad.size == 0, (it, length, stride, shift, n, bad[:5].tolist())
