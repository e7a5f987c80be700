"""Run rounds of the commit bursts (burst_kernel, zscrc_kernels.hip
run_check / run_issue / run_hash): 64 back-to-back 312-byte commit spans --
zsbench's BATCHED log layout (benchmark/zsbench.c:159-217; spans as written
by src/zeroskip-file.c:253-350) -- read as one coalesced 20 KiB grid, hashed
per 64-byte piece and folded per record by CRC linearity.  Every CRC and
status against the format oracle (FileWriter / walk), with the run rounds on
and off (tuning bit 2048), at file boundaries, stale finalise commits,
corrupt span bytes, corrupt stored CRCs at lanes 0 and 63 of a round, the
previous commit's CRC field inside a round's first piece, seeded spans, and
the writer side byte for byte."""
import struct

import numpy as np
import pytest
import torch

from oracle import oracle
from oracle import zs_format as zf
from tests.test_format_oracle import UUID
from zeroskip_amd import zsfile
from zeroskip_amd._lib import lib

pytestmark = pytest.mark.gpu

RUN_OFF = 2048  # zs::BatchDesc::opt bit: no run rounds


def _zsbench_db(per_file, gaps, seed=5):
    """zsbench BATCHED-like files (one 16-byte key + 256-byte value per
    transaction: 312-byte spans every 320 bytes) concatenated with `gaps`
    bytes between them (shifts every file's piece grid)."""
    rng = np.random.default_rng(seed)
    parts, offs, lens, commits = [], [], [], []
    base = 0
    for f, (n, gap) in enumerate(zip(per_file, gaps)):
        parts.append(bytes(rng.integers(0, 256, gap, dtype=np.uint8)))
        base += gap
        w = zf.FileWriter(UUID, idx=f)
        for t in range(n):
            w.add(b"%016d" % (f * 100000 + t), rng.integers(0, 256, 256, dtype=np.uint8).tobytes())
            w.commit()
        if f % 2:
            w.finalise()              # a stale zero-length commit after the last span
        img = w.image()
        cs, _, _ = zf.walk(img)
        for c in cs:
            offs.append(base + c["span_off"])
            lens.append(c["span_len"])
            commits.append(c)
        parts.append(img)
        base += len(img)
    host = np.frombuffer(b"".join(parts), np.uint8).copy()
    return host, np.array(offs, np.int64), np.array(lens, np.int64), commits


def _verify(d, o, ln, opt, **kw):
    lib().zscrc_set_opt(opt)
    try:
        crc, st = zsfile.verify_commits(d, o, ln, **kw)
        torch.cuda.synchronize()
    finally:
        lib().zscrc_set_opt(0)
    return crc.cpu().numpy().view(np.uint32), st.cpu().numpy()


@pytest.fixture(scope="module")
def db():
    # 2,000-odd spans: many full rounds, rounds cut by file ends and stale
    # commits, grids at every 8-byte phase of a 64-byte piece
    return _zsbench_db([700, 333, 64, 65, 900, 129], [0, 8, 24, 40, 200, 56])


@pytest.mark.parametrize("opt", [0, RUN_OFF], ids=["runs", "quad-only"])
@pytest.mark.parametrize("bound", [True, False], ids=["bounded", "classes"])
def test_runs_match_oracle(gpu, db, opt, bound):
    host, offs, lens, commits = db
    d = torch.from_numpy(host).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    crc, st = _verify(d, o, ln, opt, max_len=int(lens.max()) if bound else None)
    want = np.array([c["computed"] for c in commits], np.uint32)
    ok = np.array([c["ok"] for c in commits])
    assert (crc == want).all()
    assert ((st == 1) == ok).all() and (~ok).sum() == 3   # the three stale finalise commits


def test_runs_corruptions(gpu, db):
    host, offs, lens, commits = db
    h = host.copy()
    n = len(commits)
    span = [i for i in range(n) if lens[i] == 312]
    hit = {}
    # a span byte mid-round, stored CRCs at lanes 0 and 63 of rounds, the
    # last span byte of a round's last lane
    for i, at in ((4 * 64 + 31, 100), (3 * 64 + 63, 312 + 7), (5 * 64, 312 + 4), (7 * 64 + 63, 311)):
        assert i in span
        h[offs[i] + at] ^= 0x40
        hit[i] = True
    # the previous commit's CRC field sits in round 6's first piece: only
    # that previous commit is bad, round 6's lane 0 is not
    h[offs[6 * 64] - 2] ^= 0x01
    hit[6 * 64 - 1] = True
    d = torch.from_numpy(h).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    res = [_verify(d, o, ln, opt, max_len=312) for opt in (0, RUN_OFF)]
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    crc, st = res[0]
    hb = h.tobytes()
    for i in range(n):
        c = zf._commit_check(hb, int(offs[i] + lens[i]))
        assert crc[i] == c[4], i
    bad = set(np.nonzero(st != 1)[0].tolist()) - {i for i, c in enumerate(commits) if not c["ok"]}
    assert bad == set(hit), sorted(bad)


def test_runs_seeded(gpu, db):
    host, offs, lens, commits = db
    rng = np.random.default_rng(9)
    seeds = rng.integers(0, 2**32, len(offs), dtype=np.uint64).astype(np.uint32)
    d = torch.from_numpy(host).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    sd = torch.from_numpy(seeds.view(np.int32)).cuda()
    for opt in (0, RUN_OFF):
        crc, st = _verify(d, o, ln, opt, seed=sd, max_len=312)
        for i in range(0, len(offs), 97):
            w0, = struct.unpack_from(">Q", host, int(offs[i] + lens[i]))
            span = host[offs[i]:offs[i] + lens[i]]
            want = oracle.crc32c_hw(oracle.crc32c_hw(int(seeds[i]), span),
                                    struct.pack("<Q", w0 & 0xFFFFFFFF00000000))
            assert crc[i] == want, (opt, i)


def test_runs_writer_byte_exact(gpu, db):
    host, offs, lens, commits = db
    blank = host.copy()
    live = lens > 0
    for i in np.nonzero(live)[0]:
        e = offs[i] + lens[i]
        blank[e + 4:e + 8] = 0
    for opt in (0, RUN_OFF):
        d = torch.from_numpy(blank.copy()).cuda()
        o = torch.from_numpy(offs[live].copy()).cuda()
        ln = torch.from_numpy(lens[live].copy()).cuda()
        lib().zscrc_set_opt(opt)
        try:
            zsfile.write_commits(d, o, ln, max_len=312)
            torch.cuda.synchronize()
        finally:
            lib().zscrc_set_opt(0)
        assert np.array_equal(d.cpu().numpy(), host), opt


@pytest.mark.parametrize("opt", [0, RUN_OFF, 32768], ids=["commit_kernel", "quad-only", "burst_kernel"])
@pytest.mark.parametrize("bound", [True, False], ids=["bounded", "classes"])
def test_verdict_matches_status(gpu, db, opt, bound):
    """zscrc_device_verify_commits_verdict: the count and the set of bad
    indices equal the statuses != 1 of the per-commit verify, on a clean
    image and with corrupt spans / stored CRCs (cap smaller than the count:
    the count is still exact, the listed indices a subset)"""
    host, offs, lens, commits = db
    h = host.copy()
    for i in (5, 64 * 2 + 63, 64 * 3, 700 + 40, 1500):
        h[offs[i] + (100 if i % 2 else 312 + 5)] ^= 0x11
    d = torch.from_numpy(h).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    mx = int(lens.max()) if bound else None
    _, st = _verify(d, o, ln, 0, max_len=mx)
    want = set(np.nonzero(st != 1)[0].tolist())
    assert len(want) == 5 + 3
    lib().zscrc_set_opt(opt)
    try:
        nbad, bad = zsfile.verify_commits_verdict(d, o, ln, max_len=mx)
        nb2, bad2 = zsfile.verify_commits_verdict(d, o, ln, max_len=mx, cap=3)
        torch.cuda.synchronize()
    finally:
        lib().zscrc_set_opt(0)
    assert int(nbad.item()) == len(want)
    assert set(bad[:len(want)].cpu().tolist()) == want
    assert int(nb2.item()) == len(want) and set(bad2[:3].cpu().tolist()) <= want
    clean = torch.from_numpy(host).cuda()
    nb3, _ = zsfile.verify_commits_verdict(clean, o, ln, max_len=mx)
    assert int(nb3.item()) == 3          # the stale finalise commits only


def test_writer_without_crc_array(gpu, db):
    """write_commits with d_crc NULL: the image gets every CRC all the same"""
    host, offs, lens, commits = db
    live = lens > 0
    blank = host.copy()
    for i in np.nonzero(live)[0]:
        blank[offs[i] + lens[i] + 4:offs[i] + lens[i] + 8] = 0
    d = torch.from_numpy(blank).cuda()
    r = zsfile.write_commits(d, torch.from_numpy(offs[live].copy()).cuda(), torch.from_numpy(lens[live].copy()).cuda(),
                             max_len=312, crc=False)
    torch.cuda.synchronize()
    assert r is None and np.array_equal(d.cpu().numpy(), host)
