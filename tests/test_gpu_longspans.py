"""Long commit spans through the unbounded commit route: zsbench NOTBATCHED
layouts (benchmark/zsbench.c:159-217 writeseq: one commit per ~2 MiB file,
spans as written by src/zeroskip-file.c:253-350) and longer -- a span past the
short commit's 24-bit length takes the long commit trailer (writer
semantics, zeroskip-file.c:266-302).  Without a caller bound the batch goes
classify -> plan -> parts (xteam_kernel's parts mode for class 3, team<16>
parts for class 2) -> part fold; every CRC, status, verdict and written CRC
against the format oracle, on both class-3 routes (xteam parts and team<64>
parts, tuning bit 65536; the segment plan -- the class's bytes end to end
cut into one equal segment per wave, or 16 per wave dealt per workgroup, bit 1 << 27 -- and
per-record parts, bit 256) and both classify forms (one single-block launch
with the plans, or two passes and plan launches: bit 524288), with corruptions at a record's first byte, its
last span byte, its stored CRC and bytes either side of a part boundary."""
import numpy as np
import pytest
import torch

from oracle import zs_format as zf
from tests.test_format_oracle import UUID
from zeroskip_amd import zsfile
from zeroskip_amd._lib import lib

pytestmark = pytest.mark.gpu

TEAM64_PARTS = 65536  # zs::BatchDesc::opt: class 3 on team<64> parts instead of xteam parts
MULTI_CLASSIFY = 524288  # opt: two multi-block classify passes + plan launches (not the single-block one)
RECORD_PARTS = 256  # opt: class 3 parts cut per record instead of the segment plan
XDEAL_PARTS = 1 << 27  # opt: segment plans of 16 segments per wave dealt per workgroup (default: one per wave)
OPTS = [0, TEAM64_PARTS, MULTI_CLASSIFY, RECORD_PARTS, XDEAL_PARTS]
IDS = ["xteam-segments", "team64-parts", "multi-classify", "xteam-record-parts", "xteam-segments-dealt"]

# transaction sizes in bytes of value payload: class 3 (> g16_max) records
# of 0.3-3 MiB, one past 16 MiB (long commit), class 2 and short ones beside
SIZES = [[2_100_000, 312, 3_000_000], [1_100_000, 20_000, 300_000, 17_000_000], [9_000, 2_200_000, 5_000, 64]]


def _db(seed=11):
    rng = np.random.default_rng(seed)
    parts, commits, base = [], [], 0
    for f, sizes in enumerate(SIZES):
        w = zf.FileWriter(UUID, idx=f)
        for t, size in enumerate(sizes):
            left = size
            k = 0
            while left > 0:               # values of up to 1 MiB per key
                v = min(left, 1 << 20)
                w.add(b"%08d-%07d" % (f * 100 + t, k), rng.integers(0, 256, v, dtype=np.uint8).tobytes())
                left -= v
                k += 1
            w.commit()
        img = w.image()
        cs, _, _ = zf.walk(img)
        for c in cs:
            c = dict(c)
            c["span_off"] += base
            c["commit_off"] += base
            commits.append(c)
        parts.append(img)
        base += len(img)
    host = np.frombuffer(b"".join(parts), np.uint8).copy()
    offs = np.array([c["span_off"] for c in commits], np.int64)
    lens = np.array([c["span_len"] for c in commits], np.int64)
    return host, offs, lens, commits


@pytest.fixture(scope="module")
def db():
    return _db()


def _with_opt(opt, fn):
    lib().zscrc_set_opt(opt)
    try:
        r = fn()
        torch.cuda.synchronize()
    finally:
        lib().zscrc_set_opt(0)
    return r


def test_layout(db):
    host, offs, lens, commits = db
    assert len(commits) == sum(len(s) for s in SIZES)
    assert lens.max() > (1 << 24)             # one long commit trailer
    assert all(c["ok"] for c in commits)


@pytest.mark.parametrize("opt", OPTS, ids=IDS)
def test_long_spans_match_oracle(gpu, db, opt):
    host, offs, lens, commits = db
    d = torch.from_numpy(host).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    crc, st = _with_opt(opt, lambda: zsfile.verify_commits(d, o, ln))
    crc = crc.cpu().numpy().view(np.uint32)
    assert (crc == np.array([c["computed"] for c in commits], np.uint32)).all()
    assert (st.cpu().numpy() == 1).all()
    nbad, _ = _with_opt(opt, lambda: zsfile.verify_commits_verdict(d, o, ln))
    assert int(nbad.item()) == 0


@pytest.mark.parametrize("opt", OPTS, ids=IDS)
def test_long_spans_corruptions(gpu, db, opt):
    host, offs, lens, commits = db
    h = host.copy()
    big = [i for i in range(len(commits)) if lens[i] > 1_000_000]
    hit = {}
    i0, i1, i2, i3 = big[:4]
    h[offs[i0]] ^= 0x01                              # first span byte (the short first part)
    h[offs[i1] + lens[i1] - 1] ^= 0x80               # last span byte
    e = commits[i2]["commit_off"] + (20 if lens[i2] > (1 << 24) else 4)
    h[e] ^= 0x10                                     # the stored CRC
    h[offs[i3] + lens[i3] // 2] ^= 0x02              # mid-span, near a part boundary
    h[offs[i3] + lens[i3] // 2 + 1] ^= 0x02          # (two flips in one record)
    hit = {i0, i1, i2, i3}
    d = torch.from_numpy(h).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    crc, st = _with_opt(opt, lambda: zsfile.verify_commits(d, o, ln))
    crc = crc.cpu().numpy().view(np.uint32)
    hb = h.tobytes()
    for i, c in enumerate(commits):
        assert crc[i] == zf._commit_check(hb, c["commit_off"])[4], i
    assert set(np.nonzero(st.cpu().numpy() != 1)[0].tolist()) == hit
    nbad, bad = _with_opt(opt, lambda: zsfile.verify_commits_verdict(d, o, ln))
    assert int(nbad.item()) == len(hit) and set(bad[:len(hit)].cpu().tolist()) == hit


@pytest.mark.parametrize("opt", OPTS, ids=IDS)
def test_long_spans_writer(gpu, db, opt):
    """write_commits over blanked CRC fields: the image byte for byte"""
    host, offs, lens, commits = db
    blank = host.copy()
    for c in commits:
        at = c["commit_off"] + (20 if c["span_len"] > (1 << 24) else 4)
        blank[at:at + 4] = 0
    d = torch.from_numpy(blank).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    _with_opt(opt, lambda: zsfile.write_commits(d, o, ln, crc=False))
    assert np.array_equal(d.cpu().numpy(), host)


def test_long_spans_seeded_crc_batch(gpu, db):
    """the same spans as a plain CRC batch with per-record seeds (the fold's
    non-commit output)"""
    from oracle import oracle
    from zeroskip_amd import device
    host, offs, lens, _ = db
    rng = np.random.default_rng(3)
    seeds = rng.integers(0, 2**32, len(offs), dtype=np.uint64).astype(np.uint32)
    d = torch.from_numpy(host).cuda()
    out = device.crc_batch(d, torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda(),
                           seeds=torch.from_numpy(seeds.view(np.int32)).cuda())
    got = out.cpu().numpy().view(np.uint32)
    for i in range(len(offs)):
        assert got[i] == oracle.crc32c_hw(int(seeds[i]), host[offs[i]:offs[i] + lens[i]]), i


@pytest.mark.parametrize("nseg", [1, 3, 7, 50, 400])
def test_segment_plans(gpu, db, nseg, monkeypatch):
    """Segment plans with fewer segments than waves (ZSCRC_XSEGS): segments
    holding several records, records over many segments, a single segment
    -- every CRC, status and a corruption next to a segment boundary"""
    host, offs, lens, commits = db
    monkeypatch.setenv("ZSCRC_XSEGS", str(nseg))
    d = torch.from_numpy(host).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    crc, st = _with_opt(0, lambda: zsfile.verify_commits(d, o, ln))
    assert (crc.cpu().numpy().view(np.uint32) == np.array([c["computed"] for c in commits], np.uint32)).all()
    assert (st.cpu().numpy() == 1).all()
    big = [i for i in range(len(commits)) if lens[i] > 1_000_000]
    # the byte at a segment boundary of the class-3 records laid end to end
    klass3 = [i for i in range(len(commits)) if lens[i] > (1 << 20)]   # g16_max
    total = int(sum(lens[i] for i in klass3))
    G = max(-(-total // nseg) + 63 & ~63, 1 << 16)
    start, at = 0, None
    for i in klass3:
        j = -(-start // G) * G
        if j < start + lens[i] and j > start:
            at = (i, j - start)
            break
        start += int(lens[i])
    h = host.copy()
    hit = {big[0]}
    h[offs[big[0]] + lens[big[0]] // 3] ^= 0x40
    if at is not None:
        i, k = at
        h[offs[i] + k] ^= 0x08
        h[offs[i] + k - 1] ^= 0x01
        hit.add(i)
    d = torch.from_numpy(h).cuda()
    nbad, bad = _with_opt(0, lambda: zsfile.verify_commits_verdict(d, o, ln))
    assert int(nbad.item()) == len(hit) and set(bad[:len(hit)].cpu().tolist()) == hit


NO_ONLY3 = 1 << 28  # opt: the single-block classify's count + scatter passes instead of the fused class-3-only pass


@pytest.mark.parametrize("opt", [0, MULTI_CLASSIFY, NO_ONLY3], ids=["single-classify", "multi-classify", "no-only3"])
def test_verdict_range_long_only(gpu, db, opt):
    """zscrc_device_verify_commits_verdict_range with the walk's range: only
    the class-3 commits (every length > g16_max), so classes 0-2 get no
    launch and the classify counts commits outside the image itself -- the
    verdict equals the unranged one, corruptions and an out-of-image commit
    included."""
    host, offs, lens, commits = db
    long_i = [i for i in range(len(commits)) if lens[i] > (1 << 20)]
    h = host.copy()
    a, b = long_i[0], long_i[-1]
    h[offs[a] + 7] ^= 0x20
    h[commits[b]["commit_off"] + (20 if lens[b] > (1 << 24) else 4)] ^= 0x01
    o_np = np.concatenate([offs[long_i], [len(h) - (2 << 20)]])     # this one's record is past the end
    l_np = np.concatenate([lens[long_i], [(2 << 20) + 16]])
    d = torch.from_numpy(h).cuda()
    o, ln = torch.from_numpy(o_np).cuda(), torch.from_numpy(l_np).cuda()
    want = {long_i.index(a), long_i.index(b), len(long_i)}
    for lo in (0, int(l_np.min())):
        nbad, bad = _with_opt(opt, lambda: zsfile.verify_commits_verdict(d, o, ln, max_len=int(l_np.max()),
                                                                         min_len=lo))
        assert int(nbad.item()) == len(want) and set(bad[:len(want)].cpu().tolist()) == want, lo


@pytest.mark.parametrize("opt", [0, NO_ONLY3], ids=["only3", "count-scatter"])
def test_verdict_range_empty_entries(gpu, db, opt):
    """The fused class-3-only classify (Classify::only3) lists a commit
    outside the image as an empty entry with no parts: such entries first,
    in the middle and last, between real long commits (one corrupt), give
    the same verdict as the count + scatter passes and list every one."""
    host, offs, lens, commits = db
    long_i = [i for i in range(len(commits)) if lens[i] > (1 << 20)]
    h = host.copy()
    bad_rec = long_i[len(long_i) // 2]
    h[offs[bad_rec] + lens[bad_rec] // 2] ^= 0x10
    past = [len(h) - (1 << 20), len(h) - 5]                      # records past the image end
    o_l, l_l, want = [past[0]], [(2 << 20)], {0}
    for k, i in enumerate(long_i):
        o_l.append(offs[i])
        l_l.append(lens[i])
        if i == bad_rec:
            want.add(len(o_l) - 1)
        if k == len(long_i) // 3:
            o_l.append(past[1])
            l_l.append((1 << 21) + 9)
            want.add(len(o_l) - 1)
    o_l.append(past[0] + 3)
    l_l.append((3 << 20) + 1)
    want.add(len(o_l) - 1)
    d = torch.from_numpy(h).cuda()
    o = torch.from_numpy(np.array(o_l, np.int64)).cuda()
    ln = torch.from_numpy(np.array(l_l, np.int64)).cuda()
    nbad, bad = _with_opt(opt, lambda: zsfile.verify_commits_verdict(d, o, ln, max_len=int(max(l_l)),
                                                                     min_len=int(min(l_l))))
    assert int(nbad.item()) == len(want) and set(bad[:len(want)].cpu().tolist()) == want
    # and the per-commit arrays agree on which commits fail
    _, st = _with_opt(opt, lambda: zsfile.verify_commits(d, o, ln))
    assert set(np.nonzero(st.cpu().numpy() != 1)[0].tolist()) == want
