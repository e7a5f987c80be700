"""Class-3-only commit verdicts in two launches (xteam_kernel MODE 3 +
nbv_fold_kernel, "nbv", the default since round 6;
zscrc_device_verify_commits_verdict_range with a range above class 2, the
bench's NOTBATCHED verdict).  Every workgroup scans the commit lengths
itself, wave w hashes segment w of the commits laid end to end, finishes the
commits inside it and stores the parts of longer ones, which the fold
launch folds and checks -- so the verdict is checked here against the
format oracle (src/zeroskip-file.c:253-350's trailer semantics,
zf._commit_check) and against the three-launch route (classify + parts +
fold, tuning bit 64) on:
  * commits shorter than a segment (whole commits finished by their wave),
    several per segment, and commits over many segments (class 3 lowered to
    8 KiB with zscrc_set_teams);
  * corruptions at segment boundaries (the byte either side of G k), first
    and last span bytes and stored CRCs;
  * commits outside the image first, in the middle and last (counted by
    workgroup 0 before any part is hashed);
  * per-commit seeds, a long commit trailer (> 16 MiB span);
  * repeated calls on two streams (the verdict pairs are 0 at rest: a wrong
    reset would show up as a later call's error).
The launch count (zscrc_stats) shows the two-launch route ran."""
import numpy as np
import pytest
import torch

from oracle import zs_format as zf
from tests.test_format_oracle import UUID
from zeroskip_amd import zsfile
from zeroskip_amd._lib import DEFAULT_TEAMS, lib, stats

pytestmark = pytest.mark.gpu

NO_NBV = 64        # zs::OPT_NO_NBV: the classify + parts + fold launches
UNIT_MIN = 1 << 16  # class 3's segment floor (64-lane teams x 16 steps of 1 KiB)


def _image(seed, sizes):
    """one file, one commit per size (values split at 1 MiB per key)"""
    rng = np.random.default_rng(seed)
    w = zf.FileWriter(UUID, idx=0)
    for t, size in enumerate(sizes):
        left, k = int(size), 0
        while left > 0:
            v = min(left, 1 << 20)
            w.add(b"%07d-%05d" % (t, k), rng.integers(0, 256, v, dtype=np.uint8).tobytes())
            left -= v
            k += 1
        w.commit()
    img = np.frombuffer(w.image(), np.uint8).copy()
    cs, _, _ = zf.walk(img.tobytes())
    return img, cs


def _seg_unit(total, nseg):
    g = -(-total // nseg)
    g = (g + 63) & ~63
    return max(g, UNIT_MIN)


def _verdict(opt, d, o, ln, lo, hi, seed=None, cap=8192):
    lib().zscrc_set_opt(opt)
    try:
        before = stats()[2]
        nbad, bad = zsfile.verify_commits_verdict(d, o, ln, seed=seed, max_len=hi, min_len=lo, cap=cap)
        torch.cuda.synchronize()
        launches = stats()[2] - before
    finally:
        lib().zscrc_set_opt(0)
    n = int(nbad.item())
    return n, set(bad[:min(n, cap)].cpu().tolist()), launches


def _oracle_bad(img, offs, lens, cs_by_off, seeds=None):
    """indices whose commit does not verify (outside the image: no commit)"""
    hb = img.tobytes()
    want = set()
    for i, (o, n) in enumerate(zip(offs, lens)):
        o, n = int(o), int(n)
        if o > len(hb) or n > len(hb) - o or len(hb) - o - n < 8:
            want.add(i)
            continue
        try:
            _, _, _, stored, comp = zf._commit_check(hb, o + n, 0 if seeds is None else int(seeds[i]))
        except ValueError:
            want.add(i)
            continue
        if stored != comp:
            want.add(i)
    return want


@pytest.fixture
def small_class3(gpu):
    """class 3 from 8 KiB up: commits shorter than a 64 KiB segment exist"""
    lib().zscrc_set_teams(DEFAULT_TEAMS[0], 8192)
    yield
    lib().zscrc_set_teams(*DEFAULT_TEAMS)


def _corrupt(img, cs, offs, lens, G, rng, k):
    """flip bytes at segment boundaries, first / last span bytes, stored CRCs"""
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    total = int(lens.sum())
    hits = []
    bounds = list(range(G, total, G))
    for b in rng.choice(bounds, size=min(k, len(bounds)), replace=False):
        r = int(np.searchsorted(starts, b, side="right") - 1)
        p = int(b - starts[r])
        img[offs[r] + p] ^= 0x08
        if p:
            img[offs[r] + p - 1] ^= 0x01
        hits.append(r)
    for r in rng.choice(len(cs), size=min(k, len(cs)), replace=False):
        what = int(rng.integers(0, 3))
        if what == 0:
            img[offs[r]] ^= 0x40
        elif what == 1:
            img[offs[r] + lens[r] - 1] ^= 0x02
        else:
            img[cs[r]["commit_off"] + (20 if lens[r] > (1 << 24) else 4)] ^= 0x10
        hits.append(int(r))
    return hits


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_nbv_short_and_long_commits(small_class3, seed):
    """9 KiB .. 400 KiB commits: whole commits inside one segment, several per
    segment, commits over many; corruptions at segment boundaries"""
    rng = np.random.default_rng(100 + seed)
    sizes = rng.integers(9_000, 400_000, 500)
    img, cs = _image(seed, sizes)
    offs = np.array([c["span_off"] for c in cs], np.int64)
    lens = np.array([c["span_len"] for c in cs], np.int64)
    nseg = torch.cuda.get_device_properties(0).multi_processor_count * 16
    G = _seg_unit(int(lens.sum()), nseg)
    assert (lens < G).any() and (lens > 2 * G).any()
    _corrupt(img, cs, offs, lens, G, rng, 20)
    want = _oracle_bad(img, offs, lens, None)
    assert want
    d = torch.from_numpy(img).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    lo, hi = int(lens.min()), int(lens.max())
    n1, b1, k1 = _verdict(0, d, o, ln, lo, hi)
    assert k1 == 2, "the two-launch route did not run"
    assert n1 == len(want) and b1 == want
    n3, b3, k3 = _verdict(NO_NBV, d, o, ln, lo, hi)
    assert k3 > 1 and n3 == n1 and b3 == b1


def test_nbv_out_of_image_entries(small_class3):
    """commits past the image end first, in the middle and last: counted and
    listed, the rest checked as usual"""
    rng = np.random.default_rng(7)
    img, cs = _image(7, rng.integers(20_000, 300_000, 200))
    offs = [c["span_off"] for c in cs]
    lens = [c["span_len"] for c in cs]
    img[offs[50] + 3] ^= 0x20
    size = len(img)
    o_l = [size - 100_000] + offs[:120] + [size - 5] + offs[120:] + [size + 64]
    l_l = [150_000] + lens[:120] + [90_000] + lens[120:] + [30_000]
    o_np, l_np = np.array(o_l, np.int64), np.array(l_l, np.int64)
    want = _oracle_bad(img, o_np, l_np, None)
    assert {0, 121, len(o_l) - 1, 51} <= want
    d = torch.from_numpy(img).cuda()
    o, ln = torch.from_numpy(o_np).cuda(), torch.from_numpy(l_np).cuda()
    lo, hi = int(l_np.min()), int(l_np.max())
    n1, b1, k1 = _verdict(0, d, o, ln, lo, hi)
    assert k1 == 2 and n1 == len(want) and b1 == want
    n3, b3, _ = _verdict(NO_NBV, d, o, ln, lo, hi)
    assert n3 == n1 and b3 == b1


def test_nbv_seeded_and_long_trailer(small_class3):
    """per-commit seeds (a commit continuing an earlier CRC) and one span past
    16 MiB (the long commit trailer), default-sized and small commits"""
    rng = np.random.default_rng(9)
    sizes = list(rng.integers(10_000, 2_500_000, 60)) + [17_500_000] + list(rng.integers(10_000, 200_000, 40))
    img, cs = _image(9, sizes)
    offs = np.array([c["span_off"] for c in cs], np.int64)
    lens = np.array([c["span_len"] for c in cs], np.int64)
    assert lens.max() > (1 << 24)
    seeds = rng.integers(0, 2**32, len(cs), dtype=np.uint64).astype(np.uint32)
    seeds[::3] = 0
    want = _oracle_bad(img, offs, lens, None, seeds)   # a seeded commit fails against its stored CRC
    d = torch.from_numpy(img).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    sd = torch.from_numpy(seeds.view(np.int32)).cuda()
    lo, hi = int(lens.min()), int(lens.max())
    n1, b1, k1 = _verdict(0, d, o, ln, lo, hi, seed=sd)
    assert k1 == 2 and n1 == len(want) and b1 == want
    n3, b3, _ = _verdict(NO_NBV, d, o, ln, lo, hi, seed=sd)
    assert n3 == n1 and b3 == b1
    # unseeded: the stored CRCs all match
    n0, b0, _ = _verdict(0, d, o, ln, lo, hi)
    assert n0 == 0 and not b0


def test_nbv_repeated_calls_two_streams(small_class3):
    """the part counters and verdict pairs return to 0: alternating clean and
    corrupt images on two streams, every call equal to the oracle"""
    rng = np.random.default_rng(13)
    img, cs = _image(13, rng.integers(9_000, 500_000, 300))
    offs = np.array([c["span_off"] for c in cs], np.int64)
    lens = np.array([c["span_len"] for c in cs], np.int64)
    bad = img.copy()
    nseg = torch.cuda.get_device_properties(0).multi_processor_count * 16
    _corrupt(bad, cs, offs, lens, _seg_unit(int(lens.sum()), nseg), rng, 10)
    want_bad = _oracle_bad(bad, offs, lens, None)
    dg, db = torch.from_numpy(img).cuda(), torch.from_numpy(bad).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    lo, hi = int(lens.min()), int(lens.max())
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for k in range(6):
        with torch.cuda.stream(s1 if k % 2 else s2):
            n, b, launches = _verdict(0, db if k % 3 else dg, o, ln, lo, hi)
        assert launches == 2
        if k % 3:
            assert n == len(want_bad) and b == want_bad, k
        else:
            assert n == 0 and not b, k


def test_nbv_notbatched_shape(gpu):
    """the bench's NOTBATCHED shape at default teams: ~2 MiB commits, one per
    segment or fewer, corruptions either side of segment boundaries"""
    rng = np.random.default_rng(21)
    img, cs = _image(21, rng.integers(1_900_000, 2_300_000, 96))
    offs = np.array([c["span_off"] for c in cs], np.int64)
    lens = np.array([c["span_len"] for c in cs], np.int64)
    nseg = torch.cuda.get_device_properties(0).multi_processor_count * 16
    _corrupt(img, cs, offs, lens, _seg_unit(int(lens.sum()), nseg), rng, 12)
    want = _oracle_bad(img, offs, lens, None)
    d = torch.from_numpy(img).cuda()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    lo, hi = int(lens.min()), int(lens.max())
    n1, b1, k1 = _verdict(0, d, o, ln, lo, hi)
    assert k1 == 2 and n1 == len(want) and b1 == want
