"""A large bounded commit batch of MIXED span lengths through every form of
commit_kernel: the run-only kernel's non-run rounds -- quad
bursts, front fix-ups, lane hashing -- are otherwise only reached by the ~1 %
file-boundary rounds of the all-312-byte zsbench images.

300,000 spans of 0-640 bytes at unaligned offsets, each followed by a short
commit record (COMMIT or FINAL type) or, for some, by no commit record; some
spans verified from a seed (the chained finalise commit of
src/zeroskip-file.c:253-350 after src/mfile.c:534-546).  The commit CRCs are
written by the CPU oracle (the writer of zeroskip-file.c:303-328), a few spans
corrupted; then, under the default schedule and OPT_NO_RUNSPLIT / OPT_RO12 /
OPT_RO_LIST: per-commit CRCs and statuses, the verdict, the writer's CRC array
and the in-place writer, each against the oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle
from zeroskip_amd import zsfile
from zeroskip_amd._lib import lib

pytestmark = pytest.mark.gpu

NO_RUNSPLIT = 1 << 29
RO12 = 1 << 31
RO_LIST = 1 << 14
T_KEY, T_COMMIT, T_FINAL = 1, 4, 16
N, MAXLEN = 300_000, 640


def _commit_crc_seeded(host, off, ln, seed, final):
    c = oracle.crc32c_hw(seed, host[off:off + ln])
    return oracle.commit_crc(c, ln, final)


@pytest.fixture(scope="module")
def mixed(gpu):
    rng = np.random.default_rng(0xA11CE)
    # lengths: mostly 0-640 uniform, with extra mass on the edges (0-8, 632-640)
    lens = rng.integers(0, MAXLEN + 1, N)
    edge = rng.random(N)
    lens[edge < 0.05] = rng.integers(0, 9, int((edge < 0.05).sum()))
    lens[edge > 0.97] = rng.integers(MAXLEN - 8, MAXLEN + 1, int((edge > 0.97).sum()))
    gaps = rng.integers(0, 8, N)            # bytes between a commit record and the next span
    offs = np.zeros(N, np.int64)
    pos = 40 + 3                            # unaligned start
    for_cum = lens + 8 + gaps
    offs[0] = pos
    offs[1:] = pos + np.cumsum(for_cum)[:-1]
    size = int(offs[-1] + lens[-1] + 8 + 64)
    host = rng.integers(0, 256, size, dtype=np.uint8)
    kind = rng.random(N)
    has_rec = kind >= 0.04                  # 4 % of spans: no commit record
    final = (kind >= 0.04) & (kind < 0.10)  # 6 % FINAL records
    at = offs + lens
    host[at[~has_rec]] = T_KEY
    host[at[has_rec & ~final]] = T_COMMIT
    host[at[final]] = T_FINAL
    seeded = has_rec & (rng.random(N) < 0.05)
    seeds = np.where(seeded, rng.integers(1, 1 << 32, N, dtype=np.uint64), 0).astype(np.uint32)
    # the oracle writes the records: unseeded through its writer, seeded here
    plain = has_rec & ~seeded
    oracle.write_commits(host, offs[plain].astype(np.uint64), lens[plain].astype(np.uint64), threads=8)
    for i in np.nonzero(seeded)[0]:
        o, ln = int(offs[i]), int(lens[i])
        crc = _commit_crc_seeded(host, o, ln, int(seeds[i]), bool(final[i]))
        w = ((T_FINAL if final[i] else T_COMMIT) << 56) | (ln << 32) | crc
        host[o + ln:o + ln + 8] = np.frombuffer(w.to_bytes(8, "big"), np.uint8)
    clean = host.copy()
    # corruptions: inside spans (len > 0) and in stored CRC fields
    rec_idx = np.nonzero(has_rec)[0]
    hit = rng.choice(rec_idx, 80, replace=False)
    for j, i in enumerate(hit):
        o, ln = int(offs[i]), int(lens[i])
        if ln and j % 2 == 0:
            host[o + int(rng.integers(0, ln))] ^= 0x5A
        else:
            host[o + ln + 4 + j % 4] ^= 0x01
    # expected per-commit CRCs over the corrupted image
    want = np.zeros(N, np.uint32)
    want[plain] = oracle.commit_crcs(host, offs[plain].astype(np.uint64), lens[plain].astype(np.uint64), threads=8)
    for i in np.nonzero(seeded)[0]:
        want[i] = _commit_crc_seeded(host, int(offs[i]), int(lens[i]), int(seeds[i]), bool(final[i]))
    bad = set(hit.tolist()) | set(np.nonzero(~has_rec)[0].tolist())
    dev = gpu
    d = {
        "img": torch.from_numpy(host).to(dev), "clean": torch.from_numpy(clean).to(dev),
        "offs": torch.from_numpy(offs.astype(np.int64)).to(dev), "lens": torch.from_numpy(lens.astype(np.int64)).to(dev),
        "seed": torch.from_numpy(seeds.view(np.int32)).to(dev), "has_rec": has_rec, "seeded": seeded,
        "plain": plain, "want": want, "bad": bad, "hit": set(hit.tolist()), "host_clean": clean,
        "offs_np": offs, "lens_np": lens,
    }
    assert (N + 63) // 64 >= 256 * 12     # past the run-only split (ncu * 12 rounds)
    return d


@pytest.mark.parametrize("opt", [0, NO_RUNSPLIT, RO12, RO_LIST], ids=["default", "no_runsplit", "ro12", "ro_list"])
def test_mixed_lengths_arrays_and_verdict(mixed, opt):
    m = mixed
    lib().zscrc_set_opt(opt)
    try:
        crc, st = zsfile.verify_commits(m["img"], m["offs"], m["lens"], seed=m["seed"], max_len=MAXLEN)
        nbad, badi = zsfile.verify_commits_verdict(m["img"], m["offs"], m["lens"], seed=m["seed"], max_len=MAXLEN,
                                                   cap=1 << 16)
        torch.cuda.synchronize()
    finally:
        lib().zscrc_set_opt(0)
    crc = crc.cpu().numpy().view(np.uint32)
    st = st.cpu().numpy()
    rec = m["has_rec"]
    assert np.array_equal(crc[rec], m["want"][rec])
    assert (st[~rec] == 2).all()
    want_st = np.ones(N, np.int32)
    want_st[list(m["hit"])] = 0
    assert np.array_equal(st[rec], want_st[rec])
    k = int(nbad.item())
    assert k == len(m["bad"]) and set(badi[:k].cpu().tolist()) == m["bad"]


@pytest.mark.parametrize("opt", [0, NO_RUNSPLIT, RO12, RO_LIST, 512],
                         ids=["default", "no_runsplit", "ro12", "ro_list", "two_pass"])
def test_mixed_lengths_writer(mixed, opt):
    """The writer's CRC array and the in-place writer over the unseeded
    record spans of the clean image (the writer has no seeds): a copy with
    those CRC fields zeroed comes back byte for byte."""
    m = mixed
    sel = np.nonzero(m["plain"])[0]
    o = m["offs"][torch.from_numpy(sel).to(m["offs"].device)].contiguous()
    ln = m["lens"][torch.from_numpy(sel).to(m["offs"].device)].contiguous()
    want = oracle.commit_crcs(m["host_clean"], m["offs_np"][sel].astype(np.uint64), m["lens_np"][sel].astype(np.uint64),
                              threads=8)
    fields = (o + ln + 4).view(-1, 1) + torch.arange(4, device=o.device).view(1, -1)
    lib().zscrc_set_opt(opt)
    try:
        crcs = zsfile.commit_crcs(m["clean"], o, ln, max_len=MAXLEN)
        z = m["clean"].clone()
        z[fields.view(-1)] = 0
        zsfile.write_commits(z, o, ln, max_len=MAXLEN, crc=False)
        torch.cuda.synchronize()
    finally:
        lib().zscrc_set_opt(0)
    assert np.array_equal(crcs.cpu().numpy().view(np.uint32), want)
    assert torch.equal(z, m["clean"])


TWO_PASS = 512   # opt: the bounded writer as a CRC array + a scatter launch


def _long_word_crc(host, off, ln, w0, w2):
    c = oracle.crc32c_hw(0, host[off:off + ln])
    words = w0.to_bytes(8, "little") + ln.to_bytes(8, "little") + (w2 & (0xFF << 56)).to_bytes(8, "little")
    return oracle.crc32c_hw(c, words)


@pytest.mark.parametrize("opt", [0, TWO_PASS, TWO_PASS | RO12], ids=["in_place", "two_pass", "two_pass_ro12"])
def test_writer_short_and_long_records(gpu, opt):
    """The bounded writer over 250,000 short spans whose commit records are
    short (8 bytes, CRC at +4) or -- every 40th -- long (24 bytes, CRC at +20:
    the record form decides, src/zeroskip-file.c:266-302 / :303-328): the
    two-pass writer's scatter (status 3 = long) and the in-place writer put
    every CRC where the verifier finds it, the rest of the image untouched."""
    rng = np.random.default_rng(0xB0B)
    n = 250_000
    lens = rng.integers(0, MAXLEN + 1, n)
    long_rec = (np.arange(n) % 40) == 7
    rl = np.where(long_rec, 24, 8)
    offs = np.zeros(n, np.int64)
    offs[0] = 41
    offs[1:] = 41 + np.cumsum(lens + rl + rng.integers(0, 8, n))[:-1]
    size = int(offs[-1] + lens[-1] + 24 + 64)
    host = rng.integers(0, 256, size, dtype=np.uint8)
    at = offs + lens
    want = np.zeros(n, np.uint32)
    short_i = np.nonzero(~long_rec)[0]
    host[at[short_i]] = T_COMMIT
    for i in np.nonzero(long_rec)[0]:
        a, ln = int(at[i]), int(lens[i])
        w0 = (36 << 56)                      # T_LONG_COMMIT
        w2 = (8 << 56) | 0                   # T_2ND_HALF, CRC field zero
        host[a:a + 8] = np.frombuffer(w0.to_bytes(8, "big"), np.uint8)
        host[a + 8:a + 16] = np.frombuffer(ln.to_bytes(8, "big"), np.uint8)
        host[a + 16:a + 24] = np.frombuffer(w2.to_bytes(8, "big"), np.uint8)
        want[i] = _long_word_crc(host, int(offs[i]), ln, w0, w2)
    # short records: the oracle writer on a copy gives the expected CRCs
    ref = host.copy()
    oracle.write_commits(ref, offs[short_i].astype(np.uint64), lens[short_i].astype(np.uint64), threads=8)
    want[short_i] = ref[(at[short_i] + 4)[:, None] + np.arange(4)].view(">u4").reshape(-1)
    # the fully written image expected: short records from the oracle, long CRC fields patched
    full = ref.copy()
    li = np.nonzero(long_rec)[0]
    full[(at[li] + 20)[:, None] + np.arange(4)] = want[li].astype(">u4").view(np.uint8).reshape(-1, 4)
    # the writer's input: short CRC fields zeroed (header words in place)
    blank = full.copy()
    blank[(at[short_i] + 4)[:, None] + np.arange(4)] = 0
    blank[(at[li] + 20)[:, None] + np.arange(4)] = 0
    img = torch.from_numpy(blank).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int64)).to(gpu)
    lib().zscrc_set_opt(opt)
    try:
        crc, st = zsfile.write_commits(img, o, ln, max_len=MAXLEN, status=True)
        torch.cuda.synchronize()
    finally:
        lib().zscrc_set_opt(0)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), want)
    assert bool((st == 1).all())
    assert np.array_equal(img.cpu().numpy(), full)
    c2, s2 = zsfile.verify_commits(img, o, ln, max_len=MAXLEN)
    assert bool((s2 == 1).all())
