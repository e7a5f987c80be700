"""The writer's CRCs out of place (zscrc_device_commit_crcs_bounded, commit
mode 3) and the host-image writer built on it (zscrc_zs_fill_commits:
H2D chunks -> CRC array -> D2H of 4 B per commit -> host patches), byte for
byte against the format oracle's writer (oracle/zs_format.py, the writer of
src/zeroskip-file.c:253-350)."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from oracle import zs_format as zf
from tests.test_gpu_runs import _zsbench_db
from zeroskip_amd import zsfile
from zeroskip_amd._lib import ZscrcError

pytestmark = pytest.mark.gpu

UUID = bytes(range(16))


def _blank(img, commits):
    """The image with every writer CRC field zeroed (the record headers kept)."""
    b = img.copy()
    for c in commits:
        at = c["span_off"] + c["span_len"]
        if c["span_len"] > zf.MAX_SHORT_VAL_LEN:
            b[at + 20:at + 24] = 0
        else:
            b[at + 4:at + 8] = 0
    return b


def _writer_spans(commits):
    # the stale finalise commit chains from the previous span: not the writer's
    keep = [c for i, c in enumerate(commits) if c["span_len"] or i == 0]
    return (np.array([c["span_off"] for c in keep], np.uint64), np.array([c["span_len"] for c in keep], np.uint64),
            keep)


@pytest.fixture(scope="module")
def db():
    return _zsbench_db([700, 333, 64, 65, 900, 129], [0, 8, 24, 40, 200, 56])


@pytest.mark.parametrize("bound", [True, False], ids=["bounded", "classes"])
def test_commit_crcs_match_oracle(gpu, db, bound):
    host, offs, lens, commits = db
    d = torch.from_numpy(host).cuda()
    before = d.clone()
    o, ln = torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda()
    crc, st = zsfile.commit_crcs(d, o, ln, max_len=int(lens.max()) if bound else None, status=True)
    torch.cuda.synchronize()
    assert torch.equal(d, before), "commit mode 3 must not store into the image"
    live = lens > 0
    want = oracle.commit_crcs(host, offs[live], lens[live])
    assert np.array_equal(crc.cpu().numpy().view(np.uint32)[live], want)
    assert bool((st == 1).all())
    # a span with no commit record after it (and one past the image end)
    o2 = torch.tensor([40, host.size - 8], dtype=torch.int64, device=gpu)
    l2 = torch.tensor([8, 8], dtype=torch.int64, device=gpu)
    _, st2 = zsfile.commit_crcs(d, o2, l2, max_len=8, status=True)
    assert st2.cpu().tolist() == [2, 2]


def _log_images(seed, long_value=False):
    rng = np.random.default_rng(seed)
    parts, commits, base = [], [], 0
    for f in range(4):
        w = zf.FileWriter(UUID, idx=f)
        for t in range(150 + 40 * f):
            for _ in range(int(rng.integers(1, 3))):
                w.add(b"%016d" % int(rng.integers(0, 10**9)),
                      rng.integers(0, 256, int(rng.integers(0, 900)), dtype=np.uint8).tobytes())
            if long_value and f == 2 and t == 50:
                w.add(b"big", rng.integers(0, 256, zf.MAX_SHORT_VAL_LEN + 4000, dtype=np.uint8).tobytes())
            if t % 9 == 4:
                w.remove(b"%016d" % t)
            w.commit(final=(t == 149 + 40 * f and f == 3))
        img = w.image()
        cs, _, why = zf.walk(img)
        assert why == ("end" if f < 3 else "stop at type 16")
        if f == 3:   # the walk stops at FINAL: its span from the record itself
            w0 = int.from_bytes(img[-8:], "big")
            n = (w0 >> 32) & 0xFFFFFF
            cs = cs + [{"span_off": len(img) - 8 - n, "span_len": n}]
        for c in cs:
            c = dict(c)
            c["span_off"] += base
            commits.append(c)
        parts.append(img)
        base += len(img)
    return np.frombuffer(b"".join(parts), np.uint8).copy(), commits


@pytest.mark.parametrize("chunk", [None, 128 << 10], ids=["default", "128KiB-chunks"])
@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
def test_fill_commits_byte_exact(gpu, chunk, pinned, monkeypatch):
    img, commits = _log_images(3)
    o, ln, keep = _writer_spans(commits)
    blank = _blank(img, keep)
    assert not np.array_equal(blank, img)
    if chunk:
        monkeypatch.setenv("ZSCRC_FILL_CHUNK", str(chunk))
    if pinned:
        t = torch.from_numpy(blank).pin_memory()
        rep = zsfile.fill_commits(t, o, ln, max_len=int(ln.max()))
        out = t.numpy()
    else:
        out = blank
        rep = zsfile.fill_commits(out, o, ln)
    assert rep["staged"] == (0 if pinned else 1)
    assert rep["commits"] == len(o) and rep["no_record"] == 0
    if chunk:
        assert rep["chunks"] > 1
    assert np.array_equal(out, img)


def test_fill_commits_long_spans(gpu, monkeypatch):
    """A > 16 MiB span (long commit record) and, with 4 MiB chunks, a span
    longer than a chunk (streamed on its own)."""
    img, commits = _log_images(4, long_value=True)
    o, ln, keep = _writer_spans(commits)
    assert ln.max() > zf.MAX_SHORT_VAL_LEN
    for chunk in (None, 4 << 20):
        if chunk:
            monkeypatch.setenv("ZSCRC_FILL_CHUNK", str(chunk))
        out = _blank(img, keep)
        rep = zsfile.fill_commits(out, o, ln)
        assert rep["long_commits"] == (1 if chunk else 0) or chunk is None
        assert rep["commits"] == len(o)
        assert np.array_equal(out, img)


def test_fill_commits_edges(gpu):
    img, commits = _log_images(5)
    o, ln, keep = _writer_spans(commits)
    # a span with no commit record after it: counted, nothing written
    o2 = np.concatenate([o, [img.size - 8]]).astype(np.uint64)
    l2 = np.concatenate([ln, [8]]).astype(np.uint64)
    out = _blank(img, keep)
    rep = zsfile.fill_commits(out, o2, l2)
    assert rep["no_record"] == 1 and rep["commits"] == len(o)
    assert np.array_equal(out, img)
    # unsorted spans are refused, and the image is left as it was (every
    # span checked before the first store) -- a swap early, one
    # late in the last chunk, and an overlap
    for swap in ([3, 4], [len(o) - 2, len(o) - 1]):
        bad = o.copy()
        bad[swap] = bad[swap[::-1]]
        blank = _blank(img, keep)
        before = blank.copy()
        with pytest.raises(ZscrcError):
            zsfile.fill_commits(blank, bad, ln)
        assert np.array_equal(blank, before)
    over = ln.copy()
    over[len(o) // 2] += 64
    blank = _blank(img, keep)
    before = blank.copy()
    with pytest.raises(ZscrcError):
        zsfile.fill_commits(blank, o, over)
    assert np.array_equal(blank, before)
    # nothing to do
    assert zsfile.fill_commits(out, np.zeros(0, np.uint64), np.zeros(0, np.uint64))["commits"] == 0
    assert not os.environ.get("ZSCRC_FILL_CHUNK")


def test_release_cache_frees_and_recovers(gpu):
    """zscrc_release_cache() frees the fill pipeline's and the scalar
    offload's cached buffers; the next calls allocate them again
    and stay byte-exact."""
    from zeroskip_amd import crc32c as zc
    from zeroskip_amd._lib import lib, stats
    img, commits = _log_images(3)
    o, ln, keep = _writer_spans(commits)
    out = _blank(img, keep)
    zsfile.fill_commits(out, o, ln)
    assert np.array_equal(out, img)
    saved = (lib().zscrc_gpu_min(0), lib().zscrc_gpu_min(1))
    lib().zscrc_set_gpu_min(1 << 20)
    try:
        d = np.random.default_rng(3).integers(0, 256, (9 << 20) + 5, dtype=np.uint8).tobytes()
        assert zc.crc32c_hw(7, d) == oracle.crc32c_hw(7, d)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        lib().zscrc_release_cache()
        free1 = torch.cuda.mem_get_info()[0]
        assert free1 > free0   # device buffers went back
        lib().zscrc_release_cache()   # twice is harmless
        out = _blank(img, keep)
        zsfile.fill_commits(out, o, ln)
        assert np.array_equal(out, img)
        before = stats()
        assert zc.crc32c_hw(7, d) == oracle.crc32c_hw(7, d)
        assert stats()[1] - before[1] == 1   # offloaded again after the release
    finally:
        lib().zscrc_set_gpu_min_pair(*saved)
