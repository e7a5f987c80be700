"""GPU verification of zeroskip file images against the format oracle:
every commit CRC (span + host-order trailer) recomputed on the device."""
import numpy as np
import pytest
import torch

from oracle import zs_format as zf
from tests.test_format_oracle import UUID, build_active
from zeroskip_amd import zsfile

pytestmark = pytest.mark.gpu


def test_active_image_all_commits_ok(gpu):
    img = build_active(200, seed=11)
    rep = zsfile.verify_image(img)
    assert rep["header_rc"] == 0 and rep["header_stored"] == rep["header_computed"]
    assert rep["walk_rc"] == zsfile.END and rep["n_commits"] == 200 and rep["n_bad"] == 0


def test_corruption_located(gpu):
    img = bytearray(build_active(200, seed=12))
    commits, _, _ = zf.walk(bytes(img))
    img[commits[137]["span_off"] + 30] ^= 0x01     # key payload byte
    rep = zsfile.verify_image(bytes(img))
    assert rep["walk_rc"] == zsfile.END and rep["n_bad"] == 1 and rep["first_bad"] == 137
    # a corrupted record length derails the walk itself (as in the reference)
    img[commits[137]["span_off"] + 30] ^= 0x01
    img[commits[137]["span_off"] + 5] ^= 0x01      # value-offset bits of the key word
    rep = zsfile.verify_image(bytes(img))
    assert rep["walk_rc"] != zsfile.END or rep["n_bad"] > 0
    img2 = bytearray(build_active(50, seed=13))
    c = zf.walk(bytes(img2))[0][20]
    img2[c["commit_off"] + 7] ^= 0x80            # stored CRC byte
    rep = zsfile.verify_image(bytes(img2))
    assert rep["n_bad"] == 1 and rep["first_bad"] == 20


def test_long_commit_and_packed(gpu):
    w = zf.FileWriter(UUID)
    w.add(b"k" * 100, np.random.default_rng(3).integers(0, 256, (17 << 20) + 5, dtype=np.uint8).tobytes())
    w.commit()
    w.add(b"small", b"v")
    w.commit()
    rep = zsfile.verify_image(w.image())
    assert rep["n_commits"] == 2 and rep["n_bad"] == 0
    recs = sorted((b"%016d" % i, None if i % 11 == 0 else b"y" * (i % 300)) for i in range(5000))
    rep = zsfile.verify_image(zf.packed_file(recs, UUID, 2, 9), zsfile.PACKED)
    assert rep["walk_rc"] == 0 and rep["n_commits"] == 2 and rep["n_bad"] == 0


def test_device_commits_match_oracle_crcs(gpu):
    # several files concatenated in one device image; commit spans of all
    # sizes (empty txn commits, deletes restarting the span, multi-record txns)
    imgs, offs, lens, want = [], [], [], []
    base = 0
    for s in range(6):
        rng = np.random.default_rng(100 + s)
        w = zf.FileWriter(UUID, idx=s)
        for t in range(300):
            for _ in range(int(rng.integers(0, 5))):
                w.add(b"%016d" % int(rng.integers(0, 10**9)),
                      rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes())
            if t % 13 == 5:
                w.remove(b"%016d" % t)
            w.commit()
        img = w.image()
        commits, _, _ = zf.walk(img)
        for c in commits:
            offs.append(base + c["span_off"])
            lens.append(c["span_len"])
            want.append(c["computed"])
        imgs.append(img)
        base += len(img)
    d = torch.from_numpy(np.frombuffer(b"".join(imgs), dtype=np.uint8).copy()).cuda()
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda")
    d_len = torch.tensor(lens, dtype=torch.int64, device="cuda")
    # unbounded, the walk's exact bound, a short (wrong) bound, and the
    # one-kernel path over the short spans only
    short = [i for i, n in enumerate(lens) if n <= 640]
    for mx, ix in [(None, None), (max(lens), None), (64, None), (640, short)]:
        o, ln = (d_off, d_len) if ix is None else (d_off[ix], d_len[ix])
        crc, st = zsfile.verify_commits(d, o, ln, max_len=mx)
        torch.cuda.synchronize()
        w = np.array(want, dtype=np.uint32) if ix is None else np.array(want, dtype=np.uint32)[ix]
        assert (st.cpu().numpy() == 1).all(), mx
        assert (crc.cpu().numpy().view(np.uint32) == w).all(), mx


def test_write_commits_matches_writer(gpu):
    # GPU writer side: zero every stored CRC, recompute + store on the device,
    # compare with the oracle writer's image byte for byte
    img = build_active(300, seed=21)
    commits, _, _ = zf.walk(img)
    blank = bytearray(img)
    for c in commits:
        blank[c["commit_off"] + 4:c["commit_off"] + 8] = b"\0\0\0\0"
    d = torch.from_numpy(np.frombuffer(bytes(blank), dtype=np.uint8).copy()).cuda()
    offs = torch.tensor([c["span_off"] for c in commits], dtype=torch.int64, device="cuda")
    lens = torch.tensor([c["span_len"] for c in commits], dtype=torch.int64, device="cuda")
    crc = zsfile.write_commits(d, offs, lens)
    torch.cuda.synchronize()
    assert d.cpu().numpy().tobytes() == img
    # bounded by the walk's longest span: one kernel, same bytes
    d2 = torch.from_numpy(np.frombuffer(bytes(blank), dtype=np.uint8).copy()).cuda()
    crc2 = zsfile.write_commits(d2, offs, lens, max_len=int(lens.max().item()))
    torch.cuda.synchronize()
    assert d2.cpu().numpy().tobytes() == img and torch.equal(crc2, crc)
    assert (crc.cpu().numpy().view(np.uint32) == np.array([c["stored"] for c in commits], np.uint32)).all()


@pytest.mark.parametrize("bound", ["none", "exact", "short"])
def test_commits_bounded_by_image(gpu, bound):
    """d_status 2 (and no read or write outside the image) for spans whose
    commit word, or a long commit's 24 bytes, do not lie inside image_size;
    a commit whose word ends exactly at the image end still verifies."""
    w = zf.FileWriter(UUID)
    rng = np.random.default_rng(77)
    for t in range(40):
        w.add(b"%016d" % t, rng.integers(0, 256, int(rng.integers(0, 900)), dtype=np.uint8).tobytes())
        w.commit()
    w.add(b"L" * 16, rng.integers(0, 256, (16 << 20) + 40, dtype=np.uint8).tobytes())   # long commit last
    w.commit()
    img = w.image()
    commits, _, _ = zf.walk(img)
    assert img[commits[-1]["commit_off"]] == zf.REC_LONG_COMMIT and commits[-1]["commit_off"] + 24 == len(img)
    host = np.frombuffer(img + b"\xab" * 64, dtype=np.uint8).copy()
    full = torch.from_numpy(host).cuda()
    offs = [c["span_off"] for c in commits]
    lens = [c["span_len"] for c in commits]
    c39 = commits[39]
    # extra descriptors: span past the end, offset past the end, huge length
    offs += [c39["span_off"], len(img) + 100, 40]
    lens += [c39["span_len"] + 64, 0, 1 << 62]
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda")
    d_len = torch.tensor(lens, dtype=torch.int64, device="cuda")
    mx = {"none": None, "exact": max(lens), "short": 640}[bound]
    n = len(commits)

    def status(size):
        _, st = zsfile.verify_commits(full[:size], d_off, d_len, max_len=mx)
        torch.cuda.synchronize()
        return st.cpu().numpy()

    st = status(len(img))                        # the long commit's 24 bytes end at the image end
    assert (st[:n] == 1).all() and (st[n:] == 2).all(), st
    st = status(len(img) - 1)                    # one byte short: the long commit has no room
    assert (st[:n - 1] == 1).all() and st[n - 1] == 2 and (st[n:] == 2).all()
    st = status(commits[-1]["commit_off"] + 8)   # the long commit's first word only
    assert (st[:n - 1] == 1).all() and st[n - 1] == 2
    st = status(c39["commit_off"] + 8)           # short commit word ends at the image end
    assert (st[:40] == 1).all() and st[40] == 2
    st = status(c39["commit_off"])               # span ends at the image end: no commit word
    assert (st[:39] == 1).all() and st[39] == 2 and st[40] == 2
    # writer: a commit word outside the image is neither read nor written
    blank = host.copy()
    for c in commits:
        blank[c["commit_off"] + (20 if c is commits[-1] else 4):][:4] = 0
    d = torch.from_numpy(blank).cuda()
    size = c39["commit_off"] + 6
    _, wst = zsfile.write_commits(d[:size], d_off, d_len, max_len=mx, status=True)
    torch.cuda.synchronize()
    wst = wst.cpu().numpy()
    assert (wst[:39] == 1).all() and (wst[39:] == 2).all()
    got = d.cpu().numpy()
    want = blank.copy()
    want[:c39["commit_off"]] = host[:c39["commit_off"]]
    assert np.array_equal(got, want)
