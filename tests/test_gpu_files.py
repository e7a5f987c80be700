"""End to end from host memory (zscrc_zs_verify_files): threaded walks,
pinned staging, overlapped H2D and per-group GPU verification, against the
format oracle's verdicts -- clean DBs, corrupt commits / headers / walks,
stale finalise commits, packed files with long commits, pieces smaller than
a file and files smaller than a piece."""
import os

import numpy as np
import pytest

from oracle import zs_format as zf
from tests.test_format_oracle import UUID, build_active
from zeroskip_amd import zsfile

pytestmark = pytest.mark.gpu


def _db(seed, nfiles=40):
    rng = np.random.default_rng(seed)
    imgs, kinds = [], []
    for i in range(nfiles):
        w = zf.FileWriter(UUID, idx=i)
        for t in range(int(rng.integers(1, 60))):
            for _ in range(int(rng.integers(0, 4))):
                w.add(b"%016d" % int(rng.integers(0, 10**9)),
                      rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes())
            w.commit()
        if i % 5 == 2:
            w.finalise()          # a stale zero-length commit after a committed txn
        imgs.append(np.frombuffer(w.image(), np.uint8).copy())
        kinds.append(zsfile.FINALISED)
    recs = sorted((b"%016d" % i, bytes(rng.integers(0, 256, int(rng.integers(0, 9000)), dtype=np.uint8)))
                  for i in range(3000))
    imgs.insert(7, np.frombuffer(zf.packed_file(recs, UUID, 0, 5), np.uint8).copy())   # > 16 MiB: long commit
    kinds.insert(7, zsfile.PACKED)
    return imgs, kinds


def _expected(imgs, kinds):
    commits = bad = stale = 0
    for im, k in zip(imgs, kinds):
        b = im.tobytes()
        if k == zsfile.PACKED:
            cs = zf.packed_check(b)
            commits += 2
            bad += sum(not c["ok"] for c in cs)
            continue
        cs, _, _ = zf.walk(b)
        commits += len(cs)
        prev = None
        for c in cs:
            if not c["ok"]:
                if c["span_len"] == 0 and prev is not None and \
                        zf._commit_check(b, c["commit_off"], prev)[4] == c["stored"]:
                    stale += 1
                else:
                    bad += 1
            prev = zf.oracle.crc32c_hw(0, b[c["span_off"]:c["span_off"] + c["span_len"]])
    return commits, bad, stale


@pytest.mark.parametrize("slot,stage", [(None, "1"), (1 << 20, "1"), (4 << 20, "1"), (None, "0")],
                         ids=["staged-64M", "staged-1M", "staged-4M", "pageable"])
def test_clean_db_end_to_end(gpu, slot, stage):
    """staged (pinned slots, walks queued after each slot's copies) and
    pageable direct copies"""
    imgs, kinds = _db(1)
    if slot:
        os.environ["ZSCRC_FILES_SLOT"] = str(slot)
    os.environ["ZSCRC_FILES_STAGE"] = stage
    try:
        rep = zsfile.verify_files(imgs, kinds, threads=6)
    finally:
        os.environ.pop("ZSCRC_FILES_SLOT", None)
        os.environ.pop("ZSCRC_FILES_STAGE", None)
    assert rep["staged"] == int(stage)
    commits, bad, stale = _expected(imgs, kinds)
    assert bad == 0 and stale >= 3
    assert rep["commits"] == commits and rep["bad_commits"] == 0 and rep["stale_empty_commits"] == stale
    assert rep["header_errors"] == rep["walk_errors"] == 0 and rep["first_bad_what"] == 0
    assert rep["bytes"] == sum(im.nbytes for im in imgs) and rep["files"] == len(imgs)


@pytest.mark.parametrize("stage", ["1", "0"], ids=["staged", "pageable"])
def test_corruptions_located(gpu, stage):
    imgs, kinds = _db(2, nfiles=25)
    os.environ["ZSCRC_FILES_STAGE"] = stage
    # a payload byte of commit 3 of file 11, a header byte of file 4, a packed records byte
    c = zf.walk(imgs[11].tobytes())[0][3]
    imgs[11][c["span_off"] + 9] ^= 0x20
    imgs[4][14] ^= 1
    imgs[7][40 + 12345] ^= 0x80
    os.environ["ZSCRC_FILES_SLOT"] = str(1 << 20)
    try:
        rep = zsfile.verify_files(imgs, kinds)
    finally:
        os.environ.pop("ZSCRC_FILES_SLOT", None)
    commits, bad, stale = _expected(imgs, kinds)
    assert bad == 2 and rep["bad_commits"] == 2 and rep["commits"] == commits
    assert rep["header_errors"] == 1 and rep["first_bad_file"] == 4 and rep["first_bad_what"] == 1
    # a truncated file: the walk stops
    imgs2 = [imgs[0], imgs[1][:-3]]
    rep2 = zsfile.verify_files(imgs2, kinds[:2])
    os.environ.pop("ZSCRC_FILES_STAGE", None)
    assert rep2["walk_errors"] == 1 and rep2["first_bad_file"] == 1 and rep2["first_bad_what"] == 2


def test_empty_and_tiny(gpu):
    rep = zsfile.verify_files([])
    assert rep["files"] == 0 and rep["commits"] == 0
    img = np.frombuffer(build_active(3), np.uint8)
    rep = zsfile.verify_files([np.zeros(0, np.uint8), img])
    assert rep["header_errors"] == 1 and rep["walk_errors"] == 1 and rep["commits"] == 3
    assert rep["first_bad_file"] == 0


def test_all_empty_files(gpu):
    """zero-byte images only: no bytes to stage, every file still walked and
    reported (header and walk errors)"""
    rep = zsfile.verify_files([np.zeros(0, np.uint8)] * 3, [zsfile.FINALISED] * 3)
    assert rep["files"] == 3 and rep["commits"] == 0
    assert rep["header_errors"] == 3 and rep["walk_errors"] == 3 and rep["first_bad_file"] == 0


@pytest.mark.parametrize("devs,group", [([0, 0], None), ([0, 0, 0], 4 << 20), ([0], 3 << 20)],
                         ids=["2slots", "3slots-4MiB-groups", "1slot-3MiB-groups"])
def test_device_slots_split_region(gpu, devs, group):
    """Multi-GPU in one process (zscrc_set_devices; one GPU here, so the slots
    share it): the DB's bytes cut into one share per slot, the packed file's
    records region split across slots and into group-sized pieces whose raw
    registers the host folds -- verdicts equal the format oracle's, with a
    corrupt byte in the split region and one in a finalised file."""
    imgs, kinds = _db(3, nfiles=30)
    c = zf.walk(imgs[20].tobytes())[0][2]
    imgs[20][c["span_off"] + 30] ^= 0x04          # a key payload byte
    mid = imgs[7].nbytes // 2
    imgs[7][mid] ^= 0x10                       # the middle of the packed records region
    assert not zf.packed_check(imgs[7].tobytes())[1]["ok"]
    commits, bad, stale = _expected(imgs, kinds)
    assert bad == 2
    zsfile.set_devices(devs)
    if group:
        os.environ["ZSCRC_FILES_GROUP"] = str(group)
    try:
        assert zsfile.devices() == devs
        rep = zsfile.verify_files(imgs, kinds, threads=4)
        imgs[7][mid] ^= 0x10
        rep_ok7 = zsfile.verify_files(imgs, kinds, threads=4)
    finally:
        zsfile.set_devices(None)
        os.environ.pop("ZSCRC_FILES_GROUP", None)
    assert rep["devices"] == len(devs)
    assert rep["commits"] == commits and rep["stale_empty_commits"] == stale
    assert rep["bad_commits"] == 2 and rep["first_bad_file"] == 7 and rep["first_bad_what"] == 3
    assert rep["header_errors"] == rep["walk_errors"] == 0
    assert rep_ok7["bad_commits"] == 1 and rep_ok7["first_bad_file"] == 20


def test_three_slots_region_spans_every_bound(gpu):
    """zscrc_set_devices([0, 0, 0]): a packed file whose records region holds
    both slot bounds (it is most of the DB's bytes), so all three slots hash
    a piece of it and the host folds three raw registers; one flipped byte on
    each side of each cut is found, and the clean DB verifies."""
    rng = np.random.default_rng(21)
    recs = sorted((b"%016d" % i, bytes(rng.integers(0, 256, int(rng.integers(4000, 8000)), dtype=np.uint8)))
                  for i in range(5000))
    packed = np.frombuffer(zf.packed_file(recs, UUID, 0, 3), np.uint8).copy()
    small = [np.frombuffer(build_active(20, seed=s), np.uint8).copy() for s in (1, 2)]
    imgs = [small[0], packed, small[1]]
    kinds = [zsfile.FINALISED, zsfile.PACKED, zsfile.FINALISED]
    roff = 40
    rlen = zf.packed_check(packed.tobytes())[1]["span_len"]
    W = small[0].nbytes + (packed.nbytes - roff) + small[1].nbytes
    cuts = []
    for s in (1, 2):
        b = W * s // 3 - small[0].nbytes
        assert 0 < b < rlen
        cuts.append(roff + b // 4096 * 4096)
    zsfile.set_devices([0, 0, 0])
    try:
        rep = zsfile.verify_files(imgs, kinds, threads=6)
        assert rep["devices"] == 3 and rep["bad_commits"] == 0 and rep["commits"] == _expected(imgs, kinds)[0]
        for cut in cuts:
            for p in (cut - 1, cut):
                packed[p] ^= 0x40
                r = zsfile.verify_files(imgs, kinds, threads=6)
                packed[p] ^= 0x40
                assert r["bad_commits"] == 1 and r["first_bad_file"] == 1 and r["first_bad_what"] == 3, (p, r)
    finally:
        zsfile.set_devices(None)
