"""The GPU verifiers on images the reference's OWN writer produced, held to
the reference's OWN verifier (tests/golden/ref_format/: written and judged by
src/zeroskip-file.c / -record.c / -header.c compiled unmodified, see
tests/golden/make_ref_format.py and tests/test_reference_format.py).

* zscrc_zs_verify_image: the bad commits are exactly the ones the reference
  rejects (ZS_INVALID_DB from zs_read_and_verify_commit_record, record.c:227-231),
  finalise commits over the stale register included;
* zscrc_zs_verify_files over the whole set: the same commits, with the
  finalise commits that chain from the previous span's CRC reported as
  stale (src/mfile.c:534-546) rather than bad.
"""
import hashlib
import json
import os

import pytest

from oracle import oracle
from oracle import zs_format as zf
from zeroskip_amd import zsfile

pytestmark = pytest.mark.gpu

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_format")
MANIFEST = json.load(open(os.path.join(DIR, "manifest.json")))
IMAGES = sorted(n for n in MANIFEST if "generator" not in MANIFEST[n] and "repack" not in MANIFEST[n])


def fixture(name):
    with open(os.path.join(DIR, name + ".zs"), "rb") as f:
        return f.read()


def ref_rejected(name):
    return [c[0] for c in MANIFEST[name]["reference"]["commits"] if c[1] != 0]


def stale_chained(img):
    """Rejected zero-length commits the oracle reads as finalise commits
    chained from the previous span's CRC (FileWriter.finalise)."""
    out, prev = 0, None
    for c in zf.walk(img)[0]:
        if not c["ok"] and c["span_len"] == 0 and prev is not None:
            out += zf._commit_check(img, c["commit_off"], seed=prev)[3:5] == (c["stored"],) * 2
        if c["span_len"]:
            prev = oracle.crc32c_hw(0, bytes(img[c["span_off"]:c["commit_off"]]))
    return out


@pytest.mark.parametrize("name", [n for n in IMAGES if MANIFEST[n]["kind"] == zsfile.ACTIVE])
def test_verify_image_matches_reference_verifier(gpu, name):
    img = fixture(name)
    rep = zsfile.verify_image(img)
    ref = MANIFEST[name]["reference"]
    commits = [c["commit_off"] for c in zf.walk(img)[0]]
    bad = ref_rejected(name)
    assert rep["header_rc"] == 0 and rep["walk_rc"] == zsfile.END and rep["end_off"] == ref["stop"]
    assert rep["n_commits"] == len(ref["commits"]) + len(ref["long_commits"]) == len(commits)
    assert rep["n_bad"] == len(bad)
    if bad:
        assert commits[rep["first_bad"]] == bad[0]


def test_verify_image_packed_reference_written(gpu):
    img = fixture("packed")
    rep = zsfile.verify_image(img, zsfile.PACKED)
    assert rep["header_rc"] == 0 and rep["n_commits"] == 2 and rep["n_bad"] == 0
    bad = bytearray(img)
    bad[MANIFEST["packed"]["reference"]["stop"] + 11] ^= 0x10   # a pointer word
    rep = zsfile.verify_image(bytes(bad), zsfile.PACKED)
    assert rep["n_bad"] == 1


def test_verify_image_long_commit_reference_written(gpu):
    """The 16 MiB long-commit image, regenerated from its generator (its
    sha256 is the reference-written image's): every commit -- the long one
    on the writer's semantics -- verifies on the GPU; one flipped byte in
    the 16 MiB value is found in the long commit."""
    import hashlib
    from tests.golden import make_ref_format as mrf
    m = MANIFEST["long_value"]
    img = bytearray(mrf.long_script().fw.image())
    assert hashlib.sha256(img).hexdigest() == m["sha256"]
    rep = zsfile.verify_image(bytes(img))
    assert rep["header_rc"] == 0 and rep["walk_rc"] == zsfile.END
    assert rep["n_commits"] == 3 and rep["n_bad"] == 0
    img[8 * 1024 * 1024 + 12345] ^= 0x01
    rep = zsfile.verify_image(bytes(img))
    assert rep["n_bad"] == 1 and rep["first_bad"] == 1


def test_verify_image_packed_long_final(gpu):
    """The long-FINAL packed image (regenerated; sha256 of the
    reference-written bytes): both commits verify on the GPU, and each
    corruption the reference's packed verifier rejects is one bad commit."""
    import hashlib
    from tests.golden import make_ref_format as mrf
    m = MANIFEST["packed_long"]
    img = zf.packed_file(mrf.packed_long_records(), *mrf.PACKED_LONG_HDR)
    assert hashlib.sha256(img).hexdigest() == m["sha256"]
    rep = zsfile.verify_image(img, zsfile.PACKED)
    assert rep["header_rc"] == 0 and rep["n_commits"] == 2 and rep["n_bad"] == 0
    for k, c in m["corruptions"].items():
        bad = bytearray(img)
        bad[c["offset"]] ^= 0x01
        assert c["reference"]["rc"] == -9
        rep = zsfile.verify_image(bytes(bad), zsfile.PACKED)
        assert rep["n_bad"] == 1, (k, rep)


def test_verify_files_matches_reference_verifier(gpu):
    names = IMAGES
    imgs = [fixture(n) for n in names]
    kinds = [MANIFEST[n]["kind"] for n in names]
    rep = zsfile.verify_files(imgs, kinds)
    active = [n for n in names if MANIFEST[n]["kind"] == zsfile.ACTIVE]
    rejected = sum(len(ref_rejected(n)) for n in active)
    stale = sum(stale_chained(fixture(n)) for n in active)
    assert stale > 0
    assert rep["files"] == len(names) and rep["header_errors"] == 0 and rep["walk_errors"] == 0
    assert rep["bad_commits"] + rep["stale_empty_commits"] == rejected
    assert rep["stale_empty_commits"] == stale


@pytest.mark.parametrize("branch", [1, 2])
def test_product_repack_equals_reference_repack(gpu, tmp_path, branch):
    """zscrc_zs_repack (the product's zsdb_repack, GPU checksums) over the
    inputs the reference's own repack read (tests/golden/ref_format/repackN,
    with a .zsdb): the packed file it writes is the reference's output byte
    for byte -- branch 1 from five finalised files, branch 2 from three
    packed files (delete-free: the reference's merge quirk does not apply)."""
    import shutil
    from zeroskip_amd import repack
    m = MANIFEST[f"repack{branch}"]
    src = os.path.join(DIR, f"repack{branch}")
    for n in m["inputs"]:
        shutil.copy(os.path.join(src, n), tmp_path / n)
    curidx = 8 if branch == 1 else 10
    uuidstr = m["out_name"].split("-", 1)[1].rsplit("-", 2)[0]
    (tmp_path / ".zsdb").write_bytes(zf.dotzsdb_bytes(4096, uuidstr.encode() + b"\0", curidx))
    rep = repack.repack_dir(str(tmp_path))
    assert rep["branch"] == branch and os.path.basename(rep["path"]) == m["out_name"]
    with open(os.path.join(src, "reference_out.zs"), "rb") as f:
        want = f.read()
    with open(tmp_path / m["out_name"], "rb") as f:
        assert f.read() == want


def test_repack_reference_compat_on_deletes(gpu, tmp_path):
    """Branch 2 on packed files that hold deletes (tests/golden/ref_format/
    repack2d: the reference's own repack output on them).  With
    ZSCRC_REPACK_REFERENCE_COMPAT the product writes the reference's bytes,
    records lost to its iterator's sticky `deleted` flag included
    (src/zeroskip-iterator.c:258-259).  The default keeps them: its output is
    the format oracle's merge, and the two differ by exactly the set the
    restatement of the reference's merge (make_ref_format.ref_merge_packed)
    predicts -- the records the reference drops, and the delete record it
    writes for a source whose first record is a delete."""
    import shutil
    from tests.golden.make_ref_format import ref_merge_packed
    from zeroskip_amd import repack
    m = MANIFEST["repack2d"]
    src = os.path.join(DIR, "repack2d")
    with open(os.path.join(src, "reference_out.zs"), "rb") as f:
        ref_out = f.read()
    assert hashlib.sha256(ref_out).hexdigest() == m["sha256"]
    uuidstr = m["out_name"].split("-", 1)[1].rsplit("-", 2)[0]
    outs = {}
    for compat in (True, False):
        d = tmp_path / ("compat" if compat else "default")
        d.mkdir()
        for n in m["inputs"]:
            shutil.copy(os.path.join(src, n), d / n)
        (d / ".zsdb").write_bytes(zf.dotzsdb_bytes(4096, uuidstr.encode() + b"\0", 10))
        rep = repack.repack_dir(str(d), reference_compat=compat)
        assert rep["branch"] == 2 and os.path.basename(rep["path"]) == m["out_name"]
        with open(d / m["out_name"], "rb") as f:
            outs[compat] = f.read()
        r = zsfile.verify_image(outs[compat], zsfile.PACKED)
        assert r["n_bad"] == 0 and r["n_commits"] == 2
    assert outs[True] == ref_out
    older, newer = (open(os.path.join(src, n), "rb").read() for n in sorted(m["inputs"])[1:])
    uuid = bytes(range(16))
    assert outs[False] == zf.packed_file(zf.repack_packed(older, newer), uuid, 4, 9)
    quirk = ref_merge_packed([(2, zf.packed_records(older)), (1, zf.packed_records(newer))])
    assert zf.packed_file(quirk, uuid, 4, 9) == ref_out
    ref_recs, def_recs = zf.packed_records(ref_out), zf.packed_records(outs[False])
    kept_beyond = [r for r in def_recs if r not in ref_recs]
    ref_only = [r for r in ref_recs if r not in def_recs]
    # what the default keeps beyond the reference: every record the quirk drops
    assert len(kept_beyond) > 50 and all(v is not None for _, v in kept_beyond)
    assert set(kept_beyond) == set(zf.repack_packed(older, newer)) - set(quirk)
    # and the reference writes the newest file's leading delete as a delete record
    assert ref_only == [(b"%016d" % 0, None)]
