"""Format-layer parity pinned on the reference's OWN code.

oracle/_ref/format_demo runs the reference's writer and verifier --
src/zeroskip-file.c (records, commits :188-393), zeroskip-record.c (walk and
commit verify :188-331), zeroskip-header.c (:30-170) and mfile.c (the CRC
span, :526-546) -- compiled unmodified from /root/reference
(oracle/Makefile `ref-format`), linked against libzscrc.so.

* live (where /root/reference exists): images the reference writes from
  zsdb_add / zsdb_remove / commit steps equal oracle/zs_format.FileWriter's
  byte for byte (short and long keys, deletes restarting the span, finalise
  commits over the stale register, long values and long commits, packed
  files); the reference verifier's verdict on every short commit equals the
  oracle walk's, on clean and corrupted images; the committed fixtures
  regenerate bit for bit.
* fixtures (everywhere, no reference needed): tests/golden/ref_format/ --
  images the reference wrote and its verifier's verdicts -- against the
  oracle walk and the product's host walk / header CRC in libzscrc.  The GPU
  verifier's turn is tests/test_gpu_ref_format.py.
"""
import json
import os
import random
import subprocess

import pytest

from oracle import zs_format as zf
from tests.golden import make_ref_format as mrf
from zeroskip_amd import zsfile

REF = "/root/reference"
HAVE_REF = os.path.isdir(os.path.join(REF, "src")) and os.path.exists("/opt/conda/include/uuid/uuid.h")
live = pytest.mark.skipif(not HAVE_REF, reason="no /root/reference (or its libuuid header) here")
MANIFEST = json.load(open(os.path.join(mrf.OUTDIR, "manifest.json")))
IMAGES = sorted(n for n in MANIFEST if "generator" not in MANIFEST[n] and "repack" not in MANIFEST[n])


def fixture(name):
    with open(os.path.join(mrf.OUTDIR, name + ".zs"), "rb") as f:
        return f.read()


def ref_commit_offsets(rep):
    return sorted([c[0] for c in rep["commits"]] + rep["long_commits"])


# ---------------------------------------------------------------- fixtures
@pytest.mark.parametrize("name", IMAGES)
def test_fixture_oracle_agrees_with_reference_verdict(name):
    img, m = fixture(name), MANIFEST[name]
    rep = m["reference"]
    assert len(img) == m["size"] and rep["header"] == 0
    assert zf.header_check(img)[0]
    rc, stored, computed = zsfile.header_crc(img)
    assert rc == 0 and stored == computed
    if m["kind"] == zsfile.PACKED:
        pc = {c["kind"]: c for c in zf.packed_check(img)}
        assert pc["records"]["ok"] and pc["pointers"]["ok"]
        # the reference walk verifies the records commit, then stops at the
        # pointer count (type byte 0): zeroskip-record.c:324-325
        assert rep["commits"] == [[pc["records"]["commit_off"], 0]]
        assert rep["why"] == "stopped" and rep["stop"] == pc["pointers"]["span_off"]
        off, ln, prc = zsfile.packed_spans(img)
        assert prc == 0
        assert sorted(zip(off.tolist(), ln.tolist())) == sorted(
            (c["span_off"], c["span_len"]) for c in pc.values())
        return
    commits, end, why = zf.walk(img)
    assert why == "end" and end == rep["stop"] == len(img)
    assert [c["commit_off"] for c in commits] == ref_commit_offsets(rep)
    verdict = {c[0]: c[1] == 0 for c in rep["commits"]}
    for c in commits:
        if c["commit_off"] in verdict:
            assert c["ok"] == verdict[c["commit_off"]], c
    off, ln, wrc, wend = zsfile.walk(img)
    assert wrc == zsfile.END and wend == len(img)
    assert (off + ln).tolist() == [c["commit_off"] for c in commits]
    assert ln.tolist() == [c["span_len"] for c in commits]


def test_long_fixture_regenerates_reference_image():
    """The 16 MiB long-commit image is committed as its generator: the oracle
    writer's mirror of the script reproduces the reference-written bytes
    (sha256), and its long commit checks under the writer's semantics."""
    import hashlib
    m = MANIFEST["long_value"]
    img = mrf.long_script().fw.image()
    assert len(img) == m["size"] and hashlib.sha256(img).hexdigest() == m["sha256"]
    assert img[:40].hex() == m["header"]
    for off, words in m["commit_records"].items():
        assert img[int(off):int(off) + len(words) // 2].hex() == words
    commits, end, why = zf.walk(img)
    assert why == "end" and all(c["ok"] for c in commits)
    assert [c["commit_off"] for c in commits] == ref_commit_offsets(m["reference"])
    assert len(m["reference"]["long_commits"]) == 1
    off, ln, wrc, wend = zsfile.walk(img)
    assert wrc == zsfile.END and (off + ln).tolist() == ref_commit_offsets(m["reference"])


@pytest.fixture(scope="module")
def packed_long():
    """The long-FINAL packed image, from the oracle writer (its sha256 is
    the reference-written image's)."""
    return zf.packed_file(mrf.packed_long_records(), *mrf.PACKED_LONG_HDR)


def test_packed_long_fixture_regenerates_reference_image(packed_long):
    """A packed file whose pointer section (17.6 MB) ends in a long FINAL
    commit -- the long-trailer layout the reference's packed verifier checks
    correctly (zeroskip-packed.c:289-312): the oracle writer reproduces the
    reference writer's bytes, the oracle and libzscrc's span walk read it as
    the reference's verifier does, and both corruptions are caught."""
    import hashlib
    m = MANIFEST["packed_long"]
    img = packed_long
    assert len(img) == m["size"] and hashlib.sha256(img).hexdigest() == m["sha256"]
    assert img[:40].hex() == m["header"] and img[-24:].hex() == m["trailer"]
    assert img[-24] == zf.REC_LONG_FINAL
    pc = {c["kind"]: c for c in zf.packed_check(img)}
    assert pc["pointers"]["ok"] and pc["records"]["ok"] and pc["pointers"]["span_len"] > zf.MAX_SHORT_VAL_LEN
    assert m["reference_packed"] == {"rc": 0, "count": mrf.PACKED_LONG_N}
    off, ln, prc = zsfile.packed_spans(img)
    assert prc == 0 and sorted(zip(off.tolist(), ln.tolist())) == sorted(
        (c["span_off"], c["span_len"]) for c in pc.values())
    for k, c in m["corruptions"].items():
        bad = bytearray(img)
        bad[c["offset"]] ^= 0x01
        assert c["reference"]["rc"] == -9                 # ZS_INVALID_DB
        assert not zf.packed_check(bytes(bad))[0]["ok"], k


def _repack_dir(branch):
    d = os.path.join(mrf.OUTDIR, f"repack{branch}")
    m = MANIFEST[f"repack{branch}"]
    inputs = {n: open(os.path.join(d, n), "rb").read() for n in m["inputs"]}
    return m, inputs, open(os.path.join(d, "reference_out.zs"), "rb").read()


def test_repack_fixtures_match_oracle():
    """The reference's own repack (zeroskip-packed.c:384-473 from the memtree
    of finalised files; :617-742 over two packed files) wrote
    tests/golden/ref_format/repackN/reference_out.zs from the inputs beside
    it: the oracle's repack_finalised / repack_packed give the same bytes."""
    import hashlib
    m, inputs, out = _repack_dir(1)
    assert hashlib.sha256(out).hexdigest() == m["sha256"] and m["reference"]["rc"] == 0
    fin = [inputs[n] for n in sorted(inputs, key=lambda n: int(n.rsplit("-", 1)[1])) if n.count("-") == 7]
    assert len(fin) == 5
    assert zf.packed_file(zf.repack_finalised(fin), bytes(range(16)), m["startidx"], m["endidx"]) == out
    m, inputs, out = _repack_dir(2)
    assert hashlib.sha256(out).hexdigest() == m["sha256"] and m["reference"]["rc"] == 0
    older, newer = (inputs[f"zeroskip-{mrf.UUIDSTR}-{r}"] for r in ("4-7", "8-9"))
    assert zf.packed_file(zf.repack_packed(older, newer), bytes(range(16)), 4, 9) == out


def test_fixture_set_covers_bad_and_stale():
    bad = {k: sum(c[1] != 0 for c in MANIFEST[k]["reference"]["commits"]) for k in IMAGES}
    assert bad["active_clean"] == 0 and bad["active_corrupt"] == 3 and bad["active_stale"] > 0


# ---------------------------------------------------------------- live reference
@pytest.fixture(scope="module")
def demo():
    return mrf.build_demo()


@live
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_reference_writer_equals_oracle(demo, tmp_path, seed):
    s = mrf.mixed_script(seed, ntxn=40, long_key=seed % 2 == 0)
    img = s.run(str(tmp_path / "f"))
    assert img == s.fw.image()
    rep = mrf.ref_verify(str(tmp_path / "f"))
    commits, end, _ = zf.walk(img)
    assert rep["header"] == 0 and rep["stop"] == end == len(img)
    assert [c["commit_off"] for c in commits] == ref_commit_offsets(rep)
    assert {c[0]: c[1] == 0 for c in rep["commits"]} == {c["commit_off"]: c["ok"] for c in commits}


@live
def test_reference_verifier_on_corruption(demo, tmp_path):
    s = mrf.mixed_script(21, ntxn=60, stale=False)
    img = s.run(str(tmp_path / "f"))
    commits, _, _ = zf.walk(img)
    rng = random.Random(21)
    for trial in range(6):
        bad = bytearray(img)
        hit = sorted(rng.sample(range(len(commits)), 3))
        for i in hit:
            c = commits[i]
            if trial % 2:                      # the stored CRC in the trailer
                bad[c["commit_off"] + 7] ^= 1 << rng.randrange(8)
            else:                              # a payload byte inside the span
                k = c["span_off"] + 24 + rng.randrange(max(1, c["span_len"] - 48))
                bad[k] ^= 1 << rng.randrange(8)
        p = tmp_path / f"bad{trial}"
        p.write_bytes(bytes(bad))
        rep = mrf.ref_verify(str(p))
        got = {c[0]: c[1] for c in rep["commits"]}
        want = {c["commit_off"]: c["ok"] for c in zf.walk(bytes(bad))[0]}
        assert {o for o, r in got.items() if r != 0} == {commits[i]["commit_off"] for i in hit}
        assert {o: r == 0 for o, r in got.items()} == want


@live
def test_reference_header_verdict(demo, tmp_path):
    img = bytearray(mrf.mixed_script(5, ntxn=3).run(str(tmp_path / "f")))
    for byte in (8, 15, 30, 34, 39):           # version, uuid, start / end index, stored CRC
        bad = bytearray(img)
        bad[byte] ^= 0x04
        p = tmp_path / f"h{byte}"
        p.write_bytes(bytes(bad))
        assert mrf.ref_verify(str(p))["header"] == -9      # ZS_INVALID_DB
        assert not zf.header_check(bytes(bad))[0]
        rc, stored, computed = zsfile.header_crc(bytes(bad))
        assert stored != computed


@live
def test_reference_long_value_long_commit(demo, tmp_path):
    """A span over MAX_SHORT_VAL_LEN: long value record and long commit
    (zeroskip-file.c:266-302); the reference's verifier cannot check a long
    commit (zeroskip-record.c:258), so the oracle's long verify is held to the
    reference WRITER's bytes."""
    s = mrf.long_script()
    img = s.run(str(tmp_path / "f"))
    assert img == s.fw.image()
    rep = mrf.ref_verify(str(tmp_path / "f"))
    commits, end, _ = zf.walk(img)
    assert len(rep["long_commits"]) == 1 and all(c[1] == 0 for c in rep["commits"])
    assert [c["commit_off"] for c in commits] == ref_commit_offsets(rep)
    assert all(c["ok"] for c in commits)
    off, ln, wrc, wend = zsfile.walk(img)
    assert wrc == zsfile.END and (off + ln).tolist() == ref_commit_offsets(rep)


@live
def test_reference_packed_writer_equals_oracle(demo, tmp_path):
    rng = random.Random(9)
    recs = sorted({b"%016d" % rng.randrange(10 ** 9): (None if rng.random() < 0.3 else
                                                      bytes(rng.randrange(256) for _ in range(rng.randint(0, 200))))
                   for _ in range(700)}.items())
    ops, blob = mrf.packed_ops(bytes(range(3, 19)), 4, 9, recs)
    img = mrf.run_ops(ops, blob, str(tmp_path / "p"))
    assert img == zf.packed_file(recs, bytes(range(3, 19)), 4, 9)
    assert zf.packed_records(img) == recs


@live
def test_reference_packed_verifier_on_oracle_image(demo, tmp_path, packed_long):
    """The reference's own zs_packed_file_open over the oracle-written
    long-FINAL image and its corruptions (the manifest's verdicts were taken
    on the reference-written bytes, which the oracle's equal)."""
    p = tmp_path / "pl"
    p.write_bytes(packed_long)
    assert mrf.ref_packed(str(p)) == {"rc": 0, "count": mrf.PACKED_LONG_N}
    for k, c in MANIFEST["packed_long"]["corruptions"].items():
        bad = bytearray(packed_long)
        bad[c["offset"]] ^= 0x01
        p.write_bytes(bytes(bad))
        assert mrf.ref_packed(str(p)) == c["reference"], k
    # the small reference-written packed fixture too
    assert mrf.ref_packed(os.path.join(mrf.OUTDIR, "packed.zs")) == {"rc": 0, "count": 400}


@live
@pytest.mark.parametrize("seed", [41, 42, 43])
def test_reference_repack_finalised_equals_oracle(demo, tmp_path, seed):
    """Branch 1 on the reference's own code (finalised files -> memtree ->
    zs_packed_file_new_from_memtree): the oracle's merge (a later record of a
    key replaces an earlier one, deletes kept) byte for byte."""
    import numpy as np
    rng = np.random.default_rng(seed)
    images, paths = [], []
    for idx in range(2, 2 + int(rng.integers(2, 6))):
        w = zf.FileWriter(bytes(range(16)), idx=idx)
        for t in range(int(rng.integers(20, 120))):
            k = b"%016d" % int(rng.integers(0, 150))
            if rng.integers(0, 6) == 0:
                w.remove(k)
            else:
                w.add(k, rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes())
            if rng.integers(0, 3) == 0:
                w.commit()
        w.commit()
        images.append(w.image())
        paths.append(tmp_path / f"zeroskip-{mrf.UUIDSTR}-{idx}-{idx}")
        paths[-1].write_bytes(images[-1])
    out = tmp_path / "out"
    assert mrf.ref_repack(1, str(out), bytes(range(16)), 2, 1 + len(images), [str(p) for p in paths]) == {"rc": 0}
    want = zf.packed_file(zf.repack_finalised(images), bytes(range(16)), 2, 1 + len(images))
    assert out.read_bytes() == want


@live
def test_reference_repack_packed_and_its_delete_quirk(demo, tmp_path):
    """Branch 2 on the reference's own code (zs_iterator_* +
    zs_packed_file_new_from_packed_files).  Without deletes its output is
    the oracle's merge (the older of the two newest files wins a key)
    byte for byte -- so the product's, which the GPU tests hold to the
    oracle.  With deletes the reference loses data: its packed iterator sets
    `deleted` on the first delete it steps onto and never clears it
    (zeroskip-iterator.c:258-259), so every later record of that source is
    dropped.  ref_merge_packed restates that exactly (bytes equal); the
    product keeps the records, as the oracle does."""
    import numpy as np
    rng = np.random.default_rng(44)

    def recs(n, lo, hi, pdel):
        return sorted({b"%016d" % int(rng.integers(lo, hi)):
                       (None if pdel and rng.integers(0, pdel) == 0 else
                        rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes())
                       for _ in range(n)}.items())
    for pdel in (0, 12, 4):
        spec = {(0, 3): recs(100, 0, 900, pdel), (4, 7): recs(700, 300, 9000, pdel), (8, 9): recs(300, 0, 3000, pdel)}
        imgs = {k: zf.packed_file(r, bytes(range(16)), *k) for k, r in spec.items()}
        paths = []
        for (a, b), img in imgs.items():
            paths.append(tmp_path / f"zeroskip-{mrf.UUIDSTR}-{a}-{b}")
            paths[-1].write_bytes(img)
        out = tmp_path / f"out{pdel}"
        assert mrf.ref_repack(2, str(out), bytes(range(16)), 4, 9, [str(p) for p in paths]) == {"rc": 0}
        got = out.read_bytes()
        quirk = zf.packed_file(mrf.ref_merge_packed([(2, spec[(4, 7)]), (1, spec[(8, 9)])]), bytes(range(16)), 4, 9)
        fixed = zf.packed_file(zf.repack_packed(imgs[(4, 7)], imgs[(8, 9)]), bytes(range(16)), 4, 9)
        assert got == quirk
        assert (got == fixed) == (pdel == 0)
        if pdel:
            assert len(zf.packed_records(got)) < len(zf.packed_records(fixed))
        for p in paths:
            p.unlink()


@live
def test_committed_fixtures_regenerate(demo, tmp_path):
    for name, (img, kind) in mrf.fixtures().items():
        assert img == fixture(name), name
        p = tmp_path / name
        p.write_bytes(img)
        assert mrf.ref_verify(str(p)) == MANIFEST[name]["reference"]
        assert MANIFEST[name]["kind"] == kind
    assert mrf.long_fixture() == MANIFEST["long_value"]
    import hashlib
    for branch, inputs in ((1, mrf.repack1_inputs()), (2, mrf.repack2_inputs())):
        m, committed, out = _repack_dir(branch)
        assert inputs == committed
        srcs = [n for n in sorted(inputs) if branch == 2 or n.count("-") == 7]
        d = tmp_path / f"r{branch}"
        d.mkdir()
        for n, img in inputs.items():
            (d / n).write_bytes(img)
        assert mrf.ref_repack(branch, str(d / "o"), bytes(range(16)), m["startidx"], m["endidx"],
                              [str(d / n) for n in srcs]) == m["reference"]
        assert hashlib.sha256((d / "o").read_bytes()).hexdigest() == m["sha256"]


@live
def test_demo_links_reference_objects_unmodified(demo):
    """format_demo's CRCs resolve in libzscrc.so, and the reference objects it
    links are the ones `ref-lib` compiled from /root/reference."""
    out = subprocess.run(["ldd", demo], capture_output=True, text=True, check=True).stdout
    assert "libzscrc.so" in out and "libuuid" not in out
    und = subprocess.run(["nm", "-u", demo], capture_output=True, text=True, check=True).stdout.split()
    assert {"crc32c", "crc32c_hw"} <= set(und)
