"""The bulk C checker (oracle/zs_bulk_oracle.c) against the Python format
oracle (oracle/zs_format.py) on the same images: the record walk, packed
files, the threaded span CRC and the CPU commit writer.  These are what
bench.py's configs 4 / 5 and the GPU tests use to check full-size images, so
they are pinned here first.  CPU only."""
import struct

import numpy as np

from oracle import oracle
from oracle import zs_format as zf

UUID = bytes(range(16))


def _active(ntx, seed, long_value=False):
    rng = np.random.default_rng(seed)
    w = zf.FileWriter(UUID, idx=5)
    for t in range(ntx):
        for _ in range(int(rng.integers(1, 4))):
            w.add(b"%016d" % int(rng.integers(0, 10**9)),
                  rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8).tobytes())
        if t % 5 == 2:
            w.remove(b"%016d" % t)
        if long_value and t == ntx // 2:
            w.add(b"long", bytes(zf.MAX_SHORT_VAL_LEN + 100))   # a long commit (> 16 MiB span)
        w.commit()
    w.finalise()          # the stale zero-length commit (mfile.c:534-546)
    return np.frombuffer(w.image(), dtype=np.uint8).copy()


def _py_walk(img):
    commits, end, why = zf.walk(img.tobytes())
    return commits, end, why


def test_walk_matches_python_walk():
    imgs = [_active(40, s) for s in range(6)]
    bad = imgs[3].copy()
    c3 = _py_walk(bad)[0]
    bad[c3[7]["span_off"] + 5] ^= 0x10
    imgs.append(bad)
    out = oracle.walk_images(imgs, threads=3)
    for img, row in zip(imgs, out):
        commits, end, why = _py_walk(img)
        ok = sum(c["ok"] for c in commits)
        assert int(row[0]) == len(commits) and int(row[1]) == ok and int(row[2]) == end
        assert (int(row[3]) == 0) == (why == "end")
        first = next((c for c in commits if not c["ok"]), None)
        assert int(row[4]) == (first["commit_off"] if first else 2**64 - 1)
    # the stale finalise commit is the one failure of a clean file; the
    # corrupted span adds exactly one more
    assert [int(r[0] - r[1]) for r in out] == [1] * 6 + [2]
    assert int(out[-1][5]) == 7


def test_walk_long_commit():
    img = _active(6, 9, long_value=True)
    row = oracle.walk_images([img])[0]
    commits, end, _ = _py_walk(img)
    assert any(c["span_len"] > zf.MAX_SHORT_VAL_LEN for c in commits)
    assert int(row[0]) == len(commits) and int(row[1]) == len(commits) - 1 and int(row[2]) == end


def test_walk_truncated_and_bad_type():
    img = _active(10, 2)
    row = oracle.walk_images([img[:-3]])[0]
    assert int(row[3]) in (1, 3)
    bad = img.copy()
    bad[zf.HDR_SIZE] = zf.REC_FINAL          # the walk does not advance over FINAL
    row = oracle.walk_images([bad])[0]
    assert int(row[0]) == 0 and int(row[3]) == 2


def test_span_crc_threads():
    data = np.random.default_rng(3).integers(0, 256, (5 << 20) + 13, dtype=np.uint8)
    want = oracle.crc32c_hw(0, data)
    for t in (1, 2, 7, 16):
        assert oracle.span_crc(data, threads=t) == want


def test_packed_image():
    rng = np.random.default_rng(4)
    recs = sorted((b"%016d" % i, rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes())
                  for i in range(300))
    img = np.frombuffer(zf.packed_file(recs, UUID, 0, 7), dtype=np.uint8).copy()
    py = zf.packed_check(img.tobytes())
    got = oracle.packed_image(img, threads=4)
    assert got["pointers"]["status"] == 1 and got["records"]["status"] == 1
    assert got["pointers"]["span_off"] == py[0]["span_off"] and got["pointers"]["span_len"] == py[0]["span_len"]
    assert got["records"]["span_off"] == py[1]["span_off"] and got["records"]["span_len"] == py[1]["span_len"]
    for where, which in ((zf.HDR_SIZE + 100, "records"), (py[0]["span_off"] + 20, "pointers")):
        b = img.copy()
        b[where] ^= 1
        g = oracle.packed_image(b, threads=2)
        assert g[which]["status"] == 0
        assert g["records" if which == "pointers" else "pointers"]["status"] == 1


def test_cpu_writer_byte_exact():
    """oracle.write_commits over an image whose commit CRC fields are zero
    reproduces the format oracle's writer byte for byte (short and long
    commits, COMMIT and FINAL types), and commit_crcs returns those CRCs."""
    imgs = [_active(30, 11), _active(5, 12, long_value=True)]
    for img in imgs:
        commits, _, _ = _py_walk(img)
        blank = img.copy()
        offs, lens = [], []
        for c in commits:
            at = c["commit_off"]
            offs.append(c["span_off"])
            lens.append(c["span_len"])
            if c["span_len"] > zf.MAX_SHORT_VAL_LEN:
                blank[at + 20:at + 24] = 0
            else:
                blank[at + 4:at + 8] = 0
        # the stale finalise commit is not the writer's (it chains from the
        # previous span): leave it out, as log writers do
        keep = [i for i, c in enumerate(commits) if c["span_len"] or i == 0]
        o, ln = np.array(offs)[keep], np.array(lens)[keep]
        crcs = oracle.commit_crcs(img, o, ln, threads=2)
        assert [int(x) for x in crcs] == [commits[i]["stored"] for i in keep]
        oracle.write_commits(blank, o, ln, threads=3)
        last = commits[-1]
        if last["span_len"] == 0:
            at = last["commit_off"]
            blank[at:at + 8] = img[at:at + 8]
        assert np.array_equal(blank, img)


def test_cpu_writer_final_type():
    span = bytes(range(64))
    w = zf.commit_record(oracle.crc32c_hw(0, span), len(span), final=True)
    img = np.frombuffer(span + bytes([zf.REC_FINAL]) + bytes(7), dtype=np.uint8).copy()
    oracle.write_commits(img, [0], [64])
    assert img[64:].tobytes() == w
    assert struct.unpack(">Q", w)[0] >> 56 == zf.REC_FINAL


def test_cpu_writer_db_and_bench_checkers():
    """tools/zsdb_gen.py writer="cpu" builds a config-5-shaped DB without a
    GPU; bench.py's full-size checkers pass it and catch a corruption in each
    kind of CRC'd object."""
    import torch

    import bench
    from tools import zsdb_gen as zg
    from zeroskip_amd import consistent as cs
    db = zg.make_db(device="cpu", packed=2, packed_region_bytes=17 << 20, finalised=3, active_pairs=50,
                    writer="cpu")
    d = cs.open_db(db)
    p = bench.oracle_check_db(d, 3)
    assert p["mismatches"] == 0 and p["stale_finalise"] == 3 and p["regions_checked"] == 2
    assert p["region_bytes"] > 2 * zf.MAX_SHORT_VAL_LEN and p["dotzsdb_ok"]
    names = sorted(k for k in db if k != ".zsdb")
    for victim, at in ((names[0], 1000), (names[-1], 100), (names[-2], 39)):
        db2 = dict(db)
        t = db[victim].clone()
        t[at] ^= 4
        db2[victim] = t
        assert bench.oracle_check_db(cs.open_db(db2), 3)["mismatches"] >= 1
    # the log checker on finalised files: every commit's CRC against "GPU" crcs
    logs = torch.stack([db[n] for n in names if n.count("-") == 7 and n.split("-")[-1] == n.split("-")[-2]][:3])
    size = logs.shape[1]
    ppf = (size - 40 - 8) // 320
    offs, lens = zg.log_spans(3, ppf, True, True, "cpu")
    o, ln = offs.numpy(), lens.numpy()
    crc = oracle.commit_crcs(logs.numpy().reshape(-1), o, ln)
    r = bench.oracle_check_logs(logs.numpy(), o, ln, crc, 1)
    assert r["mismatches"] == 0 and r["commits_walked"] == len(o) and r["stale_finalise"] == 3
    crc[5] ^= 1
    assert bench.oracle_check_logs(logs.numpy(), o, ln, crc, 1)["mismatches"] == 1
