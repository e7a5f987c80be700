"""The packed-file writer (zscrc_pack_*, the repack output path of
src/zeroskip-packed.c:384-473) against the format oracle: byte-for-byte equal
files, records-region and pointer-section CRCs computed on the GPU."""
import os

import numpy as np
import pytest

from oracle import oracle
from oracle import zs_format as zf
from zeroskip_amd import repack, zsfile
from zeroskip_amd._lib import stats

pytestmark = pytest.mark.gpu

UUID = bytes(range(16))
UUIDSTR = "00010203-0405-0607-0809-0a0b0c0d0e0f"


def _records(n, seed, maxval=600, deletes=True):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        key = b"%016d" % (i * 7)
        if deletes and i % 13 == 4:
            recs.append((key, None))
        else:
            recs.append((key, rng.integers(0, 256, int(rng.integers(0, maxval)), dtype=np.uint8).tobytes()))
    return recs


def _pack(path, recs, chunk=0, start=2, end=9):
    before = stats()
    with repack.Packer(str(path), UUID, start, end, chunk_bytes=chunk) as p:
        for k, v in recs:
            p.add(k, v)
    after = stats()
    assert after[3] - before[3] >= p.report["region_bytes"], "records region not checksummed on the GPU"
    return p.report, open(path, "rb").read()


@pytest.mark.parametrize("chunk", [0, 4096, 65536 + 4096])
def test_pack_matches_oracle_short(gpu, tmp_path, chunk):
    recs = _records(3000, 5)
    rep, img = _pack(tmp_path / "p", recs, chunk)
    want = zf.packed_file(recs, UUID, 2, 9)
    assert img == want
    assert rep["records"] == len(recs) and rep["file_bytes"] == len(want)
    assert rep["region_crc"] == oracle.crc32c_hw(0, want[40:40 + rep["region_bytes"]])
    r = zsfile.verify_image(img, zsfile.PACKED)
    assert r["walk_rc"] == 0 and r["n_commits"] == 2 and r["n_bad"] == 0


def test_pack_batch_api(gpu, tmp_path):
    """zscrc_pack_add_batch (Packer.add_many / add_arrays) writes the same
    bytes as per-record adds: deletes, empty values, shared value bytes."""
    recs = _records(3000, 6)
    recs[10] = (recs[10][0], b"")
    want = zf.packed_file(recs, UUID, 2, 9)
    with repack.Packer(str(tmp_path / "m"), UUID, 2, 9, chunk_bytes=8192) as p:
        p.add_many(recs[:1000])
        p.add_many(recs[1000:])
    assert open(tmp_path / "m", "rb").read() == want
    # values sharing bytes: record i -> the same 40 bytes at offset 8 * (i % 5)
    vals = np.arange(80, dtype=np.uint8)
    keys = [b"k%07d" % i for i in range(500)]
    kb = np.frombuffer(b"".join(keys), dtype=np.uint8)
    koff = np.arange(500, dtype=np.uint64) * 8
    klen = np.full(500, 8, np.uint64)
    voff = (np.arange(500, dtype=np.uint64) % 5) * 8
    voff[7] = ~np.uint64(0)
    vlen = np.full(500, 40, np.uint64)
    with repack.Packer(str(tmp_path / "a"), UUID, 2, 9) as p:
        p.add_arrays(kb, koff, klen, vals, voff, vlen)
    recs2 = [(k, None if i == 7 else vals[8 * (i % 5):8 * (i % 5) + 40].tobytes()) for i, k in enumerate(keys)]
    assert open(tmp_path / "a", "rb").read() == zf.packed_file(recs2, UUID, 2, 9)


@pytest.mark.parametrize("chunk", [0, 1 << 20])
def test_pack_long_commit_long_records(gpu, tmp_path, chunk):
    """Records region above 16 MiB (long commit), a 17 MiB value (long value
    record), a 70,000-byte key (long key record), an empty value."""
    recs = _records(2500, 9, maxval=9000)
    big = np.random.default_rng(1).integers(0, 256, (17 << 20) + 3, dtype=np.uint8).tobytes()
    recs.insert(100, (b"%016d" % 700 + b"+big", big))
    recs.insert(200, (b"%016d" % 1400 + b"+long-key" + b"q" * 70000, b"v" * 33))
    recs.insert(300, (b"%016d" % 2100 + b"+empty", b""))
    rep, img = _pack(tmp_path / "p", recs, chunk)
    want = zf.packed_file(recs, UUID, 2, 9)
    assert rep["region_bytes"] > zf.MAX_SHORT_VAL_LEN
    assert img == want
    chk = zf.packed_check(img)
    assert all(c["ok"] for c in chk)
    assert chk[1]["stored"] == rep["commit_crc"] and chk[0]["stored"] == rep["final_crc"]


def test_pack_empty(gpu, tmp_path):
    rep, img = _pack(tmp_path / "p", [])
    assert img == zf.packed_file([], UUID, 2, 9)
    assert rep["records"] == 0 and rep["region_bytes"] == 0


def test_repack_dir_finalised_files(gpu, tmp_path):
    """zsdb_repack's CRC path over a DB directory: finalised files merged
    (newest record of a key wins, deletes kept), one packed file out."""
    rng = np.random.default_rng(3)
    merged = {}
    for idx in range(1, 6):
        w = zf.FileWriter(UUID, idx=idx)
        for t in range(200):
            k = b"%016d" % int(rng.integers(0, 500))
            if t % 17 == 3:
                w.remove(k)
                merged[k] = None
            else:
                v = rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8).tobytes()
                w.add(k, v)
                merged[k] = v
            w.commit()
        with open(tmp_path / f"zeroskip-{UUIDSTR}-{idx}-{idx}", "wb") as fh:
            fh.write(w.image())
    out = tmp_path / f"zeroskip-{UUIDSTR}-1-5"
    rep = repack.repack_dir(str(tmp_path), str(out), UUID, 1, 5)
    want = zf.packed_file(sorted(merged.items()), UUID, 1, 5)
    assert open(out, "rb").read() == want
    assert rep["records"] == len(merged)
    assert os.path.getsize(out) == rep["file_bytes"]
