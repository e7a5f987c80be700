"""The zeroskip format oracle (oracle/zs_format.py): files written with the
reference writer's semantics walk back with every commit CRC valid; corruption
is detected; header, packed and long-commit paths covered.  CPU only."""
import struct

import numpy as np

from oracle import oracle
from oracle import zs_format as zf

UUID = bytes(range(16))


def build_active(ntx=50, seed=1):
    rng = np.random.default_rng(seed)
    w = zf.FileWriter(UUID, idx=3)
    for t in range(ntx):
        for _ in range(int(rng.integers(1, 4))):
            k = b"%016d" % int(rng.integers(0, 10**9))
            v = rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8).tobytes()
            w.add(k, v)
        if t % 7 == 3:
            w.remove(b"%016d" % t)       # zeroskip.c:985 quirk: span restarts here
        w.commit()
    return w.image()


def test_header_roundtrip():
    img = build_active(3)
    ok, stored, computed = zf.header_check(img)
    assert ok and stored == computed
    assert img[:8] == b"PIKSOREZ"              # native-order signature (header.c:48)
    bad = bytearray(img)
    bad[30] ^= 1                               # startidx
    assert not zf.header_check(bytes(bad))[0]


def test_walk_all_commits_valid():
    img = build_active()
    commits, end, why = zf.walk(img)
    assert why == "end" and end == len(img)
    assert len(commits) == 50 and all(c["ok"] for c in commits)
    # the commit CRC is the chained crc32c_hw of span + LE trailer word
    c = commits[0]
    w0, = struct.unpack_from(">Q", img, c["commit_off"])
    span_crc = oracle.crc32c_hw(0, img[c["span_off"]:c["commit_off"]])
    assert oracle.crc32c_hw(span_crc, (w0 & 0xFFFFFFFF00000000).to_bytes(8, "little")) == c["stored"]


def test_corruption_detected():
    img = bytearray(build_active())
    commits, _, _ = zf.walk(bytes(img))
    victim = commits[10]
    img[victim["span_off"] + 30] ^= 0x40        # inside a key/value payload
    commits2, _, _ = zf.walk(bytes(img))
    bad = [i for i, c in enumerate(commits2) if not c["ok"]]
    assert bad == [10]


def test_packed_file():
    recs = sorted((b"%016d" % i, (b"v%d" % i) * (i % 5) if i % 9 else None) for i in range(200))
    img = zf.packed_file(recs, UUID, 1, 4)
    res = zf.packed_check(img)
    assert [r["kind"] for r in res] == ["pointers", "records"] and all(r["ok"] for r in res)
    assert res[0]["span_len"] == 8 * (1 + 200)   # count + N pointers


def test_long_commit_writer_semantics():
    # a span > 16 MiB gets the 24-byte long commit (zeroskip-file.c:266-302)
    w = zf.FileWriter(UUID)
    w.add(b"bigkey", bytes(np.random.default_rng(2).integers(0, 256, (17 << 20), dtype=np.uint8)))
    w.commit()
    img = w.image()
    commits, end, why = zf.walk(img)
    assert why == "end" and len(commits) == 1 and commits[0]["ok"]
    t1, n, w2 = struct.unpack_from(">QQQ", img, commits[0]["commit_off"])
    assert t1 >> 56 == zf.REC_LONG_COMMIT and w2 >> 56 == zf.REC_2ND_HALF and n > zf.MAX_SHORT_VAL_LEN


def test_zsbench_value_shape():
    v = zf.zsbench_values(4, 256, 0)
    assert v.shape == (4, 256) and (v[:, -1] == 0).all() and (v[:, :-1] > 32).all()
    assert len(zf.key_record(zf.zsbench_key(7))) == 40 and len(zf.value_record(v[0].tobytes())) == 272
