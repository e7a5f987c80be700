"""Host-side zeroskip parsing in libzscrc (walk, packed spans, header and .zsdb
CRC) agrees with the format oracle.  No GPU."""
import numpy as np

from oracle import zs_format as zf
from tests.test_format_oracle import UUID, build_active
from zeroskip_amd import zsfile


def test_walk_matches_oracle():
    img = build_active(80, seed=5)
    off, ln, rc, end = zsfile.walk(img)
    commits, oend, why = zf.walk(img)
    assert rc == zsfile.END and end == oend == len(img)
    assert off.tolist() == [c["span_off"] for c in commits]
    assert ln.tolist() == [c["span_len"] for c in commits]


def test_walk_stops_like_reference():
    img = build_active(5) + zf.be64(zf.REC_FINAL << 56)
    off, ln, rc, end = zsfile.walk(img)
    assert rc == zsfile.STOPPED and end == len(img) - 8 and len(off) == 5
    off, ln, rc, end = zsfile.walk(build_active(5)[:-3])
    assert rc == zsfile.TRUNCATED


def test_packed_spans():
    recs = sorted((b"%016d" % i, b"x" * (i % 40)) for i in range(300))
    img = zf.packed_file(recs, UUID, 0, 7)
    off, ln, rc = zsfile.packed_spans(img)
    ref = zf.packed_check(img)
    assert rc == 0
    assert (off[1], ln[1]) == (ref[0]["span_off"], ref[0]["span_len"])
    assert (off[0], ln[0]) == (ref[1]["span_off"], ref[1]["span_len"])


def test_header_and_dotzsdb_crc():
    img = build_active(2)
    rc, st, cp = zsfile.header_crc(img)
    assert rc == 0 and st == cp == zf.header_check(img)[1]
    dz = zf.dotzsdb_bytes(4096, b"0123e4567-e89b-12d3-a456-426614174000"[:37], 3)
    rc, st, cp = zsfile.dotzsdb_crc(dz)
    assert rc == 0 and st == cp
    bad = bytearray(dz)
    bad[20] ^= 1
    rc, st, cp = zsfile.dotzsdb_crc(bytes(bad))
    assert st != cp
