"""Host-side zeroskip parsing in libzscrc (walk, packed spans, header and .zsdb
CRC) agrees with the format oracle.  No GPU."""
import numpy as np
import pytest

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


def _key_then_long_value(voff_extra: int, vlen: int) -> bytes:
    """Header, one short key record (16-byte key) and a LONG_VALUE record
    whose 64-bit length word is `vlen` (corrupt on purpose)."""
    hdr = build_active(1)[:zf.HDR_SIZE]
    voff = 24 + 16 + voff_extra
    key = zf.be64((zf.REC_KEY << 56) | (16 << 40) | voff) + bytes(16) + b"k" * 16 + bytes(voff_extra)
    val = zf.be64(zf.REC_LONG_VALUE << 56) + zf.be64(vlen) + b"v" * 64
    return hdr + key + val


@pytest.mark.timeout(20)
@pytest.mark.parametrize("case", ["wrapped_vlen", "self_loop", "vlen_past_end", "long_delete_at_end",
                                  "long_delete_huge_klen", "long_key_huge_voff"])
def test_walk_survives_corrupt_lengths(case):
    """Every length word is file data: a corrupt one must stop the walk with
    TRUNCATED -- never loop, go backwards or read past the image."""
    voff = 24 + 16
    if case == "wrapped_vlen":
        img = _key_then_long_value(0, (1 << 64) - 8)
    elif case == "self_loop":
        # v + 16 + rup8(vlen) == off (mod 2^64): the old walk stood still forever
        img = _key_then_long_value(0, (1 << 64) - 16 - voff)
    elif case == "vlen_past_end":
        img = _key_then_long_value(0, 4096)
    elif case == "long_delete_at_end":
        # a long delete's key length sits at off + 8, past the image end
        img = build_active(2) + zf.be64(zf.REC_LONG_DELETED << 56)
    elif case == "long_delete_huge_klen":
        img = build_active(2) + zf.be64(zf.REC_LONG_DELETED << 56) + zf.be64((1 << 64) - 24) + bytes(8)
    else:
        hdr = build_active(1)[:zf.HDR_SIZE]
        img = hdr + zf.be64(zf.REC_LONG_KEY << 56) + zf.be64(16) + zf.be64((1 << 64) - 1) + b"k" * 16
    off, ln, rc, end = zsfile.walk(img)
    assert rc == zsfile.TRUNCATED, (case, rc, end)
    assert zf.HDR_SIZE <= end <= len(img)


def test_record_lister_matches_oracle():
    """zscrc_zs_records (C) lists the same records as the format oracle's
    walk (finalised files: adds, deletes, overwrites, empty values) and
    pointer section (packed files, incl. a long value record); CPU only."""
    import numpy as np
    from oracle import zs_format as zf
    from tests.test_format_oracle import UUID
    from zeroskip_amd import repack, zsfile
    rng = np.random.default_rng(31)
    w = zf.FileWriter(UUID, idx=4)
    for t in range(300):
        k = b"%016d" % int(rng.integers(0, 90))
        if t % 11 == 3:
            w.remove(k)
        else:
            w.add(k, rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8).tobytes())
        if t % 3 == 0:
            w.commit()
    w.commit()
    img = w.image()
    (ko, kl, vo, vl), rc = repack.records(img, zsfile.FINALISED)
    got = [(img[a:a + b], None if c == 2**64 - 1 else img[c:c + d]) for a, b, c, d in zip(ko, kl, vo, vl)]
    assert rc == zsfile.END and got == zf.file_records(img)
    recs = sorted({b"%08d" % i: (None if i % 7 == 1 else bytes([i % 256]) * (i % 50)) for i in range(400)}.items())
    recs[5] = (recs[5][0], b"L" * ((16 << 20) + 9))
    pimg = zf.packed_file(recs, UUID, 1, 9)
    (ko, kl, vo, vl), rc = repack.records(pimg, zsfile.PACKED)
    got = [(pimg[a:a + b], None if c == 2**64 - 1 else pimg[c:c + d]) for a, b, c, d in zip(ko, kl, vo, vl)]
    assert rc == 0 and got == zf.packed_records(pimg) == recs


def test_dotzsdb_build_matches_oracle():
    import ctypes
    from oracle import zs_format as zf
    from zeroskip_amd._lib import lib
    u = b"00010203-0405-0607-0809-0a0b0c0d0e0f"
    out = (ctypes.c_uint8 * 61)()
    assert lib().zscrc_zs_dotzsdb_build(123456789, u, 77, out) == 0
    assert bytes(out) == zf.dotzsdb_bytes(123456789, u + b"\0", 77)
