"""The host-side zeroskip parsers of libzscrc (zscrc_zs_walk / _packed_spans
/ _records / _header_crc / _dotzsdb_crc) on mutated copies of the
reference-written fixtures: every span and record they return lies inside
the image, and crc32c_hw == crc32c_sw on random slices (tests/c/parse_fuzz.c,
built here against the in-tree libzscrc.so; no GPU call).  The same driver
under AddressSanitizer + UBSan is tools/asan_fuzz.sh.

Against the format oracle: on every mutated active / finalised image the
oracle can read, libzscrc's walk either ends like the oracle's (END) with
the same spans, or stops early (TRUNCATED / STOPPED on a length that leaves
the image, where the reference would read past the mmap) with a prefix of
the oracle's spans."""
import json
import os
import random
import subprocess

import pytest

from oracle import zs_format as zf
from zeroskip_amd import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "ref_format")
FILES = ["active_clean.zs", "active_corrupt.zs", "active_stale.zs", "active_longkey.zs", "packed.zs",
         "repack1/reference_out.zs", "repack2/reference_out.zs"]


@pytest.fixture(scope="module")
def fuzzer(tmp_path_factory):
    d = tmp_path_factory.mktemp("fuzz")
    exe = d / "parse_fuzz"
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "parse_fuzz.c"), "-L", os.path.dirname(LIB_PATH),
                           "-lzscrc", f"-Wl,-rpath,{os.path.dirname(LIB_PATH)}", "-o", str(exe)])
    (d / "dotzsdb").write_bytes(zf.dotzsdb_bytes(4096, b"00010203-0405-0607-0809-0a0b0c0d0e0f\0", 8))
    return str(exe), [os.path.join(FIX, f) for f in FILES] + [str(d / "dotzsdb")]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_parsers_stay_inside_mutated_images(fuzzer, seed):
    exe, files = fuzzer
    out = subprocess.run([exe, "3000", str(seed), *files], capture_output=True, text=True, timeout=300,
                         env={**os.environ, "ZSCRC_GPU_MIN": "0"})
    assert out.returncode == 0, out.stderr[-2000:]
    rep = json.loads(out.stdout)
    assert rep["violations"] == 0 and rep["walks"] == 3000 and rep["record_lists"] == 9000


@pytest.mark.parametrize("seed", [5, 6])
def test_walk_matches_oracle_or_stops_early(seed):
    from tests import fuzzlib
    from zeroskip_amd import zsfile
    rng = random.Random(seed)
    imgs = [open(os.path.join(FIX, f), "rb").read() for f in FILES[:4]]
    full = prefix = 0
    for _ in range(1500):
        m = fuzzlib.mutate(rng, rng.choice(imgs))
        if len(m) < 40:
            continue
        o = fuzzlib.oracle_walk(m)
        if o is None:
            continue
        commits, end, why = o
        off, ln, rc, wend = zsfile.walk(m)
        got = list(zip(off.tolist(), ln.tolist()))
        want = [(c["span_off"], c["span_len"]) for c in commits]
        if rc == zsfile.END:
            assert why == "end" and end == len(m) == wend and got == want
            full += 1
        else:
            assert rc in (zsfile.TRUNCATED, zsfile.STOPPED) and want[:len(got)] == got
            prefix += 1
    assert full > 300 and prefix > 300


@pytest.mark.parametrize("seed", [7, 8])
def test_packed_spans_match_oracle(seed):
    """Mutated finalised images (the reference's packed file and both
    repack outputs): whenever zscrc_zs_packed_spans accepts one, its two
    spans are the format oracle's packed_check spans (which then never
    raises); otherwise it rejects with a parse code (STOPPED / TRUNCATED)
    or an error."""
    from tests import fuzzlib
    from zeroskip_amd import zsfile
    rng = random.Random(seed)
    imgs = [open(os.path.join(FIX, f), "rb").read() for f in FILES[4:]]
    agree = rejected = 0
    for _ in range(1500):
        m = fuzzlib.mutate(rng, rng.choice(imgs))
        if len(m) < 48:
            continue
        off, ln, rc = zsfile.packed_spans(m)
        if rc != 0:
            assert rc < 0 or rc in (zsfile.STOPPED, zsfile.TRUNCATED), rc
            rejected += 1
            continue
        want = sorted((c["span_off"], c["span_len"]) for c in zf.packed_check(m))
        assert sorted(zip(off.tolist(), ln.tolist())) == want
        agree += 1
    assert agree > 500 and rejected > 200
