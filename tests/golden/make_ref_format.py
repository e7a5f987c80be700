"""Zeroskip file images written by the reference's OWN format code, and what
the reference's OWN verifier says about them (TEST INFRASTRUCTURE ONLY).

oracle/_ref/format_demo (tests/c/format_demo.c; oracle/Makefile `ref-format`)
runs src/zeroskip-file.c, -record.c, -header.c and mfile.c compiled unmodified
from /root/reference.  `Script` feeds it a sequence of zsdb_add / zsdb_remove
/ commit steps and mirrors each step into oracle/zs_format.FileWriter, so a
test can hold the oracle to the reference byte for byte.

Run as a script (where /root/reference exists) it regenerates
tests/golden/ref_format/: a few small images (`*.zs`) and manifest.json with
the reference verifier's verdict on each.  The GPU box has no reference; the
GPU tests (tests/test_gpu_ref_format.py) read those fixtures.
"""
from __future__ import annotations

import json
import os
import random
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import zs_format as zf  # noqa: E402

DEMO = os.path.join(ROOT, "oracle", "_ref", "format_demo")
OUTDIR = os.path.join(ROOT, "tests", "golden", "ref_format")


def build_demo() -> str:
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref-format"])
    return DEMO


class Script:
    """One file's worth of format_demo ops, mirrored into the oracle writer."""

    def __init__(self, uuid: bytes, idx: int = 0):
        self.blob = bytearray()
        self.ops = [f"H {uuid.hex()} {idx} {idx}"]
        self.fw = zf.FileWriter(uuid, idx)

    def _put(self, b: bytes) -> int:
        off = len(self.blob)
        self.blob += b
        return off

    def add(self, key: bytes, val: bytes):
        self.ops.append(f"A {self._put(key)} {len(key)} {self._put(val)} {len(val)}")
        self.fw.add(key, val)

    def remove(self, key: bytes):
        self.ops.append(f"D {self._put(key)} {len(key)}")
        self.fw.remove(key)

    def commit(self):
        """zsdb_commit's file half; with no span running it is the finalise
        commit over the stale register (FileWriter.finalise)."""
        self.ops.append("C")
        if self.fw.begin is None:
            self.fw.finalise()
        else:
            self.fw.commit()

    def run(self, path: str) -> bytes:
        return run_ops(self.ops, bytes(self.blob), path)


def packed_ops(uuid: bytes, startidx: int, endidx: int, records):
    """format_demo ops for zs_packed_file_new_from_memtree's writes
    (zeroskip-packed.c:384-473) over records [(key, value-or-None)] in key
    order; returns (ops, blob)."""
    blob = bytearray()
    ops = [f"H {uuid.hex()} {startidx} {endidx}", "B"]
    ptrs, off = [], zf.HDR_SIZE
    for k, v in records:
        ptrs.append(off)
        ko = len(blob)
        blob += k
        if v is None:
            ops.append(f"d {ko} {len(k)}")
            off += len(zf.delete_record(k))
        else:
            vo = len(blob)
            blob += v
            ops.append(f"a {ko} {len(k)} {vo} {len(v)}")
            off += len(zf.key_record(k)) + len(zf.value_record(v))
    words = [len(ptrs)] + ptrs
    ops += ["C", "B"] + ["P " + " ".join(str(x) for x in words[k:k + 2048]) for k in range(0, len(words), 2048)]
    ops.append("F")
    return ops, bytes(blob)


def run_ops(ops, blob: bytes, path: str) -> bytes:
    with tempfile.NamedTemporaryFile(suffix=".blob") as b:
        b.write(blob)
        b.flush()
        if os.path.exists(path):
            os.unlink(path)
        out = subprocess.run([DEMO, "write", path, b.name], input="\n".join(ops) + "\n",
                             capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        raise RuntimeError(f"format_demo write: rc {out.returncode}: {out.stderr}")
    with open(path, "rb") as f:
        return f.read()


def ref_verify(path: str) -> dict:
    out = subprocess.run([DEMO, "verify", path], capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        raise RuntimeError(f"format_demo verify: rc {out.returncode}: {out.stderr}")
    return json.loads(out.stdout)


def mixed_script(seed: int, ntxn: int = 40, long_key: bool = False, stale: bool = True) -> Script:
    """Transactions of 1-8 adds / removes; keys 1-40 bytes (plus the 65535 /
    65536 short/long boundary when long_key), values 0-300 bytes; after some
    commits a second commit with no span running (the finalise case)."""
    rng = random.Random(seed)
    s = Script(bytes(rng.randrange(256) for _ in range(16)), rng.randrange(8))
    for t in range(ntxn):
        for _ in range(rng.randint(1, 8)):
            klen = rng.randint(1, 40)
            if long_key and rng.random() < 0.05:
                klen = rng.choice([65535, 65536, 70001])
            key = bytes(rng.randrange(256) for _ in range(klen))
            if rng.random() < 0.25 and klen <= zf.MAX_SHORT_KEY_LEN:
                s.remove(key)
            else:
                s.add(key, bytes(rng.randrange(256) for _ in range(rng.randint(0, 300))))
        s.commit()
        if stale and rng.random() < 0.1:
            s.commit()
    return s


def long_script() -> Script:
    """A span over MAX_SHORT_VAL_LEN: a 16 MiB + 9 value (long value record)
    and a 70,000-byte key (long key record) in one transaction, so a long
    commit (zeroskip-file.c:266-302), between two short ones."""
    import numpy as np
    rng = np.random.default_rng(7)
    s = Script(bytes(range(16, 32)), 3)
    s.add(b"small", b"v" * 9)
    s.commit()
    s.add(b"big-value", rng.integers(0, 256, zf.MAX_SHORT_VAL_LEN + 9, dtype=np.uint8).tobytes())
    s.add(b"k" * 70000, b"after")
    s.commit()
    s.remove(b"small")
    s.commit()
    return s


def long_fixture() -> dict:
    """The long-commit image is 16 MiB: committed as its generator
    (long_script, whose oracle mirror regenerates it) and the reference-written
    image's sha256 and commit records, not as bytes."""
    import hashlib
    import struct
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "long")
        img = long_script().run(path)
        rep = ref_verify(path)
    commits = sorted([c[0] for c in rep["commits"]] + rep["long_commits"])
    words = {str(o): img[o:o + (24 if o in rep["long_commits"] else 8)].hex() for o in commits}
    return dict(kind=0, size=len(img), generator="long_script", sha256=hashlib.sha256(img).hexdigest(),
                commit_records=words, reference=rep, header=img[:40].hex(),
                note="bytes not committed (16 MiB): regenerate with long_script().fw (the oracle writer, "
                     "equal to the reference writer byte for byte) and check sha256")


PACKED_LONG_N = 2_200_000   # pointer section 17.6 MB > MAX_SHORT_VAL_LEN: a long FINAL commit


def packed_long_records():
    """2.2 M records (8-byte keys, empty values) for a packed file whose
    pointer section ends in a long FINAL commit."""
    return [(b"%08d" % i, b"") for i in range(PACKED_LONG_N)]


PACKED_LONG_HDR = (bytes(range(16)), 1, 4)   # uuid, startidx, endidx


def ref_packed(path: str) -> dict:
    """zs_packed_file_open's verdict (the reference's packed verifier)."""
    out = subprocess.run([DEMO, "packed", path], capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        raise RuntimeError(f"format_demo packed: rc {out.returncode}: {out.stderr}")
    return json.loads(out.stdout)


def packed_long_fixture() -> dict:
    """The long-FINAL packed image (123 MB): written by the reference's own
    writer (~1 min of mmap remaps), committed as its generator, sha256 and the
    reference verifier's verdicts on it and on two corruptions."""
    import hashlib
    recs = packed_long_records()
    ops, blob = packed_ops(*PACKED_LONG_HDR, recs)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "pl")
        img = run_ops(ops, blob, path)
        clean = ref_packed(path)
        pc = {c["kind"]: c for c in zf.packed_check(img)}
        flips = {"pointer_word": pc["pointers"]["span_off"] + 8 * 5 + 3, "final_crc": len(img) - 1}
        verdicts = {}
        for k, at in flips.items():
            bad = bytearray(img)
            bad[at] ^= 0x01
            with open(path, "wb") as f:
                f.write(bad)
            verdicts[k] = dict(offset=at, reference=ref_packed(path))
    return dict(kind=2, size=len(img), generator="packed_long_records", sha256=hashlib.sha256(img).hexdigest(),
                header=img[:40].hex(), trailer=img[-24:].hex(), reference_packed=clean, corruptions=verdicts,
                note="bytes not committed (123 MB): regenerate with zs_format.packed_file(packed_long_records(), "
                     "*PACKED_LONG_HDR) (the oracle writer; equal to the reference writer byte for byte) and "
                     "check sha256")


def ref_repack(branch: int, out: str, uuid: bytes, sidx: int, eidx: int, files) -> dict:
    """zsdb_repack's branch 1 or 2 on the reference's own code (format_demo
    repack1 / repack2)."""
    r = subprocess.run([DEMO, f"repack{branch}", out, uuid.hex(), str(sidx), str(eidx), *files],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError(f"format_demo repack{branch}: rc {r.returncode}: {r.stderr}")
    return json.loads(r.stdout)


def ref_merge_packed(sources):
    """The records zs_packed_file_new_from_packed_files writes
    (zeroskip-packed.c:617-742 over zeroskip-iterator.c), restated with its
    quirks: sources = [(priority, [(key, value-or-None)])] in the order of the
    file list.  A key in several sources goes to the higher priority; the
    iterator's `deleted` flag is set when it steps onto a delete
    (zeroskip-iterator.c:258-259) and never cleared, so from a source's first
    delete after its first record on, none of that source's records is
    written; a delete as a source's FIRST record is never flagged
    (zs_iterator_begin_for_packed_files reads its key without the type) and
    is written as a delete record."""
    import heapq
    its = [dict(prio=p, recs=r, pos=0, deleted=False, done=False) for p, r in sources]
    ht, pq = {}, []

    def process(key, it):
        old = ht.get(key)
        if old is not None:
            if it["prio"] > old["prio"]:
                ht[key] = it
                step(old)
            else:
                step(it)
        else:
            ht[key] = it
            heapq.heappush(pq, key)

    def step(it):
        if it["done"]:
            return
        it["pos"] += 1
        if it["pos"] < len(it["recs"]):
            k, v = it["recs"][it["pos"]]
            if v is None:
                it["deleted"] = True
            process(k, it)
        else:
            it["done"] = True

    for it in its:
        if it["recs"]:
            process(it["recs"][0][0], it)
    out = []
    while pq:
        key = heapq.heappop(pq)
        it = ht.pop(key)
        if not it["deleted"]:
            out.append(it["recs"][it["pos"]])
        step(it)
    return out


UUIDSTR = "00010203-0405-0607-0809-0a0b0c0d0e0f"   # the repack fixtures' DB uuid (bytes 0..15)


def repack1_inputs():
    """Five finalised files (idx 3..7; adds, removes, a key often rewritten)
    and an empty active file (idx 8): zsdb_repack branch 1's input."""
    import numpy as np
    rng = np.random.default_rng(31)
    files = {}
    for idx in range(3, 8):
        w = zf.FileWriter(bytes(range(16)), idx=idx)
        for t in range(100):
            k = b"%016d" % int(rng.integers(0, 300))
            if t % 11 == 3:
                w.remove(k)
            else:
                w.add(k, rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes())
            w.commit()
        files[f"zeroskip-{UUIDSTR}-{idx}-{idx}"] = w.image()
    files[f"zeroskip-{UUIDSTR}-8"] = zf.FileWriter(bytes(range(16)), idx=8).image()
    return files


def repack2_inputs():
    """Three packed files without deletes (0-3, 4-7, 8-9): branch 2's input,
    on which the reference's merge has no quirk (ref_merge_packed)."""
    import numpy as np
    rng = np.random.default_rng(32)

    def recs(n, lo, hi, vmax):
        return sorted({b"%016d" % int(rng.integers(lo, hi)):
                       rng.integers(0, 256, int(rng.integers(0, vmax)), dtype=np.uint8).tobytes()
                       for _ in range(n)}.items())
    spec = {(0, 3): recs(100, 0, 500, 200), (4, 7): recs(400, 200, 4000, 200), (8, 9): recs(150, 0, 1000, 200)}
    return {f"zeroskip-{UUIDSTR}-{a}-{b}": zf.packed_file(r, bytes(range(16)), a, b) for (a, b), r in spec.items()}


def repack2d_inputs():
    """Three packed files WITH deletes (0-3, 4-7, 8-9) -- among them a delete
    as the first record of one merged source, and keys present in both merged
    files on either side of each source's first delete: branch 2's input on
    which the reference's merge loses records (ref_merge_packed), the
    fixture of its compat mode (ZSCRC_REPACK_REFERENCE_COMPAT)."""
    import numpy as np
    rng = np.random.default_rng(33)

    def recs(n, lo, hi, vmax, pdel):
        return {b"%016d" % int(rng.integers(lo, hi)):
                (None if rng.integers(0, pdel) == 0 else
                 rng.integers(0, 256, int(rng.integers(0, vmax)), dtype=np.uint8).tobytes())
                for _ in range(n)}
    spec = {(0, 3): recs(100, 0, 500, 200, 6), (4, 7): recs(400, 100, 2000, 200, 25),
            (8, 9): recs(200, 0, 2000, 200, 15)}
    spec[(8, 9)][b"%016d" % 0] = None          # a delete as the newest file's first record
    out = {}
    for (a, b), r in spec.items():
        out[f"zeroskip-{UUIDSTR}-{a}-{b}"] = zf.packed_file(sorted(r.items()), bytes(range(16)), a, b)
    return out


def repack_fixture(branch: int, name: str | None = None) -> dict:
    """The inputs, and the output the reference's own repack writes from them
    (format_demo repack1 / repack2), under tests/golden/ref_format/<name>/
    (repackN; "repack2d": branch 2 on sources holding deletes)."""
    import hashlib
    name = name or f"repack{branch}"
    files = repack1_inputs() if branch == 1 else repack2d_inputs() if name == "repack2d" else repack2_inputs()
    d = os.path.join(OUTDIR, name)
    os.makedirs(d, exist_ok=True)
    for f in os.listdir(d):
        os.unlink(os.path.join(d, f))
    for name, img in files.items():
        with open(os.path.join(d, name), "wb") as fh:
            fh.write(img)
    if branch == 1:
        srcs, (sidx, eidx) = [n for n in files if n.count("-") == 7], (3, 7)
    else:
        srcs, (sidx, eidx) = sorted(files), (4, 9)
    out = os.path.join(d, "reference_out.zs")
    rep = ref_repack(branch, out, bytes(range(16)), sidx, eidx, [os.path.join(d, n) for n in srcs])
    img = open(out, "rb").read()
    return dict(repack=branch, inputs=sorted(files), startidx=sidx, endidx=eidx, reference=rep, size=len(img),
                sha256=hashlib.sha256(img).hexdigest(),
                out_name=f"zeroskip-{UUIDSTR}-{sidx}-{eidx}")


def fixtures() -> dict:
    """name -> (image bytes, kind) for the committed fixture set."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        img = mixed_script(11, ntxn=60, stale=False).run(os.path.join(d, "a"))
        out["active_clean"] = (img, 0)
        bad = bytearray(img)
        commits, _, _ = zf.walk(img)
        for i in (3, 17, 40):                 # one payload byte in three spans
            c = commits[i]
            bad[c["span_off"] + c["span_len"] // 2] ^= 0x20
        out["active_corrupt"] = (bytes(bad), 0)
        out["active_stale"] = (mixed_script(12, ntxn=50, stale=True).run(os.path.join(d, "b")), 0)
        out["active_longkey"] = (mixed_script(13, ntxn=12, long_key=True).run(os.path.join(d, "c")), 0)
        rng = random.Random(14)
        recs = sorted({b"%016d" % rng.randrange(10 ** 9): (None if rng.random() < 0.2 else
                                                          bytes(rng.randrange(256) for _ in range(rng.randint(0, 90))))
                       for _ in range(400)}.items())
        ops, blob = packed_ops(bytes(range(16)), 2, 5, recs)
        out["packed"] = (run_ops(ops, blob, os.path.join(d, "p")), 2)
    return out


def main():
    build_demo()
    os.makedirs(OUTDIR, exist_ok=True)
    manifest = {}
    for name, (img, kind) in fixtures().items():
        path = os.path.join(OUTDIR, name + ".zs")
        with open(path, "wb") as f:
            f.write(img)
        manifest[name] = dict(kind=kind, size=len(img), reference=ref_verify(path))
    manifest["long_value"] = long_fixture()
    manifest["packed_long"] = packed_long_fixture()
    manifest["repack1"] = repack_fixture(1)
    manifest["repack2"] = repack_fixture(2)
    manifest["repack2d"] = repack_fixture(2, "repack2d")
    with open(os.path.join(OUTDIR, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps({k: v["size"] for k, v in manifest.items()}))


def main_repack2d():
    """Only the repack2d fixture, merged into the existing manifest."""
    build_demo()
    path = os.path.join(OUTDIR, "manifest.json")
    with open(path) as f:
        manifest = json.load(f)
    manifest["repack2d"] = repack_fixture(2, "repack2d")
    with open(path, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(manifest["repack2d"]))


if __name__ == "__main__":
    import sys
    main_repack2d() if sys.argv[1:] == ["repack2d"] else main()
