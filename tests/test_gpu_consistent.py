"""zsdb_consistent on the GPU (zeroskip_amd/consistent.py) against the oracle:
oracle-written DBs, corruptions, the GPU-side DB generator re-checked by the
oracle walker, a directory on disk, and two ranks exchanging digests."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

from oracle import zs_format as zf
from tests.test_consistent_host import OracleBackend, name, small_db
from zeroskip_amd import consistent as cs

pytestmark = pytest.mark.gpu


def gpu_report(db, world=1, rank=0):
    return cs.Consistent(cs.open_db(db), rank, world).prepare().run()


def same(a, b):
    return (a.ok, a.commits, a.bad_commits, a.stale_empty_commits, a.files, a.bytes_checked,
            sorted(map(tuple, a.header_errors)), a.issues) == \
           (b.ok, b.commits, b.bad_commits, b.stale_empty_commits, b.files, b.bytes_checked,
            sorted(map(tuple, b.header_errors)), b.issues)


def test_oracle_db_clean(gpu):
    db = small_db(long_region=True)
    g = gpu_report(db)
    o = cs.Consistent(cs.open_db(db), 0, 1, OracleBackend()).prepare().run()
    assert g.ok and same(g, o), (g.as_dict(), o.as_dict())
    assert len(g.stale_empty_commits) == 3


@pytest.mark.parametrize("what", ["finalised", "long_records", "ptrs", "header"])
def test_oracle_db_corruption(gpu, what):
    db = small_db(long_region=True)
    if what == "finalised":
        f = name(7, 7)
        img = bytearray(db[f])
        c = zf.walk(img)[0][17]
        img[c["span_off"] + c["span_len"] - 1] ^= 0x80
        want = [(f, c["commit_off"])]
    elif what in ("long_records", "ptrs"):
        f = name(4, 5)
        img = bytearray(db[f])
        c = {c["kind"]: c for c in zf.packed_check(img)}["records" if what == "long_records" else "pointers"]
        img[c["span_off"] + 12345 % c["span_len"]] ^= 4
        want = [(f, c["commit_off"])]
    else:
        f = name(0, 3)
        img = bytearray(db[f])
        img[30] ^= 1
        want = []
    db[f] = bytes(img)
    g = gpu_report(db)
    o = cs.Consistent(cs.open_db(db), 0, 1, OracleBackend()).prepare().run()
    assert not g.ok and same(g, o)
    assert g.bad_commits == want
    if what == "header":
        assert [h[0] for h in g.header_errors] == [f]


@pytest.mark.parametrize("post", ["cpass", "native", "native-overflow", "torch"])
def test_post_pass_paths(gpu, monkeypatch, post):
    """The device pass: the one-call native pass (zscrc_cpass: verdict batch,
    post kernel, one small copy), the per-commit arrays with the row kernel
    (one copy back), its overflow fallback (more mismatches than the row
    buffer) and the torch path give the oracle backend's report, with stale
    finalise commits and a corrupted commit in the same DB."""
    db = small_db(long_region=True)
    f = name(7, 7)
    img = bytearray(db[f])
    c = zf.walk(img)[0][5]
    img[c["span_off"] + 3] ^= 0x10
    db[f] = bytes(img)
    if post != "cpass":
        monkeypatch.setattr(cs.GpuBackend, "native_pass", False)
    if post == "torch":
        monkeypatch.setenv("ZS_POSTPASS", "torch")
    elif post == "native-overflow":
        monkeypatch.setattr(cs.GpuBackend, "ROWS_CAP", 2)
    g = gpu_report(db)
    o = cs.Consistent(cs.open_db(db), 0, 1, OracleBackend()).prepare().run()
    assert not g.ok and same(g, o), (g.as_dict(), o.as_dict())
    assert g.bad_commits == [(f, c["commit_off"])] and len(g.stale_empty_commits) == 3


def _gen_small(gpu):
    from tools import zsdb_gen
    return zsdb_gen.make_db(device=gpu, packed=2, packed_region_bytes=20 << 20, packed_vlen=1000,
                            finalised=5, active_pairs=100)


def test_generator_checked_by_oracle(gpu):
    """The GPU-written DB (bench config 5) is what the oracle writer would write."""
    db = _gen_small(gpu)
    nstale = 0
    for n, v in db.items():
        if n == ".zsdb":
            assert zf.dotzsdb_bytes(int.from_bytes(v[8:16], "big"), v[16:53],
                                    int.from_bytes(v[53:57], "big")) == v
            continue
        img = v.cpu().numpy().tobytes()
        assert zf.header_check(img)[0], n
        kind = cs.parse_name(n)[0]
        if kind == 2:
            assert all(c["ok"] for c in zf.packed_check(img)), n
        else:
            commits, end, why = zf.walk(img)
            assert why == "end" and end == len(img), n
            for c in commits[:-1]:
                assert c["ok"], (n, c)
            if kind == 1:
                assert commits[-1]["span_len"] == 0 and not commits[-1]["ok"]
                nstale += 1
            else:
                assert commits[-1]["ok"]
    assert nstale == 5
    rep = gpu_report(db)
    assert rep.ok and len(rep.stale_empty_commits) == 5 and not rep.issues, rep.as_dict()


def test_directory_and_cli(gpu, tmp_path):
    from tools import zsdb_gen
    db = _gen_small(gpu)
    zsdb_gen.write_dir(db, str(tmp_path))
    rep = cs.consistent(str(tmp_path))
    assert rep.ok and rep.files == len(db) - 1
    f = sorted(p for p in os.listdir(tmp_path) if cs.parse_name(p) and cs.parse_name(p)[0] == 1)[2]
    with open(tmp_path / f, "r+b") as fh:
        fh.seek(40 + 3 * 320 + 100)          # value payload of pair 3
        b = fh.read(1)
        fh.seek(40 + 3 * 320 + 100)
        fh.write(bytes([b[0] ^ 1]))
    assert cs.main([str(tmp_path)]) == 1
    rep = cs.consistent(str(tmp_path))
    assert [b[0] for b in rep.bad_commits] == [f]


def _rank_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        db = small_db(long_region=True)
        img = bytearray(db[name(4, 5)])
        c = {c["kind"]: c for c in zf.packed_check(img)}["records"]
        img[c["span_off"] + 7] ^= 1
        db[name(4, 5)] = bytes(img)
        job = cs.Consistent(cs.open_db(db), rank, world).prepare()
        rep = job.run()
        # the digest rows' exchange: one host round trip per pass
        assert rep.timing.get("host_round_trips") == 1, rep.timing
        # pipelined: two passes' rows in flight, collected in order, the same reports
        reps = []
        for _ in range(4):
            assert job.submit()
            if job.pending() > 1:
                reps.append(job.collect())
        while job.pending():
            reps.append(job.collect())
        assert len(reps) == 4
        assert all((r.ok, r.commits, r.bad_commits, r.stale_empty_commits) ==
                   (rep.ok, rep.commits, rep.bad_commits, rep.stale_empty_commits) for r in reps)
        q.put((rank, rep.ok, rep.commits, rep.bad_commits, len(rep.stale_empty_commits), c["commit_off"]))
    finally:
        dist.destroy_process_group()


def test_two_ranks_split_long_region(gpu):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = cs.Consistent(cs.open_db(small_db(long_region=True)), 0, 1, OracleBackend()).prepare().run()
    for _, ok, commits, bad, nstale, at in res:
        assert not ok and commits == single.commits and nstale == 3
        assert bad == [(name(4, 5), at)]


def test_native_entry_point(gpu, tmp_path):
    """zscrc_zs_consistent (the C entry point for zsdb_consistent) agrees with
    the Python driver, clean and corrupted, across several device groups."""
    db = small_db(long_region=True)
    for n, v in db.items():
        (tmp_path / n).write_bytes(v)
    nat = cs.consistent_native(str(tmp_path))
    py = cs.consistent(str(tmp_path))
    assert nat["consistent"] == 1 and py.ok
    assert nat["commits"] == py.commits and nat["stale_empty_commits"] == py.n_stale == 3
    assert nat["files"] == 6 and nat["dotzsdb"] == 1
    f = name(7, 7)
    img = bytearray(db[f])
    c = zf.walk(img)[0][5]
    img[c["span_off"] + 3] ^= 0x10
    (tmp_path / f).write_bytes(bytes(img))
    os.environ["ZSCRC_CONSISTENT_GROUP"] = str(1 << 20)     # one file per device pass
    try:
        nat = cs.consistent_native(str(tmp_path))
    finally:
        del os.environ["ZSCRC_CONSISTENT_GROUP"]
    assert nat["consistent"] == 0 and nat["bad_commits"] == 1
    assert nat["first_bad"].startswith(f"{f}:{c['commit_off']}:")
    (tmp_path / ".zsdb").write_bytes(b"short")
    assert cs.consistent_native(str(tmp_path))["dotzsdb"] == 0


def test_eight_slots_config5_shape(gpu, tmp_path):
    """Multi-GPU readiness on one GPU: zscrc_zs_consistent with eight device
    slots (ZSCRC_DEVICES=0,...,0 -- what an 8-GPU node gives it) on a
    config-5-shaped DB whose commit CRCs the CPU oracle wrote (two packed
    files with > 16 MiB records regions, finalised files with stale finalise
    commits, an active file): the records regions are cut at the slot bounds
    and folded on the host.  Clean, then one flipped byte on each side of
    every slot bound that falls inside a region -- each found as the one bad
    commit of that file."""
    from tools import zsdb_gen as zg
    db = zg.make_db(device="cpu", packed=2, packed_region_bytes=24 << 20, finalised=20, active_pairs=500,
                    writer="cpu")
    files = {n: (v.numpy() if hasattr(v, "numpy") else np.frombuffer(v, np.uint8)) for n, v in db.items()}
    for n, v in files.items():
        (tmp_path / n).write_bytes(v.tobytes())
    slots = 8
    os.environ["ZSCRC_DEVICES"] = ",".join(["0"] * slots)
    try:
        rep = cs.consistent_native(str(tmp_path))
        assert rep["consistent"] == 1 and rep["stale_empty_commits"] == 20 and rep["bad_commits"] == 0
        # the slot bounds (zscrc_files.cpp: W = packed files from their
        # records region on, others whole; cuts 4 KiB-aligned in a region)
        order = sorted((n for n in files if n != ".zsdb"), key=lambda n: cs.parse_name(n)[2:])
        W = sum(files[n].nbytes - (40 if cs.parse_name(n)[0] == 2 else 0) for n in order)
        at, cuts = 0, []
        for n in order:
            if cs.parse_name(n)[0] == 2:
                rlen = oracle_region_len(files[n])
                for s in range(1, slots):
                    b = W * s // slots
                    if at < b < at + rlen:
                        cuts.append((n, 40 + (b - at) // 4096 * 4096))
                at += files[n].nbytes - 40
            else:
                at += files[n].nbytes
        assert len(cuts) >= 4, cuts
        for n, cut in cuts:
            for p in (cut - 1, cut):
                img = files[n].copy()
                img[p] ^= 0x08
                (tmp_path / n).write_bytes(img.tobytes())
                r = cs.consistent_native(str(tmp_path))
                assert r["consistent"] == 0 and r["bad_commits"] == 1, (n, p, r)
                assert r["first_bad"].startswith(n + ":"), r["first_bad"]
            (tmp_path / n).write_bytes(files[n].tobytes())
        assert cs.consistent_native(str(tmp_path))["consistent"] == 1
    finally:
        del os.environ["ZSCRC_DEVICES"]


def oracle_region_len(img) -> int:
    from oracle import oracle
    return oracle.packed_image(img)["records"]["span_len"]


def test_pipelined_passes(gpu):
    """zscrc_cpass_submit / _collect (bench config 5's pipelined steps): up to
    two passes in flight in two host slots, collected in order, each report
    the same as a synchronous pass's -- and a corruption made on the device
    between two submits shows in the second report only."""
    db = small_db(long_region=True)
    job = cs.Consistent(cs.open_db(db), 0, 1).prepare()
    assert job._cpass is not None
    want = job.run()
    assert want.ok and len(want.stale_empty_commits) == 3
    reps = []
    for k in range(7):
        assert job.submit()
        if job.pending() > 1:
            reps.append(job.collect())
    while job.pending():
        reps.append(job.collect())
    assert len(reps) == 7 and all(same(r, want) for r in reps)
    with pytest.raises(RuntimeError):
        job.submit(), job.submit(), job.submit()
    while job.pending():
        job.collect()
    # a commit span flipped on the device after pass 1 is submitted: pass 1
    # clean (stream order: the flip runs after it), pass 2 reports it
    f = name(7, 7)
    fid = [i for i, x in enumerate(job.db.files) if x.name == f][0]
    c = zf.walk(bytearray(db[f]))[0][9]
    assert job.submit()
    where = job.dev_offset(fid, c["span_off"] + 1)
    job.buf[where] ^= 0x40
    assert job.submit()
    r1, r2 = job.collect(), job.collect()
    assert r1.ok and same(r1, want)
    assert not r2.ok and r2.bad_commits == [(f, c["commit_off"])]
    job.buf[where] ^= 0x40
    assert job.run().ok


def test_destroy_with_uncollected_passes(gpu):
    """A pass destroyed with two submits never collected (their completion
    the caller's own end events, recorded on the stream): zscrc_cpass_destroy
    waits for the device before freeing the host slots the post kernels
    write, and a new pass over the same DB runs clean after."""
    db = small_db(long_region=True)
    job = cs.Consistent(cs.open_db(db), 0, 1).prepare()
    assert job._cpass is not None
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(2)]
    assert job.submit(evs[0]) and job.submit(evs[1])
    assert job.pending() == 2
    from zeroskip_amd._lib import lib
    h, job._cpass = job._cpass, None
    lib().zscrc_cpass_destroy(h)
    del evs
    torch.cuda.synchronize()
    job2 = cs.Consistent(cs.open_db(db), 0, 1).prepare()
    rep = job2.run()
    assert rep.ok and len(rep.stale_empty_commits) == 3


@pytest.mark.parametrize("case", ["clean", "corrupt", "bad_2000", "bad_5000", "bad_12000"])
def test_device_row_matches_host_digest(gpu, case):
    """zscrc_cpass_submit_row's digest row (built by cpass_post_kernel's last
    workgroup: the listed verdict sorted on the device) equals the row the
    host builds from the same pass's copied-back block (Consistent._pack of
    the native digest), int64 for int64 -- clean, with a bad commit, a bad
    records region and stale commits, with more bad commits than a row lists
    (2,000 > 1,000) and more than the pass lists (5,000 and 12,000 > 4,096:
    flag 1, the caller takes the torch path).  The counts are the device's
    over every mismatch on both sides, so they agree whatever order the
    waves listed the mismatches in -- and equal the torch path's exact
    counts."""
    import ctypes
    from zeroskip_amd._lib import check, lib
    if case.startswith("bad_"):
        from tools import zsdb_gen
        db = zsdb_gen.make_db(device=gpu, packed=2, packed_region_bytes=8 << 20, packed_vlen=1000,
                              finalised=3, active_pairs=100)
    else:
        db = small_db(long_region=True)
    if case == "corrupt":
        for f, what in ((name(7, 7), None), (name(4, 5), "records")):
            img = bytearray(db[f])
            if what is None:
                c = zf.walk(img)[0][5]
                assert c["span_len"] > 3
                img[c["span_off"] + 3] ^= 0x10
            else:
                c = {c["kind"]: c for c in zf.packed_check(img)}[what]
                img[c["span_off"] + 99] ^= 2
            db[f] = bytes(img)
    job = cs.Consistent(cs.open_db(db), 0, 1).prepare()
    assert job._cpass is not None
    if case.startswith("bad_"):
        k = int(case[4:])
        live = torch.nonzero(job.d_len > 0).flatten()[:k]
        assert live.numel() == k
        job.buf[job.d_off[live]] ^= 0x5A
        if k > 4096:
            # by construction: stale finalise commits (zero-length, at the end
            # of each finalised file) lie after the 4,097th bad commit in
            # index order, so a count over only the first 4,096 listed
            # entries would miss them
            zero = torch.nonzero(job.d_len == 0).flatten()
            assert int((zero > live[4096]).sum()) >= 1
    row = job.device_row().cpu().numpy()
    res = cs.CPassResult()
    with torch.cuda.device(job.buf.device):
        check(lib().zscrc_cpass_run(job._cpass, None, ctypes.byref(res)), "zscrc_cpass_run")
    want = job._pack(job._native_digest(res))
    assert row.shape == want.shape
    if case in ("bad_5000", "bad_12000"):
        # more mismatches than the pass lists: WHICH 4,096 a pass lists depends
        # on the order its waves found them, so the lists may differ; the
        # counts may not, and the row says incomplete (the caller then
        # decides on the torch path)
        assert not res.complete and row[6] == 1 and row[1] + row[2] >= k
        assert np.array_equal(row[:3], want[:3]), (row[:3], want[:3])
        assert row[3] == job.MAX_LISTED
        exact = job._run_torch()
        assert (int(row[1]), int(row[2])) == (exact.n_bad, exact.n_stale), (row[:3], exact.as_dict())
        return
    assert row[6] == 0
    if case.startswith("bad_"):
        assert row[3] == job.MAX_LISTED
    assert np.array_equal(row, want), np.nonzero(row != want)[0][:10]
    if case == "corrupt":
        assert row[1] >= 1 and row[2] == 3


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZSCRC_SOAK_BASE", "0")),
                                      int(os.environ.get("ZSCRC_SOAK_BASE", "0")) +
                                      int(os.environ.get("ZSCRC_SOAK_CONSISTENT", "8"))))
def test_random_corruptions_match_oracle(gpu, seed):
    """zsdb_consistent on the GPU backend and on the oracle backend over the
    same DB with 1-4 random bytes flipped anywhere in its files (headers,
    spans, commit records, pointer sections, the long records region): the
    same report, field for field."""
    rng = np.random.default_rng(300 + seed)
    db = small_db(long_region=seed % 2 == 0, seed=100 + seed)
    files = sorted(k for k in db if k != ".zsdb")
    for _ in range(int(rng.integers(1, 5))):
        f = files[int(rng.integers(0, len(files)))]
        img = bytearray(db[f])
        img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
        db[f] = bytes(img)
    g = gpu_report(db)
    o = cs.Consistent(cs.open_db(db), 0, 1, OracleBackend()).prepare().run()
    assert same(g, o), (seed, g.as_dict(), o.as_dict())
    print(f"seed {seed}: ok={g.ok} bad={len(g.bad_commits)} header_errors={len(g.header_errors)} "
          f"issues={len(g.issues)}")


def test_cpass_understated_max_len(gpu):
    """A C caller's zscrc_cpass_spec.max_len below the longest span (ADVICE
    r05): the verdict launches only the length classes up to the bound, so
    zscrc_cpass_create takes the lengths' true maximum -- the corrupted
    longest commit is still found."""
    import ctypes
    from zeroskip_amd._lib import check, lib
    db = small_db(long_region=True)
    job = cs.Consistent(cs.open_db(db), 0, 1).prepare()
    i = int(torch.argmax(job.d_len))
    L = int(job.d_len[i])
    assert L > 640                         # above the one-lane length class
    job.buf[int(job.d_off[i]) + L // 2] ^= 0x21
    h = ctypes.c_void_p()
    res = cs.CPassResult()
    with torch.cuda.device(job.buf.device):
        for max_len in (1, 64, L - 1):
            spec = cs.CPassSpec(job.buf.data_ptr(), job.buf.numel(), len(job.c_off), job.d_off.data_ptr(),
                                job.d_len.data_ptr(), job.d_file.data_ptr(), max_len, 0, None, None, None)
            check(lib().zscrc_cpass_create(ctypes.byref(h), ctypes.byref(spec)), "zscrc_cpass_create")
            try:
                check(lib().zscrc_cpass_run(h, None, ctypes.byref(res)), "zscrc_cpass_run")
            finally:
                lib().zscrc_cpass_destroy(h)
            bad = list(res.bad[:res.n_listed_bad])
            assert res.complete and i in bad, (max_len, i, bad, res.n_bad)


def test_passes_alternate_streams(gpu):
    """Consecutive passes of one handle enqueued on different streams (ADVICE
    r05): each pass zeroes the counters the next one increments, so a pass on
    another stream first waits for the previous stream's work -- every
    report equals the synchronous one, with a corrupted commit counted once
    per pass."""
    db = small_db(long_region=True)
    f = name(7, 7)
    img = bytearray(db[f])
    c = zf.walk(img)[0][5]
    img[c["span_off"] + 3] ^= 0x10
    db[f] = bytes(img)
    job = cs.Consistent(cs.open_db(db), 0, 1).prepare()
    want = job.run()
    assert not want.ok and len(want.bad_commits) == 1
    streams = [torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.current_stream()]
    reps = []
    for k in range(9):
        with torch.cuda.stream(streams[k % 3]):
            assert job.submit()
            if job.pending() > 1:
                reps.append(job.collect())
    while job.pending():
        reps.append(job.collect())
    assert len(reps) == 9 and all(same(r, want) for r in reps)
    for k in range(4):
        with torch.cuda.stream(streams[k % 2]):
            assert same(job.run(), want)


def _nccl_one_rank(port, q):
    import torch.distributed as dist
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        torch.cuda.set_device(0)
        db = small_db(long_region=True)
        f = name(4, 5)
        img = bytearray(db[f])
        c = {c["kind"]: c for c in zf.packed_check(img)}["records"]
        img[c["span_off"] + 11] ^= 4
        db[f] = bytes(img)
        job = cs.Consistent(cs.open_db(db), 0, 1).prepare()
        want = job.run()
        # the world > 1 code paths under RCCL, on a one-rank group: the
        # synchronous row exchange and the pipelined one (the all-gather on
        # RCCL's stream, the copy to pinned memory on a side stream)
        sync = job._run_native_rows(None)
        job._inflight, job._next_slot = [], 0
        piped = []
        for _ in range(5):
            job._submit_rows(None, job._next_slot)
            if len(job._inflight) > 1:
                piped.append(job._collect_rows())
        while job._inflight:
            piped.append(job._collect_rows())
        q.put((same(sync, want), [same(r, want) for r in piped], want.ok, want.bad_commits,
               sync.timing.get("host_round_trips"), c["commit_off"]))
    finally:
        dist.destroy_process_group()


def test_row_exchange_over_rccl_one_rank(gpu):
    """the nccl branch of the digest-row exchange
    (Consistent._run_native_rows, _submit_rows / _collect_rows: the async
    all_gather_into_tensor on RCCL's stream, the side stream waiting on the
    work, the non-blocking copy into pinned rows) run for real on a one-rank
    RCCL group (RCCL refuses two ranks on one device): the same report as the
    one-rank native pass, pass after pass."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_one_rank, args=(port, q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    sync_ok, piped_ok, ok, bad, trips, at = res
    assert sync_ok and len(piped_ok) == 5 and all(piped_ok)
    assert not ok and bad == [(name(4, 5), at)] and trips == 1


def test_cpass_stale_rehash_ragged_spans(gpu):
    """The post kernel's finalise-quirk check rehashes the span before each
    zero-length commit (crc_run: its ragged head and tail from the aligned
    dword around them, the body in 64-byte steps, the last words loaded
    together).  Zeroskip's own spans are 8-byte aligned, so here a synthetic
    image places them at every byte alignment with lengths 1..1,500 and on
    the step edges; each span's commit record is followed by nothing but a
    zero-length commit that reuses it -- stale (the quirk) when both commits
    are of one file, bad when the file ids differ.  Counts and listed
    indices equal what the construction says.  src/zeroskip-active.c:122,
    src/mfile.c:534-546 (the quirk); src/zeroskip-file.c:266-302 (the
    commit CRC)."""
    import ctypes
    from oracle import oracle
    from zeroskip_amd._lib import check, lib
    rng = np.random.default_rng(606)
    # (length 0 is no case: the zero-length commit would then verify like its
    # predecessor, which is not the quirk)
    edges = [1, 2, 3, 4, 5, 7, 8, 60, 63, 64, 65, 67, 127, 128, 129, 131, 192, 312, 319, 320, 1023]
    lens = edges + rng.integers(1, 1501, 200).tolist()
    m = len(lens)
    size = sum(lens) + m * (8 + 7 + 64) + 4096
    img = rng.integers(0, 256, size, dtype=np.uint8)
    off, ln, fid, stale, bad = [], [], [], [], []
    pos = 1
    for k, pl in enumerate(lens):
        pos += int(rng.integers(0, 64))          # any byte alignment
        at = pos + pl
        img[at:at + 4] = (4, 0, 0, 0)            # COMMIT, length 0 in the record's header word
        S = oracle.crc32c_hw(0, img[pos:pos + pl].tobytes())
        hi = int.from_bytes(img[at:at + 4].tobytes() + b"\0\0\0\0", "big")
        c = oracle.crc32c_hw(S, hi.to_bytes(8, "little"))
        img[at + 4:at + 8] = np.frombuffer(c.to_bytes(4, "big"), np.uint8)
        same_file = k % 7 != 3
        i = len(off)
        off += [pos, at]
        ln += [pl, 0]
        fid += [2 * k, 2 * k if same_file else 2 * k + 1]
        (stale if same_file else bad).append(i + 1)
        pos = at + 8
    assert pos <= size
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(img).to(dev)
    d_off = torch.tensor(off, dtype=torch.int64, device=dev)
    d_len = torch.tensor(ln, dtype=torch.int64, device=dev)
    d_file = torch.tensor(fid, dtype=torch.int32, device=dev)
    h = ctypes.c_void_p()
    res = cs.CPassResult()
    with torch.cuda.device(dev):
        spec = cs.CPassSpec(buf.data_ptr(), buf.numel(), len(off), d_off.data_ptr(), d_len.data_ptr(),
                            d_file.data_ptr(), max(ln), 0, None, None, None)
        check(lib().zscrc_cpass_create(ctypes.byref(h), ctypes.byref(spec)), "zscrc_cpass_create")
        try:
            for _ in range(3):                    # both device blocks, and back
                check(lib().zscrc_cpass_run(h, None, ctypes.byref(res)), "zscrc_cpass_run")
                assert res.complete and res.n_undecided == 0
                assert (res.n_stale, res.n_bad) == (len(stale), len(bad)), (res.n_stale, res.n_bad)
                assert list(res.stale[:res.n_listed_stale]) == stale
                assert list(res.bad[:res.n_listed_bad]) == bad
        finally:
            lib().zscrc_cpass_destroy(h)


def _corrupt_db(seed):
    """test_random_corruptions_match_oracle's DB for `seed`."""
    rng = np.random.default_rng(300 + seed)
    db = small_db(long_region=seed % 2 == 0, seed=100 + seed)
    files = sorted(k for k in db if k != ".zsdb")
    for _ in range(int(rng.integers(1, 5))):
        f = files[int(rng.integers(0, len(files)))]
        img = bytearray(db[f])
        img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
        db[f] = bytes(img)
    return db


def _random_rank_worker(rank, world, port, seeds, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        out = []
        for seed in seeds:
            rep = cs.Consistent(cs.open_db(_corrupt_db(seed)), rank, world).prepare().run()
            out.append((seed, rep.ok, rep.commits, rep.bad_commits, rep.stale_empty_commits,
                        sorted(map(tuple, rep.header_errors)), rep.issues))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_random_corruptions_match_one_rank(gpu, world):
    """The N-rank path -- shares cut by byte weight, each rank's pass with its
    digest row built by the post kernel's last workgroup, the rows exchanged
    (gloo here: RCCL refuses two ranks on one device), split regions folded
    from the ranks' raw registers -- over the randomly corrupted DBs of
    test_random_corruptions_match_oracle: every rank's report equals the
    one-rank report, field for field."""
    import torch.multiprocessing as mp
    seeds = list(range(int(os.environ.get("ZSCRC_SOAK_BASE", "0")),
                       int(os.environ.get("ZSCRC_SOAK_BASE", "0")) + 6))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_random_rank_worker, args=(r, world, port, seeds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for seed_i, seed in enumerate(seeds):
        one = gpu_report(_corrupt_db(seed))
        want = (seed, one.ok, one.commits, one.bad_commits, one.stale_empty_commits,
                sorted(map(tuple, one.header_errors)), one.issues)
        for rank, out in res:
            assert out[seed_i] == want, (world, rank, seed, out[seed_i], want)
