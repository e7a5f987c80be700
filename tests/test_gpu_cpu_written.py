"""GPU verification of images whose commit CRCs the CPU oracle wrote
(tools/zsdb_gen.py writer="cpu": oracle/zs_bulk_oracle.c oracle_write_commits,
the writer of src/zeroskip-file.c:253-350), so the GPU writer and the GPU
verifier are never each other's only witness:

* >= 1.1 M zsbench BATCHED commits (config 4's layout, 168 log files of 2 MiB)
  verified by commit_kernel<false> -- verdict and per-commit arrays -- against
  the oracle's stored CRCs, and the GPU writer reproducing the CPU-written
  image byte for byte;
* NOTBATCHED ~2 MiB spans (the parts mode) from the CPU writer;
* a config-5-shaped DB (packed files with long commits, finalised files,
  active file) written by the CPU, checked by `consistent` on the GPU.
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from tools import zsdb_gen as zg
from zeroskip_amd import consistent as cs
from zeroskip_amd import zsfile

pytestmark = pytest.mark.gpu

UUID = bytes(range(16))


@pytest.fixture(scope="module")
def batched(gpu):
    ppf = zg.pairs_per_file(True)
    nfiles = -(-1_100_000 // ppf)   # > 2^20 commits: commit_kernel's dynamic tail is on
    g = torch.Generator(device=gpu)
    g.manual_seed(0xC0DE)
    img = zg.log_files(UUID, 0, nfiles, ppf, 0, True, g, gpu, writer="cpu")
    offs, lens = zg.log_spans(nfiles, ppf, True, True, gpu)
    torch.cuda.synchronize()
    return img, offs, lens, nfiles


def test_cpu_written_million_commits_verdict(batched):
    img, offs, lens, nfiles = batched
    assert offs.numel() >= 1_100_000 + nfiles
    nbad, bad = zsfile.verify_commits_verdict(img.view(-1), offs, lens, max_len=312)
    nbad = int(nbad.item())
    stale = torch.nonzero(lens == 0).flatten()
    assert nbad == nfiles
    assert torch.equal(torch.sort(bad[:nbad]).values, stale)


def test_cpu_written_million_commits_arrays(batched):
    img, offs, lens, nfiles = batched
    crc, st = zsfile.verify_commits(img.view(-1), offs, lens, max_len=312)
    host = img.view(-1).cpu().numpy()
    o, ln = offs.cpu().numpy(), lens.cpu().numpy()
    st = st.cpu().numpy()
    live = ln > 0
    assert (st[live] == 1).all() and (st[~live] == 0).all()
    # every computed CRC equals the oracle's (the stored field the CPU wrote)
    want = oracle.commit_crcs(host, o[live], ln[live], threads=8)
    got = crc.cpu().numpy().view(np.uint32)[live]
    assert np.array_equal(got, want)
    stored = host[(o[live] + ln[live] + 4)[:, None] + np.arange(4)].view(">u4").reshape(-1)
    assert np.array_equal(stored, want)


def test_gpu_writer_reproduces_cpu_image(batched):
    img, offs, lens, nfiles = batched
    live = lens > 0
    o, ln = offs[live].contiguous(), lens[live].contiguous()
    blank = img.clone().view(-1)
    at = (o + ln + 4)[:, None] + torch.arange(4, device=o.device)
    blank[at.reshape(-1)] = 0
    assert not torch.equal(blank, img.view(-1))
    zsfile.write_commits(blank, o, ln, max_len=312)
    torch.cuda.synchronize()
    assert torch.equal(blank, img.view(-1))


def test_cpu_written_notbatched(gpu):
    ppf = zg.pairs_per_file(False)
    g = torch.Generator(device=gpu)
    g.manual_seed(7)
    nf = 24
    img = zg.log_files(UUID, 0, nf, ppf, 0, False, g, gpu, batched=False, writer="cpu")
    o, ln = zg.log_spans(nf, ppf, False, False, gpu)
    nbad, _ = zsfile.verify_commits_verdict(img.view(-1), o, ln)
    assert int(nbad.item()) == 0
    crc, st = zsfile.verify_commits(img.view(-1), o, ln)
    assert bool((st == 1).all())
    want = oracle.commit_crcs(img.view(-1).cpu().numpy(), o.cpu().numpy(), ln.cpu().numpy(), threads=8)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), want)


def test_cpu_written_db_consistent(gpu):
    db = zg.make_db(device=gpu, packed=2, packed_region_bytes=20 << 20, finalised=12, active_pairs=300,
                    writer="cpu")
    rep = cs.consistent(db)
    assert rep.ok and rep.n_bad == 0 and rep.n_stale == 12
    # the long records commits (> 16 MiB regions) came from the CPU writer
    for name, v in db.items():
        if name.endswith("-0-7") or name.endswith("-8-15"):
            p = oracle.packed_image(v.cpu().numpy(), threads=4)
            assert p["records"]["status"] == 1 and p["records"]["span_len"] > zg.MAX_SHORT
            assert p["pointers"]["status"] == 1


def test_fill_commits_host_million(batched):
    """zscrc_zs_fill_commits on the >= 1 M-commit host image with its CRC
    fields zeroed reproduces the CPU-written image byte for byte."""
    img, offs, lens, nfiles = batched
    host = img.view(-1).cpu().numpy()
    live = (lens > 0).cpu().numpy()
    o, ln = offs.cpu().numpy()[live], lens.cpu().numpy()[live]
    blank = host.copy()
    blank[(o + ln + 4)[:, None] + np.arange(4)] = 0
    rep = zsfile.fill_commits(blank, o, ln, max_len=312)
    assert rep["commits"] == len(o) and rep["no_record"] == 0 and rep["chunks"] > 1
    assert np.array_equal(blank, host)


STATIC_ROUNDS = 1 << 22   # zs::BatchDesc::opt: commit_kernel's static schedule (rounds not dealt)
NO_RUNSPLIT = 1 << 29     # opt: one commit_kernel (not the run-only kernel + the listed leftover rounds)
RO12 = 1 << 31            # opt: the run-only commit_kernel at 12 waves per CU (default 16)
RO_LIST = 1 << 14         # opt: its other rounds listed for a second commit_kernel launch (default: quad bursts)


def test_dealt_rounds_verdicts(batched):
    """commit_kernel's rounds dealt to a workgroup's waves by an LDS counter:
    corruptions spread over the image -- the first rounds, random ones and
    the last ones -- are all found, launch after launch, and every per-commit
    CRC and status equals the static schedule's."""
    from zeroskip_amd._lib import lib
    img, offs, lens, nfiles = batched
    flat = img.view(-1).clone()
    n = offs.numel()
    rng = np.random.default_rng(9)
    live = torch.nonzero(lens > 0).flatten().cpu().numpy()
    hit = np.unique(np.concatenate([rng.choice(live, 40, replace=False), live[-64:][::7], live[:3]]))
    at = (offs.cpu().numpy()[hit] + 100).astype(np.int64)
    flat[torch.from_numpy(at).to(flat.device)] ^= 0x11
    stale = set(torch.nonzero(lens == 0).flatten().cpu().tolist())
    want = set(hit.tolist()) | stale
    for _ in range(3):
        nbad, bad = zsfile.verify_commits_verdict(flat, offs, lens, max_len=312, cap=8192)
        k = int(nbad.item())
        assert k == len(want) and set(bad[:k].cpu().tolist()) == want
    crc_d, st_d = zsfile.verify_commits(flat, offs, lens, max_len=312)
    for opt in (STATIC_ROUNDS, NO_RUNSPLIT, STATIC_ROUNDS | NO_RUNSPLIT, RO12, STATIC_ROUNDS | RO12, RO_LIST,
                RO_LIST | RO12, 0):
        lib().zscrc_set_opt(opt)
        try:
            crc_s, st_s = zsfile.verify_commits(flat, offs, lens, max_len=312)
            nbad_s, _ = zsfile.verify_commits_verdict(flat, offs, lens, max_len=312)
            torch.cuda.synchronize()
        finally:
            lib().zscrc_set_opt(0)
        assert torch.equal(crc_d, crc_s) and torch.equal(st_d, st_s) and int(nbad_s.item()) == len(want), opt
    assert set(torch.nonzero(st_d != 1).flatten().cpu().tolist()) == want
    assert n > 1 << 20


def test_split_commit_batches_writer_and_crcs(batched):
    """The run-only commit_kernel (16 or 12 waves per CU; its other rounds --
    file boundaries, stale finalise commits, the last partial round -- hashed
    in one-piece quad bursts, or listed for a second commit_kernel launch)
    against one commit_kernel: the writer's CRCs into a zeroed copy of the image byte for
    byte, the CRC array, and the per-commit arrays."""
    from zeroskip_amd._lib import lib
    img, offs, lens, nfiles = batched
    flat = img.view(-1)
    live = lens > 0
    ow, lw = offs[live].contiguous(), lens[live].contiguous()
    fields = (ow + lw + 4).view(-1, 1) + torch.arange(4, device=ow.device).view(1, -1)
    out = {}
    for opt in (0, RO12, RO_LIST, NO_RUNSPLIT):
        lib().zscrc_set_opt(opt)
        try:
            z = flat.clone()
            z[fields.view(-1)] = 0
            zsfile.write_commits(z, ow, lw, max_len=312, crc=False)
            crcs = zsfile.commit_crcs(flat, ow, lw, max_len=312)
            arr = zsfile.verify_commits(flat, offs, lens, max_len=312)
            torch.cuda.synchronize()
        finally:
            lib().zscrc_set_opt(0)
        out[opt] = (z, crcs, arr)
    assert torch.equal(out[0][0], flat)                 # the split writer restores every CRC field
    for opt in (RO12, RO_LIST, NO_RUNSPLIT):
        assert torch.equal(out[opt][0], flat), opt
        assert torch.equal(out[0][1], out[opt][1]), opt
        assert torch.equal(out[0][2][0], out[opt][2][0]) and torch.equal(out[0][2][1], out[opt][2][1]), opt


@pytest.mark.parametrize("opt", [0, RO12])
def test_verdicts_two_streams(batched, opt):
    """The run-only commit_kernel's verdicts (16 and 12 waves per CU)
    alternating between two streams, back to back, all find the same corrupt
    commits."""
    from zeroskip_amd._lib import lib
    img, offs, lens, nfiles = batched
    flat = img.view(-1).clone()
    live = torch.nonzero(lens > 0).flatten()
    hit = live[torch.tensor([0, 5000, live.numel() // 2, live.numel() - 1], device=live.device)]
    flat[offs[hit] + 37] ^= 0x5A
    want = set(hit.cpu().tolist()) | set(torch.nonzero(lens == 0).flatten().cpu().tolist())
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    lib().zscrc_set_opt(opt)
    try:
        for k in range(6):
            st = s1 if k % 2 == 0 else s2
            with torch.cuda.stream(st):
                outs.append(zsfile.verify_commits_verdict(flat, offs, lens, max_len=312, cap=8192))
        torch.cuda.synchronize()
    finally:
        lib().zscrc_set_opt(0)
    for nbad, bad in outs:
        k = int(nbad.item())
        assert k == len(want) and set(bad[:k].cpu().tolist()) == want
