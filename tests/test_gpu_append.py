"""The append path through the unchanged symbol (SURVEY.md sec 8f-4 and rows
a5 / a6): the reference's own src/mfile.c, compiled unmodified and linked to
libzscrc.so (oracle/_ref/mfile_demo, built by oracle/Makefile `ref`), runs
crc32_begin / mfile_write / crc32_end; with ZSCRC_GPU_MIN set, crc32_end's
crc32c_hw (src/mfile.c:538) runs on the GPU.  And the reference's wrappers
(crc32c_map / _iovec / _cstring / _buf, src/crc32c.c:686-711) above the
offload threshold."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle
from zeroskip_amd import crc32c as zc
from zeroskip_amd._lib import lib, stats

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "oracle", "_ref", "mfile_demo")


@pytest.mark.parametrize("piece,pieces", [(1 << 20, 48), (100003, 300)])
def test_reference_mfile_crc32_end_on_gpu(gpu, tmp_path, piece, pieces):
    assert os.path.exists(DEMO), "oracle/_ref/mfile_demo missing: run `make -C oracle ref` where /root/reference exists"
    f = tmp_path / "active"
    res = {}
    for mode, gmin in (("gpu", str(1 << 20)), ("cpu", "0")):
        out = subprocess.run([DEMO, str(f), str(piece), str(pieces)], capture_output=True, text=True, timeout=120,
                             env={**os.environ, "ZSCRC_GPU_MIN": gmin, "ZSCRC_STRICT": "1"})
        assert out.returncode == 0, out.stderr
        res[mode] = json.loads(out.stdout)
    data = open(f, "rb").read()
    want = oracle.crc32c_hw(0, data[40:])
    assert res["gpu"]["gpu_calls"] == 1 and res["cpu"]["gpu_calls"] == 0
    assert res["gpu"]["crc"] == res["cpu"]["crc"] == want
    assert res["gpu"]["span"] == piece * pieces == len(data) - 40


def test_reference_mfile_default_thresholds(gpu, tmp_path):
    """No ZSCRC_GPU_MIN in the environment: the library's measured defaults
    decide.  A process that called zscrc_warmup (mfile_demo's 4th argument)
    offloads crc32_end's span above the warm crossover, and keeps a span
    below it on the CPU; a process without a device context keeps the same
    span on the CPU (the cold crossover: the first GPU call would pay HIP
    init).  Every CRC bit-exact against the oracle."""
    assert os.path.exists(DEMO), "oracle/_ref/mfile_demo missing: run `make -C oracle ref` where /root/reference exists"
    warm = lib().zscrc_gpu_min(0)
    cold = lib().zscrc_gpu_min(1)
    assert 0 < warm < cold
    env = {k: v for k, v in os.environ.items() if not k.startswith("ZSCRC_GPU_MIN")}
    env["ZSCRC_STRICT"] = "1"
    piece = 1 << 20
    cases = [("above-warm", warm // piece + 8, ["warm"], 1), ("below-warm", max(1, warm // piece // 2), ["warm"], 0),
             ("cold", warm // piece + 8, [], 0)]
    for name, pieces, extra, gpu_calls in cases:
        f = tmp_path / name
        out = subprocess.run([DEMO, str(f), str(piece), str(pieces)] + extra, capture_output=True, text=True,
                             timeout=180, env=env)
        assert out.returncode == 0, out.stderr
        res = json.loads(out.stdout)
        data = open(f, "rb").read()
        assert res["crc"] == oracle.crc32c_hw(0, data[40:]), name
        assert res["span"] == piece * pieces and res["gpu_calls"] == gpu_calls, (name, res)
        os.unlink(f)


def test_wrappers_offloaded(gpu):
    d = np.random.default_rng(5).integers(1, 256, (3 << 20) + 11, dtype=np.uint8)   # no NUL: crc32c_buf
    raw = d.tobytes()
    want = oracle.crc32c_hw(0, raw)
    L = lib()
    saved = (L.zscrc_gpu_min(0), L.zscrc_gpu_min(1))
    before = stats()
    L.zscrc_set_gpu_min(1 << 20)
    try:
        assert L.crc32c_map(raw, len(raw)) == want
        cbuf = ctypes.create_string_buffer(raw, len(raw) + 1)
        assert L.crc32c_buf(cbuf) == want

        class CString(ctypes.Structure):
            _fields_ = [("len", ctypes.c_size_t), ("alloc", ctypes.c_size_t), ("buf", ctypes.c_char_p)]
        cs = CString(len(raw), len(raw) + 1, ctypes.cast(cbuf, ctypes.c_char_p))
        assert L.crc32c_cstring(ctypes.byref(cs)) == want

        class Iov(ctypes.Structure):
            _fields_ = [("iov_base", ctypes.c_void_p), ("iov_len", ctypes.c_size_t)]
        base = ctypes.addressof(cbuf)
        cuts = [0, 1 << 20, (1 << 20) + 5, (1 << 20) + 5, len(raw)]          # a zero-length iov too
        iov = (Iov * 4)(*[Iov(base + a, b - a) for a, b in zip(cuts[:-1], cuts[1:])])
        assert L.crc32c_iovec(iov, 4) == want
    finally:
        L.zscrc_set_gpu_min_pair(*saved)
    after = stats()
    # map, buf, cstring: one offloaded call each; iovec: its two >= 1 MiB pieces
    assert after[1] - before[1] == 5
    assert zc.crc32c(0, raw) == want
