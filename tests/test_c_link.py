"""A C program compiled against include/zscrc.h Part 1 links to libzscrc.so and
reproduces the reference's known answers through the drop-in symbols (host
scalar path; no GPU)."""
import os
import subprocess

from zeroskip_amd import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_program_links_and_matches(tmp_path):
    exe = tmp_path / "link_test"
    libdir = os.path.dirname(LIB_PATH)
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "link_test.c"), "-L", libdir, "-lzscrc",
                           f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "OK", out.stdout + out.stderr


def test_config1_harness(tmp_path):
    """BASELINE config 1 (tools/crc32bench.c) through the drop-in symbols: the
    574-byte text's CRC is the golden one under hw / sw / dispatch, and the
    1 MiB xorshift64 buffer's CRC matches the oracle."""
    import json

    import numpy as np

    from oracle import oracle
    from tests.golden.datagen import xorshift64_bytes

    exe = tmp_path / "crc32bench"
    libdir = os.path.dirname(LIB_PATH)
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tools", "crc32bench.c"), "-L", libdir, "-lzscrc", "-lz",
                           f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    out = subprocess.run([str(exe), "-r", "20"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert rep["ok"] is True
    want = oracle.batch(xorshift64_bytes(1 << 20), np.array([0], np.uint64), np.array([1 << 20], np.uint64))[0]
    assert f"(crc {int(want):08x})" in out.stdout.splitlines()[0]
