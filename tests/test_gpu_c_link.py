"""BASELINE config 1 on the MI355X host (the GPU twin of
tests/test_c_link.py::test_config1_harness): tools/crc32bench.c linked to
libzscrc.so runs the reference harness's workload (benchmark/crc32bench.c:
45-112) through the drop-in symbols with the GPU present, and its routing leg
shows the scalar offload's thresholds at work -- a 64 MiB crc32c_hw call
before any device context exists stays on the CPU (cold threshold, 5 GiB),
the same call after zscrc_warmup() runs on the GPU (warm threshold, 32 MiB),
both bit-exact against the oracle."""
import json
import os
import subprocess

import numpy as np
import pytest

from zeroskip_amd import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_config1_harness_on_gpu_host(gpu, tmp_path):
    from oracle import oracle
    from tests.golden.datagen import xorshift64_bytes

    exe = tmp_path / "crc32bench"
    libdir = os.path.dirname(LIB_PATH)
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tools", "crc32bench.c"), "-L", libdir, "-lzscrc", "-lz",
                           f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    env = {k: v for k, v in os.environ.items() if not k.startswith("ZSCRC_")}   # library defaults
    route = 64 << 20
    out = subprocess.run([str(exe), "-r", "200", "-b", str(route)], capture_output=True, text=True,
                         timeout=100, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert rep["ok"] is True and rep["ok_all"] is True, rep
    r = rep["routing"]
    assert r["cold_on_cpu"] and r["warm_on_gpu"] and r["warmup_rc"] == 0, r
    assert r["cold_threshold"] > route >= r["warm_threshold"], r
    mib = xorshift64_bytes(1 << 20)
    want = oracle.crc32c_hw(0, np.tile(mib, route >> 20))
    assert r["crc"] == f"{want:08x}", (r, hex(want))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "config1_gpu_host.json"), "w") as f:
        f.write(out.stdout.strip().splitlines()[-1] + "\n")
