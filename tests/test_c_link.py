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
