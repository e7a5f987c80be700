"""bench.py --gpus N never measures fewer GPUs than asked: without a launcher
it starts torchrun itself (one rank per GPU, 127.0.0.1) before anything
touches a GPU; a WORLD_SIZE that disagrees with --gpus is an error.  CPU only
(BENCH_LAUNCH_DRYRUN prints the launch instead of running it)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=120)


def test_gpus_without_launcher_spawns_torchrun():
    p = _run(["--gpus", "4", "--steps", "3", "--warmup", "1"], BENCH_LAUNCH_DRYRUN="1")
    assert p.returncode == 0, p.stderr
    cmd = json.loads(p.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-6:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3", "--warmup", "1"][-6:]


def test_world_size_mismatch_is_an_error():
    p = _run(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)


def test_traffic_only_for_its_own_kernel():
    """a PMC traffic record is reported only on the line of the
    kernel it was measured on (profiles/pmc_traffic.json is keyed by config
    and names its kernel)."""
    import json
    import bench
    rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    for cfg in ("config2", "config3", "config4", "config5"):
        assert cfg in rec and rec[cfg]["kernel"] and rec[cfg]["bytes_per_launch"] > 0, cfg
        assert os.path.exists(os.path.join(ROOT, rec[cfg]["record"])), rec[cfg]["record"]
        t, src = bench.traffic_for(cfg, rec[cfg]["kernel"])
        assert t == rec[cfg]["bytes_per_launch"]
        t, src = bench.traffic_for(cfg, rec[cfg]["kernel"] + "+another_kernel")
        assert t is None and "not reported" in src
