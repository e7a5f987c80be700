"""Host-CPU scaling of the oracle's timing leg on the GPU box: the crc32c_hw
class and a plain read over 512 MiB of 64 KiB chunks at several thread
counts (pinned one per physical core, dealt over L3 domains), with the
cgroup's CPU quota and throttling counters.  usage: python tools/probes/cpu_threads.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle  # noqa: E402


def rd(p):
    try:
        return open(p).read().strip()
    except OSError:
        return None


def main():
    data = np.random.default_rng(1).integers(0, 256, 512 << 20, dtype=np.uint8)
    n, L = (512 << 20) // 65536, 65536
    print(json.dumps({"cpu.max": rd("/sys/fs/cgroup/cpu.max"), "cpuset": rd("/sys/fs/cgroup/cpuset.cpus.effective"),
                      "affinity": len(os.sched_getaffinity(0)), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                      "stat0": rd("/sys/fs/cgroup/cpu.stat")}), flush=True)
    for t in (1, 4, 8, 12, 14, 15, 16, 20, 24, 32):
        row = {"threads": t}
        for impl in ("hw", "read"):
            _, el, p = oracle.batch_rate(data, n=n, stride=L, fixed_len=L, impl=impl, threads=t,
                                         cpus=oracle.pick_cpus(t), budget=1.5)
            row[impl] = round(p * n * L / el / 2**30, 2)
        _, el, p = oracle.batch_rate(data, n=n, stride=L, fixed_len=L, impl="hw", threads=t, budget=1.5)
        row["hw_unpinned"] = round(p * n * L / el / 2**30, 2)
        row["stat"] = rd("/sys/fs/cgroup/cpu.stat")
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
