"""Host-CPU scaling of the oracle's timing leg on the GPU box: the crc32c_hw
class and a plain read over 512 MiB of 64 KiB chunks at several thread
counts (pinned one per physical core, dealt over L3 domains), with the
cgroup's CPU quota and throttling counters; the core clocks (/proc/cpuinfo
MHz of the pinned CPUs, read while a leg runs).  usage: python
tools/probes/cpu_threads.py [record_bytes]  (default 65536; 64 = config 2)"""
import threading
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle  # noqa: E402


def rd(p):
    try:
        return open(p).read().strip()
    except OSError:
        return None


def cpu_mhz(cpus):
    """/proc/cpuinfo's MHz of the given logical CPUs (the kernel's last sample)."""
    out, cur = [], None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("processor"):
                cur = int(ln.split(":")[1])
            elif ln.startswith("cpu MHz") and cur in cpus:
                out.append(float(ln.split(":")[1]))
    except OSError:
        pass
    return out


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    data = np.random.default_rng(1).integers(0, 256, 512 << 20, dtype=np.uint8)
    n = (512 << 20) // L
    print(json.dumps({"cpu.max": rd("/sys/fs/cgroup/cpu.max"), "cpuset": rd("/sys/fs/cgroup/cpuset.cpus.effective"),
                      "affinity": len(os.sched_getaffinity(0)), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                      "stat0": rd("/sys/fs/cgroup/cpu.stat")}), flush=True)
    for t in (1, 4, 8, 12, 14, 15, 16, 20, 24, 32):
        row = {"threads": t}
        cpus = oracle.pick_cpus(t)
        for impl in ("hw", "read"):
            mhz = []
            th = threading.Thread(target=lambda: (time.sleep(0.7), mhz.extend(cpu_mhz(cpus))))
            th.start()
            _, el, p = oracle.batch_rate(data, n=n, stride=L, fixed_len=L, impl=impl, threads=t,
                                         cpus=cpus, budget=1.5)
            th.join()
            row[impl] = round(p * n * L / el / 2**30, 2)
            if mhz:
                row[impl + "_mhz_median"] = round(float(np.median(mhz)))
        _, el, p = oracle.batch_rate(data, n=n, stride=L, fixed_len=L, impl="hw", threads=t, budget=1.5)
        row["hw_unpinned"] = round(p * n * L / el / 2**30, 2)
        row["stat"] = rd("/sys/fs/cgroup/cpu.stat")
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
