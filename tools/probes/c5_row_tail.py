"""The parts of config 5's fixed per-step tail at N ranks,
measured on one GPU: the device pass with its digest row vs with the block
copy back (event-timed, 20 passes each, medians), the copy of N rows to the
host, and the host's unpack + merge of N rows.  Run under rocprofv3
--kernel-trace for the post kernel's duration with and without the row (round 5: cpass_row_kernel, a kernel of its own).
usage: python tools/probes/c5_row_tail.py [N=8]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import consistent as cs  # noqa: E402


def med(xs):
    return float(sorted(xs)[len(xs) // 2])


def main():
    nr = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    db = zg.make_db(device=dev, packed=2, packed_region_bytes=3072 << 20, finalised=1024)
    job = cs.Consistent(cs.open_db(db), 0, 1).prepare()
    st = torch.cuda.current_stream(dev)
    out = {"ranks": nr, "row_int64": job._row_len}
    for what in ("row", "block"):
        ts = []
        for i in range(23):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if what == "row":
                job.device_row((a, b))
            else:
                job.submit((a, b))
            torch.cuda.synchronize()
            if what == "block":
                job.collect()
            if i >= 3:
                ts.append(a.elapsed_time(b))
        out[f"pass_with_{what}_ms"] = round(med(ts), 4)
    rows_d = torch.zeros(nr * job._row_len, dtype=torch.int64, device=dev)
    ts = []
    for i in range(23):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rows = rows_d.cpu()
        ts.append(time.perf_counter() - t0)
    out["rows_d2h_us"] = round(med(ts[3:]) * 1e6, 1)
    row = job.device_row().cpu().numpy()
    job._host_all = job._host_all * nr
    ts = []
    for i in range(23):
        t0 = time.perf_counter()
        allsum = [job._unpack(r, row) for r in range(nr)]
        job._merge(allsum)
        ts.append(time.perf_counter() - t0)
    out["unpack_merge_us"] = round(med(ts[3:]) * 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
