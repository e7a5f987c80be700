"""Interleaved A/B of qteam_kernel (coalesced non-temporal 16-lane column-quad
teams) against team_kernel<16> (per-lane 64-byte piece loads) on
equal-length fixed-stride records, config 3 first.  Median of 15 HIP-event
timed launches per mode, the modes alternating launch by launch; the outputs
of the two modes compared record by record.

usage: python tools/probes/qteam_ab.py [> profiles/r02/qteam_ab.jsonl]
env QT_CASES=stride:len:n,... to pick shapes; QT_VS_XTEAM=1: xteam_kernel (the
default from 256 KiB) against qteam forced"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd._lib import QTEAM_DEFAULT, check, lib  # noqa: E402

CASES = [(65536, 65536, 65536), (8192, 8192, 1 << 19), (16384, 16384, 1 << 18), (32768, 32768, 1 << 17),
         (131072, 131072, 1 << 15), (65536, 65536, 65536)]


def main():
    dev = torch.device("cuda", 0)
    big = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
    cases = CASES
    if os.environ.get("QT_CASES"):
        cases = [tuple(int(v) for v in c.split(":")) for c in os.environ["QT_CASES"].split(",")]
    st = torch.cuda.current_stream()
    reps = int(os.environ.get("QT_REPS", "15"))
    for stride, length, n in cases:
        outs = {m: torch.empty(n, dtype=torch.int32, device=dev) for m in (0, 1)}
        ts = {0: [], 1: []}
        names = {}
        for i in range(reps + 2):
            for m in (0, 1):
                if os.environ.get("QT_VS_XTEAM"):
                    # mode 0: the default dispatch (xteam_kernel for >= 256 KiB); 1: qteam forced
                    lib().zscrc_set_xteam(1, (1 << 40) if m else (256 << 10))
                    lib().zscrc_set_qteam(1)
                else:
                    lib().zscrc_set_qteam(m)
                names[m] = lib().zscrc_fixed_kernel(big.data_ptr(), stride, length, n).decode()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                check(lib().zscrc_device_fixed(big.data_ptr(), stride, length, 0, outs[m].data_ptr(), n, 0,
                                               st.cuda_stream), "zscrc_device_fixed")
                b.record(st)
                torch.cuda.synchronize()
                if i >= 2:
                    ts[m].append(a.elapsed_time(b))
        lib().zscrc_set_qteam(QTEAM_DEFAULT)
        lib().zscrc_set_xteam(1, 256 << 10)
        row = {"stride": stride, "len": length, "n": n}
        for m in (0, 1):
            ms = sorted(ts[m])[len(ts[m]) // 2]
            row[f"{names[m]}_ms"] = round(ms, 4)
            row[f"{names[m]}_min_ms"] = round(min(ts[m]), 4)
            row[f"{names[m]}_p90_ms"] = round(sorted(ts[m])[(len(ts[m]) * 9) // 10], 4)
            row[f"{names[m]}_GBs"] = round(n * (length + 4) / ms / 1e6, 1)
        row["mismatches"] = int((outs[0] != outs[1]).sum())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
