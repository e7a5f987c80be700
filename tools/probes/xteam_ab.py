"""A/B of the fixed-stride long-record kernels on one GPU: xteam_kernel (coalesced
non-temporal whole-wave teams) against the round-1 dispatch (team<16> /
team<64> per-lane piece loads).  Median of 15 HIP-event timed launches per
case, the modes interleaved launch by launch (run back to back, the first
mode measured up to 8 % apart from the same kernel later); outputs of every
mode compared with each other.

usage: python tools/probes/xteam_ab.py [> profiles/r02/xteam_ab.jsonl]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd._lib import check, lib  # noqa: E402

CASES = [(65536, 65536, 65536), (4096, 4096, 1 << 20), (8192, 8192, 1 << 19), (16384, 16384, 1 << 18),
         (1 << 20, 1 << 20, 4096), (1 << 20, 1 << 20, 512), (65536, 65536, 4096), (5000, 5000, 800000)]


def timed_modes(data, stride, length, n, modes, reps=15):
    """median launch time per xteam mode, the modes interleaved launch by launch
    (clock and thermal drift hits every mode alike); outputs per mode"""
    st = torch.cuda.current_stream()
    outs = {m: torch.empty(n, dtype=torch.int32, device=data.device) for m in modes}
    ts = {m: [] for m in modes}
    for i in range(reps + 2):
        for m in modes:
            lib().zscrc_set_xteam(m, 4096)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            check(lib().zscrc_device_fixed(data.data_ptr(), stride, length, 0, outs[m].data_ptr(), n, 0,
                                           st.cuda_stream), "zscrc_device_fixed")
            b.record(st)
            torch.cuda.synchronize()
            if i >= 2:
                ts[m].append(a.elapsed_time(b))
    lib().zscrc_set_xteam(1, 4096)
    return {m: sorted(v)[len(v) // 2] for m, v in ts.items()}, outs


def main():
    dev = torch.device("cuda", 0)
    big = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
    modes = [int(x) for x in os.environ.get("XT_MODES", "0,1").split(",")]
    for stride, length, n in CASES:
        if (n - 1) * stride + length > big.numel():
            continue
        row = {"stride": stride, "len": length, "n": n}
        ms, outs = timed_modes(big, stride, length, n, modes)
        for m in modes:
            lib().zscrc_set_xteam(m, 4096)
            key = f"xteam{m}" if m else f"team{lib().zscrc_team_for(length, n)}"
            row[key + "_ms"] = round(ms[m], 4)
            row[key + "_GBs"] = round(n * length / ms[m] / 1e6, 1)
            if not torch.equal(outs[modes[0]], outs[m]):
                row[key + "_MISMATCH"] = int((outs[modes[0]] != outs[m]).sum())
        lib().zscrc_set_xteam(1, 4096)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
