"""Sustained back-to-back launches of the config-3 kernels: per-launch HIP
event times over a long run of each kernel (team_kernel<16>, qteam_kernel,
the nt streaming-read ceiling), an idle gap between the kernels.  Separates
a kernel that slows down under sustained load (power / clock management)
from one that is slower per launch.

usage: python tools/probes/sustain_probe.py [launches] > gpurun_out/sustain.jsonl"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd._lib import QTEAM_DEFAULT, check, lib  # noqa: E402

N, L = 65536, 65536


def main():
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    modes = os.environ.get("SP_MODES", "team16,qteam,stream,qteam,team16").split(",")
    dev = torch.device("cuda", 0)
    data = torch.randint(0, 256, (N * L,), dtype=torch.uint8, device=dev)
    out = torch.empty(N, dtype=torch.int32, device=dev)
    scratch = torch.zeros(4, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    opt = int(os.environ.get("SP_OPT", "0"))
    for mode in modes:
        lib().zscrc_set_qteam(1 if mode == "qteam" else 0)
        lib().zscrc_set_opt(opt)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
        torch.cuda.synchronize()
        for a, b in ev:
            a.record(st)
            if mode == "stream":
                check(lib().zscrc_diag_stream_read(data.data_ptr(), N * L, scratch.data_ptr(), 1, st.cuda_stream),
                      "stream read")
            else:
                check(lib().zscrc_device_fixed(data.data_ptr(), L, L, 0, out.data_ptr(), N, 0, st.cuda_stream),
                      "zscrc_device_fixed")
            b.record(st)
        torch.cuda.synchronize()
        ms = [round(a.elapsed_time(b), 4) for a, b in ev]
        s = sorted(ms)
        row = {"mode": mode, "opt": opt, "median": s[len(s) // 2], "mean": round(sum(ms) / len(ms), 4),
               "min": s[0], "max": s[-1]}
        if launches > 100:  # long runs: means per block of 25 launches
            row["block25"] = [round(sum(ms[i:i + 25]) / len(ms[i:i + 25]), 4) for i in range(0, launches, 25)]
        else:
            row["ms"] = ms
        print(json.dumps(row), flush=True)
        time.sleep(float(os.environ.get("SP_SLEEP", "3")))
    lib().zscrc_set_qteam(QTEAM_DEFAULT)
    lib().zscrc_set_opt(0)


if __name__ == "__main__":
    main()
