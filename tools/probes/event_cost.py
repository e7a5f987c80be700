"""Cost of the bench's per-step timing events: config 3's step (one
zscrc_device_fixed launch over 65,536 x 64 KiB) timed in blocks of 20 steps
with a timing-event pair around every step (bench.py's Timer) against one
pair around the block, interleaved over 8 rounds after the power settles.
usage (GPU box): python tools/probes/event_cost.py"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd._lib import check, lib  # noqa: E402

NCHUNK, CHUNK, K = 65536, 65536, 20


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    data = torch.randint(0, 256, (NCHUNK * CHUNK,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(NCHUNK, dtype=torch.int32, device=dev)

    def launch():
        check(lib().zscrc_device_fixed(data.data_ptr(), CHUNK, CHUNK, 0, out.data_ptr(), NCHUNK, 0,
                                       stream.cuda_stream), "zscrc_device_fixed")

    for _ in range(200):
        launch()
    torch.cuda.synchronize()
    rows = {"per_step_events": [], "block_events": [], "no_events": []}
    kern = {"per_step_events": [], "block_events": []}
    for _ in range(8):
        for form in rows:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if form == "block_events":
                ev[0][0].record(stream)
            for i in range(K):
                if form == "per_step_events":
                    ev[i][0].record(stream)
                launch()
                if form == "per_step_events":
                    ev[i][1].record(stream)
            if form == "block_events":
                ev[0][1].record(stream)
            torch.cuda.synchronize()
            rows[form].append((time.perf_counter() - t0) / K * 1e3)
            if form == "per_step_events":
                kern[form].append(float(np.mean([a.elapsed_time(b) for a, b in ev])))
            elif form == "block_events":
                kern[form].append(ev[0][0].elapsed_time(ev[0][1]) / K)
    print(json.dumps({"step_ms_median": {k: round(float(np.median(v)), 4) for k, v in rows.items()},
                      "event_ms_median": {k: round(float(np.median(v)), 4) for k, v in kern.items()},
                      "step_ms": {k: [round(x, 4) for x in v] for k, v in rows.items()}}), flush=True)


if __name__ == "__main__":
    main()
