"""Where the per-wave end-time spread of the persistent kernels lives
(zscrc_diag_wave_times): inside workgroups or between them, per XCD -- for
config 3's qteam_kernel, a 3 GiB span on xteam_kernel and config 5's
multi-span launch shape, so per-workgroup dealing (commit_kernel and
multi64_kernel deal their units by an LDS counter) can be judged for them.
usage (GPU box): python tools/probes/wave_spread.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd._lib import check, lib  # noqa: E402


def waves(name, fn, nwaves, per_block):
    buf = torch.zeros(nwaves * 4, dtype=torch.int64, device="cuda")
    for _ in range(30):            # the power controller settles under load (DESIGN_LOG.md 1.6)
        fn()
    torch.cuda.synchronize()
    check(lib().zscrc_diag_wave_times(buf.data_ptr()), "wave times")
    fn()
    torch.cuda.synchronize()
    check(lib().zscrc_diag_wave_times(None), "wave times off")
    a = buf.view(-1, 4).cpu().numpy().astype(np.int64)
    live = a[:, 0] > 0
    wid = np.nonzero(live)[0]
    a = a[live]
    t0 = a[:, 0].min()
    end = (a[:, 2] - t0) / 100.0
    blk = wid // per_block
    ub = np.unique(blk)
    bmax = np.array([end[blk == b].max() for b in ub])
    bmin = np.array([end[blk == b].min() for b in ub])
    xcd = ub % 8
    print(json.dumps({"case": name, "waves": int(live.sum()), "kernel_us": round(float(end.max()), 1),
                      "end_us_p10_p50_max": [round(float(np.percentile(end, q)), 1) for q in (10, 50, 100)],
                      "within_block_range_us_p50": round(float(np.median(bmax - bmin)), 1),
                      "block_end_us_p10_p50_max": [round(float(np.percentile(bmax, q)), 1) for q in (10, 50, 100)],
                      "xcd_block_end_us_median": [round(float(np.median(bmax[xcd == x])), 1) for x in range(8)],
                      "units_per_wave": sorted(set(int(x) for x in a[:, 3]))[:8]}), flush=True)


def main():
    if os.environ.get("WS_OPT"):        # e.g. 16777216: qteam parts dealt per workgroup
        lib().zscrc_set_opt(int(os.environ["WS_OPT"]))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    c4 = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(65536, dtype=torch.int32, device=dev)
    waves("config 3: 65,536 x 64 KiB (qteam_kernel)", lambda: zd.crc_fixed(c4, 65536, 65536, 65536, out=out),
          ncu * 16, 16)
    old = lib().zscrc_set_xdeal(0)
    waves("3 GiB span (xteam segments, static: two per wave)", lambda: zd.crc_span(c4[:3 << 30]), ncu * 16, 16)
    lib().zscrc_set_xdeal(old)
    waves("3 GiB span (xteam segments, 16 per wave dealt per workgroup)", lambda: zd.crc_span(c4[:3 << 30]),
          ncu * 16, 16)
    waves("4,096 x 1 MiB records (xteam_kernel)", lambda: zd.crc_fixed(c4, 1 << 20, 1 << 20, 4096), ncu * 16, 16)


if __name__ == "__main__":
    main()
