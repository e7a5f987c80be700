"""Per-wave timing of xteam_kernel launches (zscrc_diag_wave_times): the
NOTBATCHED verdict (parts mode) beside a 3 GiB span and 4,096 x 762 KiB
records (the same bytes per wave, one record each), so plan imbalance,
per-part start-up and the kernel's tail can be told apart.
usage (GPU box): python tools/probes/xparts_waves.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402
from zeroskip_amd._lib import check, lib  # noqa: E402


def waves(name, fn, nwaves):
    buf = torch.zeros(nwaves * 4, dtype=torch.int64, device="cuda")
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    check(lib().zscrc_diag_wave_times(buf.data_ptr()), "wave times")
    fn()
    torch.cuda.synchronize()
    check(lib().zscrc_diag_wave_times(None), "wave times off")
    a = buf.view(-1, 4).cpu().numpy().astype(np.int64)
    live = a[:, 0] > 0
    a = a[live]
    t0 = a[:, 0].min()
    ent, fill, end, cnt = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, (a[:, 2] - t0) / 100.0, a[:, 3]
    work = end - fill
    wave_id = np.nonzero(live)[0]
    xcd = (wave_id // 16) % 8                      # blockIdx.x % 8: the XCD a block lands on
    by_xcd = [round(float(np.median(end[xcd == x])), 1) for x in range(8)]
    row = {"case": name, "end_us_median_by_xcd": by_xcd, "waves_recorded": int(live.sum()), "kernel_us": round(float(end.max()), 1),
           "entry_us_max": round(float(ent.max()), 1), "fill_done_us_p50": round(float(np.median(fill)), 1),
           "end_us_p10_p50_p90_max": [round(float(np.percentile(end, q)), 1) for q in (10, 50, 90, 100)],
           "waves_by_items": {int(k): int((cnt == k).sum()) for k in np.unique(cnt)},
           "work_us_by_items": {int(k): round(float(work[cnt == k].mean()), 1) for k in np.unique(cnt)}}
    print(json.dumps(row), flush=True)


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nw = ncu * 16
    ppf = zg.pairs_per_file(False)
    nf = -(-10_000_000 // ppf)
    img = zg.log_files(bytes(range(16)), 0, nf, ppf, 0, False, g, dev, batched=False).view(-1)
    o, ln = zg.log_spans(nf, ppf, False, False, dev)
    vout = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(64, dtype=torch.int64, device=dev))
    waves("notbatched verdict (xteam parts)", lambda: zsfile.verify_commits_verdict(img, o, ln, out=vout), nw)
    if os.environ.get("WAVES_NB_RANGE"):  # the bench's ranged verdict: one launch (MODE 3) and tuning bit 64
        lo, hi = int(ln.min().item()), int(ln.max().item())
        for opt in (0, 64):
            lib().zscrc_set_opt(opt)
            waves(f"notbatched ranged verdict opt {opt}",
                  lambda: zsfile.verify_commits_verdict(img, o, ln, out=vout, min_len=lo, max_len=hi), nw)
        lib().zscrc_set_opt(0)
        return
    del img
    c3 = torch.randint(0, 256, (3 << 30,), dtype=torch.uint8, device=dev, generator=g)
    waves("span 3 GiB (xteam segments)", lambda: zd.crc_span(c3), nw)
    per = 762 * 1024
    waves("4096 x 762 KiB records (xteam, one per wave)", lambda: zd.crc_fixed(c3, per, per, 4096), nw)
    if os.environ.get("WAVES_C3"):  # config 3's qteam has no wave timing; its xteam form for comparison
        del c3
        c4 = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev, generator=g)
        waves("4 GiB span (xteam segments)", lambda: zd.crc_span(c4), nw)
        waves("config 3: 65,536 x 64 KiB (qteam_kernel)", lambda: zd.crc_fixed(c4, 65536, 65536, 65536), nw)


if __name__ == "__main__":
    main()
