"""Phase times of the single-block classify + plan launch
(zscrc_diag_classify_times) on config 4's NOTBATCHED layout (1,488 commits
of ~2 MiB): count pass, scatter, the class-3 plan's table load, record scan
+ part lists, tail and plan write -- for the ranged verdict, the unranged
verdict and the per-commit arrays, after 30 calls that settle the power
controller.  usage (GPU box): python tools/probes/classify_phases.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402
from zeroskip_amd._lib import check, lib  # noqa: E402

NAMES = ["count", "scatter", "plan_table", "plan_scan", "plan_tail", "plan_write", "end"]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED)
    ppf = zg.pairs_per_file(False)
    nf = -(-10_000_000 // ppf)
    img = zg.log_files(bytes(range(16)), 0, nf, ppf, 0, False, g, dev, batched=False).view(-1)
    offs, lens = zg.log_spans(nf, ppf, False, False, dev)
    lo, hi = int(lens.min().item()), int(lens.max().item())
    out = (torch.empty(1, dtype=torch.int64, device=dev), torch.empty(64, dtype=torch.int64, device=dev))
    forms = {"verdict_range": lambda: zsfile.verify_commits_verdict(img, offs, lens, out=out, min_len=lo, max_len=hi),
             "verdict": lambda: zsfile.verify_commits_verdict(img, offs, lens, out=out),
             "arrays": lambda: zsfile.verify_commits(img, offs, lens)}
    buf = torch.zeros(8, dtype=torch.int64, device=dev)
    for name, fn in forms.items():
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        rows = []
        check(lib().zscrc_diag_classify_times(buf.data_ptr()), "classify times")
        try:
            for _ in range(10):
                buf.zero_()
                fn()
                torch.cuda.synchronize()
                t = buf.cpu().numpy().astype(np.int64)
                # each phase from the last stamp before it (the fused class-3-only
                # pass stamps 0, 2, 4, 6, 7 only)
                row = []
                for k in range(7):
                    prev = max((j for j in range(k + 1) if t[j]), default=None)
                    row.append((t[k + 1] - t[prev]) / 100.0 if t[k + 1] and prev is not None else None)
                row.append((t[7] - t[0]) / 100.0 if t[7] and t[0] else None)
                rows.append(row)
        finally:
            check(lib().zscrc_diag_classify_times(None), "classify times off")
        med = {}
        for k, n in enumerate(NAMES):
            v = [r[k] for r in rows if r[k] is not None]
            med[n] = round(float(np.median(v)), 2) if v else None
        tot = [r[7] for r in rows if r[7] is not None]
        print(json.dumps({"form": name, "commits": int(offs.numel()), "phase_us_median": med,
                          "entry_to_end_us_median": round(float(np.median(tot)), 2) if tot else None}),
              flush=True)


if __name__ == "__main__":
    main()
