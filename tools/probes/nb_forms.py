"""Config 4 NOTBATCHED's three forms (ranged verdict, unranged verdict,
per-commit arrays) timed two ways, interleaved round by round: the GPU time
per call (HIP events around 20 calls back to back) and the host's
submission time per call (perf_counter around the same 20 calls, before the
synchronize) -- whether a form is bound by its kernels or by its host side.
usage (GPU box): python tools/probes/nb_forms.py"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402


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
    st = torch.cuda.current_stream(dev)
    for fn in forms.values():
        for _ in range(10):
            fn()
    torch.cuda.synchronize()
    gpu = {k: [] for k in forms}
    host = {k: [] for k in forms}
    for _ in range(7):
        for name, fn in forms.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            t0 = time.perf_counter()
            for _ in range(20):
                fn()
            t1 = time.perf_counter()
            b.record(st)
            torch.cuda.synchronize()
            gpu[name].append(a.elapsed_time(b) / 20)
            host[name].append((t1 - t0) * 1e3 / 20)
    print(json.dumps({k: {"gpu_ms_per_call": round(float(np.median(gpu[k])), 4),
                          "host_submit_ms_per_call": round(float(np.median(host[k])), 4)} for k in forms}), flush=True)
    assert int(out[0].item()) == 0


if __name__ == "__main__":
    main()
