"""zscrc_zs_verify_files end to end on config 4's BATCHED log images (host
memory) for several staging-slot sizes (env ZSCRC_FILES_SLOT, read per
call): best of 5 wall times and the library's phases.  usage: python tools/probes/slot_sweep.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    ppf = zg.pairs_per_file(True)
    nf = -(-10_000_000 // ppf)
    img = zg.log_files(bytes(range(16)), 0, nf, ppf, 0, True, g, dev)
    host = img.cpu()
    images = list(host.numpy().reshape(nf, -1))
    kinds = [zsfile.FINALISED] * nf
    del img
    for mib in (64, 16, 32, 128, 64):
        os.environ["ZSCRC_FILES_SLOT"] = str(mib << 20)
        zsfile.verify_files(images, kinds)
        best = None
        for _ in range(5):
            t0 = time.perf_counter()
            rep = zsfile.verify_files(images, kinds)
            dt = time.perf_counter() - t0
            if best is None or dt < best[0]:
                best = (dt, rep)
        dt, rep = best
        print(json.dumps({"slot_MiB": mib, "s": round(dt, 4), "GBs": round(host.numel() / dt / 1e9, 2),
                          "copy_s": round(rep["copy_s"], 4), "tail_s": round(rep["verify_tail_s"], 4),
                          "lib_s": round(rep["total_s"], 4)}), flush=True)


if __name__ == "__main__":
    main()
