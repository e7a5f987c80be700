"""Per-kernel PMC summary of a tools/pmc_case.sh run: every pass's
counters (gpurun_out/pmc_<case>_<i>/run_counter_collection.csv) summed over
the dispatches of one kernel, per dispatch and per KiB of algorithmic bytes,
with derived ratios (TA stall / busy, VMEM instructions in flight per KiB,
wave-cycles waiting per KiB).
usage: python tools/probes/pmc_summary.py <case> <kernel substring> <bytes per dispatch> [passes 1 2 3] [--box file.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    box = None
    if "--box" in args:
        i = args.index("--box")
        box = json.load(open(args[i + 1]))
        del args[i:i + 2]
    case, kname, nbytes = args[0], args[1], float(args[2])
    passes = args[3:] or ["1", "2", "3"]
    tot = defaultdict(float)
    disp = {}
    for p in passes:
        for f in glob.glob(f"gpurun_out/pmc_{case}_{p}/**/*counter_collection.csv", recursive=True):
            ids = set()
            for r in csv.DictReader(open(f)):
                if kname not in r["Kernel_Name"]:
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                ids.add(r["Dispatch_Id"])
            disp[p] = len(ids)
    n = max(disp.values()) if disp else 0
    if not n:
        raise SystemExit(f"no dispatch of {kname} in gpurun_out/pmc_{case}_*")
    kib = nbytes / 1024.0
    out = {"case": case, "kernel": kname, "dispatches_per_pass": disp, "bytes_per_dispatch": nbytes,
           "per_dispatch": {k: round(v / n, 1) for k, v in sorted(tot.items())},
           "per_KiB": {k: round(v / n / kib, 3) for k, v in sorted(tot.items()) if k.startswith("SQ_")}}
    if tot.get("TA_TA_BUSY"):
        out["ta_stall_ratio"] = round(tot["TA_ADDR_STALLED_BY_TC_CYCLES"] / tot["TA_TA_BUSY"], 3)
    if box:
        out["box"] = box
    print(json.dumps(out))


if __name__ == "__main__":
    main()
