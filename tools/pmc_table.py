"""Per-kernel PMC sums from tools/pmc_case.sh runs: one row per zs:: kernel,
counters summed over its dispatches, divided by the passes and by the bytes
one pass reads.  usage: python tools/pmc_table.py gpurun_out/pmc_config2 PASSES BYTES_PER_PASS"""
import csv
import glob
import json
import sys
from collections import defaultdict

stem, passes, nbytes = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
tot = defaultdict(lambda: defaultdict(float))
for d in sorted(glob.glob(stem + "_[0-9]")):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "zs::" not in k or "stream_read" in k:
                continue
            k = k.split("(")[0].replace("void ", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
out = {}
for k, c in tot.items():
    row = {n: v / passes for n, v in sorted(c.items())}
    per_kb = {n + "_per_KiB": round(v / passes / (nbytes / 1024), 3) for n, v in sorted(c.items())
              if n.startswith("SQ_INSTS") or n.startswith("SQ_WAIT") or n in ("SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES",
                                                                              "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU",
                                                                              "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY")}
    if c.get("TA_TA_BUSY"):
        per_kb["TA_stall_ratio"] = round(c["TA_ADDR_STALLED_BY_TC_CYCLES"] / c["TA_TA_BUSY"], 3)
    out[k] = {"per_pass": row, "per_KiB_read": per_kb}
print(json.dumps(out, indent=1))
