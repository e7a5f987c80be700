"""TA_ADDR_STALLED_BY_TC_CYCLES / TA_TA_BUSY per kernel name from a rocprofv3
--pmc counter_collection.csv (all dispatches of a name summed).
usage: python tools/probes/ta_ratio.py <rocprofv3 -d dir>"""
import csv
import glob
import json
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
busy, stall, n = defaultdict(float), defaultdict(float), defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if r["Counter_Name"] == "TA_TA_BUSY":
        busy[k] += float(r["Counter_Value"])
    elif r["Counter_Name"] == "TA_ADDR_STALLED_BY_TC_CYCLES":
        stall[k] += float(r["Counter_Value"])
    n[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
for k in busy:
    print(json.dumps({"kernel": k, "dispatches": len(n[k]), "TA_stall_ratio": round(stall[k] / busy[k], 3) if busy[k] else None}))
