"""HBM traffic per pass from tools/pmc_traffic.sh runs
(gpurun_out/pmc_<case>_FETCH_SIZE, _WRITE_SIZE): each counter summed over the
zs:: dispatches after tools/prof_case.py's marker dispatch (the stream-read
diagnostic: setup's kernels come before it), per kernel and in total,
divided by the passes;
FETCH_SIZE (KB) x2 for the gfx950 wide-read under-count, WRITE_SIZE (KB) as
read, both x1024 to bytes.
usage: python tools/traffic_summary.py <case> <passes> <algorithmic bytes per pass>"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    case, passes, alg = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"gpurun_out/pmc_{case}_{ctr}/**/*counter_collection.csv", recursive=True):
            rows = list(csv.DictReader(open(f)))
            marks = [int(r["Dispatch_Id"]) for r in rows if "stream_read" in r["Kernel_Name"]]
            cut = max(marks) if marks else -1
            for r in rows:
                k = r["Kernel_Name"]
                if "zs::" not in k or "stream_read" in k or int(r["Dispatch_Id"]) <= cut:
                    continue
                k = k.split("(")[0].replace("void ", "")
                per[k][ctr] += float(r["Counter_Value"])
                disp[(k, ctr)].add(r["Dispatch_Id"])
    kern = {}
    fetch = write = 0.0
    for k, c in per.items():
        fb = c.get("FETCH_SIZE", 0.0) * 2 * 1024 / passes
        wb = c.get("WRITE_SIZE", 0.0) * 1024 / passes
        fetch += fb
        write += wb
        kern[k] = {"fetch_bytes_per_pass": int(fb), "write_bytes_per_pass": int(wb),
                   "dispatches": len(disp[(k, "FETCH_SIZE")])}
    print(json.dumps({"case": case, "passes": passes, "fetch_bytes_per_pass": int(fetch),
                      "write_bytes_per_pass": int(write), "traffic_bytes_per_pass": int(fetch + write),
                      "algorithmic_bytes": alg, "ratio": round((fetch + write) / alg, 4), "per_kernel": kern},
                     indent=1))


if __name__ == "__main__":
    main()
