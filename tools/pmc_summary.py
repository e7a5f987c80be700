"""Average per-dispatch counters of the zs:: kernels in gpurun_out/pmc_<cfg>_<k>/ (after the marker)."""
import csv
import glob
import sys
from collections import defaultdict

cfg = sys.argv[1] if len(sys.argv) > 1 else "config4"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_{cfg}_*/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    key = lambda r: int(r.get("Dispatch_Id") or 0)  # noqa: E731
    marks = [key(r) for r in rows if "stream_read_kernel" in r["Kernel_Name"]]
    m = max(marks) if marks else -1
    for r in rows:
        if key(r) > m and "zs::" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:32s} {sum(v) / len(v):.4g}")
