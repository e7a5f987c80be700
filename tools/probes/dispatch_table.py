"""Mean duration per zs:: kernel (and per dispatch position in a pass) from a
rocprofv3 kernel_trace.csv: python3 tools/probes/dispatch_table.py <dir>"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "zs::" in r["Kernel_Name"]]
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    agg[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    print(f"{k:45s} n={len(v):4d} median_us={v2[len(v2) // 2] / 1e3:9.1f} total_ms={sum(v) / 1e6:8.3f}")
