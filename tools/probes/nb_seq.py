"""Print the kernel sequence around the NOTBATCHED verify passes of a
config-4 bench trace (tools/trace_bench.sh): durations and the gaps between
kernels.  usage: python tools/probes/nb_seq.py gpurun_out/trace_bench/config4 [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"][:56], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
big = [i for i, k in enumerate(ks) if "xteam_kernel<2>" in k[0] and k[2] - k[1] > 100_000]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for j in big[-n:]:
    s = j
    while s > 0 and "fillBuffer" not in ks[s][0]:
        s -= 1
    e = j
    while e + 1 < len(ks) and "part_fold" in ks[e + 1][0] or (e + 1 < len(ks) and e - j < 6 and "zs::" in ks[e + 1][0]):
        e += 1
    prev = None
    for name, t0, t1 in ks[s:e + 1]:
        print(f"{name:56s} {(t1 - t0) / 1000:8.2f} us  gap {(t0 - prev) / 1000 if prev else 0:7.2f}")
        prev = t1
    print(f"first start -> last end: {(ks[e][2] - ks[s][1]) / 1000:.1f} us\n")
