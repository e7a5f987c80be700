"""Kernel sequence of the last pass(es) of a tools/prof_case.py kernel trace:
every dispatch after the marker (stream_read_kernel), grouped into passes by
the first kernel name of a pass, with durations and gaps.
usage: python tools/probes/seq_trace.py <rocprofv3 -d dir> [passes]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"][:60], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
m = max(i for i, k in enumerate(ks) if "stream_read_kernel" in k[0])
ks = ks[m + 1:]
first = ks[0][0]
starts = [i for i, k in enumerate(ks) if k[0] == first]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
tot = []
for j, s in enumerate(starts):
    e = starts[j + 1] if j + 1 < len(starts) else len(ks)
    tot.append((ks[e - 1][2] - ks[s][1]) / 1000)
    if j >= len(starts) - n:
        prev = None
        for name, t0, t1 in ks[s:e]:
            print(f"{name:60s} {(t1 - t0) / 1000:8.2f} us  gap {(t0 - prev) / 1000 if prev else 0:7.2f}")
            prev = t1
        print(f"pass {j}: first start -> last end {tot[-1]:.1f} us\n")
tot.sort()
print(f"passes {len(tot)}: median first->last {tot[len(tot) // 2]:.1f} us, min {tot[0]:.1f}")
