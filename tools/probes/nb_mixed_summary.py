"""Per-form kernel times of a mixed NOTBATCHED trace (tools/prof_case.py
config4nb with C4NB_MODE=mixed: pass k runs form k % 3 -- ranged verdict,
unranged verdict, per-commit arrays -- in one process, so every form sees
the same power state): the dispatches after the marker split into passes at
each classify_kernel, the last `tail` passes of each form summarised.
usage: python tools/probes/nb_mixed_summary.py <rocprofv3 -d dir> [tail]"""
import csv
import glob
import json
import sys

import numpy as np

FORMS = ["verdict_range", "verdict", "arrays"]


def main():
    d = sys.argv[1]
    tail = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
          for r in rows]
    m = max(i for i, k in enumerate(ks) if "stream_read_kernel" in k[0])
    ks = [k for k in ks[m + 1:] if k[0].startswith("zs::")]
    passes, cur = [], None
    for k in ks:
        if k[0].startswith("zs::classify_kernel"):
            if cur:
                passes.append(cur)
            cur = []
        if cur is not None:
            cur.append(k)
    if cur:
        passes.append(cur)
    out = {}
    for fi, name in enumerate(FORMS):
        sel = [p for i, p in enumerate(passes) if i % 3 == fi][-tail:]
        span = [(p[-1][2] - p[0][1]) / 1e3 for p in sel]
        per = {}
        for p in sel:
            for n, s, e in p:
                per.setdefault(n, []).append((e - s) / 1e3)
        out[name] = {"passes": len(sel), "first_to_last_us_median": round(float(np.median(span)), 2),
                     "kernels_us_median": {n: round(float(np.median(v)), 2) for n, v in per.items()},
                     "launches_per_pass": round(sum(len(p) for p in sel) / max(1, len(sel)), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
