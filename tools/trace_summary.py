"""Per-step kernel time of a bench.py run traced by tools/trace_bench.sh:
the zs:: dispatches after the same-GPU read-ceiling probe (stream_read_kernel
x 26) grouped into the bench's steps (warmup + timed), summed per step, and
the mean over the timed steps set beside the line's kernel_ms.

usage: python tools/trace_summary.py gpurun_out/trace_bench/config4 [first_kernel_of_step] [per_launch_div]
       [last_k]   (config 2: the cold multi-batch launches are the last 2 of zs::multi64_kernel, /64)"""
import csv
import json
import os
import sys


def main():
    d = sys.argv[1]
    head = sys.argv[2] if len(sys.argv) > 2 else None
    div = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    last = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    line = json.loads(open(d + ".json").read().strip().splitlines()[-1])
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
          for r in rows if "zs::" in r["Kernel_Name"]]
    # skip to after the 26 streaming-read probe launches
    idx = [i for i, k in enumerate(ks) if k[0].startswith("zs::stream_read_kernel")]
    ks = ks[idx[-1] + 1:] if idx else ks
    head = head or ks[0][0]
    steps, cur = [], None
    for k in ks:
        if k[0].startswith(head):
            if cur:
                steps.append(cur)
            cur = []
        if cur is not None:
            cur.append(k)
    if cur:
        steps.append(cur)
    warm, timed = line["warmup"], line["steps"]
    if line["roofline"].get("note", "").startswith("kernel_ms = launch time"):
        warm, timed = 1, len(steps) - 1
    if last:
        steps = [[k] for k in ks if k[0].startswith(head)]
        sel = steps[-last:]
    else:
        sel = steps[warm:warm + timed] if len(steps) >= warm + timed else steps[-timed:]
    busy = [sum(e - s for _, s, e in st) / 1e6 / div for st in sel]          # ms of kernel time
    copies = os.path.join(d, "run_memory_copy_trace.csv")
    cp = []
    if os.path.exists(copies):
        # device->host / device->device copies inside each step's span count too
        cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(copies))]
        for st in sel:
            a, b = st[0][1], st[-1][2] + 200000
            cp.append(sum(e - s for s, e in cs if a <= s <= b) / 1e6 / div)
    span = [(st[-1][2] - st[0][1]) / 1e6 / div for st in sel]                # first start -> last end
    names = {}
    for st in sel:
        for n, s, e in st:
            names.setdefault(n, []).append((e - s) / 1e3 / div)
    out = {"trace": d, "steps_found": len(steps), "steps_used": len(sel), "line_kernel_ms": line["roofline"]["kernel_ms"],
           "trace_busy_ms_mean": round(sum(busy) / len(busy), 4), "trace_span_ms_mean": round(sum(span) / len(span), 4),
           "per_kernel_us_mean": {n: round(sum(v) / len(sel), 2) for n, v in names.items()}}
    # rocprofiler-sdk may drop async copy records under load ("... completion
    # callbacks were not delivered" on stderr); a step without any copy record
    # is then missing data, not a zero
    err = d + ".err"
    dropped = os.path.exists(err) and "not delivered" in open(err, errors="replace").read()
    if cp and not dropped and min(cp) > 0:
        out["trace_copies_ms_mean"] = round(sum(cp) / len(cp), 4)
        out["trace_busy_plus_copies_ms_mean"] = round(out["trace_busy_ms_mean"] + out["trace_copies_ms_mean"], 4)
        out["busy_plus_copies_vs_line"] = round(out["trace_busy_plus_copies_ms_mean"] / out["line_kernel_ms"], 4)
    elif os.path.exists(copies):
        out["trace_copies_ms_mean"] = "not captured"
        out["copies_note"] = ("the profiler dropped copy records" if dropped else
                              f"{sum(1 for x in cp if x == 0)} of {len(cp)} steps have no copy record") + \
            ": copy time inside the steps is unknown, not zero"
    out["busy_vs_line"] = round(out["trace_busy_ms_mean"] / out["line_kernel_ms"], 4)
    out["span_vs_line"] = round(out["trace_span_ms_mean"] / out["line_kernel_ms"], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
