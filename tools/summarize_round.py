"""Summarise tools/profile_round.sh output into profiles/<tag>/: per config the
kernel-time and HBM-traffic per pass (zs:: dispatches after the marker
dispatch of tools/prof_case.py, divided by REPS), the dominant kernel's
average duration, and the rocprofv3 --stats CSV of the config-3 bench run.
FETCH_SIZE is doubled (gfx950: it reports half the bytes of 16-byte-per-lane
reads, MI355X_MICROARCH.md "HBM").  Also refreshes profiles/pmc_traffic.json,
which bench.py reads for roofline.traffic.

usage: python tools/summarize_round.py <tag> [gpurun_out/prof] [REPS]"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UNITS = {"config2": 64}  # tools/prof_case.py config2: one pass = one 64-batch launch


def newest(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return max(fs, key=os.path.getmtime) if fs else None


def after_marker(rows, name_key):
    """zs:: rows after the last marker (stream_read_kernel) row, by dispatch id."""
    key = lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)  # noqa: E731
    rows = sorted(rows, key=key)
    marks = [key(r) for r in rows if "stream_read_kernel" in r[name_key]]
    if not marks:
        return []
    m = max(marks)
    return [r for r in rows if key(r) > m and "zs::" in r[name_key]]


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    out, traffic = {}, {}
    for cfg in ("config2", "config3", "config4", "config5"):
        tr = newest(os.path.join(src, f"{cfg}_trace"), "*kernel_trace.csv")
        st = newest(os.path.join(src, f"{cfg}_trace"), "*kernel_stats.csv")
        fe = newest(os.path.join(src, f"{cfg}_fetch"), "*counter_collection.csv")
        wr = newest(os.path.join(src, f"{cfg}_write"), "*counter_collection.csv")
        if not tr:
            continue
        if st:
            shutil.copy(st, os.path.join(dst, f"{cfg}_kernel_stats.csv"))
        disp = after_marker(list(csv.DictReader(open(tr))), "Kernel_Name")
        per_kernel = {}
        for r in disp:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            k = r["Kernel_Name"].split("(")[0]
            per_kernel.setdefault(k, []).append(d)
        dom = max(per_kernel, key=lambda k: sum(per_kernel[k])) if per_kernel else None
        units = UNITS.get(cfg, 1)  # bench.py steps per pass
        summ = {
            "passes": reps,
            "bench_steps_per_pass": units,
            "kernel_ns_per_pass": sum(sum(v) for v in per_kernel.values()) / reps,
            "dominant_kernel": dom,
            "dominant_avg_ns": sum(per_kernel[dom]) / len(per_kernel[dom]) if dom else None,
            "kernels_per_pass": {k: round(sum(v) / reps) for k, v in per_kernel.items()},
        }
        for what, f, cname in (("fetch", fe, "FETCH_SIZE"), ("write", wr, "WRITE_SIZE")):
            if not f:
                continue
            rows = [r for r in after_marker(list(csv.DictReader(open(f))), "Kernel_Name")
                    if r["Counter_Name"] == cname]
            summ[f"{what}_kb_per_pass"] = sum(float(r["Counter_Value"]) for r in rows) / reps
        if "fetch_kb_per_pass" in summ and "write_kb_per_pass" in summ:
            summ["hbm_bytes_per_pass"] = int(summ["fetch_kb_per_pass"] * 1024 * 2
                                             + summ["write_kb_per_pass"] * 1024)
            traffic[f"{cfg}_bytes_per_launch"] = summ["hbm_bytes_per_pass"] // units
        out[cfg] = summ
    b = newest(os.path.join(src, "bench_trace"), "*kernel_stats.csv")
    if b:
        shutil.copy(b, os.path.join(dst, "bench_config3_kernel_stats.csv"))
    bl = os.path.join(src, "bench.log")
    if os.path.exists(bl):
        lines = [ln for ln in open(bl) if ln.startswith("{")]
        if lines:
            open(os.path.join(dst, "bench_config3.json"), "w").write(lines[-1])
    # merge into an existing summary: a run that profiled some configs only
    # updates those
    prev_path = os.path.join(dst, "summary.json")
    if os.path.exists(prev_path):
        prev = json.load(open(prev_path))
        prev.update(out)
        out = prev
    json.dump(out, open(prev_path, "w"), indent=1)
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if traffic and os.path.exists(tpath):
        old = json.load(open(tpath))
        old.update(traffic)
        traffic = old
    if traffic:
        traffic["source"] = (f"profiles/{tag}/summary.json: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in "
                             "separate passes over tools/prof_case.py, zs:: dispatches per pass, "
                             "FETCH_SIZE x2 (gfx950 wide-read correction)")
        json.dump(traffic, open(tpath, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
