"""Summarise tools/probes/pmc_calibrate.sh: per case/depth FETCH_SIZE x2, L2 requests,
misses x 128 B and the kernel time per pass (zs:: dispatches after the marker)."""
import csv
import glob
import sys


def rows_after(f):
    rows = list(csv.DictReader(open(f)))
    key = lambda r: int(r["Dispatch_Id"])  # noqa: E731
    m = max([key(r) for r in rows if "stream_read" in r["Kernel_Name"]] or [0])
    return [r for r in rows if key(r) > m and "zs::" in r["Kernel_Name"]]


def main(d="gpurun_out/cal", reps=5):
    for f in sorted(glob.glob(f"{d}/*_fetch")):
        tag = f.split("/")[-1][:-6]
        res = {}
        for sub in ("fetch", "tcc"):
            for g in glob.glob(f"{d}/{tag}_{sub}/**/*counter_collection.csv", recursive=True):
                for r in rows_after(g):
                    res[r["Counter_Name"]] = res.get(r["Counter_Name"], 0) + float(r["Counter_Value"]) / reps
        t = 0.0
        for g in glob.glob(f"{d}/{tag}_trace/**/*kernel_trace.csv", recursive=True):
            t = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows_after(g)) / reps
        print(tag, {"fetch_GB_x2": round(res.get("FETCH_SIZE", 0) * 2048 / 1e9, 3),
                    "l2_req_M": round(res.get("TCP_TCC_READ_REQ_sum", 0) / 1e6, 2),
                    "l2_miss_GB_x128": round(res.get("TCC_MISS_sum", 0) * 128 / 1e9, 3),
                    "us": round(t / 1e3, 1)})


if __name__ == "__main__":
    main(*sys.argv[1:])
