"""Summarise tools/probes/pmc_short.sh: counters of the last crc kernel dispatch per depth."""
import collections
import csv
import glob
import sys


def main(depths=("3", "9")):
    for dp in depths:
        agg = collections.defaultdict(float)
        for f in glob.glob(f"gpurun_out/pmc_d{dp}_*/**/*counter_collection.csv", recursive=True):
            rows = [r for r in csv.DictReader(open(f))
                    if "short_kernel" in r["Kernel_Name"] or "burst_kernel" in r["Kernel_Name"]]
            if not rows:
                continue
            last = max(int(r["Dispatch_Id"]) for r in rows)
            for r in rows:
                if int(r["Dispatch_Id"]) == last:
                    agg[r["Counter_Name"]] += float(r["Counter_Value"])
        wc = agg.get("SQ_WAVE_CYCLES", 1)
        print(dp, {k: f"{v:.3e}" for k, v in sorted(agg.items())})
        print("   fractions of wave cycles:", {k: round(agg.get(k, 0) / wc, 3) for k in
                                               ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS")})


if __name__ == "__main__":
    main(sys.argv[1:] or ("3", "9"))
