"""Summarise rocprofv3 passes for one kernel: avg duration (kernel trace) and
per-launch HBM bytes from separate FETCH_SIZE / WRITE_SIZE passes.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reads exactly
half the bytes of a wide coalesced streaming read -> x2; WRITE_SIZE is exact
for 16-B-per-lane streaming stores.  Both counters are in KiB.
usage: python tools/parse_prof.py gpurun_out/prof ring_mix_kernel out.json [agents params n_gpus]
"""
import csv
import json
import statistics
import sys


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main():
    d, kname, out = sys.argv[1], sys.argv[2], sys.argv[3]
    extra = sys.argv[4:]
    stats = [r for r in rows(f"{d}/trace/run_kernel_stats.csv") if kname in r["Name"]]
    trace = [r for r in rows(f"{d}/trace/run_kernel_trace.csv") if kname in r["Kernel_Name"]]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
    res = {"kernel": kname, "calls": len(durs), "avg_ns": statistics.mean(durs) if durs else None,
           "median_ns": statistics.median(durs) if durs else None,
           "stats_avg_ns": float(stats[0]["AverageNs"]) if stats else None}
    for ctr, fn, scale in (("FETCH_SIZE", "fetch", 2.0), ("WRITE_SIZE", "write", 1.0)):
        try:
            vals = [float(r["Counter_Value"]) for r in rows(f"{d}/{fn}/run_counter_collection.csv")
                    if kname in r["Kernel_Name"] and r["Counter_Name"] == ctr]
        except FileNotFoundError:
            vals = []
        res[ctr + "_KiB_raw_median"] = statistics.median(vals) if vals else None
        res[ctr.lower() + "_bytes_per_launch"] = statistics.median(vals) * 1024 * scale if vals else None
    if res["fetch_size_bytes_per_launch"] is not None and res["write_size_bytes_per_launch"] is not None:
        res["hbm_bytes_per_launch"] = res["fetch_size_bytes_per_launch"] + res["write_size_bytes_per_launch"]
    res["corrections"] = "FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), WRITE_SIZE x1; KiB -> bytes"
    if len(extra) >= 3:
        res["agents"], res["params"], res["n_gpus"] = int(extra[0]), int(extra[1]), int(extra[2])
        res["algorithmic_bytes_per_launch"] = 2 * res["agents"] // res["n_gpus"] * res["params"] * 4
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
