"""Per-kernel summary of a tools/profile.sh run: calls, avg/median duration
(kernel trace), and per-launch HBM bytes from the separate FETCH_SIZE /
WRITE_SIZE passes (gfx950: FETCH_SIZE x2 for 16-B streaming reads, WRITE_SIZE
x1; counters in KiB).  usage: python tools/summarize_prof.py gpurun_out/prof out.json"""
import csv
import json
import re
import statistics
import sys


def rows(path):
    try:
        with open(path, newline="") as f:
            return list(csv.DictReader(f))
    except FileNotFoundError:
        return []


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name[:80]


def main():
    d, out = sys.argv[1], sys.argv[2]
    trace = rows(f"{d}/trace/run_kernel_trace.csv")
    per = {}
    for r in trace:
        k = short(r["Kernel_Name"]) + f" grid={r.get('Grid_Size_X') or r.get('Grid_Size')}"
        per.setdefault(k, {"durations_ns": []})["durations_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for ctr, fn, scale in (("FETCH_SIZE", "fetch", 2.0), ("WRITE_SIZE", "write", 1.0)):
        for r in rows(f"{d}/{fn}/run_counter_collection.csv"):
            if r["Counter_Name"] != ctr:
                continue
            k = short(r["Kernel_Name"]) + f" grid={r.get('Grid_Size')}"
            per.setdefault(k, {"durations_ns": []}).setdefault(ctr, []).append(float(r["Counter_Value"]) * 1024 * scale)
    res = {}
    for k, v in per.items():
        ds = v["durations_ns"]
        e = {"calls": len(ds)}
        if ds:
            e.update(avg_ms=statistics.mean(ds) / 1e6, median_ms=statistics.median(ds) / 1e6)
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            if v.get(ctr):
                e[ctr.lower() + "_bytes_median"] = statistics.median(v[ctr])
        if "fetch_size_bytes_median" in e and "write_size_bytes_median" in e:
            e["hbm_bytes_per_launch"] = e["fetch_size_bytes_median"] + e["write_size_bytes_median"]
            if "median_ms" in e:
                e["hbm_GBps"] = e["hbm_bytes_per_launch"] / (e["median_ms"] / 1e3) / 1e9
        res[k] = e
    res = dict(sorted(res.items(), key=lambda kv: -kv[1].get("avg_ms", 0) * kv[1]["calls"]))
    res["_corrections"] = "FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), WRITE_SIZE x1, KiB->bytes"
    json.dump(res, open(out, "w"), indent=1)
    for k, e in res.items():
        if k.startswith("_"):
            continue
        print(f"{k[:90]:90s} calls={e['calls']:4d} avg_ms={e.get('avg_ms', 0):8.3f} hbm_GB={e.get('hbm_bytes_per_launch', 0)/1e9:8.2f} GBps={e.get('hbm_GBps', 0):8.1f}")


if __name__ == "__main__":
    main()
