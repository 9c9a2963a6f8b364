"""Summarise tools/gpu_r06j.sh: per pass, per ordered pair, the eps pass's and
the ring round's median duration (kernel trace) and median counters (PMC),
for the eps_pair_counters.py run of that pass.  One JSON line per (pass, pair)."""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict


def main(root):
    for p in sorted(glob.glob(f"{root}/p*.json")):
        tag = p.rsplit("/", 1)[1][:-5]
        meta = json.loads(open(p).read().strip().splitlines()[-1])
        tr = glob.glob(f"{root}/{tag}/**/*kernel_trace.csv", recursive=True)
        pc = glob.glob(f"{root}/{tag}/**/*counter_collection.csv", recursive=True)
        if not tr or not pc:
            continue
        disp = []
        for r in csv.DictReader(open(tr[0])):
            nm = r["Kernel_Name"]
            if "ring_stream_dma_kernel" in nm or ("ring_mix_dma_kernel" in nm and "DgdEpi" not in nm):
                disp.append((int(r["Dispatch_Id"]), "eps" if "stream" in nm else "ring",
                             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
        disp.sort()
        cnt = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(pc[0])):
            cnt[int(r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        k = 0
        for pair in meta["pairs"]:
            for kind in ("eps", "ring"):
                rows = []
                for _ in range(meta["per_pair"][kind]):
                    rows.append(disp[k])
                    k += 1
                assert all(r[1] == kind for r in rows), (pair, kind, rows)
                ms = statistics.median(r[2] for r in rows)
                ctr = {}
                for name in cnt[rows[0][0]]:
                    vals = [cnt[r[0]][name] for r in rows]
                    if len(vals[0]) == 1:
                        ctr[name] = statistics.median(v[0] for v in vals)
                    else:  # per-instance values: spread across L2 channels (min / max / cv of the last launch)
                        v = vals[-1]
                        m = statistics.mean(v)
                        ctr[name] = {"n": len(v), "sum": sum(v), "min": min(v), "max": max(v),
                                     "cv": statistics.pstdev(v) / m if m else 0.0}
                print(json.dumps({"pass": tag, "pair": pair, "kernel": kind, "ms": ms, "counters": ctr}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r06j")
