# Counters for config 4's FedADMM round at 8192 x 2^20 (10 local steps,
# momentum): the one-pass round + mean (admm_ls_round_mean_kernel) and the
# two-kernel round (admm_ls_round_kernel + ordered_sum_kernel), driven by
# tools/admm_round_ab.py: kernel trace, then one rocprofv3 pass each for
# FETCH_SIZE and WRITE_SIZE.  FetchSize is doubled for gfx950
# (MI355X_MICROARCH.md, HBM section).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_admm}
mkdir -p "$OUT"
CMD="tools/admm_round_ab.py --rounds 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $CMD > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
echo "trace ok"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $ctr -d "$OUT/$ctr" -o run --output-format csv -- python3 $CMD > "$OUT/$ctr.log" 2>&1 || { echo "pmc $ctr failed"; tail -5 "$OUT/$ctr.log"; exit 1; }
  echo "pmc $ctr ok"
done
python3 - "$OUT" <<'PY'
import csv, glob, json, statistics, sys
out = sys.argv[1]
N, P = 8192, 1 << 20
row = N * P * 4
alg = {"admm_ls_round_mean_kernel": 6 * row + 2 * P * 4, "admm_ls_round_kernel": 6 * row,
       "ordered_sum_kernel": row + P * 4}
def key(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return n
res = {}
for r in csv.DictReader(open(f"{out}/trace/run_kernel_trace.csv")):
    n = key(r["Kernel_Name"])
    if any(a in n for a in alg):
        res.setdefault(n, {"durs_ns": []})["durs_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for d in glob.glob(f"{out}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(d)):
        n = key(r["Kernel_Name"])
        if any(a in n for a in alg):
            res.setdefault(n, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
summ = {}
for k, v in res.items():
    base = next(a for a in alg if a in k)
    s = {c: statistics.median(x) for c, x in v.items() if x}
    s["launches"] = len(v.get("durs_ns", []))
    s["algorithmic_bytes"] = alg[base]
    if "FETCH_SIZE" in s:
        s["hbm_read_bytes_corrected"] = 2 * s["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in s:
        s["hbm_write_bytes"] = s["WRITE_SIZE"] * 1024
    if "hbm_read_bytes_corrected" in s and "hbm_write_bytes" in s:
        s["traffic_over_algorithmic"] = (s["hbm_read_bytes_corrected"] + s["hbm_write_bytes"]) / alg[base]
    if "durs_ns" in s:
        s["achieved_GBps"] = alg[base] / s["durs_ns"]
        s["frac_of_8TBps"] = s["achieved_GBps"] / 8000.0
    summ[k] = s
json.dump(summ, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(summ, indent=1))
PY
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
rm -rf "$OUT/trace" "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE"
