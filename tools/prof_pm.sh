# Counters for the parameter-major kernels (dol_mix_csr_pm_f32 rr4 at AGENTS x
# 2^20; dol_dgd_csr_pm_f32 at 1024 x 2^20 when AGENTS=1024): kernel trace, then
# one rocprofv3 pass each for FETCH_SIZE, WRITE_SIZE, TCC_HIT_sum+TCC_MISS_sum.
# FETCH_SIZE is doubled for gfx950 (MI355X_MICROARCH.md, HBM section).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
N=${AGENTS:-1024}
OUT=${OUT:-gpurun_out/prof_pm_$N}
mkdir -p "$OUT"
DGD=""; [ "$N" = 1024 ] && DGD="--dgd-pm 1024 --dgd-topologies rr4"
[ -n "$DGD" ] || DGD="--dgd-pm"
CMD="tools/bench_configs.py --agents $N --topologies rr4-pm --mlp --dgd $DGD --reps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $CMD > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
echo "trace ok"
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -s KILL 200 rocprofv3 --pmc $ctr -d "$OUT/$tag" -o run --output-format csv -- python3 $CMD > "$OUT/$tag.log" 2>&1 || { echo "pmc $ctr failed"; tail -5 "$OUT/$tag.log"; exit 1; }
  echo "pmc $ctr ok"
done
python3 - "$OUT" "$N" <<'PY'
import csv, glob, json, statistics, sys
out, N = sys.argv[1], int(sys.argv[2])
P = 1 << 20
res = {}
def key(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
for r in csv.DictReader(open(f"{out}/trace/run_kernel_trace.csv")):
    n = r["Kernel_Name"]
    if "csr_pm_kernel" in n:
        res.setdefault(key(n), {"durs_ns": []})["durs_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for d in glob.glob(f"{out}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(d)):
        n = r["Kernel_Name"]
        if "csr_pm_kernel" in n:
            res.setdefault(key(n), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
summ = {}
for k, v in res.items():
    s = {c: statistics.median(x) for c, x in v.items() if x}
    s["launches"] = len(v.get("durs_ns", []))
    # algorithmic bytes: mix 2*N*P*4; fused round (OBJ >= 0 in the name's 8th
    # template argument) adds the target read (+ momentum read/write)
    targs = k.split("<")[1].rstrip(">").split(",")
    obj, mode = int(targs[7]), int(targs[8])
    alg = N * P * 4 * (2 + (1 if obj >= 0 else 0) + (2 if mode == 2 else 1 if mode == 1 else 0))
    s["algorithmic_bytes"] = alg
    if "FETCH_SIZE" in s:
        s["hbm_read_bytes_corrected"] = 2 * s["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in s:
        s["hbm_write_bytes"] = s["WRITE_SIZE"] * 1024
    if "hbm_read_bytes_corrected" in s and "hbm_write_bytes" in s:
        s["traffic_over_algorithmic"] = (s["hbm_read_bytes_corrected"] + s["hbm_write_bytes"]) / alg
    if "TCC_HIT_sum" in s and "TCC_MISS_sum" in s:
        s["l2_hit_rate"] = s["TCC_HIT_sum"] / max(1.0, s["TCC_HIT_sum"] + s["TCC_MISS_sum"])
    if "durs_ns" in s:
        s["achieved_GBps"] = alg / s["durs_ns"]
        s["frac_of_8TBps"] = s["achieved_GBps"] / 8000.0
    summ[k] = s
json.dump(summ, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(summ, indent=1))
PY
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
rm -rf "$OUT/trace" "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE" "$OUT/TCC_HIT_sum_TCC_MISS_sum"
