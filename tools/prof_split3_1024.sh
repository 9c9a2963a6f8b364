# MFMA utilisation of the split3 GEMM at 1024 agents x 101,770 (config 5's mix):
# separate rocprofv3 passes (MfmaUtil; GRBM_GUI_ACTIVE; SQ_WAVES + SQ_BUSY_CYCLES) + kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_split3}
mkdir -p "$OUT"
CMD="tools/bench_dense.py --agents ${AGENTS:-1024} --params 101770 --reps 3 --skip-f32-above 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $CMD > "$OUT/trace.log" 2>&1 || exit 1
echo "trace ok"
for ctr in "MfmaUtil" "GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$OUT/$tag" -o run --output-format csv -- python3 $CMD > "$OUT/$tag.log" 2>&1 || { echo "pmc $ctr failed"; exit 1; }
  echo "pmc $ctr ok"
done
python3 - "$OUT" <<'PY'
import csv, glob, os, statistics, sys, json
out = sys.argv[1]
res = {}
tr = list(csv.DictReader(open(f"{out}/trace/run_kernel_trace.csv")))
for r in tr:
    n = r["Kernel_Name"]
    if "split3" not in n:
        continue
    k = n.split("(")[0][:60]
    res.setdefault(k, {"durs": []})["durs"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for d in glob.glob(f"{out}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(d)):
        n = r["Kernel_Name"]
        if "split3" not in n:
            continue
        k = n.split("(")[0][:60]
        res.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
summ = {}
for k, v in res.items():
    summ[k] = {c: (statistics.median(x) if x else None) for c, x in v.items()}
    summ[k]["calls"] = len(v.get("durs", []))
json.dump(summ, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(summ, indent=1))
PY
rm -rf "$OUT/trace" "$OUT/MfmaUtil" "$OUT/GRBM_GUI_ACTIVE" "$OUT/SQ_BUSY_CYCLES_SQ_WAVE_CYCLES"
