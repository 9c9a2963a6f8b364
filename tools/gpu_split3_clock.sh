# Effective clock and MFMA busy of the split3 GEMMs (VERDICT r04 item 8's
# stall breakdown): one kernel-trace pass and one PMC pass of
# tools/split3_ab.py (1024 x 1024 x 101,770: the split-pass path and the fused
# FX8 path).  Per kernel: median duration, GRBM_GUI_ACTIVE cycles per launch
# (summed over the 8 XCDs) -> the effective clock, the SQ time split and
# SQ_VALU_MFMA_BUSY_CYCLES per SIMD-cycle.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/split3_clock}
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 tools/split3_ab.py > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -3 "$OUT/trace.log"; exit 1; }
echo trace ok
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES -d "$OUT/pmc" -o run --output-format csv -- python3 tools/split3_ab.py > "$OUT/pmc.log" 2>&1 || { echo "pmc rc=$?"; tail -3 "$OUT/pmc.log"; exit 1; }
echo pmc ok
python3 - "$OUT" <<'PY'
import csv, sys, collections, statistics, json, re
d = sys.argv[1]
def short(n):
    m = re.search(r"(dense_split3_\w+?|split3_\w+?)(<[^>]*>)?\(", n)
    return (m.group(1) + (m.group(2) or "")) if m else None
dur = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")):
    k = short(r["Kernel_Name"])
    if k: dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
ctr = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"{d}/pmc/run_counter_collection.csv")):
    k = short(r["Kernel_Name"])
    if k: ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k in dur:
    ms = statistics.median(dur[k])
    c = {n: statistics.median(v) for n, v in ctr[k].items()}
    e = {"median_ms": ms, "launches": len(dur[k]), **c}
    if "GRBM_GUI_ACTIVE" in c: e["effective_MHz"] = c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e3)
    if c.get("SQ_WAVE_CYCLES"):
        w = c["SQ_WAVE_CYCLES"]
        e["split"] = {"parked": c.get("SQ_WAIT_ANY", 0) / w, "issue_stall": c.get("SQ_WAIT_INST_ANY", 0) / w,
                      "active": c.get("SQ_ACTIVE_INST_ANY", 0) / w}
    if c.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        e["mfma_busy_per_busy_cycle"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_BUSY_CYCLES"]
    out[k] = e
json.dump(out, open(f"{d}/summary.json", "w"), indent=1)
for k, e in out.items():
    print(k, json.dumps({a: (round(b, 4) if isinstance(b, float) else b) for a, b in e.items()}))
PY
