# Clock / issue probe of FedLCon's eps = 5 pass vs the headline ring round
# (VERDICT r02 item 8): one kernel-trace pass and one PMC pass of
# tools/eps_pass_time.py; per kernel: mean duration, GRBM_GUI_ACTIVE cycles per
# launch -> the effective clock (cycles / duration), and the SQ time split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/clock}
mkdir -p "$OUT"
CMD="python3 tools/eps_pass_time.py --reps 5"  # DOL_RING_STREAM etc. pass through the environment
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $CMD > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -3 "$OUT/trace.log"; exit 1; }
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/pmc" -o run --output-format csv -- $CMD > "$OUT/pmc.log" 2>&1 || { echo "pmc rc=$?"; tail -3 "$OUT/pmc.log"; exit 1; }
echo pmc ok
python3 - "$OUT" <<'PY'
import csv, sys, collections, statistics, json
d = sys.argv[1]
def short(n):
    for k in ("ring_steps_kernel", "ring_stream_kernel", "ring_mix_dma_kernel", "ring_mix_kernel"):
        if k in n: return k
    return None
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
    e = {"median_ms": ms, **c}
    # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (11.8 ms of the ring kernel read 224M)
    if "GRBM_GUI_ACTIVE" in c: e["effective_MHz"] = c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e3)
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        w = c["SQ_WAVE_CYCLES"]
        e["split"] = {"parked": c.get("SQ_WAIT_ANY", 0) / w, "issue_stall": c.get("SQ_WAIT_INST_ANY", 0) / w,
                      "active": c.get("SQ_ACTIVE_INST_ANY", 0) / w, "valu_active": c.get("SQ_ACTIVE_INST_VALU", 0) / w}
    out[k] = e
json.dump(out, open(f"{d}/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
