# Box probe: tools/box_probe.py under a kernel trace and PMC passes, summarised
# per kernel (ring_mix_dma, csr_pm, ring_steps, the copy): duration, effective
# clock from GRBM_GUI_ACTIVE (summed over 8 XCDs), SQ time split, memory-side
# read requests and their in-flight level (mean read latency = level / requests,
# in L2 clocks), TA busy.  OUT=gpurun_out/box_X bash tools/gpu_box_probe.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/box}
mkdir -p "$OUT"
CMD="python3 tools/box_probe.py --reps 3"
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- $CMD > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -3 "$OUT/trace.log"; exit 1; }
echo "trace ok: $(tail -1 "$OUT/trace.log")"
pass() {  # tag, counters...
  local tag=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv -- $CMD > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "pmc $tag rc=$rc"
  case $rc in 0) return 0;; 124|137|134|139) exit $rc;; *) tail -2 "$OUT/$tag.log"; return 0;; esac
}
pass sq GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
if grep -q TCC_EA0_RDREQ_LEVEL "$OUT/avail.txt"; then pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum; else pass ea TCC_EA0_RDREQ_sum; fi
if grep -q "TA_BUSY_avr" "$OUT/avail.txt"; then pass ta TA_BUSY_avr; fi
python3 - "$OUT" <<'PY'
import csv, collections, glob, json, os, statistics, sys
d = sys.argv[1]
def short(n):
    for k in ("ring_mix_dma_kernel", "csr_pm_kernel", "ring_steps_kernel", "ring_stream_kernel", "copy"):
        if k in n:
            return k
    return None
dur = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")):
    k = short(r["Kernel_Name"])
    if k:
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
ctr = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k:
            ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, ds in dur.items():
    ms = statistics.median(ds)
    c = {n: statistics.median(v) for n, v in ctr[k].items()}
    e = {"ms": ms, "launches": len(ds)}
    if "GRBM_GUI_ACTIVE" in c:
        e["eff_MHz"] = c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e3)
    if c.get("SQ_WAVE_CYCLES"):
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in c:
                e[n + "_frac"] = c[n] / c["SQ_WAVE_CYCLES"]
    if c.get("TCC_EA0_RDREQ_sum"):
        e["rdreq"] = c["TCC_EA0_RDREQ_sum"]
        if "TCC_EA0_RDREQ_LEVEL_sum" in c:
            e["rd_latency_cycles"] = c["TCC_EA0_RDREQ_LEVEL_sum"] / c["TCC_EA0_RDREQ_sum"]
            if "GRBM_GUI_ACTIVE" in c:
                e["rd_in_flight"] = c["TCC_EA0_RDREQ_LEVEL_sum"] / (c["GRBM_GUI_ACTIVE"] / 8)
    for n, v in c.items():
        if n.startswith("TA_"):
            e[n] = v
    out[k] = e
print(json.dumps(out, indent=1))
json.dump(out, open(f"{d}/summary.json", "w"), indent=1)
PY
rm -rf "$OUT/trace" "$OUT"/sq "$OUT"/ea "$OUT"/ta
