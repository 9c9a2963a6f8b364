# PMC passes of the LDS-gather CSR kernel (1024 x 101,770, ER p = 0.1), one
# rocprofv3 run per counter group (<= 8 SQ counters each), each under its own kill timeout
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CMD="python3 $R/tools/bench_slab.py --agents 1024 --paths slab --reps 5"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $R/gpurun_out/slabpmc1 -o run --output-format csv -- $CMD > $R/gpurun_out/slabpmc1.log 2>&1 || { echo "pass1 rc=$?"; tail -5 $R/gpurun_out/slabpmc1.log; exit 1; }
echo pass1 ok
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $R/gpurun_out/slabpmc2 -o run --output-format csv -- $CMD > $R/gpurun_out/slabpmc2.log 2>&1 || { echo "pass2 rc=$?"; tail -5 $R/gpurun_out/slabpmc2.log; exit 1; }
echo pass2 ok
for d in slabpmc1 slabpmc2; do
  f=$(find $R/gpurun_out/$d -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if 'csr_slab_kernel' not in r['Kernel_Name']:
        continue
    tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(1, n[k] / 1):16.1f}  (summed over {n[k]} records)")
PY
done
