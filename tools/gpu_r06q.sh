#!/bin/bash
# r06q: PMC passes of csr_slab_kernel under variants 1 and 3 (DOL_SLAB_KERNEL), 1024 x 101,770 ER p = 0.1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06q; mkdir -p $O
CMD="python3 $R/tools/bench_slab.py --agents 1024 --paths slab --reps 5"
for v in ${VARIANTS:-1 3}; do
  DOL_SLAB_KERNEL=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/v${v}p1 -o run --output-format csv -- $CMD > $O/v${v}p1.log 2>&1 || { echo "v$v pass1 failed"; tail -5 $O/v${v}p1.log; exit 1; }
  DOL_SLAB_KERNEL=$v timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $O/v${v}p2 -o run --output-format csv -- $CMD > $O/v${v}p2.log 2>&1 || { echo "v$v pass2 failed"; tail -5 $O/v${v}p2.log; exit 1; }
  for p in p1 p2; do
    f=$(find $O/v$v$p -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$v" "$p" >> $O/summary.jsonl <<'PY'
import csv, sys, collections, json
tot = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if 'csr_slab_kernel' not in r['Kernel_Name']:
        continue
    tot[r['Counter_Name']] += float(r['Counter_Value']); disp[r['Counter_Name']].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
print(json.dumps({"variant": int(sys.argv[2]), "pass": sys.argv[3],
                  "per_dispatch": {k: tot[k] / max(1, len(disp[k])) for k in sorted(tot)},
                  "dispatches": {k: len(v) for k, v in disp.items()}}))
PY
  done
done
