#!/bin/bash
# r06m: MLP step, W1 reuse between the forward and dW1: forward staging policy x dW1 agent order
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06m; mkdir -p $O
cd $R && DOL_MLP_F1_KEEP=1 DOL_MLP_DW1_REVERSE=1 timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
cd /tmp
for rep in 1 2 3; do
  for v in "0 0" "1 0" "0 1" "1 1"; do
    set -- $v
    DOL_MLP_F1_KEEP=$1 DOL_MLP_DW1_REVERSE=$2 timeout -k 10 120 python3 $R/tools/mlp_order_ab.py >> $O/time.jsonl || exit 1
  done
done
for v in "0 0" "1 1"; do
  set -- $v
  for cn in FETCH_SIZE WRITE_SIZE; do
    DOL_MLP_F1_KEEP=$1 DOL_MLP_DW1_REVERSE=$2 timeout -s KILL 120 rocprofv3 --pmc $cn -d $O/p$1$2_$cn -o run --output-format csv -- python3 $R/tools/mlp_order_ab.py --reps 5 > $O/p$1$2_$cn.log 2>&1 || { echo "pmc failed"; exit 1; }
    f=$(find $O/p$1$2_$cn -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$1$2" "$cn" >> $O/pmc.jsonl <<'PY'
import csv, sys, json, collections
v = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    nm = 'fwd' if 'mlp_fwd_kernel' in r['Kernel_Name'] else ('dw1' if 'dw1' in r['Kernel_Name'] else None)
    if nm: v[nm][r.get('Dispatch_Id', '')] += float(r['Counter_Value'])
out = {k: sorted(d.values())[len(d) // 2] for k, d in v.items()}
print(json.dumps({"cfg": sys.argv[2], "counter": sys.argv[3], "kB_median": out}))
PY
  done
done
