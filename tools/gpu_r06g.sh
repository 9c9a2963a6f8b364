#!/bin/bash
# r06g: DGD epilogue nontemporal buffer loads as the default: bit-exact DGD tests, then time + HBM bytes (LS+momentum, logistic)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06g; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest tests/test_dgd_gpu.py tests/test_pmajor_gpu.py tests/test_parallel_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dgd or ring or DGD" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
cd /tmp
for obj in least_squares logistic; do
  for nt in 3 0 3 0; do
    DOL_DGD_EPI_NT=$nt timeout -k 10 120 python3 $R/tools/dgd_ring_ab.py --objective $obj >> $O/time.jsonl || exit 1
  done
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c -d $O/${obj}_$c -o run --output-format csv -- python3 $R/tools/dgd_ring_ab.py --reps 4 --objective $obj > $O/${obj}_$c.log 2>&1 || { echo "pmc $obj $c failed"; exit 1; }
    f=$(find $O/${obj}_$c -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$obj" "$c" >> $O/pmc.jsonl <<'PY'
import csv, sys, json, collections
v = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'ring_mix_dma_kernel' in r['Kernel_Name'] and 'DgdEpi' in r['Kernel_Name']:
        v[r.get('Dispatch_Id', '')] += float(r['Counter_Value'])
vals = sorted(v.values())
print(json.dumps({"objective": sys.argv[2], "counter": sys.argv[3], "per_dispatch_kB_median": vals[len(vals) // 2], "n": len(vals)}))
PY
  done
done
