#!/bin/bash
# r06f: ring DGD round, target / momentum loads plain vs nontemporal: time + HBM bytes (FETCH_SIZE, WRITE_SIZE passes)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f; mkdir -p $O
for nt in 0 1 3 17 18 19 0; do
  DOL_DGD_EPI_NT=$nt timeout -k 10 120 python3 $R/tools/dgd_ring_ab.py >> $O/time.jsonl || exit 1
done
for nt in 0 3 17 18 19; do
  for c in FETCH_SIZE WRITE_SIZE; do
    DOL_DGD_EPI_NT=$nt timeout -s KILL 90 rocprofv3 --pmc $c -d $O/nt${nt}_$c -o run --output-format csv -- python3 $R/tools/dgd_ring_ab.py --reps 4 > $O/nt${nt}_$c.log 2>&1 || { echo "pmc $nt $c failed"; tail -3 $O/nt${nt}_$c.log; exit 1; }
    f=$(find $O/nt${nt}_$c -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$nt" "$c" >> $O/pmc.jsonl <<'PY'
import csv, sys, json, collections
v = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'ring_mix_dma_kernel' in r['Kernel_Name'] and 'DgdEpi' in r['Kernel_Name']:
        v[r.get('Dispatch_Id', '')] += float(r['Counter_Value'])
vals = sorted(v.values())
print(json.dumps({"nt": sys.argv[2], "counter": sys.argv[3], "per_dispatch_kB_median": vals[len(vals) // 2], "n": len(vals)}))
PY
  done
done
