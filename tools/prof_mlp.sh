#!/bin/bash
# per-kernel durations of the config-5 MLP round under each launch path (rocprofv3 kernel trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-mlpprof}
mkdir -p $O
for v in ${VARIANTS:-DOL_MLP_F1_TILES=0 DOL_MLP_F1_TILES=5 DOL_MLP_SPLIT_FWD=1}; do
  env $(echo $v | tr , " ") timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/bench_configs.py --mlp 1024 --mlp-mix csr --agents > $O/run_$v.log 2>&1 || { echo "rc=$? $v"; tail -5 $O/run_$v.log; exit 1; }
  f=$(find $O/t -name 'run_kernel_stats.csv' | head -1); cp "$f" "$O/stats_$v.csv"; rm -rf $O/t
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
  if 'mlp' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
" "$O/stats_$v.csv"
done
