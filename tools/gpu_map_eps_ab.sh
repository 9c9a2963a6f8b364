#!/bin/bash
# mapped (dol_bank_alloc) vs torch-allocated headline buffers: ring round AND the eps = 5 pass / pm mix
# that run over the same buffers, alternating processes on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-map_eps_ab}
mkdir -p $O
for rep in 1 2; do
  for m in 1 0; do
    timeout -k 10 400 python bench.py --no-cpu --map-ring $m > $O/b_$m.json 2> $O/b_$m.err || { echo "bench rc=$?"; tail -3 $O/b_$m.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; e=d['fedlcon_eps5']; p=d['random_regular_pm']
print('map_ring', sys.argv[2], 'ring_ms', round(r['kernel_ms'],3), 'copy_GBps', round(r['copy_kernel_GBps']), 'eps_ms', round(e['ms_per_pass'],3), 'eps_variants', {k: round(v,2) for k,v in e['variant_ms'].items()}, 'pm_ms', round(p['ms_per_round'],3))" $O/b_$m.json $m | tee -a $O/ab.txt
  done
done
