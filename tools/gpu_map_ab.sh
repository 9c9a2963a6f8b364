#!/bin/bash
# headline ring round on mapped (dol_bank_alloc) vs torch-allocated x / y, alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-map_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bank_alloc_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "bank pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for m in 1 0; do
    timeout -k 10 300 python bench.py --no-cpu --no-primal-dual --map-ring $m > $O/b_$m.json 2> $O/b_$m.err || { echo "bench rc=$?"; tail -3 $O/b_$m.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']
print('map_ring', sys.argv[2], 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(r['kernel_ms'],4), 'copy_GBps', round(r['copy_kernel_GBps']), 'frac', round(r['frac'],4))" $O/b_$m.json $m | tee -a $O/ab.txt
  done
done
