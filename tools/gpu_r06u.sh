#!/bin/bash
# r06u: slab tests, the balance A/B (register-resident packing kernel), then the bench line (from_dense plans balanced)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06u; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_slab_gpu.py tests/test_mlp_gpu.py tests/test_graph_capture_gpu.py tests/test_kernels_gpu.py tests/test_model3_gpu.py tests/test_parallel_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python -u tools/slab_balance_ab.py > $O/ab.jsonl 2> $O/ab.err || { echo "ab failed"; tail -10 $O/ab.err; exit 1; }
cat $O/ab.jsonl
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'])
print('er_exact_mix', d['er_exact_mix']['ms_per_round'], d['er_exact_mix']['mix_ms'])
print('config5', d['config5_round']['ms_per_round'], d['config5_round']['phase_ms'])
"
timeout -k 10 300 python -u tools/mlp_stagger_ab.py > $O/stagger.jsonl 2> $O/stagger.err || { echo "stagger failed"; tail -10 $O/stagger.err; exit 1; }
cat $O/stagger.jsonl
