#!/bin/bash
# r06z: the final tree -- GPU suite, smoke, the N = 1 bench line, and the bench
# under rocprofv3 (kernel trace + FETCH_SIZE / WRITE_SIZE passes, summarised)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06z}; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { echo "suite failed"; tail -40 $O/suite.txt; exit 1; }
tail -1 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'])
print('er_exact_mix', d['er_exact_mix']['ms_per_round'], d['er_exact_mix']['mix_ms'])
print('config5', d['config5_round']['ms_per_round'], d['config5_round']['phase_ms'])
print('split3', d['dense_er_mix']['bf16_mfma_util'])
"
[ -n "$NO_PROF" ] || { export DOL_BANK_ALLOC=torch; OUT=gpurun_out/${RUN:-r06z}_prof bash tools/profile_cmd_summary.sh bench.py --steps 20 --no-cpu --map-ring 0 || { echo "profile failed"; exit 1; }; }
