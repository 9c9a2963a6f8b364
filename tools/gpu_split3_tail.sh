# split3 narrow-tail path: its tests, then the bench's dense ER round (1024 x 101,770) with the tail path on / off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "split3" -x -q --timeout 120 --timeout-method thread > gpurun_out/split3_tail_tests.log 2>&1
rc=$?; tail -2 gpurun_out/split3_tail_tests.log; [ $rc -eq 0 ] || exit $rc
for c in default 0 default 0; do for NAG in 1024 2048; do export NAG
  if [ $c = default ]; then unset DOL_SPLIT3_CUS; else export DOL_SPLIT3_CUS=$c; fi
  timeout -k 10 120 python -u -c "
import json, os, torch, bench
r = bench.dense_mix_round(torch.device('cuda', 0), N=int(os.environ.get('NAG', '1024')), reps=20)
r['DOL_SPLIT3_CUS'] = os.environ.get('DOL_SPLIT3_CUS', 'device'); print(json.dumps(r))" 2>&1 | grep '^{' || exit 1
done; done > gpurun_out/split3_tail.log 2>&1
rc=$?; cut -c1-230 gpurun_out/split3_tail.log; exit $rc
