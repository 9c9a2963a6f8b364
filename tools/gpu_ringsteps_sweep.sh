# FedLCon eps = 5 fused ring: 16-B lanes (R = 22, default) vs 8-B lanes with taller tiles
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DOL_RING_STEPS_V2=38 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "ring_steps" -x -q --timeout 120 --timeout-method thread > gpurun_out/rs_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rs_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 22 30 38 54 0 38; do
  echo "v2r=$v"
  DOL_RING_STEPS_V2=$v timeout -k 10 200 python -u tools/bench_configs.py --agents 8192 --topologies ring-eps5 --mlp --dgd --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/rs_sweep.log 2>&1
rc=$?; cut -c1-230 gpurun_out/rs_sweep.log; exit $rc
