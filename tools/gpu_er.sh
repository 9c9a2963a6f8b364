set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "er_stochastic or split3" -x -q --timeout 120 --timeout-method thread > gpurun_out/er_tests.log 2>&1
rc=$?; tail -3 gpurun_out/er_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_configs.py --agents --dgd --mlp 1024 8192 --reps 5 > gpurun_out/config5.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/config5.log | cut -c1-700
