# Config 3's fused round on the parameter-major bank: its tests, then timings
# beside the agent-major fused round of the same box (1024 x 2^20).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_pmajor_gpu.py ${EXTRA_TESTS} -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pm_dgd_tests.log 2>&1
rc=$?; tail -1 gpurun_out/pm_dgd_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/pm_dgd_tests.log | head -80; exit $rc; }
timeout -k 10 300 python -u tools/bench_configs.py --agents --mlp --dgd 1024 --dgd-pm 1024 --reps 10 \
  > gpurun_out/pm_dgd_bench.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/pm_dgd_bench.log | cut -c1-400
exit $rc
