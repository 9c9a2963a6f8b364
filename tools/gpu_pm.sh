# Parameter-major CSR mix + FedADMM-LS round on the GPU box: tests, then timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pmajor_gpu.py tests/test_admm_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pm_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/pm_tests.log | head -80; exit $rc; }
for nb in 4 3; do
  echo "NBUF=$nb"
  DOL_PM_NBUF=$nb timeout -k 10 300 python -u tools/bench_configs.py --agents 1024 8192 --topologies rr4-pm ring-pm rr4 \
    --mlp --dgd --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/pm_bench.log 2>&1
rc=$?
cat gpurun_out/pm_bench.log
exit $rc
