# split3 dense-mix diagnostics on the GPU box: PROBES="0 1 2" (full / MFMA only / staging only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "split3" -x -q --timeout 120 --timeout-method thread > gpurun_out/dense_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dense_tests.log; [ $rc -eq 0 ] || exit $rc
for probe in ${PROBES:-0 1 2}; do
  echo "probe=$probe group_m=${DOL_SPLIT3_GROUP_M:-8}"
  DOL_SPLIT3_PROBE=$probe timeout -k 10 200 python -u tools/bench_dense.py --agents 8192 1024 --params 101770 --reps 3 --skip-f32-above 0 || exit $?
done > gpurun_out/dense_probe.log 2>&1
rc=$?; cat gpurun_out/dense_probe.log; exit $rc
