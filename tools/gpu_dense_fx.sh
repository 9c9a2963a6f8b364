# fused-X split3: tests, then fused vs split-pass timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dense" -q -rf --timeout 120 --timeout-method thread > gpurun_out/dense_tests.log 2>&1
rc=$?; tail -8 gpurun_out/dense_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_dense.py --agents 1024 2048 8192 --params 101770 --reps 3 > gpurun_out/bench_dense.log 2>&1 || exit 1
cut -c1-700 gpurun_out/bench_dense.log
