set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dense" -x -v --timeout 120 --timeout-method thread > gpurun_out/dense_tests.log 2>&1
rc=$?; tail -25 gpurun_out/dense_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_dense.py --agents 1024 2048 8192 --params 101770 --reps 3 > gpurun_out/bench_dense.log 2>&1
rc=$?; cat gpurun_out/bench_dense.log; exit $rc
