# CSR mix variants on the GPU box (random 4-regular, 8192 x 2^20): tests under the variant, then a sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DOL_CSR_MODE=1 DOL_CSR_XW=24 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgd_gpu.py -k "csr or dgd" -x -q --timeout 120 --timeout-method thread > gpurun_out/csr_tests.log 2>&1
rc=$?; tail -2 gpurun_out/csr_tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-32 24 16 32 24}; do
  xw=$v
  echo "xw=$xw"
  DOL_CSR_XW=$xw timeout -k 10 200 python -u tools/bench_configs.py --agents 8192 --topologies rr4 --mlp --dgd --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/csr_sweep.log 2>&1
rc=$?; cut -c1-260 gpurun_out/csr_sweep.log; exit $rc
