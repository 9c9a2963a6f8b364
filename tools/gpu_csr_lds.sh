# LDS-slab CSR mix (DOL_CSR_MODE=3) on the GPU box: bit-exact CSR/DGD tests
# with the kernel forced at test shapes, then rr4 timings vs the XCD kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DOL_CSR_MODE=3 DOL_CSR_LDS_GRID=16 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgd_gpu.py -k "csr or dgd or rr" -x -q --timeout 120 --timeout-method thread > gpurun_out/csr_lds_tests.log 2>&1
rc=$?; tail -3 gpurun_out/csr_lds_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 1" "3 1" "3 0" "1 1" "3 1"; do
  set -- $cfg
  echo "mode=$1 nt=$2"
  DOL_CSR_MODE=$1 DOL_CSR_LDS_NT=$2 timeout -k 10 300 python -u tools/bench_configs.py --agents 1024 8192 --topologies rr4 --mlp --dgd 1024 8192 --dgd-topologies rr4 --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/csr_lds_sweep.log 2>&1
rc=$?; cut -c1-300 gpurun_out/csr_lds_sweep.log; exit $rc
