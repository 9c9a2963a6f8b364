# ring mix: nontemporal DMA loads for the rows no other tile reads (DOL_RING_NTI, default 1);
# ring tests under both settings, then bench.py A/B pairs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1; do
  DOL_RING_NTI=$v timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgd_gpu.py -k "ring or dgd" -x -q --timeout 120 --timeout-method thread > gpurun_out/nti_tests.log 2>&1 || exit $?
done
for v in 0 1 0 1 0 1; do
  DOL_RING_NTI=$v timeout -k 10 200 python -u bench.py --no-cpu --no-primal-dual --steps 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('nti=$v', round(d['value'],2), round(d['roofline']['kernel_ms'],3), round(d['roofline']['copy_kernel_GBps'],0))" || exit 1
done > gpurun_out/nti.log 2>&1
rc=$?; cat gpurun_out/nti.log; exit $rc
