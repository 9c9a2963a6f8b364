# CSR mix variants on the GPU box: bit-exact CSR/DGD tests with each variant
# forced at test shapes, then rr4 timings (1024 / 8192 agents x 2^20).
#   DOL_CSR_MODE=1 XCD-pinned tiles (r01), 3 LDS slab (<= 4096 agents), 4 persistent L2 gather
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
runt() {
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgd_gpu.py -k "csr or dgd or rr" -x -q \
    --timeout 120 --timeout-method thread
}
if [ -z "$NO_TESTS" ]; then
  DOL_CSR_MODE=3 DOL_CSR_LDS_GRID=16 runt > gpurun_out/csr_t3.log 2>&1; rc=$?; tail -1 gpurun_out/csr_t3.log; [ $rc -eq 0 ] || exit $rc
  DOL_CSR_MODE=5 DOL_CSR_LDS_GRID=16 runt > gpurun_out/csr_t5.log 2>&1; rc=$?; tail -1 gpurun_out/csr_t5.log; [ $rc -eq 0 ] || exit $rc
  DOL_CSR_MODE=6 DOL_CSR_LDS_GRID=16 runt > gpurun_out/csr_t6.log 2>&1; rc=$?; tail -1 gpurun_out/csr_t6.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-"1_8" "3_8" "4_8" "4_4" "1_8" "3_8" "4_8" "4_4"}; do
  m=${cfg%_*}; tw=${cfg#*_}
  echo "mode=$m tw=$tw"
  DOL_CSR_MODE=$m DOL_CSR_XCDP_TW=$tw timeout -k 10 300 python -u tools/bench_configs.py --agents 1024 8192 \
    --topologies rr4 --mlp --dgd 1024 8192 --dgd-topologies rr4 --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/csr_sweep2.log 2>&1
rc=$?
python3 - <<'PY'
import json
for line in open("gpurun_out/csr_sweep2.log"):
    line = line.strip()
    if line.startswith("mode"):
        print(line)
        continue
    try:
        d = json.loads(line)
    except Exception:
        print(line[:200])
        continue
    if "workload" in d:
        print("  dgd %-13s N=%5d %7.3f ms %6.0f GB/s" % (d["objective"], d["agents"], d["ms_per_round"], d["GBps"]))
    else:
        print("  mix rr4 N=%5d %7.3f ms %6.0f GB/s %.3f" % (d["agents"], d["ms_per_launch"], d["GBps"], d["frac_of_8TBps"]))
PY
exit $rc
