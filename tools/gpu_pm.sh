# Parameter-major CSR mix on the GPU box: its tests, then 1024 / 8192 x 2^20
# timings beside the agent-major kernels of the same box (ring, random 4-regular)
# and the pm kernel's own copy ceiling (DOL_PM_VARIANT=4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pmajor_gpu.py ${EXTRA_TESTS} -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pm_tests.log 2>&1
rc=$?; tail -1 gpurun_out/pm_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/pm_tests.log | head -80; exit $rc; }
{
  timeout -k 10 300 python -u tools/bench_configs.py --agents ${AGENTS:-1024 8192} --topologies ring rr4 rr4-pm ring-pm \
    --mlp --dgd --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
  echo "copy ceiling (DOL_PM_VARIANT=4)"
  DOL_PM_VARIANT=4 timeout -k 10 300 python -u tools/bench_configs.py --agents ${AGENTS:-1024 8192} --topologies rr4-pm \
    --mlp --dgd --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
} > gpurun_out/pm_bench.log 2>&1
rc=$?
python3 - <<'PY'
import json
for line in open("gpurun_out/pm_bench.log"):
    try:
        d = json.loads(line)
    except Exception:
        print(line[:200].rstrip()); continue
    print("  %-8s N=%5d %7.3f ms %6.0f GB/s %.3f" % (d["topology"], d["agents"], d["ms_per_launch"], d["GBps"], d["frac_of_8TBps"]))
PY
exit $rc
