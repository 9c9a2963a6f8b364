# csr_pm_kernel measurement variants (DOL_PM_VARIANT): 0 default, 1 nt DMA, 2 plain stores, 3 both, 4 copy ceiling
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-0 1 2 3 4 0}; do
  echo "VARIANT=$v"
  DOL_PM_VARIANT=$v timeout -k 10 300 python -u tools/bench_configs.py --agents 1024 8192 --topologies rr4-pm \
    --mlp --dgd --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/pm_sweep.log 2>&1
rc=$?
python3 - <<'PY'
import json
for line in open("gpurun_out/pm_sweep.log"):
    if line.startswith("VARIANT"):
        print(line.strip()); continue
    try:
        d = json.loads(line)
    except Exception:
        print(line[:200].rstrip()); continue
    print("  %-8s N=%5d %7.3f ms %6.0f GB/s %.3f" % (d["topology"], d["agents"], d["ms_per_launch"], d["GBps"], d["frac_of_8TBps"]))
PY
exit $rc
