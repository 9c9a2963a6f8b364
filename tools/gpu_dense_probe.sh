# split3 dense-mix diagnostics on the GPU box: PROBES="0 1 2 3 4" (full / MFMA only / staging only / MFMA only without stores / full without stores)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for probe in ${PROBES:-0 1 2 3 4}; do
  echo "probe=$probe"
  DOL_SPLIT3_PROBE=$probe timeout -k 10 200 python -u tools/bench_dense.py --agents 8192 1024 --params 101770 --reps 3 --skip-f32-above 0 || exit $?
done > gpurun_out/dense_probe.log 2>&1
