# split3 dense mix on the GPU box: tests, probes, f32-vs-split3 bench, config-5 rounds, rocprof trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_dense_probe.sh > gpurun_out/dense_probe_all.log 2>&1 || { echo "probe step failed"; exit 1; }
echo "probes ok"
timeout -k 10 300 python -u tools/bench_dense.py --agents 1024 2048 8192 --params 101770 --reps 3 > gpurun_out/bench_dense.log 2>&1 || { echo "bench_dense failed"; exit 1; }
echo "bench_dense ok"
timeout -k 10 400 python -u tools/bench_configs.py --agents --dgd --mlp 1024 8192 --reps 5 > gpurun_out/config5.log 2>&1 || { echo "config5 failed"; exit 1; }
echo "config5 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dense -o run --output-format csv -- python3 tools/bench_dense.py --agents 8192 --params 101770 --reps 3 --skip-f32-above 0 > gpurun_out/prof_dense.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo "rocprof ok"
