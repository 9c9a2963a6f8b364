# r01c profiles on the GPU box: bench trace + FETCH/WRITE passes, and MFMA PMC for the split3 dense mix
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/prof_r01c bash tools/profile.sh || exit 1
python3 tools/summarize_prof.py gpurun_out/prof_r01c gpurun_out/prof_r01c/summary.json || exit 1
timeout -s KILL 300 rocprofv3 --pmc MfmaUtil MfmaFlopsBF16 -d gpurun_out/pmc_mfma -o run --output-format csv -- python3 tools/prof_dense.py > gpurun_out/pmc_mfma.log 2>&1 || { echo "mfma pmc failed"; tail -5 gpurun_out/pmc_mfma.log; exit 1; }
echo "mfma pmc ok"
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE -d gpurun_out/pmc_clk -o run --output-format csv -- python3 tools/prof_dense.py > gpurun_out/pmc_clk.log 2>&1 || { echo "clk pmc failed"; tail -5 gpurun_out/pmc_clk.log; exit 1; }
echo "clk pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_dense -o run --output-format csv -- python3 tools/prof_dense.py > gpurun_out/trace_dense.log 2>&1 || { echo "dense trace failed"; exit 1; }
echo "dense trace ok"
