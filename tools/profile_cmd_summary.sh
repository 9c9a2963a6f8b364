# tools/profile_cmd.sh's three rocprofv3 passes over one python command, then the
# per-kernel summary on the box (only small files stay under gpurun_out/).
#   OUT=gpurun_out/prof_x bash tools/profile_cmd_summary.sh tools/bench_configs.py ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/prof_cmd}
OUT=$OUT bash tools/profile_cmd.sh "$@" || exit 1
python3 tools/summarize_prof.py "$OUT" "$OUT/summary.json" > "$OUT/summary.txt" 2>&1 || exit 1
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write"
head -12 "$OUT/summary.txt"
