# Round-2 profile of the default bench: tools/profile.sh's three passes, then the
# per-kernel summary on the box, keeping only small files under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/prof_r02}
OUT=$OUT bash tools/profile.sh || exit 1
tail -3 "$OUT/trace.log"
python3 tools/summarize_prof.py "$OUT" "$OUT/summary.json" > "$OUT/summary.txt" 2>&1 || exit 1
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write"
head -40 "$OUT/summary.txt"
