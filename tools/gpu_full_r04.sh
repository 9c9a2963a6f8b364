#!/bin/bash
# Round-4 validation on one box: the whole -m gpu suite, smoke, the default
# bench line, then the rocprof trace + FETCH/WRITE passes of the bench
# (tools/profile.sh) summarised per kernel.  Stops at the first crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r04f}
mkdir -p "$OUT"
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; if crash $rc; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; if crash $rc; then exit $rc; fi
fi
timeout -k 10 600 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench.err"; if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PROF" ]; then
  OUT="$OUT/prof" bash tools/profile.sh || exit 1
  python3 tools/summarize_prof.py "$OUT/prof" "$OUT/prof/summary.json" > "$OUT/prof/summary.txt" 2>&1 || exit 1
  cp "$OUT/prof/trace/run_kernel_stats.csv" "$OUT/prof/kernel_stats.csv"
  rm -rf "$OUT/prof/trace" "$OUT/prof/fetch" "$OUT/prof/write"
  head -25 "$OUT/prof/summary.txt"
fi
exit 0
