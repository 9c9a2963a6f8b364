#!/bin/bash
# Round-3 GPU session: named test files, the slab kernel timing, optional bench.
#   TESTS="tests/a.py tests/b.py" OUT=r03x [BENCH=1] [SLAB=1] tools/gpu_r03.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r03}
mkdir -p "$OUT"
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
  if crash $rc; then exit $rc; fi
fi
if [ -n "$SLAB" ]; then
  timeout -k 10 120 python -u tools/bench_slab.py --agents 1024 --paths slab > "$OUT/slab.jsonl" 2> "$OUT/slab.err"
  rc=$?; echo "slab rc=$rc"; cat "$OUT/slab.jsonl"
  if crash $rc; then exit $rc; fi
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench.err"
  if crash $rc; then exit $rc; fi
fi
exit 0
