#!/bin/bash
# Round-4 GPU session: named tests (+ optional -k filter), optional bench.
#   TESTS="tests/a.py tests/b.py" [KEXPR="ring_steps"] OUT=r04a [BENCH=1] [BENCH_ARGS=...] tools/gpu_r04.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r04}
mkdir -p "$OUT"
crash() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
if [ -n "$TESTS" ]; then
  if [ -n "$KEXPR" ]; then
    timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -k "$KEXPR" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  else
    timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  fi
  rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
  if crash $rc; then exit $rc; fi
fi
if [ -n "$EPS" ]; then
  for d in 8 16; do
    DOL_RING_DMA_D=$d timeout -k 10 300 python -u tools/eps_variants.py $EPS_ARGS >> "$OUT/eps.jsonl" 2> "$OUT/eps.err"
    rc=$?; echo "eps D=$d rc=$rc"; tail -1 "$OUT/eps.jsonl"
    if crash $rc; then exit $rc; fi
  done
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-500} python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.err"
  if crash $rc; then exit $rc; fi
fi
exit 0
