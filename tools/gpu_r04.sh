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
  # EPS_ENVS: space-separated env assignments, one run each (comma-joined for several vars)
  for e in ${EPS_ENVS:-DOL_RING_DMA_D=8 DOL_RING_DMA_D=16}; do
    env ${e//,/ } timeout -k 10 300 python -u tools/eps_variants.py $EPS_ARGS > "$OUT/eps_one.json" 2>> "$OUT/eps.err"
    rc=$?; echo "eps $e rc=$rc"
    python -c "import json,sys; d=json.load(open('$OUT/eps_one.json')); d['env']='$e'; print(json.dumps(d))" >> "$OUT/eps.jsonl"
    tail -1 "$OUT/eps.jsonl" | cut -c1-400
    if crash $rc; then exit $rc; fi
  done
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-500} python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.err"
  if crash $rc; then exit $rc; fi
fi
exit 0
