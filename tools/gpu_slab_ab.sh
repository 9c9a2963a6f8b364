# csr_slab A/B on one box: slab GPU tests, then tools/bench_slab.py at 1024 x 101,770
# ER p = 0.1 alternating the env settings in $VARIANTS (e.g. "DOL_SLAB_BALANCE=1 DOL_SLAB_BALANCE=0").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-slab_ab}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in ${VARIANTS:-DOL_SLAB_BALANCE=1}; do
    echo "# $v" >> "$OUT/slab.jsonl"
    env $v timeout -k 10 120 python -u tools/bench_slab.py --agents ${AGENTS:-1024} --paths slab >> "$OUT/slab.jsonl" 2>> "$OUT/slab.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -3 "$OUT/slab.err"; exit $rc; }
  done
done
cat "$OUT/slab.jsonl" | cut -c1-200
