# config-5 fused MLP step A/B on one box (r03): tests/test_mlp_gpu.py under each
# variant, then tools/bench_configs.py's MLP round (local-step ms) alternating
# the env settings in $VARIANTS, $REPS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-mlp_ab}
mkdir -p "$OUT"
for v in ${VARIANTS:-DOL_MLP_DW1_CHAINS=1 DOL_MLP_DW1_CHAINS=2}; do
  env $(echo $v | tr , " ") timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py -k "${PYTEST_K:-not bit_identical}" -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 "$OUT/pytest_$v.log")"; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
done
for rep in ${REPS:-1 2 3}; do
  for v in ${VARIANTS:-DOL_MLP_DW1_CHAINS=1 DOL_MLP_DW1_CHAINS=2}; do
    env $(echo $v | tr , " ") timeout -k 10 120 python3 tools/bench_configs.py --mlp 1024 --mlp-mix csr --dgd --dgd-pm --agents > "$OUT/run.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 "$OUT/run.log"; exit $rc; }
    echo "$v $(grep -h '"workload"' "$OUT/run.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("local_ms", round(d["kernel_ms"]["local"],4), "mix_ms", round(d["kernel_ms"]["mix"],4), "round_ms", round(d["ms_per_round"],4))')" | tee -a "$OUT/mlp.txt"
  done
done
