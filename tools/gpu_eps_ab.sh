# FedLCon eps pass A/B (r03): the register-tile kernel (DOL_RING_STREAM=0) vs the
# streaming kernel at tile heights 256 / 512 / 1024, tools/eps_pass_time.py at
# 8192 x 2^20 (eps 5 unless EPS is set), alternating twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-eps_ab}
mkdir -p "$OUT"
for rep in ${REPS:-1 2}; do
  for v in ${VARIANTS:-DOL_RING_STREAM=0 DOL_RING_STREAM_T=1024 DOL_RING_STREAM_T=2048 DOL_RING_STREAM_T=4096 DOL_RING_STREAM_PF=16}; do
    echo "# $v" >> "$OUT/eps.jsonl"
    env $(echo $v | tr , " ") timeout -k 10 120 python -u tools/eps_pass_time.py --eps ${EPS:-5} >> "$OUT/eps.jsonl" 2>> "$OUT/eps.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 "$OUT/eps.err"; exit $rc; }
  done
done
cat "$OUT/eps.jsonl"
