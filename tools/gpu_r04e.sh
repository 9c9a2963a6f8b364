#!/bin/bash
# r04 experiments: allocation modes vs the ring rate, pm stage orders (incl. 64-256),
# eps pass sweep order / tile height, dW1 tile order A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r04e}
mkdir -p "$OUT"
timeout -k 10 300 tools/alloc_probe 2 > "$OUT/alloc_probe.jsonl" 2> "$OUT/alloc_probe.err"
rc=$?; echo "alloc rc=$rc"; cat "$OUT/alloc_probe.jsonl"; [ $rc -eq 0 ] || exit $rc
for w in 1 0; do
  DOL_PM_WAIT=$w timeout -k 10 300 python -u tools/pm_nseg_sweep.py > "$OUT/pm_nseg_wait$w.json" 2>> "$OUT/pm_nseg.err"
  rc=$?; echo "pm wait=$w rc=$rc"; cut -c1-1500 "$OUT/pm_nseg_wait$w.json"; [ $rc -eq 0 ] || exit $rc
done
EPS=1 EPS_ARGS="--variants 1 3" EPS_ENVS="${EPS_ENVS:-DOL_RING_DMA_ORDER=0 DOL_RING_DMA_ORDER=1,DOL_RING_STREAM_T=64 DOL_RING_DMA_ORDER=1,DOL_RING_STREAM_T=128 DOL_RING_DMA_ORDER=1,DOL_RING_STREAM_T=256 DOL_RING_DMA_ORDER=1,DOL_RING_STREAM_T=512 DOL_RING_DMA_ORDER=1,DOL_RING_STREAM_T=128,DOL_RING_DMA_PROBE=1}" OUT=$(basename "$OUT") tools/gpu_r04.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
OUT=$(basename "$OUT")_mlp REPS="1 2" VARIANTS="DOL_MLP_DW1_XCD=0 DOL_MLP_DW1_XCD=1" timeout -k 10 900 bash tools/gpu_mlp_ab.sh
