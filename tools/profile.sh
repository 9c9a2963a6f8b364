#!/bin/bash
# rocprofv3 passes for the headline bench (run on the GPU box):
#   1) --kernel-trace --stats      -> per-kernel durations
#   2) --pmc FETCH_SIZE            -> HBM read bytes (own pass)
#   3) --pmc WRITE_SIZE            -> HBM write bytes (own pass)
# Each pass has its own hard timeout; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
ARGS=${ARGS:---steps 10 --warmup 2 --no-cpu --no-copy}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace ok"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
echo "fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "write ok"
