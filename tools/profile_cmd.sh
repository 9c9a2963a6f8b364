#!/bin/bash
# Three rocprofv3 passes over one python script (run on the GPU box):
#   trace (--kernel-trace --stats), FETCH_SIZE, WRITE_SIZE — each its own run,
#   each under its own hard time limit; stops at the first failure.
#   OUT=gpurun_out/prof_x tools/profile_cmd.sh tools/prof_kernels.py [args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_cmd}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$@" > "$OUT/trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace ok"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "$@" > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
echo "fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 "$@" > "$OUT/write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "write ok"
