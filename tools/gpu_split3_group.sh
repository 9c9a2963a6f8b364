#!/bin/bash
# split3 GEMM at 1024 agents x 101,770: XCD tile-group height (DOL_SPLIT3_GROUP_M) and wave count, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in DOL_SPLIT3_GROUP_M=8 DOL_SPLIT3_GROUP_M=1 DOL_SPLIT3_GROUP_M=2 DOL_SPLIT3_GROUP_M=4 DOL_SPLIT3_WAVES=4; do
    echo "== $v"
    env $v timeout -k 10 200 python -u tools/bench_dense.py --agents 1024 --params 101770 --reps 20 --skip-f32-above 0 2>/dev/null || exit 1
  done
done
