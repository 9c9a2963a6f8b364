# csr_slab kernel diagnostics (1024 x 101,770, ER p = 0.1): index by v_readlane
# vs uniform LDS reads, staging-only and gathers-only probes
set -e
for v in "DOL_SLAB_READLANE=1" "DOL_SLAB_READLANE=0" "DOL_SLAB_PROBE=1" "DOL_SLAB_PROBE=2" "DOL_SLAB_READLANE=1" "DOL_SLAB_READLANE=0"; do
  echo "$v"
  env $v timeout -k 10 120 python -u tools/bench_slab.py --agents 1024 --paths slab 2>/dev/null
done
