# csr_slab kernel diagnostics (1024 x 101,770, ER p = 0.1): index by uniform LDS
# reads (default) vs v_readlane (DOL_SLAB_MODE=2), staging-only and gathers-only
# probes, and the 8192-agent case
set -e
for v in "DOL_SLAB_PROBE=0" "DOL_SLAB_PROBE=1" "DOL_SLAB_PROBE=0"; do
  echo "$v"
  env $v timeout -k 10 120 python -u tools/bench_slab.py --agents 1024 --paths slab 2>/dev/null
done
timeout -k 10 120 python -u tools/bench_slab.py --agents 8192 --paths slab 2>/dev/null
