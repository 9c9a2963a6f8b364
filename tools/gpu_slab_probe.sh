set -e
for pr in 0 1 2; do
  echo "PROBE=$pr"
  DOL_SLAB_PROBE=$pr timeout -k 10 120 python -u tools/bench_slab.py --agents 1024 --paths slab 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/slabprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_slab.py --agents 1024 --paths slab > /dev/null 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/slabprof -name "*stats*" | head
