#!/bin/bash
# r06p: csr_slab_kernel variant 3 (asm stream): slab GPU tests under every variant, then the A/B
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_slab_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 240 python -u tools/slab_variant_ab.py --trials 3 --reps 20 > $O/ab.jsonl 2> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
