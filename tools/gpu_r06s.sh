#!/bin/bash
# r06s: the GPU suite, smoke and the N = 1 bench line on the current tree
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06s; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { echo "suite failed"; tail -40 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
