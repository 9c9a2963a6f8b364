#!/bin/bash
# r06r: split3 tail variants (kernel trace) + slab tests under the new default variant
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06r; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/split3_tail_ab.py > $O/ab.jsonl 2> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
" | sort -k3 -n -r | head -12
