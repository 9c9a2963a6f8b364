#!/bin/bash
# r06j: counters of slow vs fast (source, destination) pairs of FedLCon's eps pass (tools/eps_pair_counters.py);
# each pass its own process (own allocations): the kernel trace of the same run says which pairs are slow there
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06j; mkdir -p $O
i=0
for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
           "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" \
           "TCC_EA0_WRREQ TCC_EA0_RDREQ" \
           "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set -d $O/p$i -o run --output-format csv -- python3 $R/tools/eps_pair_counters.py > $O/p$i.json 2> $O/p$i.log || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i ok"
done
