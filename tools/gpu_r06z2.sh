#!/bin/bash
# r06z2: the bench under rocprofv3 (kernel trace + FETCH_SIZE / WRITE_SIZE passes, summarised)
R=$GRAFT_REPO_ROOT
cd $R
# under rocprofv3 a released mapped block does not give its memory back (r06z: free memory
# unchanged after 64 GiB of blocks were freed, then an OOM): profile on torch-allocated buffers
export DOL_BANK_ALLOC=torch
OUT=gpurun_out/r06z_prof bash tools/profile_cmd_summary.sh bench.py --steps 20 --no-cpu --map-ring 0 || { echo "profile failed"; grep "^\[bench" gpurun_out/r06z_prof/*.log | tail -20; tail -5 gpurun_out/r06z_prof/trace.log; exit 1; }
grep "^\[bench" gpurun_out/r06z_prof/trace.log 2>/dev/null | tail -12
