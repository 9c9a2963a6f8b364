# config-5 local step: rocprofv3 kernel stats of the fused MLP step (mlp_fwd / mlp_dw1) at 1024 agents
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mlpprof -o run --output-format csv -- python3 $R/tools/bench_configs.py --mlp 1024 --mlp-mix csr --dgd --dgd-pm --agents > $R/gpurun_out/mlpprof.log 2>&1
find $R/gpurun_out/mlpprof -name "*kernel_stats.csv" -exec cut -c1-220 {} \;
