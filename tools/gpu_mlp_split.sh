# (the DOL_MLP_SPLIT code this script drove was removed after the measurement: profiles/r02_mlp_split.txt)
# config-5 fused MLP step: agent pieces over two streams (DOL_MLP_SPLIT = 1 / 2 / 4), round and local-step times
set -e
R=$GRAFT_REPO_ROOT
for sp in 1 2 4 1 2 4; do
  DOL_MLP_SPLIT=$sp timeout -k 10 120 python3 $R/tools/bench_configs.py --mlp 1024 --mlp-mix csr --dgd --dgd-pm --agents > $R/gpurun_out/mlpsp.log 2>&1
  echo "split=$sp $(grep -h '"workload"' $R/gpurun_out/mlpsp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("local_ms", round(d["kernel_ms"]["local"],4), "mix_ms", round(d["kernel_ms"]["mix"],4), "round_ms", round(d["ms_per_round"],4))')"
done
