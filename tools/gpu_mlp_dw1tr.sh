# (the DOL_MLP_DW1_TR code this script drove was removed after the measurement: profiles/r02_mlp_split.txt)
# config-5 fused MLP step: transposed dW1 tiles (DOL_MLP_DW1_TR=1, 16-B W1 / momentum accesses) vs the default;
# MLP GPU tests under the variant, then local-step / round times alternating on one box
set -e
R=$GRAFT_REPO_ROOT
DOL_MLP_DW1_TR=1 timeout -k 10 300 python -u -m pytest $R/tests/test_mlp_gpu.py $R/tests/test_dropin_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
for v in 0 1 0 1; do
  DOL_MLP_DW1_TR=$v timeout -k 10 120 python3 $R/tools/bench_configs.py --mlp 1024 --mlp-mix csr --dgd --dgd-pm --agents > $R/gpurun_out/mlptr.log 2>&1
  echo "tr=$v $(grep -h '"workload"' $R/gpurun_out/mlptr.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("local_ms", round(d["kernel_ms"]["local"],4), "round_ms", round(d["ms_per_round"],4))')"
done
