# (the DOL_MLP_DW1_WPE code this script drove was removed after the measurement: profiles/r02_mlp_split.txt)
# config-5 fused MLP step: dW1 compiled for >= 5 / 6 waves per SIMD (DOL_MLP_DW1_WPE) vs the default (4);
# MLP GPU tests under each variant, then local-step / round times alternating on one box
set -e
R=$GRAFT_REPO_ROOT
for v in 5 6; do
  DOL_MLP_DW1_WPE=$v timeout -k 10 300 python -u -m pytest $R/tests/test_mlp_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
done
for v in 0 5 6 0 5 6; do
  DOL_MLP_DW1_WPE=$v timeout -k 10 120 python3 $R/tools/bench_configs.py --mlp 1024 --mlp-mix csr --dgd --dgd-pm --agents > $R/gpurun_out/mlpw.log 2>&1
  echo "wpe=$v $(grep -h '"workload"' $R/gpurun_out/mlpw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("local_ms", round(d["kernel_ms"]["local"],4), "round_ms", round(d["ms_per_round"],4))')"
done
