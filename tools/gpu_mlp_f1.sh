# (the DOL_MLP_F1 code this script drove was removed after the measurement: profiles/r02_mlp_split.txt)
# config-5 fused MLP step: F1 staging variants (DOL_MLP_F1 = 0: 32-k chunks x 3 stages, 1: 16-k x 4, 2: 16-k x 6);
# the MLP GPU tests under each, then local-step / round times alternating on one box
set -e
R=$GRAFT_REPO_ROOT
for v in 1 2; do
  DOL_MLP_F1=$v timeout -k 10 300 python -u -m pytest $R/tests/test_mlp_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
done
for v in 0 1 2 0 1 2; do
  DOL_MLP_F1=$v timeout -k 10 120 python3 $R/tools/bench_configs.py --mlp 1024 --mlp-mix csr --dgd --dgd-pm --agents > $R/gpurun_out/mlpf1.log 2>&1
  echo "f1=$v $(grep -h '"workload"' $R/gpurun_out/mlpf1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("local_ms", round(d["kernel_ms"]["local"],4), "round_ms", round(d["ms_per_round"],4))')"
done
