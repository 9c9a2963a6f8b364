# config-5 fused MLP step: F1 pipeline depth 2 / 3 / 4 (DOL_MLP_STAGES), kernel stats per setting
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for ns in 3 2 4 3; do
  rm -rf $R/gpurun_out/mlpst
  DOL_MLP_STAGES=$ns timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mlpst -o run --output-format csv -- python3 $R/tools/bench_configs.py --mlp 1024 --mlp-mix csr --dgd --dgd-pm --agents > $R/gpurun_out/mlpst.log 2>&1
  echo "stages=$ns $(grep -h '"workload"' $R/gpurun_out/mlpst.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("local_ms", round(d["kernel_ms"]["local"],4), "round_ms", round(d["ms_per_round"],4))')"
  grep -h "mlp_fwd\|mlp_dw1" $(find $R/gpurun_out/mlpst -name "*kernel_stats.csv") | cut -d, -f1,2,4 | cut -c1-40,100-200
done
