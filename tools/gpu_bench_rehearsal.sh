# N>1 bench path rehearsed on a 1-GPU box: 2 ranks on cuda:0, halos staged through gloo
# (the driver's 8-GPU run uses RCCL; this checks the sharded code path end to end)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DOL_DEVICE_MAP=0 DOL_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --agents 1024 --params 262144 \
  --no-cpu > gpurun_out/bench_rehearsal.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/bench_rehearsal.log | tail -3 | cut -c1-900; exit $rc
