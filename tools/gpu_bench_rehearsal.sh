# N>1 bench path rehearsed on a 1-GPU box: NPROC ranks (default 2) on cuda:0, halos
# and the FedADMM means staged through gloo (the driver's multi-GPU runs use RCCL;
# this checks the sharded code path end to end).  ARGS overrides the bench size.
#   NPROC=8 ARGS="--agents 8192 --params 1048576" OUT=r03b bash tools/gpu_bench_rehearsal.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-rehearsal}
mkdir -p "$OUT"
NPROC=${NPROC:-2}
DOL_DEVICE_MAP=0 DOL_DIST_BACKEND=gloo timeout -k 10 ${REH_TIMEOUT:-300} python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node $NPROC --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $NPROC --steps 5 --warmup 2 \
  ${ARGS:---agents 1024 --params 262144} --no-cpu --no-copy > "$OUT/bench_rehearsal_n$NPROC.log" 2>&1
rc=$?; grep -v amdgpu "$OUT/bench_rehearsal_n$NPROC.log" | tail -3 | cut -c1-900; exit $rc
