set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --steps 20 > gpurun_out/b1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_configs.py --agents 8192 --topologies ring ring-eps5 --mlp --dgd --reps 10 > gpurun_out/b2.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/b1.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['fedlcon_eps5'])"
grep -v amdgpu gpurun_out/b2.log | cut -c1-200
