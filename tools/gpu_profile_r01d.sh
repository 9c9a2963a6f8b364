# r01d: headline bench trace + FETCH/WRITE passes with this round's final build, then the N=2 rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/prof_${TAG:-r01d} bash tools/profile.sh || exit 1
python3 tools/summarize_prof.py gpurun_out/prof_${TAG:-r01d} gpurun_out/prof_${TAG:-r01d}/summary.json || exit 1
bash tools/gpu_bench_rehearsal.sh
