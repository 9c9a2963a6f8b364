# split3 GEMM: 4 waves (one per SIMD, 128 x 128 each) vs 8 waves (two per SIMD,
# 128 x 64 each) per 256 x 256 tile; correctness under 8 waves first
set -e
DOL_SPLIT3_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k split3 -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
for w in 4 8 4 8; do
  echo "WAVES=$w"
  DOL_SPLIT3_WAVES=$w timeout -k 10 200 python -u tools/bench_dense.py --agents 1024 8192 --reps 10 --skip-f32-above 0 2>/dev/null
done
