#!/bin/bash
# r06c: narrow-strip fused FedADMM round (column-sharded ranks' geometry) A/B + the ADMM / parallel GPU tests
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_admm_gpu.py tests/test_parallel_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "admm" > $O/tests.txt 2>&1 || exit 1
for t in 1024 256 64 0; do
  DOL_ADMM_ROUND_THREADS=$t timeout -k 10 120 python -u tools/admm_round_ab.py --params 131072 --rounds 5 >> $O/narrow_ab.jsonl || exit 1
done
timeout -k 10 120 python -u tools/admm_round_ab.py --rounds 5 >> $O/narrow_ab.jsonl || exit 1
