#!/bin/bash
# r06d: slab kernel variants (row loop vs pipelined stream): bit-exact tests under both, then the A/B timing
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_slab_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
timeout -k 10 300 python -u tools/slab_variant_ab.py --trials 3 > $O/ab.jsonl || exit 1
