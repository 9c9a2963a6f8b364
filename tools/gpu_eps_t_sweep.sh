cd "${GRAFT_REPO_ROOT}"
for v in "DOL_RING_STREAM_T=1024" "DOL_RING_STREAM_T=256" "DOL_RING_STREAM_T=2048" "DOL_RING_STREAM_T=128,DOL_RING_DMA_ORDER=1" "DOL_RING_STREAM_T=32,DOL_RING_DMA_ORDER=1"; do
  env $(echo $v | tr , " ") timeout -k 10 200 python tools/eps_variants.py --variants 3 4 --blocks 2 > gpurun_out/epst.json 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/epst.json').read().strip().splitlines()[-1]); print(sys.argv[1], d.get('best_ms'))" "$v"
done
