"""A/B/C timing of the ring-steps kernels (dol_mix_ring_steps_ex_f32 variants)
in the bench's own buffers (ShardedRing(8192, 2^20) at world 1, ld =
row_stride(P)), alternating the variants block by block so every variant
sees the same pages; the headline ring kernel timed beside them.  One JSON
line.  python tools/eps_variants.py [--eps 5] [--variants 1 2 3] [--blocks 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import ops  # noqa: E402
from dolhip.parallel import ShardedRing  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--blocks", type=int, default=3)
    ap.add_argument("--variants", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--agents", type=int, default=8192)
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--ld", type=int, default=0, help="row stride in floats (0: ShardedRing's row_stride(P))")
    ap.add_argument("--directions", action="store_true",
                    help="each variant X -> Y ('v>'), Y -> X ('v<') and alternating as FedLCon's bank.mix swaps ('v~')")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, P = a.agents, a.params
    wp = torch.rand(N)
    wn = torch.rand(N)
    ring = ShardedRing(N, P, wp, wn, dev, ld=a.ld or None)
    ring.x.normal_()
    X, Y = ring.x, ring.y

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.reps

    res = {"ring": []}
    for _ in range(a.blocks):
        res["ring"].append(timed(lambda: ops.mix_ring(X, Y, ring.w_prev, ring.w_next, P=P, n_rows=N)))
        for v in a.variants:
            def run(src, dst):
                return lambda: ops.mix_ring_steps(src, dst, ring.w_prev, ring.w_next, a.eps, P=P, n_rows=N, variant=v)
            if not a.directions:
                res.setdefault(str(v), []).append(timed(run(X, Y)))
                continue
            res.setdefault(f"{v}>", []).append(timed(run(X, Y)))
            res.setdefault(f"{v}<", []).append(timed(run(Y, X)))
            flip = [X, Y]

            def alt():
                ops.mix_ring_steps(flip[0], flip[1], ring.w_prev, ring.w_next, a.eps, P=P, n_rows=N, variant=v)
                flip.reverse()
            res.setdefault(f"{v}~", []).append(timed(alt))
    best = {k: min(v) for k, v in res.items()}
    print(json.dumps({"eps": a.eps, "agents": N, "params": P, "ld": X.stride(0),
                      "dma_d": os.environ.get("DOL_RING_DMA_D", "8"),
                      "ms": res, "best_ms": best,
                      "best_TBps": {k: 2 * N * P * 4 / v / 1e9 for k, v in best.items()}}), flush=True)


if __name__ == "__main__":
    main()
