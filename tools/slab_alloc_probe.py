"""Does config 5's exact mix (csr_slab_kernel, 1024 x 101,770, ER p = 0.1)
depend on where its X / Y landed?  K pairs of fresh [N, ld] matrices held at
once, the mix timed on each pair round-robin (so the clock's drift is not
mistaken for a pair's speed).  One JSON line per pair.
python tools/slab_alloc_probe.py [--pairs 6] [--rounds 4] [--reps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, P = 1024, 101770
    ld = row_stride(P)
    W = G.erdos_renyi_stochastic_hip(N, 0.1, seed=2028, device=dev)
    plan = G.MixingPlan.from_dense(W, dense_kernel="csr")
    pairs = []
    for k in range(a.pairs):
        X = torch.empty(N, ld, device=dev).normal_()
        Y = torch.empty_like(X)
        pairs.append((X, Y))
    for _ in range(200):  # clocks up
        plan.apply(pairs[0][0], pairs[0][1], P=P)
    torch.cuda.synchronize()
    times = {k: [] for k in range(a.pairs)}
    for _ in range(a.rounds):
        for k, (X, Y) in enumerate(pairs):
            plan.apply(X, Y, P=P)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                plan.apply(X, Y, P=P)
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / a.reps)
    for k, (X, Y) in enumerate(pairs):
        print(json.dumps({"pair": k, "ms": [round(t, 4) for t in times[k]], "X": X.data_ptr(), "Y": Y.data_ptr()}),
              flush=True)


if __name__ == "__main__":
    main()
