"""A/B of the LDS-gather CSR mix's kernel variants (dol_slab_set_variant: 1 =
a loop per (row, chunk) segment, r03; 2 = the wave's pairs as one pipelined
stream, r06) on config 5's mix: 1024 agents x 101,770 (the 784-128-10 MLP),
Erdos-Renyi p = 0.1 W drawn on the device; plus 8192 x 1024.  Variants
alternate in one process on the same buffers; every rep's output is compared
bit for bit across variants.  One JSON line per (shape, variant, trial).

  python tools/slab_variant_ab.py [--trials 3] [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip import ops  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", nargs="*", default=["1024x101770", "8192x1024"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    for shape in a.shapes:
        N, P = (int(x) for x in shape.split("x"))
        ld = row_stride(P)
        g = torch.Generator(device=dev).manual_seed(2028)
        X = torch.empty(N, ld, device=dev).normal_(generator=g)
        W = G.erdos_renyi_stochastic_hip(N, 0.1, seed=2028, device=dev)
        plan = G.MixingPlan.from_dense(W, dense_kernel="csr")
        nnz = int(plan.rowptr[-1].item())
        outs = {}
        for trial in range(a.trials):
            for v in ops.SLAB_VARIANTS:
                ops.slab_variant(v)
                Y = outs.setdefault(v, torch.empty_like(X))
                t0 = torch.cuda.Event(enable_timing=True)
                t1 = torch.cuda.Event(enable_timing=True)
                for _ in range(3):
                    plan.apply(X, Y, P=P)
                t0.record()
                for _ in range(a.reps):
                    plan.apply(X, Y, P=P)
                t1.record()
                torch.cuda.synchronize()
                ms = t0.elapsed_time(t1) / a.reps
                same = bool(torch.equal(Y[:, :P].view(torch.int32), outs[ops.SLAB_VARIANTS[0]][:, :P].view(torch.int32)))
                print(json.dumps({"agents": N, "params": P, "nnz": nnz, "variant": v, "trial": trial, "ms": ms,
                                  "lds_TBps": nnz * P * 4 / ms / 1e9, "bits_equal_variant1": same}), flush=True)
        ops.slab_variant(0)
        del X, W, plan, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
