"""Config 5's exact ER mix (LDS-gather CSR, csr_slab_kernel) at 1024 agents x
101,770 parameters vs the agent-row stride: X / Y are views of the same two
allocations at each stride; the plan (ER p = 0.1, seed 2028) is built once.
Strides alternate twice; one JSON line per (rep, stride)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
from dolhip import graph as G  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, P = 1024, 101770
    base = row_stride(P)
    lds = [base + int(x) for x in (sys.argv[1:] or "0 64 256 1024 2048 4672 6720".split())]
    ldmax = max(lds)
    fx = torch.empty(N * ldmax, device=dev).normal_()
    fy = torch.empty(N * ldmax, device=dev)
    W = G.erdos_renyi_stochastic_hip(N, 0.1, 2028, dev)
    plan = G.MixingPlan.from_dense(W, dense_kernel="csr")
    for rep in range(2):
        for ld in lds:
            X = fx[: N * ld].view(N, ld)
            Y = fy[: N * ld].view(N, ld)
            t0 = torch.cuda.Event(enable_timing=True)
            t1 = torch.cuda.Event(enable_timing=True)
            for _ in range(20):
                plan.apply(X, Y, P=P)
            torch.cuda.synchronize()
            t0.record()
            for _ in range(50):
                plan.apply(X, Y, P=P)
            t1.record()
            torch.cuda.synchronize()
            print(json.dumps({"rep": rep, "ld": ld, "ld_mod_4096": ld % 4096, "mix_ms": t0.elapsed_time(t1) / 50}),
                  flush=True)


if __name__ == "__main__":
    main()
