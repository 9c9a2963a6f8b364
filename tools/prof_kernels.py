"""Driver for rocprofv3 passes over the non-headline kernels: the fused MLP
local step (config 5, 1024 agents 784-128-10, B = 32) and the fused DGD round
(config 3, 1024 agents x 2^20, ring and random 4-regular, least squares with
momentum).  Each is launched `--reps` times after a warm-up.
  rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python3 tools/prof_kernels.py"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.bank import AgentBank  # noqa: E402
from dolhip.mlp import BatchedMLP, mlp_layout  # noqa: E402
from dolhip.synthetic import SeparableDGD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--params", type=int, default=1 << 20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.agents
    bank = AgentBank(N, mlp_layout(784, 128, 10), dev)
    mlp = BatchedMLP(bank, 784, 128, 10)
    bank.buffer("x").normal_(0, 0.05)
    X = torch.randn(N, 32, 784, device=dev)
    y = torch.randint(0, 10, (N, 32), device=dev)
    for k in range(a.reps + 1):
        mlp.step(X, y, lr=0.05, momentum=0.5, first_step=(k == 0))
    torch.cuda.synchronize()
    del bank, mlp, X, y
    torch.cuda.empty_cache()
    for topo in ("ring", "rr4"):
        if topo == "ring":
            torch.manual_seed(2028)
            plan = G.MixingPlan(G.communication_csr("circle", "stochastic", N)[0], dev)
        else:
            plan = G.MixingPlan(G.random_regular_csr(N, 4, seed=2028), dev)
        prob = SeparableDGD(plan, a.params, objective="least_squares", lr=0.01, momentum=0.5, local_steps=1)
        for _ in range(a.reps + 1):
            prob.round()
        torch.cuda.synchronize()
        del prob, plan
        torch.cuda.empty_cache()
    print("prof_kernels done")


if __name__ == "__main__":
    main()
