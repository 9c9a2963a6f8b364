"""Driver for MFMA-utilisation PMC passes (MfmaUtil, MfmaFlopsF32): the dense
fp32-MFMA mix of an Erdos-Renyi W (config 5, 2048 agents x 2^20) and the
fused MLP local step (1024 agents, 784-128-10, B = 32).
  rocprofv3 --pmc MfmaUtil MfmaFlopsF32 -d DIR -o run --output-format csv -- python3 tools/prof_dense.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.bank import AgentBank, row_stride  # noqa: E402
from dolhip.mlp import BatchedMLP, mlp_layout  # noqa: E402

dev = torch.device("cuda")
N, P = 2048, 1 << 20
gen = torch.Generator(device=dev).manual_seed(2028)
plan = G.MixingPlan.from_dense(G.erdos_renyi_stochastic(N, 0.1, gen))
X = torch.empty(N, row_stride(P), device=dev).normal_()
Y = torch.empty_like(X)
for _ in range(3):
    plan.apply(X, Y, P=P)
torch.cuda.synchronize()
del X, Y, plan
torch.cuda.empty_cache()
bank = AgentBank(1024, mlp_layout(784, 128, 10), dev)
mlp = BatchedMLP(bank, 784, 128, 10)
bank.buffer("x").normal_(0, 0.05)
Xb = torch.randn(1024, 32, 784, device=dev)
yb = torch.randint(0, 10, (1024, 32), device=dev)
for k in range(3):
    mlp.step(Xb, yb, lr=0.05, momentum=0.5, first_step=(k == 0))
torch.cuda.synchronize()
print("prof_dense done")
