"""Driver for PMC passes over the CSR mix on a random 4-regular W (8192 x 2^20
by default): one launch per mode (DOL_CSR_MODE picks XCD-pinned 512-B tiles or
4 KiB tiles), so per-kernel counters separate cleanly."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
P = 1 << 20
dev = torch.device("cuda")
plan = G.MixingPlan(G.random_regular_csr(N, 4, seed=2028), dev)
X = torch.empty(N, row_stride(P), device=dev).normal_()
Y = torch.empty_like(X)
for _ in range(3):
    plan.apply(X, Y, P=P)
torch.cuda.synchronize()
print("prof_csr done")
