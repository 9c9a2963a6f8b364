"""Config 5's fused MLP local step (1024 agents x 784-128-10, B = 32,
momentum 0.5): ms per step by HIP events for the current environment
(DOL_MLP_F1_KEEP / DOL_MLP_DW1_REVERSE experiments, r06).  One JSON line.
  python tools/mlp_order_ab.py [--reps 50]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip.bank import AgentBank  # noqa: E402
from dolhip.mlp import BatchedMLP, mlp_layout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n, B, d, h, c = 1024, 32, 784, 128, 10
    bank = AgentBank(n, mlp_layout(d, h, c), dev)
    g = torch.Generator(device=dev).manual_seed(2028)
    bank.rows().normal_(0.0, 0.05, generator=g)
    bank.buffer("mom", zero=True)
    mlp = BatchedMLP(bank, d, h, c)
    X = torch.empty(n, B, d, device=dev).normal_(generator=g)
    y = torch.randint(0, c, (n, B), device=dev, generator=g)
    mlp.step(X, y, lr=0.05, momentum=0.5, first_step=True)
    for _ in range(200):
        mlp.step(X, y, lr=0.05, momentum=0.5, first_step=False)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        mlp.step(X, y, lr=0.05, momentum=0.5, first_step=False)
    e.record()
    torch.cuda.synchronize()
    print(json.dumps({"f1_keep": os.environ.get("DOL_MLP_F1_KEEP", "0"),
                      "dw1_reverse": os.environ.get("DOL_MLP_DW1_REVERSE", "0"),
                      "ms": s.elapsed_time(e) / a.reps}), flush=True)


if __name__ == "__main__":
    main()
