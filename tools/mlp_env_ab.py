"""Config 5's fused MLP local step (1024 agents x 784-128-10, B = 32,
momentum 0.5) under settings of one environment variable the step reads per
call (--var, e.g. DOL_MLP_DW1_PAIR), alternating in one process; the updated
rows and momentum compared bit for bit against the first setting's step from
the same start.  One JSON line per (trial, setting).
  python tools/mlp_env_ab.py --var DOL_MLP_DW1_PAIR --settings 0 1 [--reps 50]"""
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
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--var", required=True)
    ap.add_argument("--settings", nargs="+", required=True)
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
    w0 = bank.rows().clone()
    m0 = bank.buffer("mom").clone()
    ref = None
    for trial in range(a.trials):
        for st in a.settings:
            os.environ[a.var] = st
            bank.rows().copy_(w0)
            bank.buffer("mom").copy_(m0)
            mlp.step(X, y, lr=0.05, momentum=0.5, first_step=False)
            torch.cuda.synchronize()
            out = torch.cat([bank.rows(), bank.buffer("mom")], 1)
            if ref is None:
                ref = out
            same = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                mlp.step(X, y, lr=0.05, momentum=0.5, first_step=False)
            e.record()
            torch.cuda.synchronize()
            print(json.dumps({"trial": trial, a.var: st, "ms": s.elapsed_time(e) / a.reps,
                              "bits_equal_first_setting": same}), flush=True)
    os.environ.pop(a.var, None)


if __name__ == "__main__":
    main()
