"""Does the fused MLP local step (config 5: 1024 agents x 784-128-10, B = 32,
momentum) depend on where its buffers landed?  K fresh banks (x + mom, and
the batch) in one process, the step timed on each: one JSON line per bank.
python tools/mlp_alloc_probe.py [--banks 6] [--reps 20]"""
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
    ap.add_argument("--banks", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n, B, d, h, c = 1024, 32, 784, 128, 10
    keep = []  # every bank held, so each new one lands on fresh memory
    for k in range(a.banks):
        bank = AgentBank(n, mlp_layout(d, h, c), dev)
        bank.rows().normal_(0.0, 0.05)
        mlp = BatchedMLP(bank, d, h, c)
        X = torch.randn(n, B, d, device=dev)
        y = torch.randint(0, c, (n, B), device=dev)
        mlp.step(X, y, lr=0.05, momentum=0.9, first_step=True)
        keep.append((bank, mlp, X, y))
    for _ in range(300):  # clocks up
        keep[0][1].step(keep[0][2], keep[0][3], lr=0.05, momentum=0.9, first_step=False)
    torch.cuda.synchronize()
    times = {k: [] for k in range(a.banks)}
    for rnd in range(a.rounds):  # round robin: a bank's own speed vs the clock's drift
        for k, (bank, mlp, X, y) in enumerate(keep):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                mlp.step(X, y, lr=0.05, momentum=0.9, first_step=False)
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / a.reps)
    for k, (bank, mlp, X, y) in enumerate(keep):
        print(json.dumps({"bank": k, "ms": times[k], "x": bank.x.data_ptr(), "mom": bank.buffer("mom").data_ptr(),
                          "X": X.data_ptr()}), flush=True)


if __name__ == "__main__":
    main()
