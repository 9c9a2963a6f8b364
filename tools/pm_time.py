"""Time the parameter-major CSR mix (dol_mix_csr_pm_f32) on a random 4-regular W
at N agents x P params; one JSON line (HIP events over `reps` launches).
  python tools/pm_time.py [--agents 8192] [--params 1048576] [--reps 10]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=8192)
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, P = a.agents, a.params
    XT = torch.randn(P, N, device=dev)
    YT = torch.empty_like(XT)
    c = G.random_regular_csr(N, 4, seed=2028)
    rp, col, val = (torch.as_tensor(t, device=dev) for t in (c.rowptr, c.col, c.val))
    for _ in range(2):
        ops.mix_csr_pm(XT, YT, rp, col, val)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        ops.mix_csr_pm(XT, YT, rp, col, val)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.reps
    print(json.dumps({"agents": N, "params": P, "nb": os.environ.get("DOL_PM_BIG_NB", "4"), "ms": ms,
                      "TBps": 2 * N * P * 4 / ms / 1e9}), flush=True)


if __name__ == "__main__":
    main()
