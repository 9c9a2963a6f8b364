"""Time the FedADMM least-squares round at BASELINE config 4's size (8192 x
2^20, 10 local steps, momentum, frac 1): the one-pass round + mean
(dol_admm_ls_round_mean_f32) and the two-kernel round (dol_admm_ls_round_f32 +
the ordered mean), each kernel by HIP events on the launch stream.  One JSON
line; run once per DOL_ADMM_ROUND_THREADS setting (read once per process).

  python tools/admm_round_ab.py [--agents N] [--params P] [--rounds R]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-optimization-and-learning_amd"))
from dolhip import ops  # noqa: E402
from dolhip.synthetic import SeparableADMM  # noqa: E402


def timed(prob, name, fn, rounds):
    evs = []

    def wrap(*a, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn(*a, **kw)
        e.record()
        evs.append((s, e))
        return out
    setattr(prob, name, wrap)
    for _ in range(rounds):
        prob.round()
    torch.cuda.synchronize()
    setattr(prob, name, fn)
    return [a.elapsed_time(b) for a, b in evs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=8192)
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    N, P = a.agents, a.params
    prob = SeparableADMM(N, P, rho=0.1, lr=0.1, momentum=0.5, local_steps=10, frac=1.0, seed=2028,
                         device=torch.device("cuda"), mean="fast", fused=True)
    prob.round()  # first momentum step
    torch.cuda.synchronize()
    fused = timed(prob, "_round_mean", ops.admm_ls_round_mean, a.rounds)
    prob.fused = False
    prob.round()
    rnd = timed(prob, "_round", ops.admm_ls_round, a.rounds)
    mean_ev = []
    osum = ops.ordered_sum

    def wrap_sum(*x, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = osum(*x, **kw)
        e.record()
        mean_ev.append((s, e))
        return out
    prob._osum = wrap_sum
    for _ in range(a.rounds):
        prob.round()
    torch.cuda.synchronize()
    mean = [x.elapsed_time(y) for x, y in mean_ev]
    row_bytes = N * P * 4
    ms_f = min(fused)
    print(json.dumps({"agents": N, "params": P, "round_threads": os.environ.get("DOL_ADMM_ROUND_THREADS", "1024"),
                      "round_mean_ms": fused, "round_mean_GBps_best": (6 * row_bytes + 8 * P) / ms_f / 1e6,
                      "client_round_ms": rnd, "client_round_GBps_best": 6 * row_bytes / min(rnd) / 1e6,
                      "ordered_mean_ms": mean, "two_kernel_best_ms": min(rnd) + min(mean)}), flush=True)


if __name__ == "__main__":
    main()
