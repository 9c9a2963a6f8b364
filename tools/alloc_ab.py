"""Headline ring round (8192 x 2^20, ld = row_stride(2^20)) on two buffer
pairs held at once in one process -- torch's caching allocator vs
dol_bank_alloc mapped blocks (bank.device_matrix(mapped=True)) -- alternating
pairs for several reps; one JSON line per (rep, allocator).  Also times the
FedLCon eps = 5 pass (the tuned kernel per pair) on both."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
from dolhip import bank as B, ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in evs:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in evs)
    return sum(ms) / len(ms), ms[0]


def main():
    dev = torch.device("cuda:0")
    N, P = 8192, 1 << 20
    ld = B.row_stride(P)
    pairs = {}
    for kind in ("torch", "mapped"):
        X = B.device_matrix(N, ld, dev, mapped=(kind == "mapped"))
        Y = B.device_matrix(N, ld, dev, mapped=(kind == "mapped"))
        X.normal_()
        Y.zero_()
        pairs[kind] = (X, Y)
    wp = torch.full((N,), 0.5, device=dev)
    wn = torch.full((N,), 0.5, device=dev)
    for X, Y in pairs.values():  # warm the clocks
        for _ in range(20):
            ops.stream_copy_rows(X, Y, P=P)
    for rep in range(4):
        for kind, (X, Y) in pairs.items():
            mean, best = timed(lambda: ops.mix_ring(X, Y, wp, wn, P=P))
            em, eb = timed(lambda: ops.mix_ring_steps(X, Y, wp, wn, 5, P=P, n_rows=N), reps=8)
            print(json.dumps({"rep": rep, "alloc": kind, "ring_ms_mean": mean, "ring_ms_min": best,
                              "ring_TBps": 2 * N * P * 4 / (mean / 1e3) / 1e12, "eps5_ms_mean": em, "eps5_ms_min": eb,
                              "eps5_pick": (ops.ring_steps_choice(X, Y, 5, P=P, n_rows=N) or {}).get("choice")}),
                  flush=True)


if __name__ == "__main__":
    main()
