"""Is bench.py's dense ER leg (split3 at 1024 x 101,770) slower because of where
it runs in the bench (after the HBM-heavy legs) rather than what it runs?
Times bench.dense_mix_round fresh, right after ~3 s of 8192 x 2^20 ring
rounds, and again after a 2 s idle; prints one JSON line per case."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
import bench  # noqa: E402
from dolhip import ops  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    out = {"fresh": bench.dense_mix_round(dev)["ms_per_round"]}
    N, P = 8192, 1 << 20
    ld = row_stride(P)
    X = torch.empty(N, ld, device=dev).normal_()
    Y = torch.empty_like(X)
    wp = torch.full((N,), 0.5, device=dev)
    wn = torch.full((N,), 0.5, device=dev)
    t0 = time.time()
    while time.time() - t0 < 3.0:
        for _ in range(20):
            ops.mix_ring(X, Y, wp, wn, P=P)
        torch.cuda.synchronize()
    out["after_ring_load"] = bench.dense_mix_round(dev)["ms_per_round"]
    del X, Y
    torch.cuda.empty_cache()
    time.sleep(2.0)
    out["after_2s_idle"] = bench.dense_mix_round(dev)["ms_per_round"]
    out["fresh_again"] = bench.dense_mix_round(dev)["ms_per_round"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
