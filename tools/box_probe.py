"""Box probe: the headline ring round, the
parameter-major random-4-regular mix and FedLCon's eps = 5 pass at 8192 x 2^20,
plus a flat copy of the same bytes, timed in one process on one box; one JSON
line.  tools/gpu_box_probe.sh runs it under rocprofv3 (trace + PMC passes) to
compare boxes.   python tools/box_probe.py [--reps 5]"""
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
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, P = 8192, 1 << 20

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.reps

    X = torch.randn(N, P, device=dev)
    Y = torch.empty_like(X)
    wp, wn = torch.rand(N, device=dev), torch.rand(N, device=dev)
    res = {"copy_ms": timed(lambda: Y.copy_(X)),
           "ring_ms": timed(lambda: ops.mix_ring(X, Y, wp, wn)),
           "eps5_ms": timed(lambda: ops.mix_ring_steps(X, Y, wp, wn, 5))}
    c = G.random_regular_csr(N, 4, seed=2028)
    rp, col, val = (torch.as_tensor(t, device=dev) for t in (c.rowptr, c.col, c.val))
    res["pm_ms"] = timed(lambda: ops.mix_csr_pm(X.view(P, N), Y.view(P, N), rp, col, val))
    b = 2 * N * P * 4
    res.update({k.replace("_ms", "_TBps"): b / v / 1e9 for k, v in list(res.items())})
    res["eps5_TBps"] *= 1  # one read + one write of the bank per pass, like the ring round
    res["ring_over_pm"] = res["ring_ms"] / res["pm_ms"]
    res["ring_over_eps5"] = res["ring_ms"] / res["eps5_ms"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
