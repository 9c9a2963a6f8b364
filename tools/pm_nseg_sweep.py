"""Parameter-major mix at 8192 x 2^20 (random 4-regular) under each stage order
(DOL_PM_NSEG, read per launch) and its own-geometry copy (DOL_PM_VARIANT=4),
beside the ring round on the same box; one JSON line.
  python tools/pm_nseg_sweep.py [--reps 3]"""
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
    ap.add_argument("--reps", type=int, default=3)
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
    c = G.random_regular_csr(N, 4, seed=2028)
    rp, col, val = (torch.as_tensor(t, device=dev) for t in (c.rowptr, c.col, c.val))
    def pm(ns):
        return lambda: ops.mix_csr_pm(X.view(P, N), Y.view(P, N), rp, col, val, nseg=ns)
    res = {"ring_ms": timed(lambda: ops.mix_ring(X, Y, wp, wn))}
    for ns in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        res[f"pm_nseg{ns}_ms"] = timed(pm(ns))
    os.environ["DOL_PM_VARIANT"] = "4"
    for ns in (8, 16, 32, 64, 256):
        res[f"pm_geometry_copy_nseg{ns}_ms"] = timed(pm(ns))
    os.environ.pop("DOL_PM_VARIANT")
    res["pm_default_ms"] = timed(pm(0))
    res["pm_tuned_ms"] = timed(pm(None))
    res["pm_tuned"] = ops.pm_stage_order_choice(Y.view(P, N), X.view(P, N), N, P=P)
    res["ring_ms_again"] = timed(lambda: ops.mix_ring(X, Y, wp, wn))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
