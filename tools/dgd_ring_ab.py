"""Config 3's fused ring DGD round (SeparableDGD: least squares + momentum
0.9, 1024 agents x 2^20, dol_dgd_ring_f32 = ring_mix_dma_kernel<DgdEpi>):
ms per round by HIP events, for the PMC passes of tools/gpu_r06f.sh.
  python tools/dgd_ring_ab.py [--reps 10] [--objective least_squares]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.synthetic import SeparableDGD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--objective", default="least_squares")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(2028)
    plan = G.MixingPlan(G.communication_csr("circle", "stochastic", a.agents)[0], dev)
    mom = 0.9 if a.objective == "least_squares" else 0.0
    prob = SeparableDGD(plan, a.params, objective=a.objective, lr=0.01, momentum=mom, local_steps=1, seed=7)
    for _ in range(3):
        prob.round()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        prob.round()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.reps
    alg = a.agents * a.params * 4 * (3 + (2 if mom else 0))
    print(json.dumps({"nt": os.environ.get("DOL_DGD_EPI_NT", "0"), "objective": a.objective, "ms": ms,
                      "frac": alg / (ms / 1e3) / 8e12, "alg_bytes": alg}), flush=True)


if __name__ == "__main__":
    main()
