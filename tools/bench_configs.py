"""Secondary mixing workloads (BASELINE configs 3 and 5): rounds/s and GB/s of
one X <- W X round for ring / random-regular / (optional) dense W.

  python tools/bench_configs.py [--agents 1024 8192] [--params 1048576] [--reps 10]
Prints one JSON line per (topology, N).  Algorithmic bytes = 2*N*P*4 (each
row read once, written once), as in the headline."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def time_plan(plan, X, Y, P, reps):
    for _ in range(2):
        plan.apply(X, Y, P=P)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        plan.apply(X, Y, P=P)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, nargs="+", default=[1024, 8192])
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--topologies", nargs="+", default=["ring", "ring-eps5", "rr4", "dense-er0.1"])
    ap.add_argument("--dense-max-agents", type=int, default=2048)
    a = ap.parse_args()
    dev = torch.device("cuda")
    P = a.params
    for N in a.agents:
        ld = row_stride(P)
        X = torch.empty(N, ld, device=dev).normal_()
        Y = torch.empty_like(X)
        for topo in a.topologies:
            t0 = time.time()
            steps = 1
            extra = {}
            if topo.startswith("ring"):
                torch.manual_seed(2028)
                plan = G.MixingPlan.from_graph(G.communication_graph("circle", "stochastic", N)[0], dev)
                if "-eps" in topo:
                    steps = int(topo.split("-eps")[1])
            elif topo.startswith("rr"):
                plan = G.MixingPlan(G.random_regular_csr(N, int(topo[2:]), seed=2028), dev)
            elif topo.startswith("dense-er"):
                if N > a.dense_max_agents:
                    continue
                p_edge = float(topo[len("dense-er"):])
                gen = torch.Generator().manual_seed(2028)
                A = (torch.rand(N, N, generator=gen) < p_edge).float()
                A.fill_diagonal_(0)
                R = torch.rand(N, N, generator=gen) * A
                R /= R.sum(0).clamp_min(1e-30)
                plan = G.MixingPlan.from_graph(R.T.contiguous(), dev, dense=True)
                extra["flops"] = 2.0 * N * N * P
            else:
                raise SystemExit(f"unknown topology {topo}")
            build_s = time.time() - t0
            if steps > 1:
                def run():
                    plan.apply_steps(X, Y, steps, P=P)
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s_.record()
                for _ in range(a.reps):
                    run()
                e_.record()
                torch.cuda.synchronize()
                ms = s_.elapsed_time(e_) / a.reps
            else:
                ms = time_plan(plan, X, Y, P, a.reps)
            alg = 2 * N * P * 4
            rec = {"topology": topo, "kernel": plan.kind, "agents": N, "params": P, "nnz": plan.csr.nnz,
                   "rounds_per_launch": steps, "ms_per_launch": ms, "rounds_per_s": steps * 1e3 / ms,
                   "GBps": alg / (ms / 1e3) / 1e9, "frac_of_8TBps": alg / (ms / 1e3) / 1e9 / 8000.0,
                   "plan_build_s": build_s}
            if "flops" in extra:
                tf = extra["flops"] / (ms / 1e3) / 1e12
                rec.update({"TFLOPs": tf, "mfma_util_vs_157TF": tf / 157.3})
            print(json.dumps(rec), flush=True)
        del X, Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
