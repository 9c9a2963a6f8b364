"""Config 5's mix (Erdos-Renyi p = 0.1 W, 101,770-parameter MLP agents) on the
three bit-exact / tolerance paths:
  slab   : dol_mix_csr_slab_f32 (LDS-gather CSR, bit-exact)      + device Neighbors
  csr    : dol_mix_csr_f32 (generic L2-gather CSR, bit-exact)
  split3 : dol_mix_dense_split3_f32 (bf16 MFMA, fp32-accurate, split pass included)

  python tools/bench_slab.py [--agents 1024 8192] [--params 101770] [--reps 20]
One JSON line per (agents, path).  LDS bound of the slab kernel: nnz * P * 4 B
of LDS reads at 256 B/clk/CU."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip import ops  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, nargs="*", default=[1024, 8192])
    ap.add_argument("--params", type=int, default=101770)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--paths", nargs="*", default=["slab", "csr", "split3"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    P = a.params
    for N in a.agents:
        ld = row_stride(P)
        g = torch.Generator(device=dev).manual_seed(2028)
        X = torch.empty(N, ld, device=dev).normal_(generator=g)
        Y = torch.empty_like(X)
        W = G.erdos_renyi_stochastic_hip(N, a.p, seed=2028, device=dev)
        state = {"plan": G.MixingPlan.from_dense(W, dense_kernel="csr")}

        def draw_csr():  # retires the previous plan (its buffers are reused)
            state["plan"] = G.MixingPlan.from_dense(W, dense_kernel="csr", reuse=state["plan"])
        t_build = timed(draw_csr, a.reps)
        plan = state["plan"]
        nnz = int(plan.rowptr[-1].item())
        base = {"agents": N, "params": P, "p_edge": a.p, "nnz": nnz, "mean_degree": nnz / N}
        for path in a.paths:
            if path == "slab":
                ms = timed(lambda: plan.apply(X, Y, P=P), a.reps)
            elif path == "csr":
                ms = timed(lambda: ops.mix_csr(X, Y, plan.rowptr, plan.col, plan.val, P=P), a.reps)
            elif path == "split3":
                if N > 8192:
                    continue
                dplan = G.MixingPlan.from_dense(W)
                ms = timed(lambda: dplan.apply(X, Y, P=P), max(2, a.reps // 4))
                del dplan
            else:
                raise SystemExit(path)
            lds_bytes = nnz * P * 4
            rec = dict(base, path=path, ms=ms, rounds_per_s=1e3 / ms,
                       hbm_GBps_2NP=2 * N * P * 4 / (ms / 1e3) / 1e9,
                       lds_GBps=lds_bytes / (ms / 1e3) / 1e9,
                       lds_frac_of_256B_clk_2p4GHz=lds_bytes / (ms / 1e3) / (256 * 256 * 2.4e9),
                       dense_TFLOPs_equiv=2.0 * N * N * P / (ms / 1e3) / 1e12,
                       neighbours_build_ms=t_build)
            print(json.dumps(rec), flush=True)
        del X, Y, W, plan, state
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
