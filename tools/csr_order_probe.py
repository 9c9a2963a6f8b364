"""Timing probe: does the ORDER in which output rows are processed change the
random-regular CSR mix's speed?  Relabels the seeded random 4-regular graph
(graph.random_regular_csr) by reverse Cuthill-McKee / BFS so that rows
processed close in time share neighbours, and times plan.apply on the
relabelled graph against the original (same nnz, same bytes).  Results of the
relabelled mix are a permutation of a different summation order, so this only
measures memory behaviour.

  python tools/csr_order_probe.py [--agents 8192] [--params 1048576]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from scipy.sparse.csgraph import breadth_first_order, reverse_cuthill_mckee  # noqa: E402
import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def relabel(csr, perm):
    """new label k = old agent perm[k]; rows and columns permuted, cols ascending."""
    n = csr.n_rows
    A = sp.csr_matrix((csr.val, csr.col, csr.rowptr.astype(np.int64)), shape=(n, n))
    B = A[perm][:, perm].tocsr()
    B.sort_indices()
    return G.CSR(n, n, B.indptr.astype(np.int32), B.indices.astype(np.int32), B.data.astype(np.float32))


def time_apply(plan, X, Y, P, reps):
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
    ap.add_argument("--agents", type=int, default=8192)
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    N, P = a.agents, a.params
    dev = torch.device("cuda", 0)
    csr = G.random_regular_csr(N, 4, seed=2028)
    A = sp.csr_matrix((csr.val, csr.col, csr.rowptr.astype(np.int64)), shape=(N, N))
    orders = {"original": np.arange(N),
              "rcm": reverse_cuthill_mckee(A, symmetric_mode=True),
              "bfs": breadth_first_order(A, 0, directed=False, return_predecessors=False)}
    X = torch.empty(N, row_stride(P), device=dev).normal_()
    # controls under the same kernel: degree-1 graphs (each row read once) in
    # order (identity) and in a random order (a permutation)
    one = np.ones(N, np.float32)
    rp = np.arange(N + 1, dtype=np.int32)
    for name, col in (("identity-d1", np.arange(N, dtype=np.int32)),
                      ("permutation-d1", torch.randperm(N, generator=torch.Generator().manual_seed(1)).numpy().astype(np.int32))):
        plan = G.MixingPlan(G.CSR(N, N, rp, col, one), dev, allow_ring=False)
        ms = time_apply(plan, X, torch.empty_like(X), P, a.reps)
        print(json.dumps({"order": name, "agents": N, "params": P, "ms": ms, "GBps": 2 * N * P * 4 / (ms / 1e3) / 1e9,
                          "csr_mode": os.environ.get("DOL_CSR_MODE", "auto")}), flush=True)
    Y = torch.empty_like(X)
    for name, perm in orders.items():
        c2 = relabel(csr, np.asarray(perm))
        bw = int(np.max(np.abs(np.repeat(np.arange(N), np.diff(c2.rowptr)) - c2.col)))
        ms = time_apply(G.MixingPlan(c2, dev), X, Y, P, a.reps)
        print(json.dumps({"order": name, "agents": N, "params": P, "bandwidth": bw, "ms": ms,
                          "GBps": 2 * N * P * 4 / (ms / 1e3) / 1e9,
                          "csr_mode": os.environ.get("DOL_CSR_MODE", "auto")}), flush=True)


if __name__ == "__main__":
    main()
