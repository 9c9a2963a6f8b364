"""Where does the parameter-major mix differ from the oracle? (debug aid)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from dolhip import graph as G, ops  # noqa: E402

gpu = torch.device("cuda")
for n, P in [(6, 154), (6, 40), (5, 10), (7, 33), (16, 154), (9, 100)]:
    torch.manual_seed(2028)
    c = G.communication_csr("circle", "stochastic", n)[0]
    X = np.random.default_rng(1).standard_normal((n, P)).astype(np.float32)
    ld = (n + 3) // 4 * 4
    XT = torch.full((P, ld), float("nan"), device=gpu)
    XT[:, :n] = torch.as_tensor(X.T.copy(), device=gpu)
    YT = torch.full((P, ld), 7.0, device=gpu)
    rp = torch.as_tensor(c.rowptr, device=gpu)
    col = torch.as_tensor(c.col, device=gpu)
    val = torch.as_tensor(c.val, device=gpu)
    ops.mix_csr_pm(XT, YT, rp, col, val)
    got = YT.cpu().numpy()[:, :n].T
    want = oracle.mix_csr(X, c.rowptr, c.col, c.val)
    bad = ~((got == want) | (np.isnan(got) & np.isnan(want)))
    print(f"n={n} P={P} mismatches={bad.sum()} agents={sorted(set(np.nonzero(bad)[0].tolist()))} "
          f"p={sorted(set(np.nonzero(bad)[1].tolist()))[:40]}")
    if bad.any():
        i, p = np.argwhere(bad)[0]
        print("   first bad", i, p, got[i, p], want[i, p], "7.0 means unwritten")
