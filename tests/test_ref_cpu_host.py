"""bench.py's CPU baseline for the headline (oracle/ref_cpu.py: the
reference-structured Neighbors scan + consensus + load_state_dict round, and
the vectorised torch ring round beside it) computes the same mixing as the
reference and as the oracle the kernels are pinned to (the
headline's CPU leg had no test), so the line's GPU/CPU ratio compares like
with like.  Reference: DIST/simulators.py:91-97,147-152, DIST/clients.py:61-69."""
import numpy as np
import pytest
import torch

import oracle
from conftest import golden
from oracle import bits_equal, ref_cpu


def _cases():
    mix = golden("mix")
    return sorted(k[:-3] for k in mix.files if k.endswith("__X"))


@pytest.mark.parametrize("case", _cases())
def test_ref_cpu_mixing_round_matches_reference_golden(case):
    """One reference-structured round on the reference's own W (graphs.npz),
    against the reference's consensus output (mix.npz) and oracle.mix_csr --
    every topology incl. the dynamic schedule's NaN rows (isolated agents -> 0)."""
    mix, graphs, csr = golden("mix"), golden("graphs"), golden("csr")
    gkey, _layout, t = case.split("__")
    W = torch.from_numpy(np.ascontiguousarray(graphs[gkey][int(t[1:])]))
    X = torch.from_numpy(mix[case + "__X"].copy())
    agents = [ref_cpu.Agent({"w": X[i]}) for i in range(X.shape[0])]
    ref_cpu.mixing_round(W, agents)
    got = X.numpy()
    assert bits_equal(got, mix[case + "__Y"])
    c = f"{gkey}__{t}"
    want = oracle.mix_csr(mix[case + "__X"], csr[c + "__rowptr"], csr[c + "__col"], csr[c + "__val"])
    assert bits_equal(got, want)


@pytest.mark.parametrize("n,P", [(7, 257), (64, 1000), (6, 1)])
def test_ref_cpu_rounds_match_oracle_ring(n, P):
    """time_rounds' loop (several rounds, rows of one matrix as the agents)
    and the vectorised ring round both equal oracle.mix_ring round for round
    on communication_graph('circle', 'stochastic', n); the vectorised form only
    differs in the sign of a zero (no +0 start), so it is compared by value."""
    from dolhip import graph as G
    torch.manual_seed(2028)
    W = G.communication_graph("circle", "stochastic", n)[0]
    rw = G.csr_from_dense(W).ring_weights()
    X0 = np.random.default_rng(n).standard_normal((n, P)).astype(np.float32)
    X0[0, 0] = -0.0
    X = torch.from_numpy(X0.copy())
    rounds, _ = ref_cpu.time_rounds(W, X, min_seconds=0.0, max_rounds=3, warmup=True)
    want = X0
    for _ in range(rounds + 1):  # + the warm-up round
        want = oracle.mix_ring(want, rw[0], rw[1])
    assert bits_equal(X.numpy(), want)
    Xv, Yv = torch.from_numpy(X0.copy()), torch.empty(n, P)
    ref_cpu.vectorized_ring_round(Xv, Yv, torch.from_numpy(rw[0]), torch.from_numpy(rw[1]))
    np.testing.assert_array_equal(Yv.numpy(), oracle.mix_ring(X0, rw[0], rw[1]))
