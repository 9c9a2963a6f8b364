"""Host logic: communication_graph / CSR extraction vs the reference's own
outputs (tests/golden/graphs.npz, csr.npz), ring detection, Sinkhorn guard,
random-regular generator, shard bounds."""
import numpy as np
import pytest
import torch

from conftest import golden
from dolhip import graph as G
from dolhip.parallel import shard_bounds


def _graph_keys():
    return sorted(golden("graphs").files)


def _parse(key):
    parts = key.split("_")
    return parts[0], "_".join(parts[1:-1]), int(parts[-1])


@pytest.mark.parametrize("key", _graph_keys())
def test_communication_graph_bit_exact(key):
    """Simulator.communication_graph (DIST/simulators.py:40-86), seed 2028."""
    topo, mode, n = _parse(key)
    torch.manual_seed(2028)
    gs = G.communication_graph(topo, mode, n)
    arr = np.ascontiguousarray(np.stack([np.asarray(g.numpy() if torch.is_tensor(g) else g) for g in gs]))
    ref = golden("graphs")[key]
    assert arr.dtype == ref.dtype and arr.shape == ref.shape
    assert arr.tobytes() == ref.tobytes()


@pytest.mark.parametrize("key", _graph_keys())
def test_csr_equals_reference_neighbors(key):
    """Simulator.Neighbors (DIST/simulators.py:91-97) for every row and step."""
    topo, mode, n = _parse(key)
    torch.manual_seed(2028)
    gs = G.communication_graph(topo, mode, n)
    csr = golden("csr")
    for t, g in enumerate(gs):
        c = G.csr_from_dense(g)
        k = f"{key}__t{t}"
        assert np.array_equal(c.rowptr, csr[k + "__rowptr"])
        assert np.array_equal(c.col, csr[k + "__col"])
        assert c.val.tobytes() == csr[k + "__val"].tobytes()


def test_rng_consumption_matches_reference():
    """Exactly one torch.rand(n, n) per weighted call (order matters: W is drawn
    after model init in Simulator.__init__)."""
    torch.manual_seed(5)
    G.communication_graph("circle", "stochastic", 7)
    a = torch.rand(3)
    torch.manual_seed(5)
    torch.rand(7, 7)
    b = torch.rand(3)
    assert torch.equal(a, b)


def test_dynamic_stochastic_isolated_rows_are_empty():
    torch.manual_seed(2028)
    gs = G.communication_graph("dynamic", "stochastic", 6)
    assert len(gs) == 6
    c = G.csr_from_dense(gs[0])
    deg = np.diff(c.rowptr)
    assert deg[0] == 1 and deg[1] == 1 and deg[2:].sum() == 0  # NaN rows drop out


def test_ring_detection():
    torch.manual_seed(0)
    for n in (3, 4, 5, 64):
        c = G.csr_from_dense(G.communication_graph("circle", "stochastic", n)[0])
        wp, wn = c.ring_weights()
        d = c.dense()
        i = np.arange(n)
        assert np.array_equal(wp, d[i, (i - 1) % n]) and np.array_equal(wn, d[i, (i + 1) % n])
    for topo in ("star", "compelete"):
        c = G.csr_from_dense(G.communication_graph(topo, "stochastic", 6)[0])
        assert c.ring_weights() is None
    assert G.csr_from_dense(G.communication_graph("circle", "stochastic", 2)[0]).ring_weights() is None


def test_complete_alias():
    torch.manual_seed(1)
    a = G.communication_graph("compelete", "stochastic", 5)[0]
    torch.manual_seed(1)
    b = G.communication_graph("complete", "stochastic", 5)[0]
    assert torch.equal(a, b)


def test_sinkhorn_bounded_raises_where_reference_hangs():
    torch.manual_seed(2028)
    with pytest.raises(G.SinkhornNotConverged):
        G.communication_graph("star", "double_stochastic", 6, sinkhorn_max_iters=200)
    torch.manual_seed(2028)
    w = G.communication_graph("compelete", "double_stochastic", 16, sinkhorn_max_iters=10_000,
                              sinkhorn_tol=1e-6)[0].numpy()
    assert np.abs(w.sum(0) - 1).max() <= 1e-6 and np.abs(w.sum(1) - 1).max() <= 1e-6


def test_unknown_topology_builds_nothing():
    assert G.communication_graph("torus", "stochastic", 4) == []


def test_random_regular():
    c = G.random_regular_csr(256, 4, seed=3)
    deg = np.diff(c.rowptr)
    assert np.all(deg == 4)
    d = c.dense()
    assert np.all(np.diag(d) == 0)
    assert np.abs(d.sum(1) - 1).max() < 1e-6
    assert np.array_equal(d > 0, (d > 0).T)  # symmetric support
    c2 = G.random_regular_csr(256, 4, seed=3)
    assert np.array_equal(c.col, c2.col) and c.val.tobytes() == c2.val.tobytes()


@pytest.mark.parametrize("n,world", [(8192, 1), (8192, 8), (10, 3), (7, 2), (1024, 8)])
def test_shard_bounds_partition(n, world):
    b = [shard_bounds(n, world, r) for r in range(world)]
    assert b[0][0] == 0 and b[-1][1] == n
    for (a0, a1), (b0, b1) in zip(b, b[1:]):
        assert a1 == b0
    sizes = [hi - lo for lo, hi in b]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("topo,mode,n", [("circle", "stochastic", n) for n in (1, 2, 3, 5, 6, 16, 64, 300)] +
                         [("dynamic", "stochastic", n) for n in (2, 3, 6, 17)] +
                         [("circle", "none", 6), ("dynamic", "none", 5), ("star", "stochastic", 6),
                          ("compelete", "stochastic", 5), ("circle", "double_stochastic", 6)])
def test_communication_csr_equals_dense_path(topo, mode, n):
    """The sparse builder gives bit-identical CSRs and consumes the same RNG."""
    torch.manual_seed(2028)
    dense = [G.csr_from_dense(g) for g in G.communication_graph(topo, mode, n)]
    after_dense = torch.rand(3)
    torch.manual_seed(2028)
    sparse = G.communication_csr(topo, mode, n)
    assert torch.equal(torch.rand(3), after_dense)
    assert len(dense) == len(sparse)
    for a, b in zip(dense, sparse):
        assert np.array_equal(a.rowptr, b.rowptr) and np.array_equal(a.col, b.col)
        assert a.val.tobytes() == b.val.tobytes()


def test_dynamic_8192_is_sparse_and_fast():
    import time
    torch.manual_seed(2028)
    t = time.time()
    gs = G.communication_csr("dynamic", "stochastic", 8192)
    assert len(gs) == 8192 and all(g.nnz == 2 for g in gs[:10])
    assert time.time() - t < 60


def test_csr_validate_rejects_malformed():
    """A malformed CSR is an error when a MixingPlan is built, not an
    out-of-bounds device read (advisor finding)."""
    from dolhip.graph import CSR
    ok = CSR(3, 3, np.array([0, 1, 3, 3], np.int32), np.array([1, 0, 2], np.int32), np.ones(3, np.float32))
    assert ok.validate() is ok
    bad = [
        CSR(3, 3, np.array([0, 1, 3], np.int32), np.array([1, 0, 2], np.int32), np.ones(3, np.float32)),
        CSR(3, 3, np.array([1, 1, 3, 3], np.int32), np.array([1, 0, 2], np.int32), np.ones(3, np.float32)),
        CSR(3, 3, np.array([0, 2, 1, 3], np.int32), np.array([1, 0, 2], np.int32), np.ones(3, np.float32)),
        CSR(3, 3, np.array([0, 1, 3, 4], np.int32), np.array([1, 0, 2], np.int32), np.ones(3, np.float32)),
        CSR(3, 3, np.array([0, 1, 3, 3], np.int32), np.array([1, 0, 3], np.int32), np.ones(3, np.float32)),
        CSR(3, 3, np.array([0, 1, 3, 3], np.int32), np.array([1, -1, 2], np.int32), np.ones(3, np.float32)),
        CSR(3, 3, np.array([0, 1, 3, 3], np.int32), np.array([1, 0, 2], np.int32), np.ones(2, np.float32)),
    ]
    for c in bad:
        with pytest.raises(ValueError):
            c.validate()
