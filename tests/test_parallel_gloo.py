"""Multi-rank logic on CPU with the gloo backend (world sizes 2 and 3).

The kernels are the HIP ops in production; here the sharding, halo exchange,
boundary-row handling and ordered chain reduce are exercised with the CPU
oracle injected as the arithmetic (the checker), and the gathered result is
compared bit-for-bit with a single-process oracle run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from dolhip import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cpu_mix_ring(X, Y, w_prev, w_next, halo_prev=None, halo_next=None, P=None, n_rows=None):
    n = X.shape[0] if n_rows is None else n_rows
    P = X.shape[1] if P is None else P
    hp = None if halo_prev is None else halo_prev[:P].numpy()
    hn = None if halo_next is None else halo_next[:P].numpy()
    out = oracle.mix_ring(X[:n, :P].numpy(), w_prev[:n].numpy(), w_next[:n].numpy(), hp, hn)
    Y[:n, :P] = torch.from_numpy(out)
    return Y


def cpu_mix_ring_edges(X, Y, w_prev, w_next, halo_prev, halo_next, P=None, n_rows=None):
    """CPU stand-in for dol_mix_ring_edges_f32: rows 0 and n-1 of the block."""
    n = X.shape[0] if n_rows is None else n_rows
    P = X.shape[1] if P is None else P
    hp, hn = halo_prev[:P].numpy(), halo_next[:P].numpy()
    nxt0 = X[1, :P].numpy() if n > 1 else hn
    Y[0, :P] = torch.from_numpy(oracle.mix_ring(X[0:1, :P].numpy(), w_prev[0:1].numpy(), w_next[0:1].numpy(),
                                                hp, nxt0))
    if n > 1:
        Y[n - 1, :P] = torch.from_numpy(oracle.mix_ring(X[n - 1:n, :P].numpy(), w_prev[n - 1:n].numpy(),
                                                        w_next[n - 1:n].numpy(), X[n - 2, :P].numpy(), hn))
    return Y


def cpu_ordered_sum(W, order, acc_in=None, out=None, scale=1.0, P=None):
    if W is None or order.numel() == 0:
        res = acc_in[:P].numpy().astype(np.float32)
        if scale != 1.0:
            res = (res / np.float32(scale)).astype(np.float32)
    else:
        res = oracle.ordered_sum(W[:, :P].numpy(), order.numpy(),
                                 None if acc_in is None else acc_in[:P].numpy(), scale)
    out[:P] = torch.from_numpy(res)
    return out


def _worker(rank, world, port, N, P, rounds, order, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    try:
        rng = np.random.default_rng(11)
        X = rng.standard_normal((N, P)).astype(np.float32)
        wp = rng.random(N).astype(np.float32)
        wn = rng.random(N).astype(np.float32)
        ring = parallel.ShardedRing(N, P, wp, wn, "cpu", ld=P + 3, mix_ring=cpu_mix_ring,
                                    mix_edges=cpu_mix_ring_edges if rank % 2 else None)
        ring.x[:, :P] = torch.from_numpy(X[ring.lo:ring.hi])
        for _ in range(rounds):
            ring.step()
        mixed = ring.x[:, :P].clone()
        exact = parallel.global_mean_exact(ring.x, ring.lo, ring.hi, order, P, ordered_sum=cpu_ordered_sum)
        local = [g - ring.lo for g in order if ring.lo <= g < ring.hi]
        fast = parallel.global_mean(ring.x, local, len(order), P, ordered_sum=cpu_ordered_sum)
        q.put((rank, ring.lo, ring.hi, mixed.numpy(), exact.numpy()[:P].copy(), fast.numpy()[:P].copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 10), (3, 11), (2, 4), (8, 35)])
def test_sharded_ring_and_means_match_single_process(world, N):
    P, rounds = 37, 3
    order = [7 % N, 0, N - 1, 3, 1, 2]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, P, rounds, order, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # single-process reference run of the same arithmetic
    rng = np.random.default_rng(11)
    X = rng.standard_normal((N, P)).astype(np.float32)
    wp = rng.random(N).astype(np.float32)
    wn = rng.random(N).astype(np.float32)
    for _ in range(rounds):
        X = oracle.mix_ring(X, wp, wn)
    got = np.concatenate([r[3] for r in res])
    assert oracle.bits_equal(got, X)
    want_mean = oracle.ordered_mean(X, np.array(order))
    for r in res:
        assert oracle.bits_equal(r[4], want_mean)  # exact chain: bit-identical on every rank
        np.testing.assert_allclose(r[5], want_mean, rtol=1e-5, atol=1e-6)  # all_reduce form


def _exact_mean_worker(rank, world, port, N, P, orders, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    try:
        X = np.random.default_rng(29).standard_normal((N, P)).astype(np.float32)
        X[3, 5] = -0.0
        X[N - 1, :3] = [np.inf, -1e-42, 3e38]
        lo, hi = parallel.shard_bounds(N, world, rank)
        rows = torch.zeros(max(hi - lo, 1), P + 5)  # ld = P + 5: rows are strided views
        rows[:hi - lo, :P] = torch.from_numpy(X[lo:hi])
        outs = [parallel.global_mean_exact(rows, lo, hi, list(o), P, ordered_sum=cpu_ordered_sum)[:P].clone().numpy()
                for o in orders]
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,P", [(2, 10, 37), (3, 11, 200), (8, 35, 1000), (8, 64, 65)])
def test_exact_mean_all_to_all_matches_reference_order(world, N, P):
    """parallel.global_mean_exact (one all_to_all of the sampled rows to
    column blocks, an ordered sum per block, one all_gather) is bit-identical
    to average_weights' sequential order (DEC/servers.py:42-48) for random
    full permutations, partial samples, one agent, every sample on one rank,
    and ranks that own no columns (P = 65 over 8 ranks) or no sampled rows."""
    rng = np.random.default_rng(31)
    orders = [rng.permutation(N), rng.choice(N, N // 3, replace=False), np.array([N - 1]),
              np.arange(N)[::-1], np.array([0, 1, 2]), np.array([N - 1, 0, N // 2, 3, 1])]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exact_mean_worker, args=(r, world, port, N, P, orders, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X = np.random.default_rng(29).standard_normal((N, P)).astype(np.float32)
    X[3, 5] = -0.0
    X[N - 1, :3] = [np.inf, -1e-42, 3e38]
    for k, o in enumerate(orders):
        want = oracle.ordered_mean(X, o)
        for r in range(world):
            assert oracle.bits_equal(res[r][k], want), f"order {k}, rank {r}"


def test_exact_mean_plan_bookkeeping():
    """perm maps the k-th sampled agent to its row in the received block
    (sources in rank order, each source's rows in global order)."""
    bounds = [(0, 3), (3, 7), (7, 8)]
    order = [5, 0, 7, 3, 2]
    mine, counts, perm, cols = parallel.exact_mean_plan(order, bounds, 130, 3, 1)
    assert mine.tolist() == [2, 0] and counts.tolist() == [2, 2, 1]
    # received block: rank 0's [0, 2], rank 1's [5, 3], rank 2's [7]
    assert perm.tolist() == [2, 0, 4, 3, 1]
    assert cols == [(0, 64), (64, 128), (128, 130)]
    with pytest.raises(ValueError):
        parallel.exact_mean_plan([8], bounds, 130, 3, 0)


def cpu_apply_csr(csr):
    def apply(X, Y, P=None):
        Y[:, :P] = torch.from_numpy(oracle.mix_csr(X[:, :P].numpy(), csr.rowptr, csr.col, csr.val))
        return Y
    return apply


def cpu_apply_dgd(csr):
    def apply_dgd(X, Y, target, mom=None, objective="least_squares", steps=1, lr=0.01, momentum=0.0,
                  first_step=False, P=None):
        mixed = oracle.mix_csr(X[:, :P].numpy(), csr.rowptr, csr.col, csr.val)
        y, m = oracle.dgd_local(mixed, target[:, :P].numpy(), None if mom is None else mom[:, :P].numpy(),
                                objective, steps, lr, momentum, first_step)
        Y[:, :P] = torch.from_numpy(y)
        if mom is not None and m is not None:
            mom[:, :P] = torch.from_numpy(m)
        return Y
    return apply_dgd


def _column_worker(rank, world, port, N, P, rounds, q):
    from dolhip import graph as G
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    try:
        csr = G.random_regular_csr(N, 4, seed=5)
        plan = type("Plan", (), {"n_rows": N})()  # host stand-in: the arithmetic is injected
        rng = np.random.default_rng(8)
        X = rng.standard_normal((N, P)).astype(np.float32)
        T = rng.standard_normal((N, P)).astype(np.float32)
        sh = parallel.ColumnSharded(plan, P, "cpu", apply=cpu_apply_csr(csr), apply_dgd=cpu_apply_dgd(csr))
        sh.x[:, :sh.Pl] = torch.from_numpy(X[:, sh.c0:sh.c1])
        t_loc = torch.from_numpy(np.ascontiguousarray(T[:, sh.c0:sh.c1]))
        m_loc = torch.zeros(N, sh.Pl)
        for k in range(rounds):
            sh.step()
            sh.dgd_step(t_loc, mom=m_loc, steps=2, lr=0.1, momentum=0.5, first_step=(k == 0))
        full = sh.gather(0)
        q.put((rank, None if full is None else full.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P", [(2, 300), (3, 130), (4, 100)])
def test_column_sharded_mix_and_dgd_match_single_process(world, P):
    """Parameter-dimension sharding: no data-path communication,
    gathered result bit-identical to one process (incl. ranks with no columns)."""
    from dolhip import graph as G
    N, rounds = 24, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_column_worker, args=(r, world, port, N, P, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    csr = G.random_regular_csr(N, 4, seed=5)
    rng = np.random.default_rng(8)
    X = rng.standard_normal((N, P)).astype(np.float32)
    T = rng.standard_normal((N, P)).astype(np.float32)
    M = np.zeros((N, P), np.float32)
    for k in range(rounds):
        X = oracle.mix_csr(X, csr.rowptr, csr.col, csr.val)
        X, M = oracle.dgd_local(oracle.mix_csr(X, csr.rowptr, csr.col, csr.val), T, M, "least_squares", 2, 0.1,
                                0.5, k == 0)
    assert oracle.bits_equal(res[0], X)


def cpu_dgd_ring(X, Y, w_prev, w_next, target, mom=None, halo_prev=None, halo_next=None, P=None, n_rows=None,
                 objective="least_squares", steps=1, lr=0.01, momentum=0.0, first_step=False):
    n = X.shape[0] if n_rows is None else n_rows
    hp = None if halo_prev is None else halo_prev[:P].numpy()
    hn = None if halo_next is None else halo_next[:P].numpy()
    mixed = oracle.mix_ring(X[:n, :P].numpy(), w_prev[:n].numpy(), w_next[:n].numpy(), hp, hn)
    y, m = oracle.dgd_local(mixed, target[:n, :P].numpy(), None if mom is None else mom[:n, :P].numpy(),
                            objective, steps, lr, momentum, first_step)
    Y[:n, :P] = torch.from_numpy(y)
    if mom is not None and m is not None:
        mom[:n, :P] = torch.from_numpy(m)
    return Y


def _dgd_ring_worker(rank, world, port, N, P, rounds, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    try:
        rng = np.random.default_rng(12)
        X = rng.standard_normal((N, P)).astype(np.float32)
        T = rng.standard_normal((N, P)).astype(np.float32)
        wp = rng.random(N).astype(np.float32)
        wn = rng.random(N).astype(np.float32)
        ring = parallel.ShardedRing(N, P, wp, wn, "cpu", ld=P + 5, mix_ring=cpu_mix_ring, dgd_ring=cpu_dgd_ring)
        ring.x[:, :P] = torch.from_numpy(X[ring.lo:ring.hi])
        t_loc = torch.from_numpy(np.ascontiguousarray(T[ring.lo:ring.hi]))
        m_loc = torch.zeros(ring.n_local, P)
        for k in range(rounds):
            ring.dgd_step(t_loc, mom=m_loc, steps=2, lr=0.1, momentum=0.5, first_step=(k == 0))
        q.put((rank, ring.x[:, :P].numpy().copy(), m_loc.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 10), (3, 11), (8, 40)])
def test_sharded_dgd_ring_matches_single_process(world, N):
    """Agent-sharded config-3 rounds over the halo exchange (up to 8 ranks, the
    node size) are bit-identical to one process."""
    P, rounds = 29, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dgd_ring_worker, args=(r, world, port, N, P, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(12)
    X = rng.standard_normal((N, P)).astype(np.float32)
    T = rng.standard_normal((N, P)).astype(np.float32)
    wp = rng.random(N).astype(np.float32)
    wn = rng.random(N).astype(np.float32)
    M = np.zeros((N, P), np.float32)
    for k in range(rounds):
        X, M = oracle.dgd_local(oracle.mix_ring(X, wp, wn), T, M, "least_squares", 2, 0.1, 0.5, k == 0)
    assert oracle.bits_equal(np.concatenate([r[1] for r in res]), X)
    assert oracle.bits_equal(np.concatenate([r[2] for r in res]), M)


def test_column_sharded_set_plan_swaps_the_mix():
    """Time-varying W (config 5): set_plan installs the new plan's kernels and
    refuses a W of another shape; one process, CPU stand-in plans."""
    from types import SimpleNamespace
    calls = []

    def plan_of(tag, n=6, m=6):
        return SimpleNamespace(n_rows=n, n_cols=m, apply=lambda x, y, P=None: calls.append(tag),
                               apply_dgd=lambda *a, **k: calls.append(tag + "-dgd"))
    sh = parallel.ColumnSharded(plan_of("a"), 10, "cpu")
    sh.step()
    sh.set_plan(plan_of("b"))
    sh.step()
    sh.dgd_step(torch.zeros(6, sh.ld))
    assert calls == ["a", "b", "b-dgd"]
    with pytest.raises(ValueError):
        sh.set_plan(plan_of("c", n=7, m=7))


def test_column_sharded_set_plan_keeps_injected_entries():
    """Entries injected at construction (the CPU-checker hook) survive set_plan
    (ADVICE r02): only un-injected entries follow the new plan."""
    from types import SimpleNamespace
    calls = []

    def plan_of(tag):
        return SimpleNamespace(n_rows=6, n_cols=6, apply=lambda x, y, P=None: calls.append(tag),
                               apply_dgd=lambda *a, **k: calls.append(tag + "-dgd"))
    sh = parallel.ColumnSharded(plan_of("a"), 10, "cpu", apply=lambda x, y, P=None: calls.append("checker"))
    sh.step()
    sh.set_plan(plan_of("b"))
    sh.step()
    sh.dgd_step(torch.zeros(6, sh.ld))
    sh.set_plan(plan_of("c"), apply_dgd=lambda *a, **k: calls.append("dgd-checker"))
    sh.dgd_step(torch.zeros(6, sh.ld))
    sh.step()
    assert calls == ["checker", "checker", "b-dgd", "dgd-checker", "checker"]


def _transpose_worker(rank, world, port, N, P, rounds, q, chunks=0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    try:
        rng = np.random.default_rng(21)
        X = rng.standard_normal((N, P)).astype(np.float32)
        tr = parallel.AgentColumnTranspose(N, P, "cpu")
        rows = torch.from_numpy(np.ascontiguousarray(X[tr.lo:tr.hi]))
        for k in range(rounds):  # a new W every round (config 5), the same on every rank
            csr = _er_csr(N, 0.3, seed=100 + k)
            tr._apply = cpu_apply_csr(csr)
            if chunks:  # the local step in pieces, each piece's exchange posted behind it
                tr.mix_with_local_steps(rows, lambda a, b: rows[a:b].mul_(0.5).add_(0.25), chunks=chunks)
            else:
                rows.mul_(0.5).add_(0.25)  # a stand-in local step on the agent-major block
                tr.mix(rows)
        q.put((rank, tr.lo, rows.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _er_csr(n, p, seed):
    from dolhip import graph as G
    r = np.random.default_rng(seed)
    A = (r.random((n, n)) < p).astype(np.float32)
    np.fill_diagonal(A, 0)
    R = r.random((n, n)).astype(np.float32) * A
    with np.errstate(invalid="ignore", divide="ignore"):
        W = (R / R.sum(0, dtype=np.float32)).T.astype(np.float32)
    return G.csr_from_dense(W)


@pytest.mark.parametrize("chunks", [0, 2, 3])
@pytest.mark.parametrize("world,N,P", [(2, 30, 300), (3, 25, 130), (4, 9, 70)])
def test_agent_column_transpose_mix_matches_single_process(world, N, P, chunks):
    """Config 5 across ranks (parallel.AgentColumnTranspose): agent-major blocks
    for the local step, one all_to_all to parameter-column blocks, the mix with a
    new W per round on every block, one all_to_all back -- bit-identical to one
    process (uneven agent and column blocks, a rank with no columns at P = 70).
    chunks > 0: mix_with_local_steps, the step in pieces whose first exchange
    is posted piece by piece (empty pieces at N = 9 over 4 ranks)."""
    rounds = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transpose_worker, args=(r, world, port, N, P, rounds, q, chunks))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X = np.random.default_rng(21).standard_normal((N, P)).astype(np.float32)
    for k in range(rounds):
        c = _er_csr(N, 0.3, seed=100 + k)
        X = ((X * np.float32(0.5)).astype(np.float32) + np.float32(0.25)).astype(np.float32)
        X = oracle.mix_csr(X, c.rowptr, c.col, c.val)
    assert oracle.bits_equal(np.concatenate([r[2] for r in res]), X)


def _stall_worker(rank, world, port, what, timeout_s, q):
    """Rank 0 runs one step of `what`; rank 1 joins the group and then stops
    participating (alive, silent) for longer than the timeout."""
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=timeout_s)
    if rank == 1:
        time.sleep(3 * timeout_s + 2)
        q.put((rank, "stalled", 0.0))
        q.close()
        q.join_thread()  # flush the queue, then leave without a teardown handshake
        os._exit(0)
    saved = parallel.DEFAULT_TIMEOUT_S
    parallel.DEFAULT_TIMEOUT_S = timeout_s
    t0 = time.perf_counter()
    try:
        N, P = 6, 8
        if what == "ring":
            ring = parallel.ShardedRing(N, P, np.ones(N, np.float32), np.ones(N, np.float32), "cpu",
                                        mix_ring=cpu_mix_ring, mix_edges=cpu_mix_ring_edges)
            ring.x.zero_()
            ring.step()
        elif what == "mean_exact":
            x = torch.zeros(3, P)
            parallel.global_mean_exact(x, 0, 3, [4, 0], P, ordered_sum=cpu_ordered_sum)
        elif what == "mean_fast":
            x = torch.zeros(3, P)
            parallel.global_mean(x, [0], 2, P, ordered_sum=cpu_ordered_sum)
        elif what == "all_to_all":
            tr = parallel.AgentColumnTranspose(N, P, "cpu", apply=lambda X, Y, P=None: Y)
            tr.mix(torch.zeros(tr.n_local, P))
        q.put((rank, "returned", time.perf_counter() - t0))
    except Exception as e:  # noqa: BLE001 - the point: it raises
        q.put((rank, type(e).__name__, time.perf_counter() - t0))
    finally:
        parallel.DEFAULT_TIMEOUT_S = saved
        q.close()
        q.join_thread()
        os._exit(0)


@pytest.mark.parametrize("what", ["ring", "mean_exact", "mean_fast", "all_to_all"])
def test_stalled_rank_raises_within_timeout(what):
    """SURVEY §5 fail-fast: when a peer stops participating, the halo exchange,
    the exact chain mean, the all_reduce mean and config 5's all_to_all raise
    on the waiting rank within the process group's timeout
    (parallel.init_process_group) instead of hanging."""
    timeout_s = 2.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stall_worker, args=(r, 2, port, what, timeout_s, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict((r, (s, t)) for r, s, t in (q.get(timeout=60) for _ in range(2)))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    status, elapsed = res[0]
    assert status != "returned", f"{what}: rank 0 returned although its peer never took part"
    assert elapsed < 3 * timeout_s, f"{what}: raised only after {elapsed:.1f} s (timeout {timeout_s} s)"


# ---------------------------------------------------------------------------
# every line RCCL would run, executed on the CPU tier
# ---------------------------------------------------------------------------

def cpu_dgd_ring_edges(X, Y, w_prev, w_next, target, halo_prev, halo_next, mom=None, P=None, n_rows=None, **kw):
    """CPU stand-in for dol_dgd_ring_edges_f32: rows 0 and n-1 of the block."""
    n = X.shape[0] if n_rows is None else n_rows
    m0 = None if mom is None else mom[0:1]
    cpu_dgd_ring(X[0:1], Y[0:1], w_prev[0:1], w_next[0:1], target[0:1], mom=m0, halo_prev=halo_prev,
                 halo_next=X[1] if n > 1 else halo_next, P=P, n_rows=1, **kw)
    if n > 1:
        m1 = None if mom is None else mom[n - 1:n]
        cpu_dgd_ring(X[n - 1:n], Y[n - 1:n], w_prev[n - 1:n], w_next[n - 1:n], target[n - 1:n], mom=m1,
                     halo_prev=X[n - 2], halo_next=halo_next, P=P, n_rows=1, **kw)
    return Y


class _FakeEvent:
    def record(self, *a):
        pass


def _line_tracer(path, hits):
    import sys

    def local(frame, event, arg):
        if event == "line":
            hits.add(frame.f_lineno)
        return local

    def glob(frame, event, arg):
        if frame.f_code.co_filename == path:
            return local
        return None
    sys.settrace(glob)


def _exercise_parallel(world, rank):
    """Every entry of dolhip.parallel on CPU tensors: ring (mix + DGD, with and
    without the one-launch edge entries), column sharding (+ set_plan, gather),
    the agent/column transpose (direct and staged-copy blocks, the piecewise
    overlapped form), the fast and exact means (a rank with and without
    sampled rows, host and tensor orders)."""
    from types import SimpleNamespace
    N, P = 11, 130
    rng = np.random.default_rng(3)
    X = rng.standard_normal((N, P)).astype(np.float32)
    wp, wn = rng.random(N).astype(np.float32), rng.random(N).astype(np.float32)
    for edges in (True, False):
        ring = parallel.ShardedRing(N, P, wp, wn, "cpu", ld=P + 2, mix_ring=cpu_mix_ring, dgd_ring=cpu_dgd_ring,
                                    mix_edges=cpu_mix_ring_edges if edges else None,
                                    dgd_edges=cpu_dgd_ring_edges if edges else None,
                                    stage_sends=True if edges else None)  # True: the GPU default at world > 1
        ring.x[:, :P] = torch.from_numpy(X[ring.lo:ring.hi])
        ring.kernel_events = (_FakeEvent(), _FakeEvent())
        ring.step()
        ring.step(ring.x, ring.y)
        t = torch.from_numpy(X[ring.lo:ring.hi].copy())
        ring.dgd_step(t, mom=torch.zeros_like(t), steps=1, lr=0.1, momentum=0.5, first_step=True)
        ring.dgd_step(t, steps=1, lr=0.1)
    csr = _er_csr(N, 0.4, seed=1)
    plan = SimpleNamespace(n_rows=N, n_cols=N, apply=cpu_apply_csr(csr), apply_dgd=cpu_apply_dgd(csr))
    sh = parallel.ColumnSharded(plan, P, "cpu")
    sh.x[:, :sh.Pl] = torch.from_numpy(np.ascontiguousarray(X[:, sh.c0:sh.c1]))
    sh.step()
    sh.dgd_step(torch.from_numpy(np.ascontiguousarray(X[:, sh.c0:sh.c1])), steps=1, lr=0.1)
    sh.set_plan(plan)
    sh.set_plan(plan, apply=cpu_apply_csr(csr))
    sh.local_cols(torch.zeros(N, P))
    sh.gather(0)
    tr = parallel.AgentColumnTranspose(N, P, "cpu")
    tr.set_plan(plan)
    rows = torch.from_numpy(np.ascontiguousarray(X[tr.lo:tr.hi]))
    tr.mix(rows)
    tr.to_columns(rows)
    tr.cols_out.copy_(tr.cols)
    tr.from_columns(rows)
    tr.mix_with_local_steps(rows, lambda a, b: rows[a:b].mul_(0.5), chunks=2, out=rows.clone(),
                            before_mix=lambda: None)
    tr.mix_with_local_steps(rows, lambda a, b: None, chunks=1)
    parallel.AgentColumnTranspose(N, P, "cpu", apply=cpu_apply_csr(csr)).mix(rows)  # an injected block mix
    Xl = torch.zeros(max(tr.n_local, 1), P + 3)
    Xl[:tr.n_local, :P] = torch.from_numpy(X[tr.lo:tr.hi])
    for order in ([0, N - 1, 5, 2], [N - 1]):  # rank 0 has no sampled row in the second
        local = [g - tr.lo for g in order if tr.lo <= g < tr.hi]
        parallel.global_mean(Xl, local, len(order), P, ordered_sum=cpu_ordered_sum)
        parallel.global_mean(Xl, torch.tensor(local, dtype=torch.int32), len(order), P, ordered_sum=cpu_ordered_sum)
        parallel.global_mean_exact(Xl, tr.lo, tr.hi, order, P, ordered_sum=cpu_ordered_sum)


def _coverage_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    hits = set()
    try:
        # every backend-dependent branch answers as it would over RCCL; the
        # transport underneath stays gloo (CPU tensors: nothing is staged)
        real_backend = parallel._backend
        parallel._backend = lambda group=None: (real_backend(group), "nccl")[1]
        _line_tracer(parallel.__file__, hits)
        _exercise_parallel(world, rank)
    finally:
        import sys
        sys.settrace(None)
        q.put((rank, sorted(hits)))
        dist.destroy_process_group()


def _parallel_lines_rccl_runs():
    """Line numbers of the statements in dolhip/parallel.py's functions, minus
    the ones RCCL never runs: host staging for gloo (`# staged`), gloo's
    bounded host wait (`# gloo-only`), raises (error paths) and docstrings.
    `# device-only` lines (CUDA events / side streams) need a GPU and run in
    tests/test_parallel_gpu.py; they are returned separately."""
    import ast
    src = open(parallel.__file__).read()
    text = src.splitlines()
    want, device = set(), set()
    for fn in ast.walk(ast.parse(src)):
        if not isinstance(fn, (ast.FunctionDef, ast.AsyncFunctionDef)):
            continue
        body = fn.body
        if body and isinstance(body[0], ast.Expr) and isinstance(getattr(body[0], "value", None), ast.Constant):
            body = body[1:]
        for stmt in body:
            for node in ast.walk(stmt):
                if not isinstance(node, ast.stmt) or isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
                    continue
                line = text[node.lineno - 1]
                if isinstance(node, ast.Raise) or "# staged" in line or "# gloo-only" in line:
                    continue
                (device if "# device-only" in line else want).add(node.lineno)
    return want, device


def test_every_rccl_line_runs_under_gloo():
    """the branches only RCCL takes (unstaged device
    tensors through send/recv, all_to_all and all_reduce, the
    all_gather_into_tensor gather, stream-side waits) execute here: gloo
    ranks of CPU tensors with parallel._backend answering "nccl", every entry
    of dolhip.parallel called at world 2 and 3 (plus world 1 and the nccl
    set-up of init_process_group in this process), and every statement RCCL
    would run is hit."""
    import sys
    want, device = _parallel_lines_rccl_runs()
    hits = set()
    for world in (2, 3):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_coverage_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        for _ in range(world):
            hits.update(q.get(timeout=180)[1])
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    # world 1 (no process group) and init_process_group's RCCL set-up (recorded, not run)
    local = set()
    seen = {}
    real_init = dist.init_process_group
    saved_env = os.environ.get("TORCH_NCCL_ASYNC_ERROR_HANDLING")
    dist.init_process_group = lambda backend, **kw: seen.update(backend=backend, **kw)
    _line_tracer(parallel.__file__, local)
    try:
        parallel.init_process_group("nccl", rank=0, world_size=1, device="cpu", timeout_s=5)
        _exercise_parallel(1, 0)
    finally:
        sys.settrace(None)
        dist.init_process_group = real_init
        if saved_env is None:
            os.environ.pop("TORCH_NCCL_ASYNC_ERROR_HANDLING", None)
        else:
            os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] = saved_env
    assert seen["backend"] == "nccl" and str(seen["device_id"]) == "cpu" and seen["world_size"] == 1
    hits |= local
    missing = sorted(want - hits)
    text = open(parallel.__file__).read().splitlines()
    assert not missing, "lines RCCL runs that no CPU test executed:\n" + "\n".join(
        f"{n}: {text[n - 1].strip()}" for n in missing)
    assert device and not (device & hits)  # the device-only lines really are (no CUDA here)
