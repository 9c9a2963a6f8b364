"""FedADMM on least squares (BASELINE config 4's primal/dual side), CPU tier.

* The oracle's fused client round (oracle/dol_oracle.c oracle_admm_ls_round_f32)
  plus its ordered mean replays the REFERENCE's own FedAdmm_Server.run on a
  least-squares model (tests/golden/make_golden_admm.py: the shipped
  update_weights / update_model / SGD.step / update_duals / average_weights)
  bit for bit: every round's theta, and the final w, momentum and alpha rows.
* dolhip.synthetic.SeparableADMM's round logic (sampling order, first-step
  flags, the ordered / all-reduce means) sharded over gloo ranks with the oracle
  injected as the arithmetic is bit-identical to one process ("exact" mean),
  and within fp32 association error of it ("fast" mean)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from dolhip import parallel
from conftest import golden
from oracle import bits_equal

CASES = ("mini_mom", "flat_nomom", "mini_full")


def replay_oracle(g, case):
    N, frac, rounds, steps, lr, mom, rho = g[f"{case}__params"]
    N, rounds, steps = int(N), int(rounds), int(steps)
    T = g[f"{case}__targets"]
    P = T.shape[1]
    w = np.zeros((N, P), np.float32)
    buf = np.zeros((N, P), np.float32) if mom != 0 else None
    alpha = np.zeros((N, P), np.float32)
    theta = g[f"{case}__theta0"].copy()
    started = np.zeros(N, bool)
    thetas = []
    for r in range(rounds):
        order = g[f"{case}__orders"][r]
        first = (~started[order]).astype(np.int32)
        w, buf, alpha, rw, ra = oracle.admm_ls_round(w, buf, alpha, T, theta, order, first, np.float32(rho),
                                                     np.float32(lr), np.float32(mom), steps)
        started[order] = True
        theta = oracle.ordered_mean(w, order)
        thetas.append(theta)
    return np.stack(thetas), w, buf, alpha, started


@pytest.mark.parametrize("case", CASES)
def test_oracle_admm_ls_replays_reference_server(case):
    g = golden("admm_ls")
    thetas, w, buf, alpha, started = replay_oracle(g, case)
    assert bits_equal(thetas, g[f"{case}__thetas"])
    # clients never sampled keep their initial (reference: the global init) weights; compare the sampled ones
    assert bits_equal(w[started], g[f"{case}__w"][started])
    assert bits_equal(alpha, g[f"{case}__alpha"])
    if buf is not None:
        assert bits_equal(buf, g[f"{case}__mom"])


def test_oracle_admm_ls_residual_outputs():
    rng = np.random.default_rng(4)
    N, P = 5, 301
    T = rng.standard_normal((N, P)).astype(np.float32)
    A = rng.standard_normal((N, P)).astype(np.float32)
    th = rng.standard_normal(P).astype(np.float32)
    order = np.array([3, 1], np.int32)
    w, _, a, rw, ra = oracle.admm_ls_round(np.zeros((N, P), np.float32), None, A, T, th, order, None,
                                           0.1, 0.1, 0.0, 2)
    for k, i in enumerate(order):
        d = (w[i] - th).astype(np.float64)  # fl(w - theta), squared and summed in fp64
        assert rw[k] == pytest.approx(float(d @ d), rel=1e-12)
        assert ra[k] == pytest.approx(float(a[i].astype(np.float64) @ a[i].astype(np.float64)), rel=1e-12)
    untouched = [i for i in range(N) if i not in order]
    assert bits_equal(a[untouched], A[untouched])


# ---------------------------------------------------------------------------
# SeparableADMM over gloo ranks with the oracle as the arithmetic
# ---------------------------------------------------------------------------

def cpu_admm_ls_round(w, alpha, target, theta, agents=None, first=None, buf=None, rho=0.1, lr=0.1, momentum=0.0,
                      local_steps=1, resid_sq=None, alpha_sq=None, work=None, P=None):
    P = w.shape[1] if P is None else P
    ag = agents.numpy() if agents is not None else np.arange(w.shape[0])
    fs = first.numpy() if first is not None else None
    wn, bn, an, rw, ra = oracle.admm_ls_round(w[:, :P].numpy(), None if buf is None else buf[:, :P].numpy(),
                                              alpha[:, :P].numpy(), target[:, :P].numpy(), theta[:P].numpy(), ag,
                                              fs, rho, lr, momentum, local_steps)
    w[:, :P] = torch.from_numpy(wn)
    alpha[:, :P] = torch.from_numpy(an)
    if buf is not None and bn is not None:
        buf[:, :P] = torch.from_numpy(bn)
    if resid_sq is not None:
        resid_sq[:] = torch.from_numpy(rw)
        alpha_sq[:] = torch.from_numpy(ra)


def cpu_ordered_sum(W, order, acc_in=None, out=None, scale=1.0, P=None):
    if W is None or order.numel() == 0:
        res = acc_in[:P].numpy().astype(np.float32)
        if scale != 1.0:
            res = (res / np.float32(scale)).astype(np.float32)
    else:
        res = oracle.ordered_sum(W[:, :P].numpy(), order.numpy(), None if acc_in is None else acc_in[:P].numpy(),
                                 scale)
    out[:P] = torch.from_numpy(res)
    return out


def _run(N, P, rounds, mean, **kw):
    from dolhip.synthetic import SeparableADMM
    s = SeparableADMM(N, P, device="cpu", mean=mean, round_fn=cpu_admm_ls_round, ordered_sum=cpu_ordered_sum,
                      **kw)
    for _ in range(rounds):
        s.round()
    return s


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, P, rounds, mean, kw, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    try:
        s = _run(N, P, rounds, mean, **kw)
        q.put((rank, s.lo, s.hi, s.w[:s.n, :P].numpy().copy(), s.alpha[:s.n, :P].numpy().copy(),
               s.theta[:P].numpy().copy(), [h["primal_resid_sq"] for h in s.history]))
    finally:
        dist.destroy_process_group()


KW = dict(rho=0.1, lr=0.1, momentum=0.5, local_steps=3, frac=0.6, seed=5)


@pytest.mark.parametrize("world,mean", [(2, "exact"), (3, "exact"), (2, "fast"), (8, "exact")])
def test_sharded_admm_matches_single_process(world, mean):
    N, P, rounds = 13, 45, 4
    ref = _run(N, P, rounds, "exact", **KW)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, P, rounds, mean, KW, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = np.concatenate([r[3] for r in res])
    a = np.concatenate([r[4] for r in res])
    hist = [h["primal_resid_sq"] for h in ref.history]
    for r in res:
        if mean == "exact":
            assert bits_equal(r[5], ref.theta[:P].numpy())
        else:
            np.testing.assert_allclose(r[5], ref.theta[:P].numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(r[6], hist, rtol=1e-9 if mean == "exact" else 1e-4)
    if mean == "exact":
        assert bits_equal(w, ref.w[:N, :P].numpy())
        assert bits_equal(a, ref.alpha[:N, :P].numpy())


def _column_worker(rank, world, port, N, P, rounds, kw, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    parallel.init_process_group("gloo", rank=rank, world_size=world, timeout_s=120)
    try:
        from dolhip.synthetic import SeparableADMM
        calls = []
        real_all_reduce, real_all_gather = dist.all_reduce, dist.all_gather_into_tensor

        def counting(fn, name):
            def wrapped(*a, **k):
                calls.append(name)
                return fn(*a, **k)
            return wrapped
        s = SeparableADMM(N, P, device="cpu", round_fn=cpu_admm_ls_round, ordered_sum=cpu_ordered_sum,
                          shard="columns", **kw)
        # the round path: no collective at all
        dist.all_reduce = counting(real_all_reduce, "all_reduce")
        dist.all_gather_into_tensor = counting(real_all_gather, "all_gather")
        try:
            for _ in range(rounds):
                s.round()
            n_round_calls = len(calls)
        finally:
            dist.all_reduce, dist.all_gather_into_tensor = real_all_reduce, real_all_gather
        theta = s.full_theta().numpy().copy()
        hist = [(h["primal_resid_sq"], h["dual_sq"]) for h in s.history]
        q.put((rank, s.c0, s.c1, s.w[:N, :s.Pl].numpy().copy(), s.alpha[:N, :s.Pl].numpy().copy(), theta, hist,
               n_round_calls, s.distance_to_fixed_point()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P", [(2, 300), (3, 300), (8, 600), (8, 65)])
def test_column_sharded_admm_matches_single_process(world, P):
    """SeparableADMM(shard="columns") -- every rank runs
    all sampled agents on its parameter columns, in the global sampled order
    -- is bit-identical to one process (rows, duals and theta; theta is
    DEC/servers.py:42-48's order exactly) with no collective on the round path;
    ranks without columns (P = 65 over 8) take part; the residual metrics
    (per-rank partials summed when `history` is read) agree to fp64 rounding."""
    N, rounds = 13, 4
    ref = _run(N, P, rounds, "exact", **KW)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_column_worker, args=(r, world, port, N, P, rounds, KW, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [parallel.column_bounds(P, world, k)[0] for k in range(world)]
    w = np.concatenate([r[3] for r in res], axis=1)
    a = np.concatenate([r[4] for r in res], axis=1)
    assert bits_equal(w, ref.w[:N, :P].numpy())
    assert bits_equal(a, ref.alpha[:N, :P].numpy())
    hist = [(h["primal_resid_sq"], h["dual_sq"]) for h in ref.history]
    for r in res:
        assert bits_equal(r[5], ref.theta[:P].numpy())
        np.testing.assert_allclose(np.array(r[6]), np.array(hist), rtol=1e-12)
        assert r[7] == 0, f"rank {r[0]}: {r[7]} collectives on the round path"
        assert r[8] == pytest.approx(ref.distance_to_fixed_point(), rel=1e-9)


def test_column_sharded_admm_one_process_is_the_agent_path():
    """shard="columns" at world 1 is the plain one-process problem (same bits)."""
    from dolhip.synthetic import SeparableADMM
    a = _run(11, 70, 3, "exact", **KW)
    b = SeparableADMM(11, 70, device="cpu", round_fn=cpu_admm_ls_round, ordered_sum=cpu_ordered_sum, shard="columns",
                      **KW)
    for _ in range(3):
        b.round()
    assert bits_equal(b.theta[:70].numpy(), a.theta[:70].numpy())
    assert bits_equal(b.w[:11, :70].numpy(), a.w[:11, :70].numpy())
    with pytest.raises(ValueError):
        SeparableADMM(4, 8, device="cpu", round_fn=cpu_admm_ls_round, ordered_sum=cpu_ordered_sum, shard="rows")


def test_separable_admm_converges_to_reference_fixed_point():
    """Full participation: theta -> (mean t + rho theta_0) / (1 + rho), the fixed
    point of the reference's iteration (its server averages w only), NOT mean t;
    the primal residual vanishes."""
    s = _run(9, 33, 80, "exact", rho=0.1, lr=0.2, momentum=0.5, local_steps=2, frac=1.0, seed=3)
    assert s.distance_to_fixed_point() < 1e-5
    assert s.distance_to_optimum() > 0.01  # the bias is real
    h = s.history
    assert h[-1]["primal_resid_sq"] < 1e-3 * h[0]["primal_resid_sq"]


def test_separable_admm_rejects_bad_orders():
    from dolhip.synthetic import SeparableADMM
    s = SeparableADMM(4, 8, device="cpu", round_fn=cpu_admm_ls_round, ordered_sum=cpu_ordered_sum)
    for bad in ([4], [-1], [1, 1], []):
        with pytest.raises(ValueError):
            s.round(order=bad)


def test_ref_cpu_admm_baseline_matches_oracle():
    """bench.py's CPU FedADMM leg (oracle/ref_cpu.py, reference-structured torch
    code) computes the same round as the oracle the kernels are pinned to, so
    the GPU/CPU ratio compares like with like."""
    import copy
    from oracle import ref_cpu
    n, P, steps, rho, lr, mu = 5, 37, 3, 0.1, 0.1, 0.5
    g = torch.Generator().manual_seed(4)
    T = [torch.randn(P, generator=g) for _ in range(n)]
    clients = [ref_cpu.AdmmClient(t, rho, lr, mu, steps) for t in T]
    theta = {"w": torch.randn(P, generator=g)}
    w0 = np.zeros((n, P), np.float32)
    b0 = np.zeros((n, P), np.float32)
    a0 = np.zeros((n, P), np.float32)
    Tn = np.stack([t.numpy() for t in T])
    th = theta["w"].numpy().copy()
    first = np.ones(n, np.int32)
    order = np.arange(n, dtype=np.int32)
    for _ in range(2):
        local = [copy.deepcopy(c.update_weights(theta)) for c in clients]
        theta = ref_cpu.average_weights(local)
        w0, b0, a0, _, _ = oracle.admm_ls_round(w0, b0, a0, Tn, th, order, first, rho, lr, mu, steps)
        th = oracle.ordered_mean(w0, order)
        first = np.zeros(n, np.int32)
        assert bits_equal(np.stack([c.model.w.detach().numpy() for c in clients]), w0)
        assert bits_equal(np.stack([c.alpha["w"].numpy() for c in clients]), a0)
        assert bits_equal(theta["w"].numpy(), th)
