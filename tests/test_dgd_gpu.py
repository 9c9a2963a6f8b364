"""Fused decentralised-gradient round (BASELINE config 3): X <- W X, then
`steps` local momentum-SGD iterations per agent on a separable synthetic loss,
in one kernel (dol_dgd_ring_f32 / dol_dgd_csr_f32) — checked against the CPU
oracle (oracle_mix_* then oracle_dgd_local_f32).

Least squares is bit-exact (every operation has one rounding on both sides).
Logistic calls expf, whose last bit may differ between the device libm and
glibc: a 1-ulp gradient difference moves x by ~1 ulp of |x| = O(1), so the
tolerance is rtol 2e-6 / atol 1e-6 (8 ulp at 1.0; observed 1.2e-7)."""
import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from dolhip import graph as G
from dolhip import ops
from dolhip.synthetic import SeparableDGD

pytestmark = pytest.mark.gpu

LOGISTIC_TOL = dict(rtol=2e-6, atol=1e-6)


def dev(a, gpu):
    return torch.as_tensor(np.ascontiguousarray(a)).to(gpu)


def _inputs(n, P, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, P)).astype(np.float32)
    T = rng.standard_normal((n, P)).astype(np.float32)
    M = rng.standard_normal((n, P)).astype(np.float32)
    return X, T, M


def _check(got, want, objective):
    if objective == "least_squares":
        assert bits_equal(got, want)
    else:
        np.testing.assert_allclose(got, want, **LOGISTIC_TOL)


@pytest.mark.parametrize("objective", ["least_squares", "logistic"])
@pytest.mark.parametrize("momentum,first", [(0.0, False), (0.5, True), (0.5, False)])
@pytest.mark.parametrize("steps", [1, 3])
@pytest.mark.parametrize("n,P", [(5, 1027), (64, 4096), (7, 3)])
def test_dgd_ring_vs_oracle(objective, momentum, first, steps, n, P, gpu):
    X, T, M = _inputs(n, P, n + P + steps)
    rng = np.random.default_rng(1)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    Xd, Td, Md = dev(X, gpu), dev(T, gpu), dev(M, gpu)
    Yd = torch.empty_like(Xd)
    ops.dgd_ring(Xd, Yd, dev(wp, gpu), dev(wn, gpu), Td, mom=Md if momentum else None, objective=objective,
                 steps=steps, lr=0.05, momentum=momentum, first_step=first)
    torch.cuda.synchronize()
    Y, Mw = oracle.dgd_local(oracle.mix_ring(X, wp, wn), T, M if momentum else None, objective, steps, 0.05,
                             momentum, first)
    _check(Yd.cpu().numpy(), Y, objective)
    if momentum:
        _check(Md.cpu().numpy(), Mw, objective)


@pytest.mark.parametrize("objective", ["least_squares", "logistic"])
@pytest.mark.parametrize("n,P,deg", [(16, 4099, 4), (600, 256, 4), (33, 4096, 6), (520, 4098, 4)])
def test_dgd_csr_vs_oracle(objective, n, P, deg, gpu):
    """Covers the XCD-pinned CSR kernel (n >= 512), the 4 KiB-tile one, the
    leftover f4 columns and the scalar tail, each with the epilogue."""
    csr = G.random_regular_csr(n, deg, seed=3)
    X, T, M = _inputs(n, P, n * P)
    Xd, Td, Md = dev(X, gpu), dev(T, gpu), dev(M, gpu)
    Yd = torch.empty_like(Xd)
    plan = G.MixingPlan(csr, gpu)
    plan.apply_dgd(Xd, Yd, Td, mom=Md, objective=objective, steps=2, lr=0.1, momentum=0.5, first_step=False)
    torch.cuda.synchronize()
    Y, Mw = oracle.dgd_local(oracle.mix_csr(X, csr.rowptr, csr.col, csr.val), T, M, objective, 2, 0.1, 0.5, False)
    _check(Yd.cpu().numpy(), Y, objective)
    _check(Md.cpu().numpy(), Mw, objective)


def test_dgd_ring_halos_match_wraparound(gpu):
    """The sharded form (interior rows with halo pointers + the two boundary rows)
    equals the one-shot wrap-around launch bit for bit."""
    n, P = 9, 2051
    X, T, M = _inputs(n, P, 5)
    rng = np.random.default_rng(2)
    wp, wn = dev(rng.random(n).astype(np.float32), gpu), dev(rng.random(n).astype(np.float32), gpu)
    Xd, Td = dev(X, gpu), dev(T, gpu)
    M1, M2 = dev(M, gpu), dev(M, gpu)
    Y1, Y2 = torch.empty_like(Xd), torch.empty_like(Xd)
    kw = dict(objective="least_squares", steps=2, lr=0.1, momentum=0.9, first_step=False)
    ops.dgd_ring(Xd, Y1, wp, wn, Td, mom=M1, **kw)
    ops.dgd_ring(Xd[1:], Y2[1:], wp[1:], wn[1:], Td[1:], mom=M2[1:], halo_prev=Xd[0], halo_next=Xd[n - 1],
                 n_rows=n - 2, **kw)
    ops.dgd_ring(Xd[0:1], Y2[0:1], wp[0:1], wn[0:1], Td[0:1], mom=M2[0:1], halo_prev=Xd[n - 1], halo_next=Xd[1],
                 n_rows=1, **kw)
    ops.dgd_ring(Xd[n - 1:], Y2[n - 1:], wp[n - 1:], wn[n - 1:], Td[n - 1:], mom=M2[n - 1:], halo_prev=Xd[n - 2],
                 halo_next=Xd[0], n_rows=1, **kw)
    torch.cuda.synchronize()
    assert bits_equal(Y1.cpu().numpy(), Y2.cpu().numpy())
    assert bits_equal(M1.cpu().numpy(), M2.cpu().numpy())


def test_separable_dgd_least_squares_reaches_mean_of_targets(gpu):
    """Known answer: for f_i = 1/2 ||x - t_i||^2 one round is
    x <- (1 - lr) W x + lr t, so (real arithmetic) the iterates contract at
    rate (1 - lr) to x* = lr (I - (1 - lr) W)^-1 t, and with a doubly
    stochastic W the agents' mean moves as mean <- (1 - lr) mean + lr mean(t)
    and mean(x*) = mean(t) (the centralised optimum).  Tolerances cover fp32
    rounding of the rounds (contractive, so it does not accumulate) and of the
    N-term means: rtol 1e-4 / atol 1e-5; 600 rounds leave (0.98)^600 = 5e-6."""
    n, P, lr = 64, 1 << 14, 0.02
    torch.manual_seed(2028)
    W = G.communication_graph("circle", "double_stochastic", n)[0]
    prob = SeparableDGD(G.MixingPlan.from_graph(W, gpu), P, objective="least_squares", lr=lr, momentum=0.0,
                        local_steps=1, seed=4)
    t = prob.targets().double().cpu()
    x_mean0 = prob.params().mean(0)
    prob.round()
    torch.cuda.synchronize()
    want = (1 - lr) * x_mean0 + lr * prob.targets().mean(0)
    torch.testing.assert_close(prob.params().mean(0), want, rtol=1e-4, atol=1e-5)
    for _ in range(600):
        prob.round()
    Wd = torch.as_tensor(np.asarray(W, np.float64))
    x_star = lr * torch.linalg.solve(torch.eye(n, dtype=torch.float64) - (1 - lr) * Wd, t)
    got = prob.params().double().cpu()
    torch.testing.assert_close(got, x_star, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(got.mean(0), t.mean(0), rtol=1e-4, atol=1e-4)


def test_separable_dgd_full_size_rows_vs_oracle(gpu):
    """1024 agents x 2^20 params (config 3's size), ring: sampled rows of one fused
    round against the oracle on their three-row neighbourhoods (bit-exact)."""
    n, P = 1024, 1 << 20
    torch.manual_seed(2028)
    plan = G.MixingPlan(G.communication_csr("circle", "stochastic", n)[0], gpu)
    prob = SeparableDGD(plan, P, objective="least_squares", lr=0.05, momentum=0.5, local_steps=2, seed=9)
    x0 = prob.params().clone()
    m0 = prob.momentum_rows().clone()
    prob.round()
    torch.cuda.synchronize()
    wp, wn = plan.w_prev.cpu().numpy(), plan.w_next.cpu().numpy()
    for i in (0, 1, 511, 1022, 1023):
        xs = x0[[(i - 1) % n, (i + 1) % n]].cpu().numpy()
        mixed = oracle.mix_ring(np.stack([xs[0], np.zeros(P, np.float32), xs[1]]),
                                np.array([0, wp[i], 0], np.float32), np.array([0, wn[i], 0], np.float32))[1]
        Y, Mw = oracle.dgd_local(mixed[None, :], prob.targets()[i:i + 1].cpu().numpy(), m0[i:i + 1].cpu().numpy(),
                                 "least_squares", 2, 0.05, 0.5, True)
        assert bits_equal(prob.params()[i].cpu().numpy(), Y[0])
        assert bits_equal(prob.momentum_rows()[i].cpu().numpy(), Mw[0])
    del prob, x0, m0
    torch.cuda.empty_cache()
