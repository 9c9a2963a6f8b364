"""FedADMM on least squares (BASELINE config 4's primal/dual side) on the GPU:
dol_admm_ls_round_f32 + the ordered mean through dolhip.synthetic.SeparableADMM.

* Replays the REFERENCE's own FedAdmm_Server.run on a least-squares model
  (tests/golden/admm_ls.npz, made by tests/golden/make_golden_admm.py) bit for
  bit: every round's theta, the final w / momentum / alpha rows.
* Matches the oracle bit for bit at ragged and unaligned sizes (vector and
  scalar paths), with the fp64 residual outputs within rtol 1e-12 (their
  reduction order differs from the oracle's sequential sum).
* Converges to the reference iteration's closed-form fixed point."""
import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from conftest import golden
from dolhip import ops
from dolhip.synthetic import SeparableADMM

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("case", ["mini_mom", "flat_nomom", "mini_full"])
def test_admm_ls_replays_reference_server(case, fused, gpu):
    """fused: the client round + mean in one pass (dol_admm_ls_round_mean_f32,
    the default at one process); else the two-kernel round."""
    g = golden("admm_ls")
    N, frac, rounds, steps, lr, mom, rho = g[f"{case}__params"]
    N, rounds, steps = int(N), int(rounds), int(steps)
    T = g[f"{case}__targets"]
    P = T.shape[1]
    s = SeparableADMM(N, P, rho=rho, lr=lr, momentum=mom, local_steps=steps, frac=frac, device=gpu, fused=fused)
    assert s.fused == fused
    s.target[:, :P] = torch.as_tensor(T, device=gpu)
    s.theta[:P] = torch.as_tensor(g[f"{case}__theta0"], device=gpu)
    sampled = np.zeros(N, bool)
    for r in range(rounds):
        order = g[f"{case}__orders"][r]
        s.round(order=order)
        sampled[order] = True
        assert bits_equal(s.theta[:P].cpu().numpy(), g[f"{case}__thetas"][r]), f"round {r}"
    assert bits_equal(s.w[:N, :P].cpu().numpy()[sampled], g[f"{case}__w"][sampled])
    assert bits_equal(s.alpha[:N, :P].cpu().numpy(), g[f"{case}__alpha"])
    if mom != 0:
        assert bits_equal(s.mom[:N, :P].cpu().numpy(), g[f"{case}__mom"])
    assert len(s.history) == rounds


@pytest.mark.parametrize("P,extra", [(4096, 0), (1031, 0), (1031, 1), (3, 0), (5000, 3)])
@pytest.mark.parametrize("mom,steps", [(0.5, 3), (0.0, 1), (0.9, 0)])
def test_admm_ls_round_vs_oracle(P, extra, mom, steps, gpu):
    rng = np.random.default_rng(P + steps)
    N, m = 9, 5
    ld = P + extra  # extra = 1 / 3: rows not 16-B aligned -> the scalar path

    def mat(a):
        t = torch.full((N, ld), float("nan"), device=gpu)
        t[:, :P] = torch.as_tensor(a, device=gpu)
        return t
    T = rng.standard_normal((N, P)).astype(np.float32)
    A = (0.1 * rng.standard_normal((N, P))).astype(np.float32)
    B = rng.standard_normal((N, P)).astype(np.float32)
    th = rng.standard_normal(P).astype(np.float32)
    T[1, :3] = [np.inf, -0.0, 1e-40]
    order = np.array([7, 2, 0, 8, 5], np.int32)
    first = np.array([1, 0, 1, 0, 0], np.int32)
    w, a, b, t = mat(np.zeros((N, P), np.float32)), mat(A), mat(B), mat(T)
    rw = torch.empty(m, dtype=torch.float64, device=gpu)
    ra = torch.empty(m, dtype=torch.float64, device=gpu)
    ops.admm_ls_round(w, a, t, torch.as_tensor(th, device=gpu), agents=torch.as_tensor(order, device=gpu),
                      first=torch.as_tensor(first, device=gpu), buf=b if mom else None, rho=0.1, lr=0.05,
                      momentum=mom, local_steps=steps, resid_sq=rw, alpha_sq=ra, P=P)
    torch.cuda.synchronize()
    w1, b1, a1, rw1, ra1 = oracle.admm_ls_round(np.zeros((N, P), np.float32), B if mom else None, A, T, th, order,
                                                first, 0.1, 0.05, mom, steps)
    assert bits_equal(w.cpu().numpy()[order][:, :P], w1[order])
    assert bits_equal(a.cpu().numpy()[:, :P], a1)
    if mom:
        assert bits_equal(b.cpu().numpy()[:, :P], b1)
    np.testing.assert_allclose(rw.cpu().numpy(), rw1, rtol=1e-12)
    fin = np.isfinite(ra1)
    np.testing.assert_allclose(ra.cpu().numpy()[fin], ra1[fin], rtol=1e-12)


def test_separable_admm_converges_to_reference_fixed_point(gpu):
    s = SeparableADMM(64, 10000, rho=0.1, lr=0.2, momentum=0.5, local_steps=2, frac=1.0, device=gpu, seed=4)
    for _ in range(80):
        s.round()
    assert s.distance_to_fixed_point() < 1e-5
    h = s.history
    assert h[-1]["primal_resid_sq"] < 1e-3 * h[0]["primal_resid_sq"]


def test_separable_admm_fast_mean_close_to_exact(gpu):
    """The all-reduce-shaped 'fast' mean (one process: the same ordered sum) is
    bit-identical to the exact one at world size 1."""
    a = SeparableADMM(20, 777, frac=0.5, device=gpu, seed=2, mean="exact")
    b = SeparableADMM(20, 777, frac=0.5, device=gpu, seed=2, mean="fast")
    for _ in range(4):
        a.round()
        b.round()
    assert bits_equal(a.theta.cpu().numpy(), b.theta.cpu().numpy())


def test_admm_ls_round_argument_errors(gpu):
    w = torch.zeros(4, 8, device=gpu)
    th = torch.zeros(8, device=gpu)
    with pytest.raises(ValueError, match="buf"):
        ops.admm_ls_round(w, w.clone(), w.clone(), th, momentum=0.5)
    with pytest.raises(ValueError, match="both"):
        ops.admm_ls_round(w, w.clone(), w.clone(), th, resid_sq=torch.zeros(4, dtype=torch.float64, device=gpu))
    with pytest.raises(ValueError, match="first"):
        ops.admm_ls_round(w, w.clone(), w.clone(), th, first=torch.zeros(2, dtype=torch.int32, device=gpu))


@pytest.mark.parametrize("P,extra", [(4096, 0), (1031, 0), (1031, 1), (3, 0), (5000, 3), (70001, 0)])
@pytest.mark.parametrize("mom,steps", [(0.5, 3), (0.0, 1), (0.9, 0)])
@pytest.mark.parametrize("m", [5, 1, 6, 9])
def test_admm_ls_round_mean_vs_oracle(P, extra, mom, steps, m, gpu):
    """dol_admm_ls_round_mean_f32 (client round + ordered mean in one pass):
    rows bit-identical to oracle.admm_ls_round, theta_out to oracle.ordered_mean
    of the new rows in the sampled order (DEC/servers.py:42-48), the raw sum
    (scale 1) to the ordered sum, and the residual totals to the per-agent
    oracle values summed (rtol 1e-12: another fp64 summation order).  extra =
    1 / 3: rows not 16-B aligned -> the scalar path; P % 4 != 0: the tail."""
    rng = np.random.default_rng(P + 7 * steps + m)
    N = 9
    ld = P + extra

    def mat(a):
        t = torch.full((N, ld), float("nan"), device=gpu)
        t[:, :P] = torch.as_tensor(a, device=gpu)
        return t
    T = rng.standard_normal((N, P)).astype(np.float32)
    A = (0.1 * rng.standard_normal((N, P))).astype(np.float32)
    B = rng.standard_normal((N, P)).astype(np.float32)
    th = rng.standard_normal(P).astype(np.float32)
    T[1, :3] = [np.inf, -0.0, 1e-40][:min(3, P)]
    # groups of three agents in flight: m = 6 / 9 end on a full group, 5 / 1 on a partial one
    order = np.array([7, 2, 0, 8, 5, 3, 6, 4, 1], np.int32)[:m]
    first = np.array([1, 0, 1, 0, 0, 1, 1, 0, 0], np.int32)[:m]
    for scale in (None, 1.0):
        w, a, b, t = mat(np.zeros((N, P), np.float32)), mat(A), mat(B), mat(T)
        tot = torch.full((2,), float("nan"), dtype=torch.float64, device=gpu)
        out = ops.admm_ls_round_mean(w, a, t, torch.as_tensor(th, device=gpu), agents=torch.as_tensor(order, device=gpu),
                                     first=torch.as_tensor(first, device=gpu), buf=b if mom else None, rho=0.1, lr=0.05,
                                     momentum=mom, local_steps=steps, scale=scale, resid_total=tot, P=P)
        torch.cuda.synchronize()
        w1, b1, a1, rw1, ra1 = oracle.admm_ls_round(np.zeros((N, P), np.float32), B if mom else None, A, T, th, order,
                                                    first, 0.1, 0.05, mom, steps)
        assert bits_equal(w.cpu().numpy()[order][:, :P], w1[order])
        assert bits_equal(a.cpu().numpy()[:, :P], a1)
        if mom:
            assert bits_equal(b.cpu().numpy()[:, :P], b1)
        want = oracle.ordered_mean(w1, order) if scale is None else oracle.ordered_sum(w1, order)
        assert bits_equal(out.cpu().numpy(), want)
        got = tot.cpu().numpy()
        np.testing.assert_allclose(got[0], rw1.sum(), rtol=1e-12)
        if np.isfinite(ra1).all():
            np.testing.assert_allclose(got[1], ra1.sum(), rtol=1e-12)


def test_admm_ls_round_mean_theta_in_place(gpu):
    """theta_out may be theta itself (each column is read before it is written)."""
    rng = np.random.default_rng(3)
    N, P = 6, 2051
    T = torch.as_tensor(rng.standard_normal((N, P)).astype(np.float32), device=gpu)
    th = torch.as_tensor(rng.standard_normal(P).astype(np.float32), device=gpu)
    order = torch.as_tensor([4, 1, 3], dtype=torch.int32, device=gpu)
    w1, a1, w2, a2 = (torch.zeros(N, P, device=gpu) for _ in range(4))
    ref = ops.admm_ls_round_mean(w1, a1, T, th, agents=order, local_steps=2, P=P)
    th2 = th.clone()
    ops.admm_ls_round_mean(w2, a2, T, th2, agents=order, local_steps=2, out=th2, P=P)
    torch.cuda.synchronize()
    assert bits_equal(th2.cpu().numpy(), ref.cpu().numpy())
    assert bits_equal(w2.cpu().numpy(), w1.cpu().numpy())


def test_separable_admm_fused_matches_two_kernel_round(gpu):
    """SeparableADMM with the one-pass round vs the two-kernel round over 5
    rounds of partial participation with momentum: theta, w, alpha, momentum
    bit-identical; the residual totals within fp64 summation-order rounding."""
    kw = dict(rho=0.1, lr=0.1, momentum=0.5, local_steps=3, frac=0.6, seed=9, device=gpu)
    a = SeparableADMM(37, 20003, fused=True, **kw)
    b = SeparableADMM(37, 20003, fused=False, **kw)
    for _ in range(5):
        a.round()
        b.round()
    torch.cuda.synchronize()
    for x, y in ((a.theta, b.theta), (a.w, b.w), (a.alpha, b.alpha), (a.mom, b.mom)):
        assert bits_equal(x.cpu().numpy(), y.cpu().numpy())
    for ha, hb in zip(a.history, b.history):
        np.testing.assert_allclose(ha["primal_resid_sq"], hb["primal_resid_sq"], rtol=1e-12)
        np.testing.assert_allclose(ha["dual_sq"], hb["dual_sq"], rtol=1e-12)


def test_admm_ls_round_mean_argument_errors(gpu):
    w = torch.zeros(4, 8, device=gpu)
    th = torch.zeros(8, device=gpu)
    with pytest.raises(ValueError, match="buf"):
        ops.admm_ls_round_mean(w, w.clone(), w.clone(), th, momentum=0.5)
    with pytest.raises(ValueError, match="resid_total"):
        ops.admm_ls_round_mean(w, w.clone(), w.clone(), th, resid_total=torch.zeros(1, dtype=torch.float64, device=gpu))
    with pytest.raises(ValueError, match="at least one"):
        ops.admm_ls_round_mean(w, w.clone(), w.clone(), th, agents=torch.zeros(0, dtype=torch.int32, device=gpu))
    # the kernel prefetches the next agents' rows before storing the
    # current ones, so repeated or out-of-range ids are refused on the host
    for bad in ([1, 2, 1], [0, 4], [-1, 0], [0, 1, 2, 3, 0]):
        with pytest.raises(ValueError, match="agents"):
            ops.admm_ls_round_mean(w, w.clone(), w.clone(), th,
                                   agents=torch.tensor(bad, dtype=torch.int32, device=gpu))


def test_admm_ls_round_mean_defaults_and_no_metrics(gpu):
    """agents=None means rows 0..n-1 in order (same bits as passing arange), and
    a round without residual outputs (metrics=False: the RESID-free kernel)
    leaves the same rows and theta as one with them."""
    rng = np.random.default_rng(11)
    N, P = 7, 4099
    T = torch.as_tensor(rng.standard_normal((N, P)).astype(np.float32), device=gpu)
    A0 = torch.as_tensor((0.1 * rng.standard_normal((N, P))).astype(np.float32), device=gpu)
    th = torch.as_tensor(rng.standard_normal(P).astype(np.float32), device=gpu)
    outs = []
    for agents, tot in ((None, None), (torch.arange(N, dtype=torch.int32, device=gpu),
                                       torch.zeros(2, dtype=torch.float64, device=gpu))):
        w, a, b = torch.zeros(N, P, device=gpu), A0.clone(), torch.zeros(N, P, device=gpu)
        o = ops.admm_ls_round_mean(w, a, T, th, agents=agents, buf=b, momentum=0.5, local_steps=3, resid_total=tot,
                                   P=P)
        torch.cuda.synchronize()
        outs.append([x.cpu().numpy() for x in (w, a, b, o)])
    for x, y in zip(*outs):
        assert bits_equal(x, y)
    kw = dict(rho=0.1, lr=0.1, momentum=0.5, local_steps=2, frac=0.5, seed=3, device=gpu)
    s1 = SeparableADMM(21, 3001, metrics=False, **kw)
    s2 = SeparableADMM(21, 3001, metrics=True, **kw)
    assert s1.fused and s2.fused
    for _ in range(3):
        s1.round()
        s2.round()
    torch.cuda.synchronize()
    assert bits_equal(s1.theta.cpu().numpy(), s2.theta.cpu().numpy())
    assert bits_equal(s1.alpha.cpu().numpy(), s2.alpha.cpu().numpy())
    assert s1.history == [] and len(s2.history) == 3
