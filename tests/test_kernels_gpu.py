"""HIP kernels (through the C-ABI) vs the oracle and the reference's golden
vectors.  Mixing, dual update, ordered mean and the fused local step are
bit-exact (fp32, same rounding sequence as the reference's torch CPU path);
the only tolerance is on the fp64 residual norm (a diagnostic whose
reduction order differs): rtol 1e-12."""
import os

import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from conftest import golden
from dolhip import graph as G
from dolhip import ops

pytestmark = pytest.mark.gpu


def dev(a, gpu, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(device=gpu, dtype=dtype)


def padded(a, gpu, extra):
    """Device copy with leading dimension P + extra (extra=1 forces the scalar path)."""
    n, P = a.shape
    t = torch.full((n, P + extra), float("nan"), dtype=torch.float32, device=gpu)
    t[:, :P] = dev(a, gpu)
    return t


def _mix_cases():
    return sorted(k[:-3] for k in golden("mix").files if k.endswith("__X"))


def _ring_weights(case):
    csr = golden("csr")
    gkey, _l, t = case.split("__")
    c = f"{gkey}__{t}"
    n = len(csr[c + "__rowptr"]) - 1
    return G.CSR(n, n, csr[c + "__rowptr"], csr[c + "__col"], csr[c + "__val"]).ring_weights()


def _ring_cases():
    """The golden cases whose W is a ring (the ring kernel's domain)."""
    return [c for c in _mix_cases() if _ring_weights(c) is not None]


@pytest.mark.parametrize("extra", [0, 1, 60])
@pytest.mark.parametrize("case", _mix_cases())
def test_mix_csr_golden(case, extra, gpu):
    mix, csr = golden("mix"), golden("csr")
    gkey, _l, t = case.split("__")
    c = f"{gkey}__{t}"
    X = mix[case + "__X"]
    n, P = X.shape
    Xd = padded(X, gpu, extra)
    Yd = padded(np.zeros_like(X), gpu, extra)
    ops.mix_csr(Xd, Yd, dev(csr[c + "__rowptr"], gpu, torch.int32), dev(csr[c + "__col"], gpu, torch.int32),
                dev(csr[c + "__val"], gpu), P=P)
    torch.cuda.synchronize()
    assert bits_equal(Yd[:, :P].cpu().numpy(), mix[case + "__Y"])


@pytest.mark.parametrize("extra", [0, 1])
@pytest.mark.parametrize("case", _ring_cases())
def test_mix_ring_golden(case, extra, gpu):
    mix = golden("mix")
    rw = _ring_weights(case)
    X = mix[case + "__X"]
    P = X.shape[1]
    Xd, Yd = padded(X, gpu, extra), padded(np.zeros_like(X), gpu, extra)
    ops.mix_ring(Xd, Yd, dev(rw[0], gpu), dev(rw[1], gpu), P=P)
    torch.cuda.synchronize()
    assert bits_equal(Yd[:, :P].cpu().numpy(), mix[case + "__Y"])


@pytest.mark.parametrize("n,P", [(3, 5), (4, 1027), (5, 4096), (64, (1 << 16) + 3), (257, 12289), (1000, 1024)])
def test_mix_ring_random_vs_oracle(n, P, gpu):
    rng = np.random.default_rng(n * 7 + P)
    X = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    Xd, Yd = dev(X, gpu), torch.empty(n, P, device=gpu)
    ops.mix_ring(Xd, Yd, dev(wp, gpu), dev(wn, gpu))
    torch.cuda.synchronize()
    assert bits_equal(Yd.cpu().numpy(), oracle.mix_ring(X, wp, wn))


def test_mix_ring_halos_and_subblocks(gpu):
    """The halo form used by the sharded ring equals the wrap form."""
    rng = np.random.default_rng(3)
    n, P = 37, 5003
    X = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    want = oracle.mix_ring(X, wp, wn)
    Xd, Yd = dev(X, gpu), torch.zeros(n, P, device=gpu)
    wpd, wnd = dev(wp, gpu), dev(wn, gpu)
    ops.mix_ring(Xd[1:], Yd[1:], wpd[1:], wnd[1:], halo_prev=Xd[0], halo_next=Xd[n - 1], n_rows=n - 2)
    ops.mix_ring(Xd[0:1], Yd[0:1], wpd[0:1], wnd[0:1], halo_prev=Xd[n - 1].clone(), halo_next=Xd[1], n_rows=1)
    ops.mix_ring(Xd[n - 1:], Yd[n - 1:], wpd[n - 1:], wnd[n - 1:], halo_prev=Xd[n - 2], halo_next=Xd[0].clone(),
                 n_rows=1)
    torch.cuda.synchronize()
    assert bits_equal(Yd.cpu().numpy(), want)


def test_mix_signed_zero_and_nonfinite(gpu):
    n, P = 8, 4100
    X = np.full((n, P), -0.0, np.float32)
    X[3, 10] = np.inf
    X[5, 11] = np.nan
    wp = np.full(n, 0.25, np.float32)
    wn = np.full(n, 0.75, np.float32)
    Yd = torch.empty(n, P, device=gpu)
    ops.mix_ring(dev(X, gpu), Yd, dev(wp, gpu), dev(wn, gpu))
    Y = Yd.cpu().numpy()
    want = oracle.mix_ring(X, wp, wn)
    assert bits_equal(Y, want)
    assert Y[0, 0].view(np.uint32) == 0  # (+0 + -0) + -0 == +0, as torch.zeros_like + ...


@pytest.mark.parametrize("n,deg,P", [(64, 4, 4099), (300, 4, 1024), (50, 12, 777)])
def test_mix_csr_random_regular_vs_oracle(n, deg, P, gpu):
    c = G.random_regular_csr(n, deg, seed=n)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((n, P)).astype(np.float32)
    plan = G.MixingPlan(c, gpu)
    assert plan.kind == "csr"
    Yd = torch.empty(n, P, device=gpu)
    plan.apply(dev(X, gpu), Yd)
    torch.cuda.synchronize()
    assert bits_equal(Yd.cpu().numpy(), oracle.mix_csr(X, c.rowptr, c.col, c.val))


def test_multi_round_mix_plan_and_bank(gpu):
    from dolhip.bank import AgentBank
    torch.manual_seed(2028)
    W = G.communication_graph("circle", "stochastic", 16)[0]
    plan = G.MixingPlan.from_graph(W, gpu)
    assert plan.kind == "ring"
    rng = np.random.default_rng(4)
    X = rng.standard_normal((16, 999)).astype(np.float32)
    bank = AgentBank(16, 999, gpu)
    bank.rows()[:] = dev(X, gpu)
    bank.mix(plan, steps=5)
    c = plan.csr
    want = X
    for _ in range(5):
        want = oracle.mix_csr(want, c.rowptr, c.col, c.val)
    assert bits_equal(bank.rows().cpu().numpy(), want)


def _local_keys():
    L = golden("local_steps")
    return sorted({k.rsplit("__", 1)[0] for k in L.files})


@pytest.mark.parametrize("key", _local_keys())
def test_fused_local_step_golden(key, gpu):
    L = golden("local_steps")
    rho, lr, mom = (float(v) for v in L[key + "__params"])
    cls = key.split("__")[0]
    th = None if cls == "FedAvg_Client" else dev(L[key + "__theta"], gpu)
    al = dev(L[key + "__alpha"][None], gpu) if cls == "FedAdmm_Client" else None
    for t in range(L[key + "__w"].shape[0]):
        w = dev(L[key + "__w"][t][None], gpu)
        b = dev(L[key + "__buf"][t][None], gpu)
        g = dev(L[key + "__g"][t][None], gpu)
        ops.prox_admm_sgd(w, g, buf=b, theta=th, alpha=al, rho=rho, lr=lr, momentum=mom, first_step=(t == 0))
        torch.cuda.synchronize()
        assert bits_equal(g.cpu().numpy()[0], L[key + "__gp"][t])
        assert bits_equal(w.cpu().numpy()[0], L[key + "__w1"][t])
        if mom != 0:
            assert bits_equal(b.cpu().numpy()[0], L[key + "__buf1"][t])


@pytest.mark.parametrize("variant", ["avg", "prox", "admm"])
@pytest.mark.parametrize("mom,first", [(0.0, False), (0.5, True), (0.5, False), (0.9, False)])
@pytest.mark.parametrize("extra", [0, 1])
def test_fused_local_step_random_vs_oracle(variant, mom, first, extra, gpu):
    rng = np.random.default_rng(9)
    n, P = 5, 20000 + 3
    w, g, b = (rng.standard_normal((n, P)).astype(np.float32) for _ in range(3))
    th = rng.standard_normal(P).astype(np.float32) if variant != "avg" else None
    al = rng.standard_normal((n, P)).astype(np.float32) if variant == "admm" else None
    wd, gd, bd = padded(w, gpu, extra), padded(g, gpu, extra), padded(b, gpu, extra)
    ald = padded(al, gpu, extra) if al is not None else None
    ops.prox_admm_sgd(wd, gd, buf=bd, theta=None if th is None else dev(th, gpu), alpha=ald, rho=0.1, lr=0.05,
                      momentum=mom, first_step=first, P=P)
    torch.cuda.synchronize()
    w1, b1, g1 = oracle.prox_admm_sgd(w, b, g, th, al, 0.1, 0.05, mom, first)
    assert bits_equal(wd[:, :P].cpu().numpy(), w1)
    assert bits_equal(gd[:, :P].cpu().numpy(), g1)
    if mom != 0:
        assert bits_equal(bd[:, :P].cpu().numpy(), b1)


@pytest.mark.parametrize("rho", ["0.1", "0.01", "1.0"])
def test_dual_golden(rho, gpu):
    D = golden("duals")
    k = f"rho{rho}"
    a = dev(D[k + "__alpha"], gpu)
    r = torch.zeros(a.shape[0], dtype=torch.float64, device=gpu)
    ops.admm_dual(a, dev(D[k + "__w"], gpu), dev(D[k + "__theta"], gpu), float(D[k + "__rho"][0]), resid_sq=r)
    torch.cuda.synchronize()
    assert bits_equal(a.cpu().numpy(), D[k + "__alpha1"])


@pytest.mark.parametrize("n,P,extra", [(3, 5, 0), (7, 4096 * 3 + 2, 0), (4, 100003, 1), (2, (1 << 20) + 1, 0)])
def test_dual_random_with_residual(n, P, extra, gpu):
    rng = np.random.default_rng(P)
    a, w = (rng.standard_normal((n, P)).astype(np.float32) for _ in range(2))
    th = rng.standard_normal(P).astype(np.float32)
    ad = padded(a, gpu, extra)
    r = torch.zeros(n, dtype=torch.float64, device=gpu)
    ops.admm_dual(ad, padded(w, gpu, extra), dev(th, gpu), 0.1, resid_sq=r, P=P)
    torch.cuda.synchronize()
    a1, r1 = oracle.admm_dual(a, w, th, 0.1)
    assert bits_equal(ad[:, :P].cpu().numpy(), a1)
    np.testing.assert_allclose(r.cpu().numpy(), r1, rtol=1e-12)


@pytest.mark.parametrize("name", ["m7_mini", "m1_mini", "m10_flat1031", "m3_flat4097"])
def test_ordered_mean_golden(name, gpu):
    A = golden("average")
    W = A[name + "__W"]
    order = torch.arange(W.shape[0], dtype=torch.int32, device=gpu)
    th = ops.ordered_mean(dev(W, gpu), order)
    torch.cuda.synchronize()
    assert bits_equal(th.cpu().numpy(), A[name + "__theta"])


@pytest.mark.parametrize("N,m,P", [(100, 10, 1663370), (64, 64, 4097), (2000, 17, 3)])
def test_ordered_mean_sampled_order_vs_oracle(N, m, P, gpu):
    rng = np.random.default_rng(m)
    W = rng.standard_normal((N, P)).astype(np.float32)
    order = rng.choice(N, m, replace=False).astype(np.int32)
    th = ops.ordered_mean(dev(W, gpu), dev(order, gpu, torch.int32))
    torch.cuda.synchronize()
    assert bits_equal(th.cpu().numpy(), oracle.ordered_mean(W, order))


def test_stream_copy(gpu):
    x = torch.randn(1 << 20 | 3, device=gpu)
    y = torch.empty_like(x)
    ops.stream_copy(x, y)
    assert torch.equal(x, y)


def test_errors_surface_as_exceptions(gpu):
    x = torch.zeros(4, 8, device=gpu)
    with pytest.raises(ValueError):
        ops.mix_ring(x, x, torch.ones(4, device=gpu), torch.ones(4, device=gpu))
    with pytest.raises(ValueError):
        ops.ordered_mean(x, torch.zeros(0, dtype=torch.int32, device=gpu))


def test_full_size_ring_sampled_rows(gpu):
    """BASELINE size (8192 agents x 2^20 params, 2 x 32 GiB): every output row
    depends on two input rows, so sampled rows are checked bit-exactly against
    the oracle, and a global checksum against an independent fp64 restatement."""
    N, P = 8192, 1 << 20
    torch.manual_seed(2028)
    W = G.communication_graph("circle", "stochastic", N)[0]
    plan = G.MixingPlan.from_graph(W, gpu)
    assert plan.kind == "ring"
    g = torch.Generator(device=gpu).manual_seed(1)
    X = torch.randn(N, P, device=gpu, generator=g)
    Y = torch.empty_like(X)
    plan.apply(X, Y)
    torch.cuda.synchronize()
    wp, wn = plan.csr.ring_weights()
    for i in [0, 1, 2, 4095, 4096, N - 2, N - 1] + list(np.random.default_rng(0).integers(0, N, 8)):
        i = int(i)
        rows = X[[(i - 1) % N, (i + 1) % N]].cpu().numpy()
        want = oracle.mix_ring(np.stack([rows[0], np.zeros(P, np.float32), rows[1]]),
                               np.array([0, wp[i], 0], np.float32), np.array([0, wn[i], 0], np.float32))[1]
        assert bits_equal(Y[i].cpu().numpy(), want), i
    # column sums: sum_i y_i = sum_j (W^T 1)_j x_j, checked in fp64 on 64 columns
    cols = torch.arange(0, P, P // 64, device=gpu)
    colw = torch.from_numpy(plan.csr.dense().sum(0).astype(np.float64)).to(gpu)
    lhs = Y[:, cols].double().sum(0)
    rhs = (colw[:, None] * X[:, cols].double()).sum(0)
    torch.testing.assert_close(lhs, rhs, rtol=1e-5, atol=1e-3)
    del X, Y
    torch.cuda.empty_cache()


@pytest.mark.parametrize("N", [1024, 8192])
def test_full_size_random_regular_sampled_rows(N, gpu):
    """BASELINE config 3 at full size on the agent-major bank: a random
    4-regular W over N agents x 2^20 (the XCD-pinned CSR kernel): sampled output
    rows bit-exact against the oracle on their four input rows, and the
    column-sum identity in fp64 on 64 columns."""
    P = 1 << 20
    plan = G.MixingPlan(G.random_regular_csr(N, 4, seed=2028), gpu)
    g = torch.Generator(device=gpu).manual_seed(2)
    X = torch.randn(N, P, device=gpu, generator=g)
    Y = torch.empty_like(X)
    plan.apply(X, Y)
    torch.cuda.synchronize()
    c = plan.csr
    for i in [0, 1, N // 2, N - 1] + list(np.random.default_rng(1).integers(0, N, 8)):
        i = int(i)
        e0, e1 = int(c.rowptr[i]), int(c.rowptr[i + 1])
        cols = c.col[e0:e1]
        rows = X[torch.as_tensor(cols, dtype=torch.int64, device=gpu)].cpu().numpy()
        want = oracle.mix_csr(rows, np.array([0, e1 - e0], np.int32), np.arange(e1 - e0, dtype=np.int32),
                              c.val[e0:e1])[0]
        assert bits_equal(Y[i].cpu().numpy(), want), i
    cols = torch.arange(0, P, P // 64, device=gpu)
    colw = np.zeros(N, np.float64)
    np.add.at(colw, c.col, c.val.astype(np.float64))
    lhs = Y[:, cols].double().sum(0)
    rhs = (torch.from_numpy(colw).to(gpu)[:, None] * X[:, cols].double()).sum(0)
    torch.testing.assert_close(lhs, rhs, rtol=1e-5, atol=1e-3)
    del X, Y
    torch.cuda.empty_cache()


# --------------------------------------------------------------------------- dense (MFMA) mix
def _gamma_bound(W, X):
    """Rigorous bound for an fp32 fma chain of length K: |Y - Y64| <= gamma_K * sum|W||X|,
    gamma_K = K u / (1 - K u), u = 2^-24."""
    K = W.shape[1]
    u = 2.0 ** -24
    return (K * u / (1 - K * u)) * (np.abs(W.astype(np.float64)) @ np.abs(X.astype(np.float64)))


@pytest.mark.parametrize("M,K,P", [(256, 256, 1024), (130, 37, 1031), (64, 64, 3)])
def test_mix_dense_identity_and_permutation_exact(M, K, P, gpu):
    rng = np.random.default_rng(M + K)
    X = rng.standard_normal((K, P)).astype(np.float32)
    for name in ("id", "perm"):
        W = np.zeros((M, K), np.float32)
        src = np.arange(M) % K if name == "id" else rng.integers(0, K, M)
        W[np.arange(M), src] = 1.0
        Y = torch.empty(M, P, device=gpu)
        ops.mix_dense(dev(W, gpu), dev(X, gpu), Y)
        torch.cuda.synchronize()
        assert bits_equal(Y.cpu().numpy(), X[src]), name  # one nonzero per row: fma chain is exact


@pytest.mark.parametrize("n,P", [(16, 4099), (256, 8192), (1000, 513)])
def test_mix_dense_stochastic_within_gamma_bound(n, P, gpu):
    torch.manual_seed(2028)
    Wt = G.communication_graph("compelete", "stochastic", n)[0]
    plan = G.MixingPlan.from_graph(Wt, gpu, dense=True, dense_kernel="f32")
    assert plan.kind == "dense"
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, P)).astype(np.float32)
    Y = torch.empty(n, P, device=gpu)
    plan.apply(dev(X, gpu), Y)
    torch.cuda.synchronize()
    Wd = plan.csr.dense()
    want64 = Wd.astype(np.float64) @ X.astype(np.float64)
    err = np.abs(Y.cpu().numpy().astype(np.float64) - want64)
    assert np.all(err <= _gamma_bound(Wd, X) + 1e-30)
    # and close to the bit-exact CSR path
    exact = oracle.mix_csr(X, plan.csr.rowptr, plan.csr.col, plan.csr.val)
    assert np.all(np.abs(Y.cpu().numpy() - exact) <= 2 * _gamma_bound(Wd, X) + 1e-30)


def _split3_bound(W, X):
    """Bound for the split3 path (dol_hip.h): the dropped piece products
    (<= 2^-23 |w x| each term) plus fp32 accumulation of 6 K' piece products,
    priced at u = 2^-23 so it holds for any rounding mode inside the MFMA."""
    K = -(-W.shape[1] // 16) * 16
    u = 2.0 ** -23
    n = 6 * K
    return (n * u / (1 - n * u) + 2.0 ** -23) * (np.abs(W.astype(np.float64)) @ np.abs(X.astype(np.float64)))


@pytest.mark.parametrize("M,K,P", [(256, 256, 1024), (130, 37, 1031), (64, 64, 3), (513, 300, 700)])
def test_mix_dense_split3_identity_and_permutation_exact(M, K, P, gpu):
    """One weight of 1.0 per row: the three pieces of x re-sum exactly."""
    rng = np.random.default_rng(M + K + 1)
    X = rng.standard_normal((K, P)).astype(np.float32)
    X[0, :3] = [3.0e38, -1.0e-30, 0.0]  # near the top of the range (truncated x0), tiny, zero
    for name in ("id", "perm"):
        W = np.zeros((M, K), np.float32)
        src = np.arange(M) % K if name == "id" else rng.integers(0, K, M)
        W[np.arange(M), src] = 1.0
        Y = torch.empty(M, P, device=gpu)
        ops.mix_dense_split3(dev(W, gpu), dev(X, gpu), Y)
        torch.cuda.synchronize()
        assert bits_equal(Y.cpu().numpy(), X[src]), name


@pytest.mark.parametrize("n,P,extra", [(16, 4099, 0), (256, 8192, 3), (1000, 513, 0), (300, 20000, 5)])
def test_mix_dense_split3_stochastic_within_bound(n, P, extra, gpu):
    """complete/stochastic W (DIST/simulators.py:54-58,65-70) through the plan:
    within the rigorous bound vs fp64, and at least as close to fp64 as the
    reference's own sequential fp32 sum (oracle.mix_csr) up to 2x."""
    torch.manual_seed(2028)
    Wt = G.communication_graph("compelete", "stochastic", n)[0]
    plan = G.MixingPlan.from_graph(Wt, gpu, dense=True, dense_kernel="split3")
    rng = np.random.default_rng(n + 7)
    X = rng.standard_normal((n, P)).astype(np.float32)
    Xd = padded(X, gpu, extra)
    Y = padded(np.zeros_like(X), gpu, extra)
    for it in range(2):  # second call reuses the split W (w_ready)
        Y.fill_(float("nan"))
        plan.apply(Xd, Y, P=P)
        torch.cuda.synchronize()
        got = Y[:, :P].cpu().numpy()
        assert np.isnan(Y[:, P:].cpu().numpy()).all()  # padding untouched
        Wd = plan.csr.dense()
        want64 = Wd.astype(np.float64) @ X.astype(np.float64)
        err = np.abs(got.astype(np.float64) - want64)
        assert np.all(err <= _split3_bound(Wd, X) + 1e-30), it
        ref = oracle.mix_csr(X, plan.csr.rowptr, plan.csr.col, plan.csr.val)
        ref_err = np.abs(ref.astype(np.float64) - want64)
        assert err.max() <= 2 * ref_err.max() + 1e-30, (err.max(), ref_err.max())
        assert np.sqrt((err ** 2).mean()) <= 2 * np.sqrt((ref_err ** 2).mean()) + 1e-30


def test_mix_dense_split3_matches_f32_kernel_and_ragged_rows(gpu):
    """Erdos-Renyi-style W with M != K (a row block) against the exact-f32 MFMA
    kernel and fp64; the W_READY reuse must give the same bits as a fresh split."""
    rng = np.random.default_rng(5)
    M, K, P = 200, 777, 3001
    A = (rng.random((M, K)) < 0.1).astype(np.float32)
    W = (A * rng.random((M, K))).astype(np.float32)
    X = (rng.standard_normal((K, P)) * 10.0 ** rng.integers(-3, 4, (K, 1))).astype(np.float32)
    Wd, Xd = dev(W, gpu), dev(X, gpu)
    Y1, Y2, Y3 = (torch.empty(M, P, device=gpu) for _ in range(3))
    work = torch.empty(ops.dense_split3_workspace_bytes(M, K, P, 0), dtype=torch.uint8, device=gpu)
    ops.mix_dense_split3(Wd, Xd, Y1, work=work)
    ops.mix_dense_split3(Wd, Xd, Y2, work=work, w_ready=True)
    ops.mix_dense(Wd, Xd, Y3)
    torch.cuda.synchronize()
    assert bits_equal(Y1.cpu().numpy(), Y2.cpu().numpy())
    want64 = W.astype(np.float64) @ X.astype(np.float64)
    e_split = np.abs(Y1.cpu().numpy() - want64)
    e_f32 = np.abs(Y3.cpu().numpy() - want64)
    assert np.all(e_split <= _split3_bound(W, X) + 1e-30)
    assert e_split.max() <= 2 * e_f32.max() + 1e-30


@pytest.mark.parametrize("fuse", [False, None])
@pytest.mark.parametrize("M,K,P,cus", [(300, 300, 2148, 16), (256, 777, 5137, 20), (513, 64, 3001, 32),
                                       (300, 300, 2148, 14), (513, 64, 3001, 10), (1024, 1024, 101770, None)])
def test_mix_dense_split3_narrow_tail_bit_identical(M, K, P, cus, fuse, gpu, monkeypatch):
    """The last partial wave of 256 x 256 tiles runs as 256 x 64 quarters
    (dense_split3_kernel<.., NB = 1>) when it would fill <= 1/4 of the CUs, as
    256 x 128 halves (NB = 2) when <= 1/2 (cus = 14, 10 here);
    DOL_SPLIT3_CUS pretends a CU count so small shapes take that path (None:
    the device's own, 1592 tiles at the bench shape = 6 x 256 + 56).  Same bits
    as all-wide tiles (DOL_SPLIT3_CUS=0), incl. ragged rows / columns / K and
    padding columns past P left untouched."""
    rng = np.random.default_rng(M + K + P)
    W = ((rng.random((M, K)) < 0.2) * rng.random((M, K))).astype(np.float32)
    X = rng.standard_normal((K, P)).astype(np.float32)
    Wd, Xd = dev(W, gpu), padded(X, gpu, 3)
    Y1, Y2 = padded(np.zeros((M, P), np.float32), gpu, 3), padded(np.zeros((M, P), np.float32), gpu, 3)
    if cus is None:
        monkeypatch.delenv("DOL_SPLIT3_CUS", raising=False)
    else:
        monkeypatch.setenv("DOL_SPLIT3_CUS", str(cus))
    ops.mix_dense_split3(Wd, Xd, Y1, P=P, fuse=fuse)  # None: the default (fused where the rows allow)
    monkeypatch.setenv("DOL_SPLIT3_CUS", "0")
    ops.mix_dense_split3(Wd, Xd, Y2, P=P, fuse=fuse)
    torch.cuda.synchronize()
    assert bits_equal(Y1[:, :P].cpu().numpy(), Y2[:, :P].cpu().numpy())
    assert np.isnan(Y1[:, P:].cpu().numpy()).all()
    if M * K * P <= 1 << 31:
        want64 = W.astype(np.float64) @ X.astype(np.float64)
        assert np.all(np.abs(Y1[:, :P].cpu().numpy() - want64) <= _split3_bound(W, X) + 1e-30)


@pytest.mark.parametrize("main", ["fxw", "fx8"])
@pytest.mark.parametrize("M,K,P,extra", [(256, 256, 1024, 0), (130, 37, 1031, 1), (300, 600, 5000, 4),
                                         (64, 20, 4, 0), (513, 300, 701, 3), (200, 50, 999, 0)])
def test_mix_dense_split3_fused_x_equals_split_pass(M, K, P, extra, main, gpu, monkeypatch):
    """X split inside the GEMM (rows 16-B readable) gives the same bits as the
    split pass, at ragged K / P tiles, NaN padding past P, values near the bf16
    overflow threshold (the wave's scalar fallback), subnormals and signed
    zeros; ld % 4 != 0 falls back to the split pass.  Main tiles on
    dense_split3_fxw_kernel (default) or dense_split3_fx8_kernel
    (DOL_SPLIT3_FXW=0, read per call)."""
    monkeypatch.setenv("DOL_SPLIT3_FXW", "0" if main == "fx8" else "1")
    rng = np.random.default_rng(M * 7 + K)
    W = ((rng.random((M, K)) < 0.3) * rng.random((M, K))).astype(np.float32)
    X = rng.standard_normal((K, P)).astype(np.float32)
    X[0, :4] = [3.0e38, -3.3e38, 1e-40, -0.0]
    if K > 3:
        X[3, -1] = 3.3895e38
    Wd, Xd = dev(W, gpu), padded(X, gpu, extra)
    fused = ops.split3_x_flags(Xd, P) != 0
    assert fused == (((P + extra) % 4 == 0) and P >= 4)
    Y1, Y2 = padded(np.zeros((M, P), np.float32), gpu, extra), padded(np.zeros((M, P), np.float32), gpu, extra)
    ops.mix_dense_split3(Wd, Xd, Y1, P=P, fuse=True)
    ops.mix_dense_split3(Wd, Xd, Y2, P=P, fuse=False)
    torch.cuda.synchronize()
    a, b = Y1[:, :P].cpu().numpy(), Y2[:, :P].cpu().numpy()
    assert bits_equal(a, b)
    assert np.isnan(Y1[:, P:].cpu().numpy()).all()
    want64 = W.astype(np.float64) @ X.astype(np.float64)
    big = (W[:, 0] > 0) | ((W[:, 3] > 0) if K > 3 else False)
    ok = ~big  # rows that do not touch the ~3e38 entries: inside the bound
    err = np.abs(a[ok].astype(np.float64) - want64[ok])
    assert np.all(err <= _split3_bound(W[ok], X) + 1e-30)


@pytest.mark.parametrize("main", ["fxw", "fx8"])
@pytest.mark.parametrize("M,K,P,cus", [(300, 300, 2148, 16), (513, 64, 3001, 32), (256, 777, 5137, 0),
                                       (1024, 1024, 101770, None)])
def test_mix_dense_split3_fx8_tiles_and_tail_bit_identical(M, K, P, cus, main, gpu, monkeypatch):
    """The fused X split (r05) on 256 x 256 tiles -- dense_split3_fxw_kernel
    (default: the record kernel's 2 x 4 waves, each lane splitting one record
    into LDS) or dense_split3_fx8_kernel (DOL_SPLIT3_FXW=0: each wave splits
    its own 32 columns once and runs 8 row blocks) -- and, for the last partial
    wave of tiles, FX8's 256 x 64 quarters (DOL_SPLIT3_CUS pretends a CU count
    so small shapes take that path; None: the device's own, 1592 tiles at the
    bench's 1024 x 101,770): the same bits as the split pass + the
    record-staged GEMM, padding past P untouched."""
    monkeypatch.setenv("DOL_SPLIT3_FXW", "0" if main == "fx8" else "1")
    rng = np.random.default_rng(M + 3 * K + P)
    W = ((rng.random((M, K)) < 0.2) * rng.random((M, K))).astype(np.float32)
    X = rng.standard_normal((K, P)).astype(np.float32)
    extra = (-P) % 4 + 4  # rows readable up to round_up(P, 4): the fused path
    Wd, Xd = dev(W, gpu), padded(X, gpu, extra)
    assert ops.split3_x_flags(Xd, P) != 0
    Y1, Y2 = padded(np.zeros((M, P), np.float32), gpu, 3), padded(np.zeros((M, P), np.float32), gpu, 3)
    if cus is None:
        monkeypatch.delenv("DOL_SPLIT3_CUS", raising=False)
    else:
        monkeypatch.setenv("DOL_SPLIT3_CUS", str(cus))
    ops.mix_dense_split3(Wd, Xd, Y1, P=P, fuse=True)
    ops.mix_dense_split3(Wd, Xd, Y2, P=P, fuse=False)
    torch.cuda.synchronize()
    assert bits_equal(Y1[:, :P].cpu().numpy(), Y2[:, :P].cpu().numpy())
    assert np.isnan(Y1[:, P:].cpu().numpy()).all()
    Y3 = padded(np.zeros((M, P), np.float32), gpu, 3)
    ops.mix_dense_split3(Wd, Xd, Y3, P=P)  # the default picks the fused path for these rows: same bits
    torch.cuda.synchronize()
    assert bits_equal(Y3[:, :P].cpu().numpy(), Y2[:, :P].cpu().numpy())


def _er_hip_numpy(n, p, seed):
    """numpy restatement of graph_draw.hip (hash, keys, G = R o A, W = (G / colsum)^T)."""
    M64 = (1 << 64) - 1

    def splitmix(z):
        z = (z + 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    h = splitmix(seed)
    k_edge, k_w = np.uint32(h & 0xFFFFFFFF), np.uint32(((h >> 32) ^ 0x5BD1E995) & 0xFFFFFFFF)

    def mix32(x):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7FEB352D)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846CA68B)
        return x ^ (x >> np.uint32(16))

    def u01(key, idx):
        with np.errstate(over="ignore"):
            return (mix32(idx * np.uint32(0x9E3779B9) + key) >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)

    i, j = np.meshgrid(np.arange(n, dtype=np.uint32), np.arange(n, dtype=np.uint32), indexing="ij")
    a, b = np.minimum(i, j), np.maximum(i, j)
    with np.errstate(over="ignore"):
        edge = (u01(k_edge, a * np.uint32(n) + b) < np.float32(p)) & (i != j)
        g = np.where(edge, u01(k_w, i * np.uint32(n) + j), np.float32(0))
    with np.errstate(invalid="ignore", divide="ignore"):
        W = (g / g.sum(0, dtype=np.float64).astype(np.float32)).T
    return np.where(W > 0, W, 0).astype(np.float32)


@pytest.mark.parametrize("n,p", [(1, 0.5), (7, 0.3), (257, 0.1), (1000, 0.02), (64, 0.0), (64, 1.0)])
def test_er_stochastic_hip_structure(n, p, gpu):
    """Config 5's per-round W drawn by one kernel: undirected G(n, p) pattern
    with a zero diagonal, rows summing to 1 (empty rows all zero), edge density
    within 5 sigma of p, deterministic per seed, and equal to a numpy
    restatement of the kernel's hash (pattern exactly, values to 2 ulp-ish:
    the colsum order differs)."""
    W = G.erdos_renyi_stochastic_hip(n, p, 11, gpu)
    W2 = G.erdos_renyi_stochastic_hip(n, p, 11, gpu)
    W3 = G.erdos_renyi_stochastic_hip(n, p, 12, gpu)
    torch.cuda.synchronize()
    Wn = W.cpu().numpy()
    assert bits_equal(Wn, W2.cpu().numpy())
    if n > 8 and 0 < p < 1:
        assert not np.array_equal(Wn, W3.cpu().numpy())
    assert (np.diag(Wn) == 0).all() and np.isfinite(Wn).all()
    A = Wn > 0
    assert (A == A.T).all()
    rs = Wn.astype(np.float64).sum(1)
    has = A.any(1)
    assert np.allclose(rs[has], 1.0, atol=2e-6) and (Wn[~has] == 0).all()
    if p == 1.0:
        assert (A == ~np.eye(n, dtype=bool)).all()
    if p == 0.0:
        assert not A.any()
    if n >= 257 and 0 < p < 1:
        m = n * (n - 1) / 2
        assert abs(A.sum() / 2 / m - p) <= 5 * np.sqrt(p * (1 - p) / m)
    want = _er_hip_numpy(n, p, 11)
    assert ((want > 0) == A).all()
    np.testing.assert_allclose(Wn, want, rtol=1e-6, atol=0)


def test_mix_dense_split3_argument_errors(gpu):
    W = torch.zeros(8, 8, device=gpu)
    X = torch.zeros(8, 16, device=gpu)
    with pytest.raises(ValueError):
        ops.mix_dense_split3(W, X, X)
    small = torch.empty(16, dtype=torch.uint8, device=gpu)
    with pytest.raises(ValueError):
        ops.mix_dense_split3(W, X, torch.empty(8, 16, device=gpu), work=small)


@pytest.mark.parametrize("admm", [False, True])
@pytest.mark.parametrize("extra", [0, 1])
def test_prox_grad_term_vs_oracle(admm, extra, gpu):
    rng = np.random.default_rng(21)
    n, P = 3, 70001
    g, w = (rng.standard_normal((n, P)).astype(np.float32) for _ in range(2))
    th = rng.standard_normal(P).astype(np.float32)
    al = rng.standard_normal((n, P)).astype(np.float32) if admm else None
    gd = padded(g, gpu, extra)
    ops.prox_grad(gd, padded(w, gpu, extra), dev(th, gpu), 0.1, alpha=padded(al, gpu, extra) if admm else None, P=P)
    torch.cuda.synchronize()
    assert bits_equal(gd[:, :P].cpu().numpy(), oracle.prox_grad(g, w, th, al, 0.1))


@pytest.fixture(params=list(ops.RING_STEPS_VARIANTS), ids=lambda v: {1: "tiles", 2: "stream", 3: "dma", 4: "dmasync", 5: "dmasweep"}[v])
def ring_variant(request):
    """dol_ring_steps_set_variant for the test, restored after it."""
    prev = ops.ring_steps_variant(request.param)
    yield request.param
    ops.ring_steps_variant(prev)


@pytest.mark.parametrize("steps", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("n,P", [(3, 8), (17, 4100), (64, 1024 * 5), (200, 1024), (1001, 2048), (1600, 4100),
                                 (2048, 1024)])
def test_ring_steps_bit_identical_to_single_rounds(steps, n, P, ring_variant, gpu):
    """Both kernels of the fused pass: the register tiles and ring_stream_kernel
    (when n >= 2 steps + 17; 1024-row tiles: 1600 / 2048 rows have interior
    tiles, wrap-around edge tiles and a short last tile; smaller rings fall back
    to the tiles)."""
    rng = np.random.default_rng(steps * 100 + n)
    X = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    want = X
    for _ in range(steps):
        want = oracle.mix_ring(want, wp, wn)
    Y = torch.empty(n, P, device=gpu)
    ops.mix_ring_steps(dev(X, gpu), Y, dev(wp, gpu), dev(wn, gpu), steps)
    torch.cuda.synchronize()
    assert bits_equal(Y.cpu().numpy(), want)


@pytest.mark.parametrize("steps", [2, 5, 8])
def test_ring_steps_interior_tiles(steps, ring_variant, gpu):
    """ring_stream_kernel's interior path (1024-row tiles with every input row and
    weight in range: here the tiles at rows 1024 and 2048 of 4096) next to the
    wrap-around edge tiles, on a ragged column count."""
    n, P = 4096, 1028
    rng = np.random.default_rng(steps + 40)
    X = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    want = X
    for _ in range(steps):
        want = oracle.mix_ring(want, wp, wn)
    Y = torch.empty(n, P, device=gpu)
    ops.mix_ring_steps(dev(X, gpu), Y, dev(wp, gpu), dev(wn, gpu), steps)
    torch.cuda.synchronize()
    assert bits_equal(Y.cpu().numpy(), want)


def test_ring_steps_variant_tuner(gpu):
    """tune_ring_steps_variant keeps the faster kernel for the process; the pass
    gives the same bits after it."""
    n, P = 1600, 4100
    rng = np.random.default_rng(7)
    X = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    want = X
    for _ in range(5):
        want = oracle.mix_ring(want, wp, wn)
    Xd, wpd, wnd = dev(X, gpu), dev(wp, gpu), dev(wn, gpu)
    Y = torch.empty(n, P, device=gpu)
    prev = ops.ring_steps_variant(0)
    try:
        tuned = ops.tune_ring_steps_variant(lambda: ops.mix_ring_steps(Xd, Y, wpd, wnd, 5), reps=1)
        assert tuned["variant"] in ops.RING_STEPS_VARIANTS and set(tuned["ms"]) == set(ops.RING_STEPS_VARIANTS)
        assert ops.ring_steps_variant(tuned["variant"]) == tuned["variant"]
        Y.zero_()
        ops.mix_ring_steps(Xd, Y, wpd, wnd, 5)
        torch.cuda.synchronize()
        assert bits_equal(Y.cpu().numpy(), want)
    finally:
        ops.ring_steps_variant(prev)


def test_ring_steps_autotuned_per_buffers(gpu, monkeypatch):
    """The product path's tuning (ops.mix_ring_steps with variant=None): the
    first call on a buffer pair times every variant on those buffers and caches
    the winner per (pair, geometry) -- the swapped pair hits the same entry --
    without touching the process-wide setting; the bits never change."""
    monkeypatch.setattr(ops, "AUTOTUNE_MIN_BYTES", 0)
    monkeypatch.setattr(ops, "_TUNED", {})
    n, P = 1600, 4100
    rng = np.random.default_rng(9)
    X = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    want = X
    for _ in range(5):
        want = oracle.mix_ring(want, wp, wn)
    Xd, wpd, wnd = dev(X, gpu), dev(wp, gpu), dev(wn, gpu)
    Y = torch.full((n, P), float("nan"), device=gpu)
    prev = ops.ring_steps_variant(0)
    ops.mix_ring_steps(Xd, Y, wpd, wnd, 5)
    torch.cuda.synchronize()
    assert bits_equal(Y.cpu().numpy(), want)
    tuned = ops.tuned_choices()
    assert len(tuned) == 1
    (entry,) = tuned.values()
    assert entry["choice"] in ops.RING_STEPS_VARIANTS and set(entry["ms"]) == set(ops.RING_STEPS_VARIANTS)
    assert ops.ring_steps_variant(0) == 0  # the process setting is untouched
    ops.mix_ring_steps(Y.clone(), Xd, wpd, wnd, 5)  # a new pair: tuned separately
    ops.mix_ring_steps(Y, Xd, wpd, wnd, 5)  # the swapped first pair: cached
    torch.cuda.synchronize()
    assert len(ops.tuned_choices()) == 2
    ops.ring_steps_variant(prev)


def test_pm_stage_order_autotuned_per_buffers(gpu, monkeypatch):
    """mix_csr_pm / dgd_csr_pm with nseg=None: the order is tuned once per
    buffer pair (on the plain mix) and both calls give the bits of an explicit order."""
    monkeypatch.setattr(ops, "AUTOTUNE_MIN_BYTES", 0)
    monkeypatch.setattr(ops, "_TUNED", {})
    from dolhip import graph as G
    n, P = 1000, 2500
    c = G.random_regular_csr(n, 4, seed=11)
    rp, col, val = (torch.as_tensor(a, device=gpu) for a in (c.rowptr, c.col, c.val))
    rng = np.random.default_rng(4)
    XT = dev(rng.standard_normal((P, 1000)).astype(np.float32), gpu)
    TT = dev(rng.standard_normal((P, 1000)).astype(np.float32), gpu)
    YT = torch.empty_like(XT)
    want = torch.empty_like(XT)
    ops.mix_csr_pm(XT, want, rp, col, val, nseg=8)
    ops.mix_csr_pm(XT, YT, rp, col, val)
    torch.cuda.synchronize()
    assert torch.equal(YT.view(torch.int32), want.view(torch.int32))
    assert len(ops.tuned_choices()) == 1
    ops.dgd_csr_pm(XT, want, rp, col, val, TT, steps=2, lr=0.1, nseg=16)
    ops.dgd_csr_pm(XT, YT, rp, col, val, TT, steps=2, lr=0.1)
    torch.cuda.synchronize()
    assert torch.equal(YT.view(torch.int32), want.view(torch.int32))
    assert len(ops.tuned_choices()) == 1  # the dgd round reused the mix's entry


@pytest.mark.parametrize("steps", [2, 5, 8])
def test_ring_steps_signed_zeros_and_underflow(steps, gpu):
    """The fused pass's intermediate levels use fma(wp, a, +0) + wn*b, which may
    hold -0 where single rounds hold +0; the last level must still match the
    single rounds bit for bit.  Inputs full of +-0, denormals and values whose
    products with the (partly negative, partly tiny) weights underflow."""
    n, P = 97, 1024
    rng = np.random.default_rng(steps)
    X = rng.standard_normal((n, P)).astype(np.float32)
    pick = rng.random((n, P))
    X[pick < 0.25] = 0.0
    X[(pick >= 0.25) & (pick < 0.5)] = -0.0
    X[(pick >= 0.5) & (pick < 0.6)] = np.float32(1e-42) * np.sign(rng.standard_normal(int(((pick >= 0.5) & (pick < 0.6)).sum())))
    X[(pick >= 0.6) & (pick < 0.65)] = np.float32(1e-30)
    X[0, :4] = [np.inf, -np.inf, np.nan, 3e38]
    wp = rng.random(n).astype(np.float32)
    wn = rng.random(n).astype(np.float32)
    wp[::3] *= -1
    wn[1::4] = np.float32(1e-20)
    wp[2::5] = 0.0
    want = X
    for _ in range(steps):
        want = oracle.mix_ring(want, wp, wn)
    assert np.signbit(want[want == 0]).sum() == 0, "single rounds never produce -0"
    Y = torch.empty(n, P, device=gpu)
    ops.mix_ring_steps(dev(X, gpu), Y, dev(wp, gpu), dev(wn, gpu), steps)
    torch.cuda.synchronize()
    assert bits_equal(Y.cpu().numpy(), want)


def test_bank_mix_fused_equals_unfused(gpu):
    from dolhip.bank import AgentBank
    torch.manual_seed(5)
    W = G.communication_graph("circle", "stochastic", 33)[0]
    plan = G.MixingPlan.from_graph(W, gpu)
    X = torch.randn(33, 2048, device=gpu)
    a, b = AgentBank(33, 2048, gpu), AgentBank(33, 2048, gpu)
    a.rows()[:] = X
    b.rows()[:] = X
    a.mix(plan, steps=13, fuse=True)     # 8 + 5 fused
    b.mix(plan, steps=13, fuse=False)    # 13 single rounds
    assert bits_equal(a.rows().cpu().numpy(), b.rows().cpu().numpy())


@pytest.mark.parametrize("n,deg,P", [(600, 4, 1024 * 8 + 12), (2048, 6, 4096), (513, 2, 128 + 4 * 32 + 3)])
def test_mix_csr_xcd_path_vs_oracle(n, deg, P, gpu):
    """Large graphs take the XCD-pinned 512-B-tile path (plus the 4 KiB-tile
    remainder and the scalar tail)."""
    c = G.random_regular_csr(n, deg, seed=n + 1)
    rng = np.random.default_rng(2)
    X = rng.standard_normal((n, P)).astype(np.float32)
    plan = G.MixingPlan(c, gpu)
    Yd = torch.empty(n, P, device=gpu)
    plan.apply(dev(X, gpu), Yd)
    torch.cuda.synchronize()
    assert bits_equal(Yd.cpu().numpy(), oracle.mix_csr(X, c.rowptr, c.col, c.val))


@pytest.mark.parametrize("mom,first", [(0.0, False), (0.5, True), (0.5, False)])
@pytest.mark.parametrize("extra", [0, 1])
def test_admm_step_dual_equals_two_calls(mom, first, extra, gpu):
    rng = np.random.default_rng(31)
    n, P = 4, 30001
    w, g, b, al = (rng.standard_normal((n, P)).astype(np.float32) for _ in range(4))
    th = rng.standard_normal(P).astype(np.float32)
    wd, gd, bd, ad = (padded(a, gpu, extra) for a in (w, g, b, al))
    ops.admm_step_dual(wd, gd, dev(th, gpu), ad, buf=bd, rho=0.1, lr=0.05, momentum=mom, first_step=first, P=P)
    torch.cuda.synchronize()
    w1, b1, g1 = oracle.prox_admm_sgd(w, b, g, th, al, 0.1, 0.05, mom, first)
    a1, _ = oracle.admm_dual(al, w1, th, 0.1)
    assert bits_equal(wd[:, :P].cpu().numpy(), w1)
    assert bits_equal(ad[:, :P].cpu().numpy(), a1)
    assert bits_equal(gd[:, :P].cpu().numpy(), g1)
    if mom != 0:
        assert bits_equal(bd[:, :P].cpu().numpy(), b1)


def test_erdos_renyi_device_plan_within_gamma_bound(gpu):
    """Config 5's per-round W: undirected ER support (symmetric, zero diagonal),
    the reference's 'stochastic' weighting (rows of W sum to 1), and the dense
    MFMA mix of it within the fp32 fma-chain bound of the bit-exact CSR mix."""
    n, P = 300, 1031
    gen = torch.Generator(device=gpu).manual_seed(5)
    W = G.erdos_renyi_stochastic(n, 0.1, gen)
    Wc = W.cpu().numpy()
    assert np.all(np.diag(Wc) == 0)
    assert np.array_equal(Wc > 0, (Wc > 0).T)
    nz = (Wc > 0).any(1)
    np.testing.assert_allclose(Wc[nz].astype(np.float64).sum(1), 1.0, rtol=1e-5)
    plan = G.MixingPlan.from_dense(W)
    assert plan.kind == "dense" and abs(plan.density - (Wc > 0).mean()) < 1e-12
    rng = np.random.default_rng(6)
    X = rng.standard_normal((n, P)).astype(np.float32)
    Y = torch.empty(n, P, device=gpu)
    plan.apply(dev(X, gpu), Y)
    torch.cuda.synchronize()
    csr = G.csr_from_dense(Wc)
    exact = oracle.mix_csr(X, csr.rowptr, csr.col, csr.val)
    assert np.all(np.abs(Y.cpu().numpy() - exact) <= 2 * _gamma_bound(Wc, X) + 1e-30)


def test_stream_copy_rows_is_a_copy(gpu):
    """The roofline calibration copy (the ring kernel with the stencil replaced
    by the row itself) reproduces X exactly, including the last partial tile."""
    X = torch.randn(11, 4096 + 64, device=gpu)
    Y = torch.full_like(X, 3.0)
    ops.stream_copy_rows(X, Y, P=4096)
    torch.cuda.synchronize()
    assert torch.equal(Y[:, :4096], X[:, :4096])
    assert (Y[:, 4096:] == 3.0).all()
    with pytest.raises(ops.DolNativeError):
        ops.stream_copy_rows(X, Y, P=4095)


@pytest.mark.parametrize("n,P,extra", [(1, 37, 0), (2, 1000, 0), (5, 4099, 3), (7, 4096, 1)])
def test_ring_edges_match_oracle(n, P, extra, gpu):
    """dol_mix_ring_edges_f32 / dol_dgd_ring_edges_f32 (the sharded round's two
    boundary rows in one launch): rows 0 and n-1 bit-exact vs the oracle's ring
    with halos, every other row untouched; f4 and scalar-tail paths."""
    rng = np.random.default_rng(n * 31 + P)
    X = rng.standard_normal((n, P)).astype(np.float32)
    T = rng.standard_normal((n, P)).astype(np.float32)
    M = rng.standard_normal((n, P)).astype(np.float32)
    hp, hn = (rng.standard_normal(P).astype(np.float32) for _ in range(2))
    X[0, :3] = [np.inf, -0.0, 1e-40]
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    ld = P + extra

    def dev(a, fill=float("nan")):
        t = torch.full((a.shape[0], ld), fill, device=gpu)
        t[:, :P] = torch.from_numpy(a).to(gpu)
        return t
    Xd, Yd, Td, Md = dev(X), dev(np.full((n, P), 5.0, np.float32)), dev(T), dev(M)
    hpd, hnd = torch.from_numpy(hp).to(gpu), torch.from_numpy(hn).to(gpu)
    wpd, wnd = torch.from_numpy(wp).to(gpu), torch.from_numpy(wn).to(gpu)
    ops.mix_ring_edges(Xd, Yd, wpd, wnd, hpd, hnd, P=P, n_rows=n)
    torch.cuda.synchronize()
    want = oracle.mix_ring(X, wp, wn, hp, hn)
    got = Yd[:, :P].cpu().numpy()
    edges = [0, n - 1]
    assert bits_equal(got[edges], want[edges])
    assert (got[1:n - 1] == 5.0).all(), "interior rows touched"
    Yd2 = dev(np.full((n, P), 5.0, np.float32))
    ops.dgd_ring_edges(Xd, Yd2, wpd, wnd, Td, hpd, hnd, mom=Md, steps=2, lr=0.05, momentum=0.9, P=P, n_rows=n)
    torch.cuda.synchronize()
    wy, wm = oracle.dgd_local(want, T, M, "least_squares", 2, 0.05, 0.9, False)
    assert bits_equal(Yd2[:, :P].cpu().numpy()[edges], wy[edges])
    gm = Md[:, :P].cpu().numpy()
    assert bits_equal(gm[edges], wm[edges])
    assert bits_equal(gm[1:n - 1], M[1:n - 1]), "interior momentum touched"


_STREAM_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import oracle
from dolhip import ops
dev = torch.device("cuda:0")
for steps, n, P in ((5, 4096, 1028), (2, 1600, 4100), (8, 2048, 1024), (3, 40, 256)):
    rng = np.random.default_rng(steps * 7 + n)
    X = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    want = X
    for _ in range(steps):
        want = oracle.mix_ring(want, wp, wn)
    Y = torch.empty(n, P, device=dev)
    ops.mix_ring_steps(torch.from_numpy(X).to(dev), Y, torch.from_numpy(wp).to(dev), torch.from_numpy(wn).to(dev), steps)
    torch.cuda.synchronize()
    assert oracle.bits_equal(Y.cpu().numpy(), want), (steps, n, P)
print("ok")
"""


@pytest.mark.parametrize("env", [{"DOL_RING_STREAM": "1"}, {"DOL_RING_STREAM": "1", "DOL_RING_STREAM_NT": "0",
                                                               "DOL_RING_STREAM_T": "2048"}])
def test_ring_stream_kernel_opt_in_bit_identical(env, gpu):
    """The opt-in streaming eps pass (DOL_RING_STREAM=1, read once per process:
    run in a child) is bit-identical to single rounds: interior and edge tiles,
    short last tiles, and the small-ring fallback to the register tiles."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _STREAM_CHILD, root,
                        os.path.join(root, "distributed-optimization-and-learning_amd")],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
