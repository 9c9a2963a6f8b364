"""The parameter-major (transposed) bank: dol_mix_csr_pm_f32 and
dol_transpose_f32 through the C-ABI.  The mix is bit-exact against the
reference's own consensus vectors (tests/golden/mix.npz, transposed) and
against the oracle on random-regular, long-row, empty-row, rectangular and
non-finite inputs, at ragged agent counts up to the 8192 limit, and on sampled
parameter rows at BASELINE config 3's full 1024 x 2^20."""
import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from conftest import golden
from dolhip import graph as G
from dolhip import ops

pytestmark = pytest.mark.gpu


def csr_dev(c, gpu):
    return (torch.as_tensor(np.asarray(c.rowptr, np.int32), device=gpu),
            torch.as_tensor(np.asarray(c.col, np.int32), device=gpu),
            torch.as_tensor(np.asarray(c.val, np.float32), device=gpu))


def pm(X, gpu, extra=0):
    """Parameter-major device copy of agent-major X [n, P]: [P, round_up(n, 4) + extra], NaN padding."""
    n, P = X.shape
    ld = (n + 3) // 4 * 4 + extra
    t = torch.full((P, ld), float("nan"), dtype=torch.float32, device=gpu)
    t[:, :n] = torch.as_tensor(np.ascontiguousarray(X.T), device=gpu)
    return t


def run_pm(X, c, gpu, x_agents=None, extra=0):
    rp, col, val = csr_dev(c, gpu)
    XT = pm(X, gpu, extra)
    n = len(c.rowptr) - 1
    YT = torch.full((X.shape[1], (n + 3) // 4 * 4 + extra), 7.0, device=gpu)
    ops.mix_csr_pm(XT, YT, rp, col, val, x_agents=x_agents if x_agents is not None else X.shape[0])
    torch.cuda.synchronize()
    out = YT.cpu().numpy()
    assert (out[:, n:] == 7.0).all(), "wrote past the last agent"
    return np.ascontiguousarray(out[:, :n].T)


def _mix_cases():
    return sorted(k[:-3] for k in golden("mix").files if k.endswith("__X"))


@pytest.mark.parametrize("case", _mix_cases())
def test_pm_mix_matches_reference_consensus(case, gpu):
    mix, csr = golden("mix"), golden("csr")
    gkey, _l, t = case.split("__")
    k = f"{gkey}__{t}"
    n = len(csr[k + "__rowptr"]) - 1
    c = G.CSR(n, n, csr[k + "__rowptr"], csr[k + "__col"], csr[k + "__val"])
    assert bits_equal(run_pm(mix[case + "__X"], c, gpu), mix[case + "__Y"])


@pytest.mark.parametrize("n", [5, 64, 100, 257, 1000, 1024, 1025, 2047, 4096, 4097, 5000, 8192])
@pytest.mark.parametrize("P", [1, 7, 300])
def test_pm_mix_random_regular_vs_oracle(n, P, gpu):
    c = G.random_regular_csr(n, 4, seed=n + 3)
    X = np.random.default_rng(n * 7 + P).standard_normal((n, P)).astype(np.float32)
    assert bits_equal(run_pm(X, c, gpu, extra=4 * (n % 3)), oracle.mix_csr(X, c.rowptr, c.col, c.val))


@pytest.mark.parametrize("n,P", [(1024, 4099), (4097, 3000), (8192, 4096)])
def test_pm_mix_many_stages_per_workgroup(n, P, gpu):
    """Enough p-rows that every persistent workgroup cycles through its whole
    LDS-DMA ring many times (beyond 4096 agents: five 32-KiB buffers, one p-row
    each), bit-exact vs the oracle."""
    c = G.random_regular_csr(n, 4, seed=n + 11)
    X = np.random.default_rng(n + P).standard_normal((n, P)).astype(np.float32)
    assert bits_equal(run_pm(X, c, gpu), oracle.mix_csr(X, c.rowptr, c.col, c.val))


@pytest.mark.parametrize("nseg", ["1", "3", "8"])
def test_pm_mix_stage_orders_bit_identical(nseg, gpu, monkeypatch):
    """The stage order (DOL_PM_NSEG segments walked side by side) is a speed
    choice only; 3 does not divide the grid and falls back to one sweep."""
    monkeypatch.setenv("DOL_PM_NSEG", nseg)
    torch.manual_seed(2028)
    c = G.communication_csr("circle", "stochastic", 1000)[0]
    X = np.random.default_rng(1).standard_normal((1000, 2500)).astype(np.float32)
    assert bits_equal(run_pm(X, c, gpu), oracle.mix_csr(X, c.rowptr, c.col, c.val))


@pytest.mark.parametrize("nseg", [16, 32, 7])
def test_pm_stage_order_setter_bit_identical(nseg, gpu):
    """dol_pm_set_stage_order overrides DOL_PM_NSEG for the process (7 does not
    divide the grid: one sweep); the tuner keeps the fastest candidate; the bits
    never change."""
    torch.manual_seed(2028)
    c = G.communication_csr("circle", "stochastic", 1000)[0]
    X = np.random.default_rng(1).standard_normal((1000, 2500)).astype(np.float32)
    prev = ops.pm_stage_order(nseg)
    try:
        assert ops.pm_stage_order(nseg) == nseg
        assert bits_equal(run_pm(X, c, gpu), oracle.mix_csr(X, c.rowptr, c.col, c.val))
        XT = torch.as_tensor(np.ascontiguousarray(X.T), device=gpu)
        YT = torch.empty_like(XT)
        rp, col, val = csr_dev(c, gpu)
        tuned = ops.tune_pm_stage_order(lambda: ops.mix_csr_pm(XT, YT, rp, col, val), candidates=(1, 8, 16), reps=1)
        assert tuned["nseg"] in (1, 8, 16) and ops.pm_stage_order(0) == tuned["nseg"]
        assert bits_equal(np.ascontiguousarray(YT.cpu().numpy().T), oracle.mix_csr(X, c.rowptr, c.col, c.val))
    finally:
        ops.pm_stage_order(prev)


def test_pm_mix_long_empty_rectangular_and_nonfinite(gpu):
    rng = np.random.default_rng(5)
    # long rows: the complete graph (degree n - 1) and a dense-ish Erdos-Renyi
    torch.manual_seed(2028)
    W = G.communication_graph("compelete", "stochastic", 40)[0]
    c = G.csr_from_dense(W)
    X = rng.standard_normal((40, 333)).astype(np.float32)
    X[3, 7], X[9, 8], X[11, 9], X[12, 10] = np.inf, np.nan, -0.0, 1e-40
    assert bits_equal(run_pm(X, c, gpu), oracle.mix_csr(X, c.rowptr, c.col, c.val))
    # empty rows (the dynamic topology: one edge per step) and Inf/NaN next to
    # skipped register slots (no 0 * Inf)
    torch.manual_seed(2028)
    for Wt in G.communication_graph("dynamic", "stochastic", 9)[:3]:
        c = G.csr_from_dense(Wt)
        X = rng.standard_normal((9, 50)).astype(np.float32)
        X[0, :5] = np.inf
        X[1, 5:9] = np.nan
        assert bits_equal(run_pm(X, c, gpu), oracle.mix_csr(X, c.rowptr, c.col, c.val))
    # rectangular: 50 output agents gathering from 70 input agents, mixed degrees
    rowptr, col, val = [0], [], []
    for i in range(50):
        d = int(rng.integers(0, 9))
        cols = np.sort(rng.choice(70, d, replace=False))
        col += cols.tolist()
        val += rng.random(d).astype(np.float32).tolist()
        rowptr.append(len(col))
    c = G.CSR(50, 70, np.array(rowptr, np.int32), np.array(col, np.int32), np.array(val, np.float32))
    X = rng.standard_normal((70, 123)).astype(np.float32)
    want = oracle.mix_csr(X, c.rowptr, c.col, c.val)
    assert bits_equal(run_pm(X, c, gpu), want)


def test_pm_mix_full_size_sampled_rows(gpu):
    """BASELINE config 3 at full size, 1024 agents x 2^20 on a random 4-regular
    W: 64 sampled parameter rows (and the last one) bit-exact vs the oracle,
    plus the column-sum identity sum_i YT[p][i] = sum_j colsum(W)_j XT[p][j]
    (fp64, rtol 1e-5) on every row."""
    n, P = 1024, 1 << 20
    c = G.random_regular_csr(n, 4, seed=2028)
    rp, col, val = csr_dev(c, gpu)
    g = torch.Generator(device=gpu).manual_seed(9)
    XT = torch.empty(P, n, device=gpu).normal_(generator=g)
    YT = torch.empty_like(XT)
    ops.mix_csr_pm(XT, YT, rp, col, val)
    torch.cuda.synchronize()
    rows = np.concatenate([np.random.default_rng(3).choice(P, 64, replace=False), [P - 1]])
    Xs = XT[torch.as_tensor(rows, device=gpu)].cpu().numpy()
    want = oracle.mix_csr(np.ascontiguousarray(Xs.T), c.rowptr, c.col, c.val)
    got = YT[torch.as_tensor(rows, device=gpu)].cpu().numpy().T
    assert bits_equal(got, want)
    colsum = np.zeros(n, np.float64)
    np.add.at(colsum, c.col, c.val.astype(np.float64))
    lhs = YT.double().sum(1)
    rhs = XT.double() @ torch.as_tensor(colsum, device=gpu)
    torch.testing.assert_close(lhs, rhs, rtol=1e-5, atol=1e-6 * float(rhs.abs().max()))


@pytest.mark.parametrize("rows,cols", [(1, 1), (5, 300), (1024, 4099), (333, 64), (70, 1)])
def test_transpose_roundtrip(rows, cols, gpu):
    A = torch.randn(rows, cols + 3, device=gpu)
    B = torch.full((cols, rows + 5), 9.0, device=gpu)
    ops.transpose(A, B, rows, cols)
    C = torch.full((rows, cols + 3), 4.0, device=gpu)
    ops.transpose(B, C, cols, rows)
    torch.cuda.synchronize()
    assert torch.equal(B[:, :rows], A[:, :cols].T)
    assert (B[:, rows:] == 9.0).all()
    assert torch.equal(C[:, :cols], A[:, :cols])


def test_pm_mix_argument_errors(gpu):
    c = G.random_regular_csr(16, 4, seed=1)
    rp, col, val = csr_dev(c, gpu)
    XT = torch.zeros(10, 16, device=gpu)
    with pytest.raises(ops.DolNativeError, match="at most"):
        ops.mix_csr_pm(torch.zeros(2, 8196, device=gpu), torch.zeros(2, 8196, device=gpu), rp, col, val,
                       x_agents=8193)
    with pytest.raises(ops.DolNativeError, match="multiples of 4"):
        ops.mix_csr_pm(torch.zeros(10, 18, device=gpu)[:, :17], torch.zeros(10, 16, device=gpu), rp, col, val)
    with pytest.raises(ValueError, match="alias"):
        ops.mix_csr_pm(XT, XT, rp, col, val)


# --- config 3's fused round on the parameter-major bank (dol_dgd_csr_pm_f32) ---

def _dgd_pm(X, T, M, c, gpu, objective, steps, lr, momentum, first, extra=0):
    rp, col, val = csr_dev(c, gpu)
    n = len(c.rowptr) - 1
    XT, TT = pm(X, gpu, extra), pm(T, gpu, extra)
    MT = pm(M, gpu, extra) if momentum else None
    YT = torch.full((X.shape[1], (n + 3) // 4 * 4 + extra), 7.0, device=gpu)
    ops.dgd_csr_pm(XT, YT, rp, col, val, TT, MT, objective=objective, steps=steps, lr=lr, momentum=momentum,
                   first_step=first, x_agents=X.shape[0])
    torch.cuda.synchronize()
    out = YT.cpu().numpy()
    assert (out[:, n:] == 7.0).all(), "wrote past the last agent"
    Mo = None
    if momentum:
        mo = MT.cpu().numpy()
        assert np.isnan(mo[:, n:]).all(), "momentum written past the last agent"
        Mo = np.ascontiguousarray(mo[:, :n].T)
    return np.ascontiguousarray(out[:, :n].T), Mo


MODES = [(0.0, False), (0.9, True), (0.9, False)]


@pytest.mark.parametrize("momentum,first", MODES)
@pytest.mark.parametrize("n", [5, 100, 1000, 1024, 1025, 2047, 4096])
@pytest.mark.parametrize("P", [1, 7, 300])
def test_pm_dgd_least_squares_vs_oracle(n, P, momentum, first, gpu):
    """Least squares: bit-exact against oracle.mix_csr then oracle.dgd_local
    (one rounding per operation on both sides), momentum written back."""
    c = G.random_regular_csr(n, 4, seed=n + 11)
    rng = np.random.default_rng(n + 13 * P)
    X, T, M = (rng.standard_normal((n, P)).astype(np.float32) for _ in range(3))
    got_y, got_m = _dgd_pm(X, T, M, c, gpu, "least_squares", 3, 0.05, momentum, first, extra=4 * (n % 2))
    want_y, want_m = oracle.dgd_local(oracle.mix_csr(X, c.rowptr, c.col, c.val), T, M if momentum else None,
                                      "least_squares", 3, 0.05, momentum, first)
    assert bits_equal(got_y, want_y)
    if momentum:
        assert bits_equal(got_m, want_m)


@pytest.mark.parametrize("momentum,first", MODES)
@pytest.mark.parametrize("n,P", [(64, 100), (1000, 257), (4096, 33)])
def test_pm_dgd_logistic_matches_agent_major_kernel(n, P, momentum, first, gpu):
    """Logistic calls expf: bit-identical to the agent-major fused kernel
    (dol_dgd_csr_f32, same device libm) and within test_dgd_gpu's stated
    tolerance (rtol 2e-6, atol 1e-6) of the glibc oracle."""
    c = G.random_regular_csr(n, 4, seed=n)
    rng = np.random.default_rng(n + P)
    X, T, M = (rng.standard_normal((n, P)).astype(np.float32) for _ in range(3))
    got_y, got_m = _dgd_pm(X, T, M, c, gpu, "logistic", 2, 0.1, momentum, first)
    rp, col, val = csr_dev(c, gpu)
    Xd, Td = (torch.as_tensor(a, device=gpu) for a in (X, T))
    Md = torch.as_tensor(M, device=gpu) if momentum else None
    Yd = torch.empty_like(Xd)
    ops.dgd_csr(Xd, Yd, rp, col, val, Td, Md, objective="logistic", steps=2, lr=0.1, momentum=momentum,
                first_step=first)
    assert bits_equal(got_y, Yd.cpu().numpy())
    if momentum:
        assert bits_equal(got_m, Md.cpu().numpy())
    want_y, _ = oracle.dgd_local(oracle.mix_csr(X, c.rowptr, c.col, c.val), T, M if momentum else None,
                                 "logistic", 2, 0.1, momentum, first)
    np.testing.assert_allclose(got_y, want_y, rtol=2e-6, atol=1e-6)


def test_pm_dgd_full_size_sampled_rows(gpu):
    """BASELINE config 3's round at full size (1024 x 2^20, random 4-regular W,
    least squares, 2 local steps, momentum 0.9 continuing): 48 sampled
    parameter rows and the last one bit-exact vs the oracle, Y and momentum."""
    n, P = 1024, 1 << 20
    c = G.random_regular_csr(n, 4, seed=2028)
    rp, col, val = csr_dev(c, gpu)
    g = torch.Generator(device=gpu).manual_seed(5)
    XT, TT, MT = (torch.empty(P, n, device=gpu).normal_(generator=g) for _ in range(3))
    M0 = MT.clone()
    YT = torch.empty_like(XT)
    ops.dgd_csr_pm(XT, YT, rp, col, val, TT, MT, steps=2, lr=0.05, momentum=0.9)
    torch.cuda.synchronize()
    rows = torch.as_tensor(np.concatenate([np.random.default_rng(4).choice(P, 48, replace=False), [P - 1]]),
                           device=gpu)
    sel = [np.ascontiguousarray(a[rows].cpu().numpy().T) for a in (XT, TT, M0)]
    want_y, want_m = oracle.dgd_local(oracle.mix_csr(sel[0], c.rowptr, c.col, c.val), sel[1], sel[2],
                                      "least_squares", 2, 0.05, 0.9, False)
    assert bits_equal(YT[rows].cpu().numpy().T, want_y)
    assert bits_equal(MT[rows].cpu().numpy().T, want_m)


def test_pm_dgd_argument_errors(gpu):
    c = G.random_regular_csr(4100, 4, seed=1)
    rp, col, val = csr_dev(c, gpu)
    Z = torch.zeros(3, 4100, device=gpu)
    with pytest.raises(ops.DolNativeError, match="at most 4096"):
        ops.dgd_csr_pm(Z, Z.clone(), rp, col, val, Z.clone())
    c = G.random_regular_csr(16, 4, seed=1)
    rp, col, val = csr_dev(c, gpu)
    XT = torch.zeros(10, 16, device=gpu)
    with pytest.raises(ValueError, match="needs MT"):
        ops.dgd_csr_pm(XT, XT.clone(), rp, col, val, XT.clone(), momentum=0.9)
    with pytest.raises(ops.DolNativeError, match="ldt / ldm"):
        ops.dgd_csr_pm(XT, XT.clone(), rp, col, val, torch.zeros(10, 18, device=gpu)[:, :17])


@pytest.mark.parametrize("objective,momentum", [("least_squares", 0.9), ("logistic", 0.0), ("least_squares", 0.0)])
def test_separable_dgd_pm_trajectory_matches_agent_major(objective, momentum, gpu):
    """SeparableDGDPM.from_agent_major continues a SeparableDGD bit-identically:
    5 rounds on each layout (random 4-regular W, 777 agents, 2 local steps)
    give the same parameters and momentum bits."""
    from dolhip.synthetic import SeparableDGD, SeparableDGDPM
    plan = G.MixingPlan(G.random_regular_csr(777, 4, seed=3), gpu)
    a = SeparableDGD(plan, 1001, objective=objective, lr=0.05, momentum=momentum, local_steps=2, seed=11)
    a.round()
    b = SeparableDGDPM.from_agent_major(a)
    for _ in range(5):
        a.round()
        b.round()
    torch.cuda.synchronize()
    assert b.rounds == a.rounds == 6
    assert bits_equal(b.params().cpu().numpy(), a.params().cpu().numpy())
    if momentum:
        assert bits_equal(b.momentum_rows().cpu().numpy(), a.momentum_rows().cpu().numpy())
    assert abs(b.consensus_error() - a.consensus_error()) <= 1e-6 * max(1.0, a.consensus_error())
