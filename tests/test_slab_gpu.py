"""The LDS-gather CSR mix for high-degree graphs (dol_mix_csr_slab_f32) and the
device-side Neighbors selection (dol_dense_to_csr_f32): bit-exact against the
oracle's restatement of DIST/clients.py:61-69 (ascending j, +0 start,
separately rounded mul and add) and bit-identical to the generic CSR kernel;
the device CSR equals graph.csr_from_dense (DIST/simulators.py:91-97) entry
for entry."""
import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from dolhip import graph as G
from dolhip import ops

pytestmark = pytest.mark.gpu


def er_csr(n, p, seed, m=None, empty_rows=()):
    """Host CSR of a seeded G(n, p) under the 'stochastic' rule (W = G^T of the
    column-normalised R o A), with chosen rows emptied (Neighbors drops NaN)."""
    m = n if m is None else m
    rng = np.random.default_rng(seed)
    A = (rng.random((m, n)) < p).astype(np.float32)
    if m == n:
        np.fill_diagonal(A, 0)
    R = rng.random((m, n)).astype(np.float32) * A
    cs = R.sum(0, dtype=np.float32)
    with np.errstate(invalid="ignore", divide="ignore"):
        W = (R / cs).T.astype(np.float32)
    for r in empty_rows:
        W[r, :] = np.nan
    return G.csr_from_dense(W)


def special_x(n, P, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, P)).astype(np.float32)
    X[rng.integers(0, n, 3), rng.integers(0, P, 3)] = np.nan
    X[rng.integers(0, n, 3), rng.integers(0, P, 3)] = np.inf
    X[rng.integers(0, n, 3), rng.integers(0, P, 3)] = -np.inf
    X[rng.integers(0, n, 5), rng.integers(0, P, 5)] = -0.0
    X[rng.integers(0, n, 5), rng.integers(0, P, 5)] = 3e38
    X[rng.integers(0, n, 5), rng.integers(0, P, 5)] = 1e-40  # denormal
    return X


def bank_like(X, gpu, ld):
    n, P = X.shape
    t = torch.full((n, ld), float("nan"), dtype=torch.float32, device=gpu)
    t[:, :P] = torch.from_numpy(X).to(gpu)
    return t


@pytest.mark.parametrize("n,P,p,ld_extra", [
    (64, 1000, 0.3, 0),
    (70, 257, 0.5, 3),       # x_rows % 64 != 0, rows % 16 != 0, a partial last lane, ld % 4 == 0
    (300, 4099, 0.1, 1),     # P % 4 != 0 (ld rounded up to a multiple of 4)
    (1024, 2560, 0.1, 0),
    (512, 700, 0.9, 0),      # over-full index blocks: the global-memory index path
    (100, 1024, 1.0, 0),     # the complete graph
])
def test_slab_mix_matches_oracle(n, P, p, ld_extra, gpu):
    csr = er_csr(n, p, seed=n + P, empty_rows=(1, n - 1))
    plan = G.MixingPlan(csr, gpu, slab=True)
    assert plan.kind == "csr" and plan.ent is not None
    X = special_x(n, P, seed=P)
    ld = -(-(P + ld_extra) // 4) * 4
    Xd, Yd = bank_like(X, gpu, ld), bank_like(np.zeros_like(X), gpu, ld)
    assert ops.slab_layout_ok(Xd, Yd, P)
    plan.apply(Xd, Yd, P=P)
    Yg = torch.empty_like(Yd)
    ops.mix_csr(Xd, Yg, plan.rowptr, plan.col, plan.val, P=P)  # the generic kernel
    torch.cuda.synchronize()
    want = oracle.mix_csr(X, csr.rowptr, csr.col, csr.val)
    got = Yd[:, :P].cpu().numpy()
    assert bits_equal(got, want)
    assert bits_equal(Yg[:, :P].cpu().numpy(), got)
    assert torch.isnan(Yd[:, P:]).all(), "wrote past P"


def test_slab_rectangular_and_low_degree_rows(gpu):
    """More X rows than Y rows (a column block of agents), rows of degree 0, 1
    and every column, neighbours confined to one chunk or spread over all."""
    n, m, P = 40, 200, 512
    rng = np.random.default_rng(5)
    W = np.zeros((n, m), np.float32)
    W[0, :] = rng.random(m).astype(np.float32) + 0.1      # every column
    W[1, 130] = 0.5                                        # degree 1, chunk 2
    W[3, 64:128] = 0.25                                    # one whole chunk
    W[4:, :] = (rng.random((n - 4, m)) < 0.2) * rng.random((n - 4, m)).astype(np.float32)
    W[2, :] = 0.0                                          # empty row
    csr = G.csr_from_dense(W)
    plan = G.MixingPlan(csr, gpu, slab=True)
    plan.n_cols = m
    X = special_x(m, P, seed=9)
    Xd, Yd = bank_like(X, gpu, P), bank_like(np.zeros((n, P), np.float32), gpu, P)
    ops.mix_csr_slab(Xd, Yd, plan.ent, plan.hdr, n, x_rows=m, P=P)
    torch.cuda.synchronize()
    assert bits_equal(Yd.cpu().numpy(), oracle.mix_csr(X, csr.rowptr, csr.col, csr.val))


def slab_pack_host(csr, x_rows):
    """Host restatement of dol_csr_slab_pack: rows in groups of SLAB_ROWS; for
    group g, chunk k the rows' chunk-k entries contiguous in (row, column)
    order, each row's segment padded to an even length with a pad entry (offset
    SLAB_ZERO_OFFSET = the stage's zero piece, weight 0); entry = (LDS byte
    offset (col % 64) * 1024, weight bits); entries stored in PAIRS as (offset
    0, offset 1, weight 0, weight 1); header word = segment start | (1 if
    padded).  Returns (hdr, entries as an [n, 2] (offset, weight) array)."""
    R, C = ops.SLAB_ROWS, ops.SLAB_CHUNK
    nk = -(-x_rows // C)
    n_rg = -(-csr.n_rows // R)
    hdr = np.zeros((n_rg, nk, R + 1), np.int64)
    ent = []
    for g in range(n_rg):
        for k in range(nk):
            for i in range(R + 1):
                hdr[g, k, i] = len(ent)
                r = g * R + i
                if i == R or r >= csr.n_rows:
                    continue
                cols = csr.col[csr.rowptr[r]:csr.rowptr[r + 1]]
                vals = csr.val[csr.rowptr[r]:csr.rowptr[r + 1]]
                sel = (cols >= k * C) & (cols < (k + 1) * C)
                for c, v in zip(cols[sel], vals[sel]):
                    ent.append(((int(c) % C) * 1024, int(np.float32(v).view(np.int32))))
                if sel.sum() % 2:
                    ent.append((SLAB_ZERO_OFFSET, 0))
                    hdr[g, k, i] |= 1
    return hdr, np.array(ent, np.int64).reshape(-1, 2)


SLAB_ZERO_OFFSET = 64 * 1024  # csr_slab.hip kZeroRel: the zero piece after each 64-KiB X stage


@pytest.mark.parametrize("n,p", [(200, 0.2), (300, 0.05)])
def test_slab_pack_matches_host(n, p, gpu):
    csr = er_csr(n, p, seed=3, empty_rows=(7,))
    plan = G.MixingPlan(csr, gpu, slab=True)
    hdr, ent = slab_pack_host(csr, n)
    got_h = plan.hdr[: hdr.size].cpu().numpy().reshape(hdr.shape)
    assert np.array_equal(got_h, hdr)
    pairs = plan.ent[: 2 * len(ent)].cpu().numpy().reshape(-1, 4)  # (off0, off1, w0, w1)
    got_e = np.stack([pairs[:, [0, 1]].reshape(-1), pairs[:, [2, 3]].reshape(-1)], axis=1)
    assert np.array_equal(got_e, ent)


@pytest.mark.parametrize("n,p", [(1024, 0.1), (333, 0.5)])
def test_dense_to_csr_on_device(n, p, gpu):
    W = G.erdos_renyi_stochastic_hip(n, p, seed=77, device=gpu)
    W[5, :] = float("nan")   # a NaN row (Neighbors drops NaN)
    W[6, :7] = -1.0          # negatives dropped
    rowptr, col, val = ops.dense_to_csr(W)
    torch.cuda.synchronize()
    host = G.csr_from_dense(W.cpu())
    nnz = int(rowptr[-1].item())
    assert nnz == host.nnz
    assert np.array_equal(rowptr.cpu().numpy(), host.rowptr)
    assert np.array_equal(col[:nnz].cpu().numpy(), host.col)
    assert bits_equal(val[:nnz].cpu().numpy(), host.val)


def test_from_dense_csr_plan_reuse_and_mix(gpu):
    """Config 5's per-round path: W drawn on the device, Neighbors on the
    device, LDS-gather mix; two rounds reuse the first plan's buffers."""
    n, P = 512, 3000
    X = special_x(n, P, seed=1)
    ld = 3008
    Xd, Yd = bank_like(X, gpu, ld), bank_like(np.zeros_like(X), gpu, ld)
    plan = None
    for rnd in range(2):
        W = G.erdos_renyi_stochastic_hip(n, 0.1, seed=1000 + rnd, device=gpu)
        prev = plan
        plan = G.MixingPlan.from_dense(W, dense_kernel="csr", reuse=plan)
        if prev is not None:  # the lender is retired: its buffers now hold this round's W
            assert prev.kind == "stale"
            with pytest.raises(RuntimeError, match="lent its buffers"):
                prev.apply(Xd, Yd, P=P)
        plan.apply(Xd, Yd, P=P)
        torch.cuda.synchronize()
        host = G.csr_from_dense(W.cpu())
        assert bits_equal(Yd[:, :P].cpu().numpy(), oracle.mix_csr(X, host.rowptr, host.col, host.val))


def test_slab_full_size_config5(gpu):
    """1024 agents x 101,770 (config 5's MLP), ER p = 0.1: bit-identical to the
    generic CSR kernel everywhere and to the oracle on sampled rows."""
    from dolhip.bank import row_stride
    n, P = 1024, 101770
    ld = row_stride(P)
    W = G.erdos_renyi_stochastic_hip(n, 0.1, seed=2028, device=gpu)
    plan = G.MixingPlan.from_dense(W, dense_kernel="csr")
    g = torch.Generator(device=gpu).manual_seed(3)
    Xd = torch.empty(n, ld, device=gpu).normal_(generator=g)
    Yd, Yg = torch.empty_like(Xd), torch.empty_like(Xd)
    plan.apply(Xd, Yd, P=P)
    ops.mix_csr(Xd, Yg, plan.rowptr, plan.col, plan.val, P=P)
    torch.cuda.synchronize()
    assert torch.equal(Yd[:, :P].view(torch.int32), Yg[:, :P].view(torch.int32))
    host = G.csr_from_dense(W.cpu())
    rows = np.array([0, 1, 511, 777, 1023])
    sub = G.CSR(len(rows), n, np.concatenate([[0], np.cumsum(np.diff(host.rowptr)[rows])]).astype(np.int32),
                np.concatenate([host.col[host.rowptr[r]:host.rowptr[r + 1]] for r in rows]),
                np.concatenate([host.val[host.rowptr[r]:host.rowptr[r + 1]] for r in rows]))
    cols = slice(P - 5000, P)
    Xs = Xd[:, cols].cpu().numpy()
    assert bits_equal(Yd[rows][:, cols].cpu().numpy(), oracle.mix_csr(Xs, sub.rowptr, sub.col, sub.val))


def test_slab_8192_agents(gpu):
    n, P = 8192, 1024
    W = G.erdos_renyi_stochastic_hip(n, 0.1, seed=11, device=gpu)
    plan = G.MixingPlan.from_dense(W, dense_kernel="csr")
    g = torch.Generator(device=gpu).manual_seed(4)
    Xd = torch.empty(n, P, device=gpu).normal_(generator=g)
    Yd, Yg = torch.empty_like(Xd), torch.empty_like(Xd)
    plan.apply(Xd, Yd)
    ops.mix_csr(Xd, Yg, plan.rowptr, plan.col, plan.val)
    torch.cuda.synchronize()
    assert torch.equal(Yd.view(torch.int32), Yg.view(torch.int32))
