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


@pytest.fixture(params=ops.SLAB_VARIANTS)
def slab_variant(request):
    """Every slab test runs under each kernel variant (dol_slab_set_variant)."""
    prev = ops.slab_variant(request.param)
    yield request.param
    ops.slab_variant(prev)


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
def test_slab_mix_matches_oracle(n, P, p, ld_extra, gpu, slab_variant):
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


def test_slab_rectangular_and_low_degree_rows(gpu, slab_variant):
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


def slab_balance_host(counts):
    """Host restatement of slab_balance_kernel for one row group: counts[i, k]
    = padded entries of row i in chunk k.  Rows by total (descending, ties by
    index), each to the wave (< RW rows) minimising sum_k c_k (2 L_wk + c_k)
    (ties: lowest wave); slot = wave * RW + the wave's fill.  Returns slot[i]."""
    R, WV = counts.shape[0], 16
    RW = R // WV
    tot = counts.sum(1)
    order = sorted(range(R), key=lambda i: (-tot[i], i))
    L = np.zeros((WV, counts.shape[1]), np.int64)
    fill = np.zeros(WV, np.int64)
    slot = np.zeros(R, np.int64)
    for i in order:
        c = counts[i].astype(np.int64)
        cost = [(int((c * (2 * L[w] + c)).sum()), w) for w in range(WV) if fill[w] < RW]
        w = min(cost)[1]
        slot[i] = w * RW + fill[w]
        fill[w] += 1
        L[w] += c
    return slot


def slab_pack_host(csr, x_rows, balance=False):
    """Host restatement of dol_csr_slab_pack: rows in groups of SLAB_ROWS, dealt
    to slots by slab_balance_host (balance) or in row order; for group g, chunk k the slots' chunk-k
    entries contiguous in (slot, column) order, each segment padded to an even
    length with a pad entry (offset SLAB_ZERO_OFFSET = the stage's zero piece,
    weight 0); entry = (LDS byte offset (col % 64) * 1024, weight bits); entries
    stored in PAIRS as (weight 0, offset 0, weight 1, offset 1); header word =
    segment start | (1 if padded); then perm[g][slot] = row (-1: none) and
    inv[row] = slot.  Returns (hdr blocks, entries as an [n, 2] (offset, weight)
    array, perm, inv)."""
    R, C = ops.SLAB_ROWS, ops.SLAB_CHUNK
    nk = -(-x_rows // C)
    n_rg = -(-csr.n_rows // R)
    hdr = np.zeros((n_rg, nk, R + 1), np.int64)
    perm = np.full((n_rg, R), -1, np.int64)
    inv = np.zeros(n_rg * R, np.int64)
    ent = []
    for g in range(n_rg):
        sel_rows = {}
        counts = np.zeros((R, nk), np.int64)
        for i in range(R):
            r = g * R + i
            if r < csr.n_rows:
                cols = csr.col[csr.rowptr[r]:csr.rowptr[r + 1]]
                for k in range(nk):
                    n = int(((cols >= k * C) & (cols < (k + 1) * C)).sum())
                    counts[i, k] = n + (n & 1)
        slot = slab_balance_host(counts) if balance else np.arange(R)
        for i in range(R):
            r = g * R + i
            if r < csr.n_rows:
                perm[g, slot[i]] = r
                inv[r] = slot[i]
        for k in range(nk):
            for sl in range(R + 1):
                hdr[g, k, sl] = len(ent)
                r = perm[g, sl] if sl < R else -1
                if r < 0:
                    continue
                cols = csr.col[csr.rowptr[r]:csr.rowptr[r + 1]]
                vals = csr.val[csr.rowptr[r]:csr.rowptr[r + 1]]
                sel = (cols >= k * C) & (cols < (k + 1) * C)
                for c, v in zip(cols[sel], vals[sel]):
                    ent.append(((int(c) % C) * 1024, int(np.float32(v).view(np.int32))))
                if sel.sum() % 2:
                    ent.append((SLAB_ZERO_OFFSET, 0))
                    hdr[g, k, sl] |= 1
    return hdr, np.array(ent, np.int64).reshape(-1, 2), perm, inv[:csr.n_rows]


SLAB_ZERO_OFFSET = 64 * 1024  # csr_slab.hip kZeroRel: the zero piece after each 64-KiB X stage


@pytest.mark.parametrize("balance", [False, True])
@pytest.mark.parametrize("n,p", [(200, 0.2), (300, 0.05), (1024, 0.1),
                                 (2000, 0.05),    # 32 chunks: the 64-chunk register packing kernel
                                 (4200, 0.01)])   # 66 chunks: the LDS packing kernel
def test_slab_pack_matches_host(n, p, balance, gpu):
    csr = er_csr(n, p, seed=3, empty_rows=(7,))
    plan = G.MixingPlan(csr, gpu, slab=True)
    rp, col, val = (torch.as_tensor(a, device=gpu) for a in (csr.rowptr, csr.col, csr.val))
    ent_d, hdr_d = ops.csr_slab_pack(rp, col, val, n, balance=balance)
    hdr, ent, perm, inv = slab_pack_host(csr, n, balance)
    H = hdr_d.cpu().numpy()
    nb = hdr.size
    assert np.array_equal(H[:nb].reshape(hdr.shape), hdr)
    assert np.array_equal(H[nb:nb + perm.size].reshape(perm.shape), perm)
    assert np.array_equal(H[nb + perm.size:nb + perm.size + n], inv)
    pairs = ent_d[: 2 * len(ent)].cpu().numpy().reshape(-1, 4)  # (w0, off0, w1, off1)
    got_e = np.stack([pairs[:, [1, 3]].reshape(-1), pairs[:, [0, 2]].reshape(-1)], axis=1)
    assert np.array_equal(got_e, ent)
    # r06: pad entries right after the last block (the stream kernel reads up to two pairs past a run)
    tail = ent_d[2 * len(ent): 2 * len(ent) + 16].cpu().numpy().reshape(-1, 2)
    assert np.array_equal(tail, np.tile([0, SLAB_ZERO_OFFSET], (8, 1)))


@pytest.mark.parametrize("n,P,p", [(1024, 2560, 0.1), (300, 1001, 0.3)])
def test_slab_balanced_pack_mixes_bit_exactly(n, P, p, gpu, slab_variant):
    """Rows dealt to waves by the greedy packing: the same sums in the same
    order, so the same bits as the row-order packing and the oracle."""
    csr = er_csr(n, p, seed=n + 7, empty_rows=(2,))
    rp, col, val = (torch.as_tensor(a, device=gpu) for a in (csr.rowptr, csr.col, csr.val))
    ent, hdr = ops.csr_slab_pack(rp, col, val, n, balance=True)
    X = special_x(n, P, seed=P + 1)
    ld = -(-P // 4) * 4
    Xd, Yd = bank_like(X, gpu, ld), bank_like(np.zeros_like(X), gpu, ld)
    ops.mix_csr_slab(Xd, Yd, ent, hdr, n, x_rows=n, P=P)
    torch.cuda.synchronize()
    assert bits_equal(Yd[:, :P].cpu().numpy(), oracle.mix_csr(X, csr.rowptr, csr.col, csr.val))


def test_slab_balancing_evens_the_chunk_loads():
    """The balancing's point (host restatement, the kernel is pinned to it
    above): at ER p = 0.1, 1024 agents, the sum over chunks of the busiest
    wave's entries drops well below row-order dealing."""
    rng = np.random.default_rng(1)
    n, R, C, WV = 1024, ops.SLAB_ROWS, ops.SLAB_CHUNK, 16
    A = rng.random((n, n)) < 0.1
    np.fill_diagonal(A, False)
    cnt = A.reshape(n, n // C, C).sum(2)
    cnt = cnt + (cnt & 1)
    natural = balanced = 0
    for g in range(n // R):
        c = cnt[g * R:(g + 1) * R]
        natural += c.reshape(WV, R // WV, -1).sum(1).max(0).sum()
        slot = slab_balance_host(c)
        L = np.zeros((WV, c.shape[1]), np.int64)
        for i in range(R):
            L[slot[i] // (R // WV)] += c[i]
        balanced += L.max(0).sum()
    assert balanced < 0.93 * natural


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


def test_slab_full_size_config5(gpu, slab_variant):
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


def test_slab_8192_agents(gpu, slab_variant):
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


@pytest.mark.parametrize("balance", [False, True])
def test_from_dense_plan_balanced_or_not_mixes_bit_exactly(balance, gpu):
    """MixingPlan.from_dense(W, 'csr', balance=...): the device-built plan, with
    or without the wave-balanced pack (TimeVaryingMLPGossip packs balanced on
    its side stream), gives the oracle's bits."""
    n, P = 300, 1001
    csr = er_csr(n, 0.2, seed=11)
    W = np.zeros((n, n), np.float32)
    for i in range(n):
        W[i, csr.col[csr.rowptr[i]:csr.rowptr[i + 1]]] = csr.val[csr.rowptr[i]:csr.rowptr[i + 1]]
    plan = G.MixingPlan.from_dense(torch.as_tensor(W, device=gpu), dense_kernel="csr", balance=balance)
    X = special_x(n, P, seed=5)
    ld = -(-P // 4) * 4
    Xd, Yd = bank_like(X, gpu, ld), bank_like(np.zeros_like(X), gpu, ld)
    plan.apply(Xd, Yd, P=P)
    torch.cuda.synchronize()
    assert bits_equal(Yd[:, :P].cpu().numpy(), oracle.mix_csr(X, csr.rowptr, csr.col, csr.val))
