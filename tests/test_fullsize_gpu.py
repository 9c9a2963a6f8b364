"""Parity at the sizes bench.py times (BASELINE config 4's 8192 agents x 2^20
params), in the bench's own buffer geometry, for the kernels whose bench claims
were only checked at smaller shapes before round 3:

* the parameter-major CSR mix (csr_pm_kernel, five 32-KiB LDS-DMA buffers
  beyond 4096 agents) on random 4-regular W, XT = [2^20, 8192] with ld = 8192
  exactly like bench.random_regular_pm_round: every element bit-identical to
  the agent-major CSR kernel (itself pinned to the oracle), sampled p-rows and
  whole p-row ranges at the stage-segment boundaries bit-exact vs the oracle,
  and the column-sum identity in fp64 on every p-row;
* the FedADMM least-squares client round + server mean (admm_ls_round_kernel +
  the ordered mean, "fast" and "exact") over all 8192 agents with 10 local
  momentum-SGD steps, two rounds (first step ever, then continuing momentum):
  every row at sampled columns (the round is elementwise per column) and
  sampled rows at every column bit-exact vs oracle.admm_ls_round, theta on the
  sampled columns vs oracle.ordered_mean;
* FedLCon's eps = 5 fused pass (ring_steps_kernel) and the headline ring round
  in ShardedRing's buffers (ld = row_stride(2^20)): every row on contiguous
  column ranges (start, end, interior, tile-straddling) bit-exact vs 5 / 1
  oracle rounds.

Reference semantics: DIST/clients.py:61-69 (consensus), DIST/simulators.py:
190-196 (FedLCon eps loop), DEC/clients.py:36-53,125-144 (update_weights,
update_model, update_duals), DEC/servers.py:42-48 (average_weights)."""
import gc

import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from dolhip import graph as G
from dolhip import ops

pytestmark = pytest.mark.gpu

N, P = 8192, 1 << 20


def _free():
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _csr_dev(c, gpu):
    return (torch.as_tensor(np.asarray(c.rowptr, np.int32), device=gpu),
            torch.as_tensor(np.asarray(c.col, np.int32), device=gpu),
            torch.as_tensor(np.asarray(c.val, np.float32), device=gpu))


def _equal_chunked(a, b, what):
    for p0 in range(0, a.shape[0], 1 << 16):
        assert torch.equal(a[p0:p0 + (1 << 16)].view(torch.int32), b[p0:p0 + (1 << 16)].view(torch.int32)), \
            f"{what}: rows {p0}.."


def test_pm_mix_8192_full_size(gpu):
    """Every stage order ops.PM_STAGE_ORDERS offers (what the product path's
    tuner may pick for these buffers) and the tuned call itself give the same
    bits; those bits are checked against the oracle and the agent-major kernel."""
    c = G.random_regular_csr(N, 4, seed=2028)  # bench.random_regular_pm_round's W
    rp, col, val = _csr_dev(c, gpu)
    g = torch.Generator(device=gpu).manual_seed(17)
    XT = torch.empty(P, N, device=gpu).normal_(generator=g)  # ld = N = 8192, the bench's view
    YT = torch.empty_like(XT)
    ops.mix_csr_pm(XT, YT, rp, col, val, nseg=ops.PM_STAGE_ORDERS[0])
    torch.cuda.synchronize()
    Yk = torch.empty_like(XT)
    for nseg in ops.PM_STAGE_ORDERS[1:] + (None,):
        Yk.fill_(float("nan"))
        ops.mix_csr_pm(XT, Yk, rp, col, val, nseg=nseg)
        torch.cuda.synchronize()
        _equal_chunked(Yk, YT, f"stage order {nseg} vs {ops.PM_STAGE_ORDERS[0]}")
    del Yk
    _free()
    # (1) sampled p-rows and whole p-row ranges at the 8 stage segments' starts
    #     and ends (XCD x walks segment x) vs the oracle
    seg = P // 8
    rows = np.unique(np.concatenate([
        np.random.default_rng(3).choice(P, 48, replace=False),
        np.arange(0, 6), np.arange(P - 6, P),
        *[np.arange(s * seg - 3, s * seg + 3) for s in range(1, 8)]]))
    ridx = torch.as_tensor(rows, device=gpu)
    want = oracle.mix_csr(np.ascontiguousarray(XT[ridx].cpu().numpy().T), c.rowptr, c.col, c.val)
    assert bits_equal(YT[ridx].cpu().numpy().T, want)
    # (2) column-sum identity on every p-row (fp64, chunked)
    colsum = np.zeros(N, np.float64)
    np.add.at(colsum, c.col, c.val.astype(np.float64))
    cs = torch.as_tensor(colsum, device=gpu)
    for p0 in range(0, P, 1 << 16):
        lhs = YT[p0:p0 + (1 << 16)].double().sum(1)
        rhs = XT[p0:p0 + (1 << 16)].double() @ cs
        torch.testing.assert_close(lhs, rhs, rtol=1e-5, atol=1e-6 * float(rhs.abs().max()))
    # (3) every element vs the agent-major CSR kernel (bit-exact vs the oracle
    #     in test_kernels_gpu / test_full_size_random_regular_sampled_rows)
    X = torch.empty(N, P, device=gpu)
    ops.transpose(XT, X, P, N)
    del XT
    _free()
    Y = torch.empty(N, P, device=gpu)
    ops.mix_csr(X, Y, rp, col, val)
    del X
    _free()
    YT2 = torch.empty(P, N, device=gpu)
    ops.transpose(Y, YT2, N, P)
    torch.cuda.synchronize()
    del Y
    _free()
    for p0 in range(0, P, 1 << 16):
        a, b = YT[p0:p0 + (1 << 16)], YT2[p0:p0 + (1 << 16)]
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), f"p-rows {p0}.."
    del YT, YT2
    _free()


@pytest.mark.parametrize("mean", ["fast", "exact"])
def test_admm_ls_round_8192_full_size(mean, gpu):
    """bench.primal_dual_round's problem: SeparableADMM(8192, 2^20, rho 0.1,
    lr 0.1, momentum 0.5, 10 local steps, frac 1, seed 2028)."""
    from dolhip.synthetic import SeparableADMM
    rho, lr, mu, steps = 0.1, 0.1, 0.5, 10
    prob = SeparableADMM(N, P, rho=rho, lr=lr, momentum=mu, local_steps=steps, frac=1.0, seed=2028,
                         device=gpu, mean=mean)
    cols = np.unique(np.concatenate([np.random.default_rng(5).choice(P, 56, replace=False),
                                     [0, 1, 2, 3, P - 4, P - 3, P - 2, P - 1]]))
    cidx = torch.as_tensor(cols, device=gpu)
    rows = np.unique(np.concatenate([[0, 1, N // 2, N - 1], np.random.default_rng(6).choice(N, 8, replace=False)]))
    ridx = torch.as_tensor(rows, device=gpu)
    T_c = prob.target[:N][:, cidx].cpu().numpy()
    T_r = prob.target[ridx][:, :P].cpu().numpy()
    for rnd in range(2):
        first = (~prob.mom_started[:N]).astype(np.int32)
        th = prob.theta[:P].cpu().numpy()
        snap_c = [t[:N][:, cidx].cpu().numpy() for t in (prob.w, prob.mom, prob.alpha)]
        snap_r = [t[ridx][:, :P].cpu().numpy() for t in (prob.w, prob.mom, prob.alpha)]
        order = prob.sample()
        prob.round(order=order)
        torch.cuda.synchronize()
        # every agent on the sampled columns: the client round, then the mean
        w1, b1, a1, _, _ = oracle.admm_ls_round(snap_c[0], snap_c[1], snap_c[2], T_c, th[cols], order, first[order],
                                                rho, lr, mu, steps)
        assert bits_equal(prob.w[:N][:, cidx].cpu().numpy(), w1), f"round {rnd}: w on sampled columns"
        assert bits_equal(prob.mom[:N][:, cidx].cpu().numpy(), b1), f"round {rnd}: momentum"
        assert bits_equal(prob.alpha[:N][:, cidx].cpu().numpy(), a1), f"round {rnd}: alpha"
        assert bits_equal(prob.theta[cidx].cpu().numpy(), oracle.ordered_mean(w1, order)), f"round {rnd}: theta"
        # sampled agents on every column (the kernel's column chunks)
        loc = np.arange(len(rows), dtype=np.int32)
        w1, b1, a1, rw, ra = oracle.admm_ls_round(snap_r[0], snap_r[1], snap_r[2], T_r, th, loc, first[rows],
                                                  rho, lr, mu, steps)
        assert bits_equal(prob.w[ridx][:, :P].cpu().numpy(), w1), f"round {rnd}: sampled rows w"
        assert bits_equal(prob.mom[ridx][:, :P].cpu().numpy(), b1), f"round {rnd}: sampled rows momentum"
        assert bits_equal(prob.alpha[ridx][:, :P].cpu().numpy(), a1), f"round {rnd}: sampled rows alpha"
        assert prob.mom_started[:N].all()
    h = prob.history
    assert len(h) == 2 and all(np.isfinite(e["primal_resid_sq"]) for e in h)
    del prob
    _free()


def _ring_buffers(gpu):
    """bench.main's buffers: ShardedRing(8192, 2^20) at world 1, ld = row_stride(P)."""
    from dolhip.parallel import ShardedRing
    torch.manual_seed(2028)
    rw = G.communication_csr("circle", "stochastic", N)[0].ring_weights()
    ring = ShardedRing(N, P, rw[0], rw[1], gpu)
    ring.x.normal_(generator=torch.Generator(device=gpu).manual_seed(2029))
    ring.y.zero_()
    return ring, rw


# contiguous column ranges: the first and last, one straddling the 2^19
# midpoint, one at an odd 16-B offset, and one ragged to a non-multiple of 64
COL_RANGES = [(0, 2048), (P - 2048, P), ((1 << 19) - 1000, (1 << 19) + 1000), (123_456, 125_504), (777_004, 777_672)]


def _check_cols(X0, Y, wp, wn, rounds):
    for c0, c1 in COL_RANGES:
        x = X0[:N, c0:c1].cpu().numpy()
        for _ in range(rounds):
            x = oracle.mix_ring(x, wp, wn)
        assert bits_equal(Y[:N, c0:c1].cpu().numpy(), x), f"columns {c0}:{c1}"


def test_ring_headline_round_8192_full_size(gpu):
    ring, (wp, wn) = _ring_buffers(gpu)
    x0 = ring.x
    ring.step()
    torch.cuda.synchronize()
    _check_cols(x0, ring.x, wp, wn, 1)
    del ring, x0
    _free()


@pytest.mark.parametrize("variant", list(ops.RING_STEPS_VARIANTS))
def test_fedlcon_eps5_pass_8192_full_size(variant, gpu):
    """Each kernel the product path's tuner may pick (ops.RING_STEPS_VARIANTS)
    at the bench's geometry: 2^33 elements, ld = row_stride(2^20)."""
    ring, (wp, wn) = _ring_buffers(gpu)
    ring.y.fill_(float("nan"))
    ops.mix_ring_steps(ring.x, ring.y, ring.w_prev, ring.w_next, 5, P=P, n_rows=N, variant=variant)
    torch.cuda.synchronize()
    _check_cols(ring.x, ring.y, wp, wn, 5)
    # sampled rows at every column: each output row depends on 11 input rows
    for i in [0, 3, 4095, 4096, N - 5, N - 1] + list(np.random.default_rng(7).integers(0, N, 6)):
        i = int(i)
        idx = [(i + d) % N for d in range(-5, 6)]
        x = ring.x[torch.as_tensor(idx, device=gpu)][:, :P].cpu().numpy()
        # the 11-row window as a chain with the ring's weights; row k of the
        # window is agent idx[k], valid rows shrink by one per round
        for r in range(5):
            y = np.zeros_like(x)
            for k in range(r + 1, 10 - r):
                a = idx[k]
                # ascending agent order (DIST/clients.py:61-69 over Neighbors' ascending j)
                terms = sorted([((a - 1) % N, x[k - 1], wp[a]), ((a + 1) % N, x[k + 1], wn[a])], key=lambda t: t[0])
                acc = np.zeros(P, np.float32)
                for _j, xv, wv in terms:
                    acc = (acc + (xv * np.float32(wv)).astype(np.float32)).astype(np.float32)
                y[k] = acc
            x = y
        assert bits_equal(ring.y[i, :P].cpu().numpy(), x[5]), f"row {i}"
    del ring
    _free()


def test_fedlcon_eps5_product_path_8192_full_size(gpu):
    """The call FedLCon.run makes (weighted_average/simulators.py:233 ->
    AgentBank.mix(plan, steps=5) -> MixingPlan.apply_steps -> ops.mix_ring_steps
    with the kernel tuned for the bank's buffers): the same bits as every
    variant, and the tuning is recorded for those buffers."""
    from dolhip.bank import AgentBank
    ring, (wp, wn) = _ring_buffers(gpu)
    torch.manual_seed(2028)
    plan = G.MixingPlan(G.communication_csr("circle", "stochastic", N)[0], gpu)
    assert plan.kind == "ring"
    bank = AgentBank(N, P, gpu, ld=ring.x.stride(0))
    bank.adopt("x", ring.x)
    bank.adopt("y", ring.y)
    x0 = ring.x
    want = torch.empty_like(x0)
    ops.mix_ring_steps(x0, want, ring.w_prev, ring.w_next, 5, P=P, n_rows=N, variant=ops.RING_STEPS_VARIANTS[0])
    bank.mix(plan, steps=5)
    torch.cuda.synchronize()
    # Jacobi swap: the pass wrote "y" -- ring.y, or a fresh destination when the
    # bank's destination check found the (x, y) pair a slow one
    assert bank.x.data_ptr() != x0.data_ptr()
    if len(bank.pair_probes) <= 1:
        assert bank.x.data_ptr() == ring.y.data_ptr()
    _equal_chunked(bank.x, want, "bank.mix(plan, 5) vs the tile kernel")
    keys = [k for k in ops.tuned_choices() if "ring_steps" in k]
    assert ops.autotune_enabled() and keys, "the product call did not tune the eps kernel"
    del ring, bank, plan, x0, want
    _free()
