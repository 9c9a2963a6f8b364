"""Bank buffers in one mapped physical allocation (dol_bank_alloc /
dol_bank_free through bank.device_matrix): usable by torch and by the kernels
like any device tensor, same bits as a torch-allocated buffer, freed with the
last tensor that references it."""
import gc

import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from dolhip import bank as B
from dolhip import ops

pytestmark = pytest.mark.gpu


def test_mapped_matrix_round_trip_and_mix(gpu, monkeypatch):
    monkeypatch.setattr(B, "MAPPED_MIN_BYTES", 0)
    monkeypatch.setenv("DOL_BANK_ALLOC", "vmm")
    n, P = 37, 4100
    X = B.device_matrix(n, P + 60, gpu)
    Y = B.device_matrix(n, P + 60, gpu, zero=True)
    assert X.device == gpu and X.dtype == torch.float32 and X.is_contiguous()
    assert float(Y.abs().sum()) == 0.0
    rng = np.random.default_rng(3)
    Xh = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    X[:, :P] = torch.from_numpy(Xh).to(gpu)
    ops.mix_ring(X, Y, torch.from_numpy(wp).to(gpu), torch.from_numpy(wn).to(gpu), P=P)
    torch.cuda.synchronize()
    assert bits_equal(Y[:, :P].cpu().numpy(), oracle.mix_ring(Xh, wp, wn))
    view = X[3:5, 10:20]  # a view keeps the block alive after X is gone
    want = view.cpu().clone()
    del X
    gc.collect()
    assert torch.equal(view.cpu(), want)
    del view, Y
    gc.collect()
    torch.cuda.synchronize()


def _remap_cycle(gpu, n, P, plan_csr, k, check):
    """One cycle of the r04 fault's sequence on fresh exact-size mapped blocks:
    map X / Y / T / M, fill them with torch (normal_ / zero_), run every bank
    kernel on the LAST rows (row views ending at the block's last byte), free."""
    ld = B.row_stride(P)
    assert (n * ld * 4) % (2 << 20) == 0  # the data ends exactly where the mapping ends
    X, Y, T, M = (B.device_matrix(n, ld, gpu, mapped=True) for _ in range(4))
    g = torch.Generator(device=gpu).manual_seed(100 + k)
    X.normal_(generator=g)
    T.normal_(generator=g)
    M.zero_()
    Y.zero_()
    w = torch.rand(n, generator=g, device=gpu)
    wn = 1.0 - w
    rp, col, val = plan_csr
    # config 3's DGD rounds (ring, then random-regular CSR), first step then continuing momentum
    for first in (True, False):
        ops.dgd_ring(X, Y, w, wn, T, mom=M, steps=2, lr=0.01, momentum=0.5, first_step=first, P=P)
        ops.dgd_csr(Y, X, rp, col, val, T, mom=M, steps=1, lr=0.01, momentum=0.5, first_step=False, P=P)
    # the last rows as a sharded block: interior mix with halo rows + both edges
    t = 3
    hp, hn = X[n - t - 1, :P].contiguous(), X[0, :P].contiguous()
    ops.mix_ring(X[n - t:], Y[n - t:], w[n - t:], wn[n - t:], halo_prev=hp, halo_next=hn, P=P)
    ops.mix_ring_edges(X[n - t:], Y[n - t:], w[n - t:], wn[n - t:], hp, hn, P=P)
    # FedLCon's eps pass under every kernel the tuner may pick, the ordered mean, the ADMM / dual / prox updates
    P4 = P // 4 * 4
    for v in ops.RING_STEPS_VARIANTS:
        ops.mix_ring_steps(X, Y, w, wn, 5, P=P4, n_rows=n, variant=v)
    order = torch.arange(n - 1, n - 9, -1, dtype=torch.int32, device=gpu)
    theta = ops.ordered_mean(X, order, P=P)
    ops.admm_ls_round(X, M, T, theta, agents=order, first=torch.zeros(8, dtype=torch.int32, device=gpu), buf=Y,
                      rho=0.1, lr=0.1, momentum=0.5, local_steps=2, P=P)
    ops.admm_dual(M[n - 2:], X[n - 2:], theta, 0.1, P=P)
    ops.prox_admm_sgd(X[n - 2:], T[n - 2:], buf=Y[n - 2:], theta=theta, alpha=M[n - 2:], rho=0.1, lr=0.1,
                      momentum=0.5, first_step=False, P=P)
    torch.cuda.synchronize()
    if check:  # the last row's mix after everything above, against the oracle
        Xl = X[n - 3:, :P].cpu().numpy()
        ops.mix_ring(X[n - 3:], Y[n - 3:], w[n - 3:], wn[n - 3:], halo_prev=hp, halo_next=hn, P=P)
        torch.cuda.synchronize()
        want = oracle.mix_ring(Xl, w[n - 3:].cpu().numpy(), wn[n - 3:].cpu().numpy(), hp.cpu().numpy(),
                               hn.cpu().numpy())
        assert bits_equal(Y[n - 3:, :P].cpu().numpy(), want)
    del X, Y, T, M, hp, hn, theta
    gc.collect()
    torch.cuda.synchronize()


def test_mapped_blocks_survive_map_free_remap_cycles(gpu):
    """the r04k fault came after a process had mapped and
    freed seven 4 GiB dol_bank_alloc blocks.  Twelve cycles of exact-size
    mapped blocks (512 rows x (2^20 - 5) floats, ld 2^20 + 2048: 2 GiB + 4 MiB
    each, ending on the mapping's last byte) with every bank kernel on their
    last rows, freed and re-mapped each cycle, the last rows' mix checked
    against the oracle every cycle.  With the freed virtual ranges handed out
    again (the r04 dol_bank_free, DOL_BANK_FREE_VA=1) this failed from cycle 1
    on (profiles/r05c_vmm_remap_probe.jsonl: 7 of 11 re-mapped cycles wrong);
    dol_bank_free now retires the range.  The kernels stay inside their rows
    (host restatement: tests/test_kernel_extents.py)."""
    from dolhip import graph as G
    n, P = 512, (1 << 20) - 5
    c = G.random_regular_csr(n, 4, seed=2028)
    csr = (torch.as_tensor(np.asarray(c.rowptr, np.int32), device=gpu),
           torch.as_tensor(np.asarray(c.col, np.int32), device=gpu),
           torch.as_tensor(np.asarray(c.val, np.float32), device=gpu))
    for k in range(12):
        _remap_cycle(gpu, n, P, csr, k, check=True)
    assert B.release_leaked() == 0


def test_bank_maps_large_state_when_asked(gpu, monkeypatch):
    made = []

    class Spy(B._MappedBlock):
        def __init__(self, *a):
            super().__init__(*a)
            made.append(self.ptr)

    monkeypatch.setattr(B, "_MappedBlock", Spy)
    monkeypatch.setattr(B, "MAPPED_MIN_BYTES", 1 << 20)
    monkeypatch.setenv("DOL_BANK_ALLOC", "torch")
    B.AgentBank(64, 8192, gpu).buffer("x")  # opted out: torch's allocator
    assert made == []
    monkeypatch.delenv("DOL_BANK_ALLOC", raising=False)
    bank = B.AgentBank(64, 8192, gpu)  # default (r05): 2 MiB per buffer >= the threshold: mapped
    x = bank.buffer("x", zero=True)
    assert made == [x.data_ptr()] and float(x.abs().sum()) == 0.0
    small = B.AgentBank(4, 64, gpu).buffer("x")  # below the threshold: torch's allocator
    assert len(made) == 1 and small.data_ptr() != made[0]
    monkeypatch.setenv("DOL_BANK_ALLOC", "torch")
    B.AgentBank(64, 8192, gpu).buffer("x")
    assert len(made) == 1


def test_fused_pass_destination_check_replaces_a_slow_pair(gpu, monkeypatch):
    """AgentBank.mix's destination check (r05): before a fused
    ring pass first writes "y" from a given "x", the pair is timed; a pair whose
    pass is slower than PAIR_RATIO x one ring round gets a fresh destination
    (its contents are dead).  Injected timer: the first pair reads slow, every
    later one fast -> exactly one replacement, both directions checked once, and
    the mixed state bit-identical to a bank without the check (and the oracle)."""
    from dolhip import graph as G
    monkeypatch.setattr(B, "PAIR_PROBE_MIN_BYTES", 0)
    n, P = 96, 1000
    rng = np.random.default_rng(31)
    X0 = rng.standard_normal((n, P)).astype(np.float32)
    plan = G.MixingPlan(G.communication_csr("circle", "stochastic", n)[0], gpu)
    assert plan.kind == "ring"
    calls = []

    def timer(x, y, plan_, steps, P_):
        calls.append((x.data_ptr(), y.data_ptr(), steps))
        return (2.0, 1.0) if len(calls) == 1 else (1.0, 1.0)

    def run(check):
        monkeypatch.setenv("DOL_BANK_PAIR_PROBE", "1" if check else "0")
        bank = B.AgentBank(n, P, gpu)
        bank._pair_timer = timer
        bank.rows().copy_(torch.from_numpy(X0).to(gpu))
        y_first = bank.buffer("y").data_ptr()
        for _ in range(3):
            bank.mix(plan, steps=5)
        torch.cuda.synchronize()
        return bank, y_first, bank.rows().cpu().numpy()

    bank, y_first, got = run(True)
    assert len(calls) == 3  # pair 1 slow -> replaced and re-timed; the swapped pair once; then cached
    assert calls[0][1] == y_first and calls[1][1] != y_first and calls[0][0] == calls[1][0]
    assert [p["attempt"] for p in bank.pair_probes] == [0, 1, 0]
    _, _, plain = run(False)
    assert bits_equal(got, plain)
    want = X0
    wp, wn = (t.cpu().numpy() for t in (plan.w_prev, plan.w_next))
    for _ in range(15):
        want = oracle.mix_ring(want, wp, wn)
    assert bits_equal(got, want)
