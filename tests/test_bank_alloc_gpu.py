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


def _ring_bank(gpu, monkeypatch, n=96, P=1000, alloc="torch"):
    from dolhip import graph as G
    monkeypatch.setattr(B, "PAIR_PROBE_MIN_BYTES", 0)
    monkeypatch.setenv("DOL_BANK_PAIR_PROBE", "1")
    monkeypatch.setenv("DOL_BANK_ALLOC", alloc)
    plan = G.MixingPlan(G.communication_csr("circle", "stochastic", n)[0], gpu)
    bank = B.AgentBank(n, P, gpu)
    bank.rows().copy_(torch.from_numpy(np.random.default_rng(5).standard_normal((n, P)).astype(np.float32)).to(gpu))
    return bank, plan


def test_destination_check_probes_at_the_calibrated_step_count(gpu, monkeypatch):
    """a longer fused pass carries more arithmetic per byte, so its
    pass / round ratio rises with the step count.  The check times the pair
    at PAIR_PROBE_STEPS (the count PAIR_RATIO was calibrated on) whatever the
    pass's own count: with a timer whose ratio is 1 + 0.02 * steps, mix(steps
    = 8) keeps its buffers (1.10 at 5 rounds; 1.16 at 8 would read as slow)."""
    bank, plan = _ring_bank(gpu, monkeypatch)
    seen = []

    def timer(x, y, plan_, steps, P_):
        seen.append(steps)
        return 1.0 + 0.02 * steps, 1.0
    bank._pair_timer = timer
    y0, x0 = bank.buffer("y").data_ptr(), bank.buffer("x").data_ptr()
    bank.mix(plan, steps=8)
    bank.mix(plan, steps=16)
    torch.cuda.synchronize()
    assert seen == [B.PAIR_PROBE_STEPS, B.PAIR_PROBE_STEPS]  # each direction once, at the calibrated count
    assert {bank.x.data_ptr(), bank.buffer("y").data_ptr()} == {x0, y0}
    assert all(p["steps"] == B.PAIR_PROBE_STEPS and p["attempt"] == 0 for p in bank.pair_probes)


def test_destination_check_holds_one_candidate_and_stops_on_a_reused_block(gpu, monkeypatch):
    """Every pair reads slow: the losing candidate is dropped before the next
    allocation (at most one buffer besides the best is held), and when torch's
    caching allocator hands the dropped block straight back the search stops
    instead of re-measuring it."""
    bank, plan = _ring_bank(gpu, monkeypatch)
    nbytes = bank.n * bank.ld * 4
    bank._pair_timer = lambda x, y, p, steps, P_: (2.0, 1.0)
    y0 = bank.buffer("y").data_ptr()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(gpu)
    torch.cuda.reset_peak_memory_stats(gpu)
    bank.mix(plan, steps=5)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(gpu) - base
    assert peak <= nbytes + (4 << 20)  # the best so far + ONE fresh candidate, never two
    probes = bank.pair_probes
    assert [p["attempt"] for p in probes] == [0, 1] and probes[-1].get("same_block")
    assert bank.x.data_ptr() == y0  # the first (equally slow) destination was kept and written


def test_destination_check_keeps_adopted_buffers(gpu, monkeypatch):
    """Buffers handed in with adopt() stay the caller's: a slow pair is
    recorded, not replaced -- unless adopted with replaceable=True."""
    bank, plan = _ring_bank(gpu, monkeypatch)
    bank._pair_timer = lambda x, y, p, steps, P_: (2.0, 1.0)
    mine = torch.empty_like(bank.buffer("y"))
    bank.adopt("y", mine)
    bank.mix(plan, steps=5)
    assert bank.x.data_ptr() == mine.data_ptr()
    assert bank.pair_probes[-1].get("kept_adopted") and len(bank.pair_probes) == 1
    bank2, plan2 = _ring_bank(gpu, monkeypatch)
    bank2._pair_timer = lambda x, y, p, steps, P_: (2.0, 1.0)
    mine2 = torch.empty_like(bank2.buffer("y"))
    bank2.adopt("y", mine2, replaceable=True)
    bank2.mix(plan2, steps=5)
    assert len(bank2.pair_probes) >= 2  # replaced and re-timed
    torch.cuda.synchronize()


def test_retired_address_space_is_counted_and_capped(gpu, monkeypatch):
    """ADVICE r05 / VERDICT r05 item 8: dol_bank_free retires the virtual range
    of a mapped block; the retired bytes are counted through the C-ABI, and
    past DOL_BANK_RETIRED_VA_CAP_GIB dol_bank_alloc refuses (DOL_ECAP):
    mapped=True raises, the default falls back to torch's allocator with a
    warning.  200 map/free cycles keep the process working."""
    from dolhip._native import DolNativeError
    monkeypatch.setattr(B, "MAPPED_MIN_BYTES", 0)
    monkeypatch.delenv("DOL_BANK_ALLOC", raising=False)
    monkeypatch.delenv("DOL_BANK_RETIRED_VA_CAP_GIB", raising=False)
    before = B.retired_va()
    for k in range(200):
        X = B.device_matrix(64, 8192, gpu, mapped=True)  # 2 MiB
        X.fill_(float(k))
        assert float(X[63, 8191]) == float(k)
        del X
        gc.collect()
    torch.cuda.synchronize()
    after = B.retired_va()
    assert after["blocks"] == before["blocks"] + 200
    assert after["bytes"] >= before["bytes"] + 200 * 64 * 8192 * 4
    assert after["cap_bytes"] == 4096 << 30
    monkeypatch.setenv("DOL_BANK_RETIRED_VA_CAP_GIB", "0")  # a cap below what is already retired
    assert B.retired_va()["cap_bytes"] == 0
    with pytest.raises(DolNativeError, match="DOL_BANK_RETIRED_VA_CAP_GIB"):
        B.device_matrix(64, 8192, gpu, mapped=True)
    monkeypatch.setattr(B, "_CAP_WARNED", [])
    with pytest.warns(ResourceWarning):
        t = B.device_matrix(64, 8192, gpu)  # default: torch's allocator instead
    t.fill_(1.0)
    assert float(t.sum()) == 64 * 8192
    monkeypatch.delenv("DOL_BANK_RETIRED_VA_CAP_GIB")
    X = B.device_matrix(64, 8192, gpu, mapped=True)
    del X, t
    gc.collect()
    torch.cuda.synchronize()
