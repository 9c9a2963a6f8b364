"""Model3's real layout on the GPU (a13: DIST/models.py:36-57, DEC/models.py:
31-51): P = 1,105,098 floats in state_dict key order, P mod 4 = 2, so every
agent row ends in a ragged 8-B tail.  A bank of real Model3 agents (default
init under seeds; agent 0 is pinned to the reference's own Model3 init by
tests/golden/host.npz, made by tests/golden/make_golden.py's gen_host) is
mixed, stepped, dual-updated and averaged through the C-ABI, each result
bit-exact against the oracle (oracle/dol_oracle.c):

* one gossip round for circle / complete / double-stochastic circle W
  (ring kernel, agent-major CSR kernel, LDS-gather CSR kernel), and FedLCon's
  eps = 3 rounds (the ragged P takes the single-round path);
* the fused FedADMM local step (ADMM term + momentum SGD, DEC/clients.py:
  125-139 + SGD.step) on the bank rows;
* update_duals (DEC/clients.py:141-144) and average_weights
  (DEC/servers.py:42-48) in a sampled order.
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import golden
from oracle import bits_equal
from dolhip import graph as G

pytestmark = pytest.mark.gpu

P3 = 1_105_098


def _model3_bank(n, gpu):
    """n real Model3 agents as rows of an AgentBank (agent i: manual_seed(2028 + i))."""
    from dolhip.bank import AgentBank, layout_of
    from dolhip.models import Model3
    rows = []
    layout = None
    for i in range(n):
        torch.manual_seed(2028 + i)
        m = Model3()
        layout = layout_of(m)
        rows.append(np.concatenate([v.numpy().reshape(-1) for v in m.state_dict().values()]))
    X = np.stack(rows).astype(np.float32)
    bank = AgentBank(n, layout, gpu)
    assert bank.P == P3 and P3 % 4 == 2
    bank.rows()[:] = torch.from_numpy(X).to(gpu)
    return bank, X


def test_model3_bank_rows_are_reference_inits(gpu):
    bank, X = _model3_bank(2, gpu)
    h = golden("host")
    assert int(h["Model3__P"][0]) == P3
    assert X[0][::4999].tobytes() == h["Model3__sample"].tobytes()
    assert bank.rows()[0].cpu().numpy()[::4999].tobytes() == h["Model3__sample"].tobytes()


def _plan(topology, mode, n, gpu, slab=None):
    torch.manual_seed(2028)
    csr = G.csr_from_dense(G.communication_graph(topology, mode, n)[0])
    return G.MixingPlan(csr, gpu, slab=slab), csr


@pytest.mark.parametrize("topology,mode,n,slab,kind", [
    ("circle", "stochastic", 6, None, "ring"),
    ("circle", "double_stochastic", 16, None, "ring"),
    ("compelete", "stochastic", 16, None, "csr"),
    ("compelete", "stochastic", 16, True, "csr"),  # the LDS-gather CSR kernel
])
def test_model3_mix_round(topology, mode, n, slab, kind, gpu):
    bank, X = _model3_bank(n, gpu)
    plan, csr = _plan(topology, mode, n, gpu, slab)
    assert plan.kind == kind and (slab is None or plan.ent is not None)
    bank.mix(plan)
    torch.cuda.synchronize()
    assert bits_equal(bank.rows().cpu().numpy(), oracle.mix_csr(X, csr.rowptr, csr.col, csr.val))


def test_model3_fedlcon_eps3(gpu):
    n = 6
    bank, X = _model3_bank(n, gpu)
    plan, csr = _plan("circle", "stochastic", n, gpu)
    bank.mix(plan, steps=3)
    torch.cuda.synchronize()
    want = X
    for _ in range(3):
        want = oracle.mix_csr(want, csr.rowptr, csr.col, csr.val)
    assert bits_equal(bank.rows().cpu().numpy(), want)


@pytest.mark.parametrize("first", [True, False])
def test_model3_admm_local_step_duals_and_average(first, gpu):
    n, rho, lr, mu = 6, 0.1, 0.05, 0.5
    bank, X = _model3_bank(n, gpu)
    rng = np.random.default_rng(31)
    G_ = rng.standard_normal((n, P3), dtype=np.float32)
    B = rng.standard_normal((n, P3), dtype=np.float32)
    A = rng.standard_normal((n, P3), dtype=np.float32) * np.float32(0.01)
    th = rng.standard_normal(P3, dtype=np.float32)
    bank.rows("grad")[:] = torch.from_numpy(G_).to(gpu)
    bank.rows("mom")[:] = torch.from_numpy(B).to(gpu)
    bank.rows("alpha")[:] = torch.from_numpy(A).to(gpu)
    theta = torch.from_numpy(th).to(gpu)
    bank.local_step(lr=lr, momentum=mu, first_step=first, theta=theta, rho=rho, admm=True)
    w1, b1, g1 = oracle.prox_admm_sgd(X, B, G_, th, A, rho, lr, mu, first)
    bank.dual_update(theta, rho)
    a1, _ = oracle.admm_dual(A, w1, th, np.float32(rho))
    order = [4, 0, 5, 2]
    mean = bank.ordered_mean(order)
    torch.cuda.synchronize()
    assert bits_equal(bank.rows().cpu().numpy(), w1)
    assert bits_equal(bank.rows("mom").cpu().numpy(), b1)
    assert bits_equal(bank.rows("grad").cpu().numpy(), g1)
    assert bits_equal(bank.rows("alpha").cpu().numpy(), a1)
    assert bits_equal(mean[:P3].cpu().numpy(), oracle.ordered_mean(w1, np.array(order)))
