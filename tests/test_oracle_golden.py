"""The CPU oracle (oracle/dol_oracle.c) against vectors produced by the
reference itself (tests/golden/make_golden.py).  Bit-exact."""
import numpy as np
import pytest

import oracle
from oracle import bits_equal
from conftest import golden


def _mix_cases():
    mix = golden("mix")
    return sorted(k[:-3] for k in mix.files if k.endswith("__X"))


@pytest.mark.parametrize("case", _mix_cases())
def test_mix_csr_matches_reference_consensus(case):
    """Neighbors + Client.consensus (DIST/simulators.py:91-97, DIST/clients.py:61-69)."""
    mix, csr = golden("mix"), golden("csr")
    gkey, _layout, t = case.split("__")
    c = f"{gkey}__{t}"
    Y = oracle.mix_csr(mix[case + "__X"], csr[c + "__rowptr"], csr[c + "__col"], csr[c + "__val"])
    assert bits_equal(Y, mix[case + "__Y"])


def test_mix_ring_form_equals_csr_form():
    from dolhip.graph import CSR
    mix, csr = golden("mix"), golden("csr")
    for case in _mix_cases():
        gkey, _l, t = case.split("__")
        c = f"{gkey}__{t}"
        n = len(csr[c + "__rowptr"]) - 1
        g = CSR(n, n, csr[c + "__rowptr"], csr[c + "__col"], csr[c + "__val"])
        rw = g.ring_weights()
        if rw is None:
            continue
        Y = oracle.mix_ring(mix[case + "__X"], rw[0], rw[1])
        assert bits_equal(Y, mix[case + "__Y"]), case


def _local_keys():
    L = golden("local_steps")
    return sorted({k.rsplit("__", 1)[0] for k in L.files})


@pytest.mark.parametrize("key", _local_keys())
def test_local_step_matches_reference_update_model_and_sgd(key):
    """FedAvg/FedProx/FedAdmm update_model (DEC/clients.py:85-139) + SGD.step."""
    L = golden("local_steps")
    rho, lr, mom = (float(v) for v in L[key + "__params"])
    cls = key.split("__")[0]
    theta = None if cls == "FedAvg_Client" else L[key + "__theta"]
    alpha = L[key + "__alpha"][None] if cls == "FedAdmm_Client" else None
    for t in range(L[key + "__w"].shape[0]):
        w1, b1, g1 = oracle.prox_admm_sgd(L[key + "__w"][t][None], L[key + "__buf"][t][None],
                                          L[key + "__g"][t][None], theta, alpha, rho, lr, mom,
                                          first_step=(t == 0))
        assert bits_equal(g1[0], L[key + "__gp"][t])
        assert bits_equal(w1[0], L[key + "__w1"][t])
        if mom != 0:
            assert bits_equal(b1[0], L[key + "__buf1"][t])
    if cls == "FedAdmm_Client":
        a1, _ = oracle.admm_dual(alpha, L[key + "__wfinal"][None], L[key + "__theta"], rho)
        assert bits_equal(a1[0], L[key + "__alpha1"])


@pytest.mark.parametrize("rho", ["0.1", "0.01", "1.0"])
def test_dual_update_matches_reference(rho):
    """FedAdmm_Client.update_duals (DEC/clients.py:141-144)."""
    D = golden("duals")
    k = f"rho{rho}"
    a1, r = oracle.admm_dual(D[k + "__alpha"], D[k + "__w"], D[k + "__theta"], float(D[k + "__rho"][0]))
    assert bits_equal(a1, D[k + "__alpha1"])
    d = D[k + "__w"].astype(np.float32) - D[k + "__theta"].astype(np.float32)[None]
    np.testing.assert_allclose(r, (d.astype(np.float64) ** 2).sum(1), rtol=1e-12)


@pytest.mark.parametrize("name", ["m7_mini", "m1_mini", "m10_flat1031", "m3_flat4097"])
def test_ordered_mean_matches_reference_average_weights(name):
    """Server.average_weights (DEC/servers.py:42-48)."""
    A = golden("average")
    W = A[name + "__W"]
    assert bits_equal(oracle.ordered_mean(W, np.arange(W.shape[0])), A[name + "__theta"])
    # the partial-sum form composes to the same value
    m = W.shape[0]
    if m > 2:
        part = oracle.ordered_sum(W, np.arange(2))
        full = oracle.ordered_sum(W, np.arange(2, m), acc_in=part, scale=float(m))
        assert bits_equal(full, A[name + "__theta"])


@pytest.mark.parametrize("momentum,first", [(0.0, False), (0.5, True), (0.5, False)])
def test_dgd_local_step_is_the_pinned_sgd_step(momentum, first):
    """Config 3's local step (oracle_dgd_local_f32, least squares) is the
    reference-pinned SGD update above (oracle_prox_admm_sgd_f32, no prox term)
    applied to g = fl(x - t) — which is exactly what torch autograd returns for
    0.5 * sum((x - t)**2) (the *2 and *0.5 scalings are exact)."""
    import torch
    rng = np.random.default_rng(3)
    Y = rng.standard_normal((4, 301)).astype(np.float32)
    T = rng.standard_normal((4, 301)).astype(np.float32)
    M = rng.standard_normal((4, 301)).astype(np.float32)
    x = torch.from_numpy(Y.copy()).requires_grad_(True)
    (0.5 * ((x - torch.from_numpy(T)) ** 2).sum()).backward()
    g = (Y - T).astype(np.float32)
    assert bits_equal(x.grad.numpy(), g)
    got_y, got_m = oracle.dgd_local(Y, T, M if momentum else None, "least_squares", 1, 0.05, momentum, first)
    want_w, want_b, _ = oracle.prox_admm_sgd(Y, M if momentum else None, g, None, None, 0.0, 0.05, momentum, first)
    assert bits_equal(got_y, want_w)
    if momentum:
        assert bits_equal(got_m, want_b)
