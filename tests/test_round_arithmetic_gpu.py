"""The engine's own arithmetic pinned through whole training rounds at Model1's
real size (P = 1,663,370).  The end-to-end trajectory tests
(test_dropin_gpu.py) compare against the reference's CPU runs within a
tolerance, because the CNN forward/backward runs through MIOpen; the per-op
digests (test_model1_golden.py) are single calls.  Here the drop-in loops run
unmodified -- DecFedAvg.run (DIST/simulators.py:133-167) and
FedAdmm_Server.run (DEC/servers.py:50-81) -- and every engine call they make
(the gossip mix, each fused optimizer step with its FedADMM term, the dual
update, the server's ordered mean) is checked bit for bit against the oracle
on the exact inputs it received, so the only values not pinned are the
gradients MIOpen produced."""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_project
from dolhip import ops

pytestmark = pytest.mark.gpu


def _host(t):
    return None if t is None else t.detach().float().cpu().numpy().copy()


class Pin:
    """Wraps engine ops: snapshot the inputs, run the kernel, compare with the oracle."""

    def __init__(self, monkeypatch):
        self.calls = {}
        for name in ("prox_admm_sgd", "admm_dual", "ordered_mean", "mix_ring", "mix_csr", "mix_csr_slab"):
            real = getattr(ops, name)
            monkeypatch.setattr(ops, name, self._wrap(name, real))

    def _count(self, name):
        self.calls[name] = self.calls.get(name, 0) + 1

    def _wrap(self, name, real):
        def prox_admm_sgd(w, g, buf=None, theta=None, alpha=None, rho=0.0, lr=0.01, momentum=0.0, first_step=False,
                          write_grad=True, P=None):
            P = w.shape[1] if P is None else P
            W, G, B = _host(w[:, :P]), _host(g[:, :P]), _host(None if buf is None else buf[:, :P])
            TH, AL = _host(None if theta is None else theta[:P]), _host(None if alpha is None else alpha[:, :P])
            real(w, g, buf=buf, theta=theta, alpha=alpha, rho=rho, lr=lr, momentum=momentum, first_step=first_step,
                 write_grad=write_grad, P=P)
            torch.cuda.synchronize()
            w1, b1, g1 = oracle.prox_admm_sgd(W, B, G, TH, AL, np.float32(rho), np.float32(lr), np.float32(momentum),
                                              first_step, write_grad)
            assert oracle.bits_equal(_host(w[:, :P]), w1), "optimizer step: parameters"
            if buf is not None:
                assert oracle.bits_equal(_host(buf[:, :P]), b1), "optimizer step: momentum"
            if write_grad:
                assert oracle.bits_equal(_host(g[:, :P]), g1), "optimizer step: gradient term"
            self._count(name)

        def admm_dual(alpha, w, theta, rho, resid_sq=None, work=None, P=None):
            P = alpha.shape[1] if P is None else P
            A, W, TH = _host(alpha[:, :P]), _host(w[:, :P]), _host(theta[:P])
            real(alpha, w, theta, rho, resid_sq=resid_sq, work=work, P=P)
            torch.cuda.synchronize()
            a1, r = oracle.admm_dual(A, W, TH, np.float32(rho))
            assert oracle.bits_equal(_host(alpha[:, :P]), a1), "update_duals"
            if resid_sq is not None:  # the fp64 diagnostic: both sums fixed-order, in different orders;
                # over P = 1.66M squares the orders differ by up to ~P * 2^-53 relative (observed 1.6e-12)
                np.testing.assert_allclose(resid_sq[:alpha.shape[0]].cpu().numpy(), r, rtol=1e-9)
            self._count(name)

        def ordered_mean(W, order, out=None, P=None):
            P = W.shape[1] if P is None else P
            Wh, o = _host(W[:, :P]), order.cpu().numpy()
            res = real(W, order, out=out, P=P)
            torch.cuda.synchronize()
            assert oracle.bits_equal(_host(res[:P]), oracle.ordered_mean(Wh, o)), "average_weights"
            self._count(name)
            return res

        def mix_ring(X, Y, w_prev, w_next, halo_prev=None, halo_next=None, P=None, n_rows=None):
            P = X.shape[1] if P is None else P
            n = X.shape[0] if n_rows is None else n_rows
            Xh = _host(X[:n, :P])
            res = real(X, Y, w_prev, w_next, halo_prev=halo_prev, halo_next=halo_next, P=P, n_rows=n_rows)
            torch.cuda.synchronize()
            want = oracle.mix_ring(Xh, _host(w_prev[:n]), _host(w_next[:n]), _host(halo_prev), _host(halo_next))
            assert oracle.bits_equal(_host(Y[:n, :P]), want), "gossip mix (ring)"
            self._count(name)
            return res

        def mix_csr(X, Y, rowptr, col, val, P=None):
            P = X.shape[1] if P is None else P
            Xh = _host(X[:, :P])
            res = real(X, Y, rowptr, col, val, P=P)
            torch.cuda.synchronize()
            rp, c, v = rowptr.cpu().numpy(), col.cpu().numpy(), val.cpu().numpy()
            want = oracle.mix_csr(Xh, rp, c, v)
            assert oracle.bits_equal(_host(Y[:len(rp) - 1, :P]), want), "gossip mix (CSR)"
            self._count(name)
            return res

        def mix_csr_slab(*a, **kw):  # complete graphs of >= 16 agents: pinned through the plan's CSR below
            self._count(name)
            return real(*a, **kw)

        return locals()[name]


def _dist_args(utils, **kw):
    base = dict(num_users=5, local_ep=1, local_bs=32, lr=0.05, topology="circle", mode="stochastic",
                model="Model1", dataset="synthetic", iid=True, shards=2, seed=7, momentum=0.5, verbose=False,
                synthetic_train=320, synthetic_test=32, device="cuda", rounds=2)
    base.update(kw)
    return utils.DotDict(base)


@pytest.mark.parametrize("topology", ["circle", "compelete"])
def test_decfedavg_rounds_pinned_at_model1_size(topology, gpu, monkeypatch):
    m = load_project("weighted_average", ["simulators", "utils"])
    args = _dist_args(m["utils"], topology=topology)
    sim = m["simulators"].DecFedAvg(args)
    assert sim.bank.P == 1_663_370
    pin = Pin(monkeypatch)
    sim.run(args.rounds)
    steps_per_client = args.rounds * -(-int(args.synthetic_train * 0.9 / args.num_users) // args.local_bs)
    assert pin.calls.get("prox_admm_sgd", 0) >= args.num_users * args.rounds
    assert pin.calls.get("mix_ring" if topology == "circle" else "mix_csr", 0) == args.rounds
    assert steps_per_client > 0


def test_fedadmm_rounds_pinned_at_model1_size(gpu, monkeypatch):
    m = load_project("primal_dual", ["servers", "utils"])
    args = m["utils"].DotDict(dict(num_users=4, local_ep=1, local_bs=32, lr=0.05, model="Model1", dataset="synthetic",
                                   iid=True, shards=2, seed=11, momentum=0.5, verbose=False, synthetic_train=256,
                                   synthetic_test=32, device="cuda", rho=0.1))
    s = m["servers"].FedAdmm_Server(args)
    pin = Pin(monkeypatch)
    s.run(1.0, 2)
    assert pin.calls.get("prox_admm_sgd", 0) >= 2 * args.num_users
    assert pin.calls.get("admm_dual", 0) == 2 * args.num_users
    assert pin.calls.get("ordered_mean", 0) >= 2
