"""Fused per-agent MLP local step (dol_mlp_step_f32, csrc/mlp_step.hip) vs one
nn.Module per agent — the reference's per-agent loop structure
(DIST/clients.py:34-59; prox/ADMM terms DEC/clients.py:101-139).

The reference checks are torch fp64 on the CPU.  The kernel's GEMMs are fp32
fma chains over K = d (forward) and K = B (dW1), so its results carry fp32
rounding of ~K ulps on dot products of O(1) terms.  Tolerance, stated once:
loss rtol 1e-5 / atol 1e-6, gradients and parameters rtol 1e-4 / atol 1e-5
(the observed max deviation is ~1e-6 at 784-128-10)."""
import numpy as np
import pytest
import torch

from dolhip import ops
from dolhip.bank import AgentBank
from dolhip.mlp import BatchedMLP, mlp_layout

pytestmark = pytest.mark.gpu

LOSS_TOL = dict(rtol=1e-5, atol=1e-6)
TOL = dict(rtol=1e-4, atol=1e-5)

SHAPES = [(3, 7, 20, 32, 5), (8, 32, 784, 128, 10), (5, 64, 36, 64, 3), (2, 1, 4, 256, 32), (4, 33, 100, 96, 17),
          (6, 32, 12, 160, 2)]


def _modules(n, d, h, c, seed):
    torch.manual_seed(seed)
    return [torch.nn.Sequential(torch.nn.Linear(d, h), torch.nn.ReLU(), torch.nn.Linear(h, c)) for _ in range(n)]


def _flat(m, grad=False):
    return torch.cat([(p.grad if grad else p.detach()).reshape(-1) for p in m.parameters()])


def _setup(n, B, d, h, c, gpu, seed=0):
    bank = AgentBank(n, mlp_layout(d, h, c), gpu)
    mlp = BatchedMLP(bank, d, h, c)
    mods = _modules(n, d, h, c, seed)
    for i, m in enumerate(mods):
        bank.load_module(i, m)
    g = torch.Generator().manual_seed(seed + 1)
    X = torch.randn(n, B, d, generator=g)
    y = torch.randint(0, c, (n, B), generator=g)
    return bank, mlp, mods, X, y


def _ref_grad(m, X, y):
    m64 = [p.detach().double().clone().requires_grad_(True) for p in m.parameters()]
    W1, b1, W2, b2 = m64
    z = torch.relu(X.double() @ W1.T + b1) @ W2.T + b2
    loss = torch.nn.functional.cross_entropy(z, y)
    loss.backward()
    return loss.detach(), torch.cat([p.grad.reshape(-1) for p in m64])


@pytest.mark.parametrize("n,B,d,h,c", SHAPES)
def test_fused_forward_backward_matches_per_agent_modules(n, B, d, h, c, gpu):
    bank, mlp, mods, X, y = _setup(n, B, d, h, c, gpu)
    loss = mlp.forward_backward(X.to(gpu), y.to(gpu))
    torch.cuda.synchronize()
    for i, m in enumerate(mods):
        li, gi = _ref_grad(m, X[i], y[i])
        torch.testing.assert_close(loss[i].double().cpu(), li, **LOSS_TOL)
        torch.testing.assert_close(bank.rows("grad")[i].double().cpu(), gi, **TOL)


def test_fused_matches_bmm_formulation(gpu):
    n, B, d, h, c = 16, 32, 784, 128, 10
    bank, mlp, _, X, y = _setup(n, B, d, h, c, gpu, seed=3)
    Xd, yd = X.to(gpu), y.to(gpu)
    l1 = mlp.forward_backward(Xd, yd)
    g1 = bank.rows("grad").clone()
    l2 = mlp.forward_backward_torch(Xd, yd)
    torch.testing.assert_close(l1, l2, **LOSS_TOL)
    torch.testing.assert_close(g1, bank.rows("grad"), **TOL)


@pytest.mark.parametrize("momentum", [0.0, 0.5])
def test_fused_sgd_steps_match_torch_sgd(momentum, gpu):
    n, B, d, h, c = 4, 16, 40, 64, 6
    bank, mlp, mods, _, _ = _setup(n, B, d, h, c, gpu, seed=1)
    mods = [m.double() for m in mods]
    opts = [torch.optim.SGD(m.parameters(), lr=0.1, momentum=momentum) for m in mods]
    g = torch.Generator().manual_seed(11)
    for step in range(3):
        X = torch.randn(n, B, d, generator=g)
        y = torch.randint(0, c, (n, B), generator=g)
        loss = mlp.step(X.to(gpu), y.to(gpu), lr=0.1, momentum=momentum, first_step=(step == 0))
        for i, (m, o) in enumerate(zip(mods, opts)):
            o.zero_grad()
            li = torch.nn.functional.cross_entropy(m(X[i].double()), y[i])
            li.backward()
            o.step()
            torch.testing.assert_close(loss[i].double().cpu(), li.detach(), **LOSS_TOL)
    for i, m in enumerate(mods):
        torch.testing.assert_close(bank.rows()[i].double().cpu(), _flat(m), **TOL)


@pytest.mark.parametrize("admm", [False, True])
def test_fused_prox_admm_step(admm, gpu):
    """FedProx (g += rho (w - theta)) / FedADMM (g += alpha + rho (w - theta)) then
    SGD with momentum, DEC/clients.py:101-115 / :125-139; g' written back to grad."""
    n, B, d, h, c = 3, 32, 64, 32, 4
    rho, lr, mu = 0.1, 0.05, 0.5
    bank, mlp, mods, X, y = _setup(n, B, d, h, c, gpu, seed=5)
    P = bank.P
    gen = torch.Generator().manual_seed(9)
    theta = torch.randn(P, generator=gen)
    alpha = torch.randn(n, P, generator=gen) if admm else torch.zeros(n, P)
    mom0 = torch.randn(n, P, generator=gen)
    bank.buffer("mom", zero=True)[:, :P] = mom0.to(gpu)
    if admm:
        bank.buffer("alpha", zero=True)[:, :P] = alpha.to(gpu)
    w0 = bank.rows().double().cpu().clone()
    mlp.step(X.to(gpu), y.to(gpu), lr=lr, momentum=mu, first_step=False, theta=theta.to(gpu), rho=rho, admm=admm,
             write_grad=True)
    torch.cuda.synchronize()
    for i, m in enumerate(mods):
        _, g = _ref_grad(m, X[i], y[i])
        t = rho * (w0[i] - theta.double())
        if admm:
            t = alpha[i].double() + t
        g2 = g + t
        buf = mom0[i].double() * mu + g2
        torch.testing.assert_close(bank.rows("grad")[i].double().cpu(), g2, **TOL)
        torch.testing.assert_close(bank.rows("mom")[i].double().cpu(), buf, **TOL)
        torch.testing.assert_close(bank.rows()[i].double().cpu(), w0[i] - lr * buf, **TOL)


def test_fused_step_leaves_padding_and_neighbours_untouched(gpu):
    """Only the P parameter floats of each row are written; the row padding and
    the X / label inputs are not."""
    n, B, d, h, c = 5, 8, 28, 32, 3
    bank, mlp, _, X, y = _setup(n, B, d, h, c, gpu, seed=7)
    x = bank.buffer("x")
    x[:, bank.P:] = 12345.0
    Xd, yd = X.to(gpu), y.to(gpu)
    mlp.step(Xd, yd, lr=0.1, momentum=0.0, first_step=True)
    torch.cuda.synchronize()
    assert torch.all(x[:, bank.P:] == 12345.0)
    assert torch.equal(Xd.cpu(), X) and torch.equal(yd.cpu(), y)


def test_out_of_range_label_gives_nan_loss(gpu):
    n, B, d, h, c = 2, 4, 8, 32, 3
    bank, mlp, _, X, y = _setup(n, B, d, h, c, gpu)
    y[1, 2] = c  # invalid for agent 1 only
    loss = mlp.forward_backward(X.to(gpu), y.to(gpu)).cpu()
    assert torch.isfinite(loss[0]) and torch.isnan(loss[1])


def test_rejects_unsupported_shapes(gpu):
    bank = AgentBank(2, mlp_layout(8, 48, 3), gpu)
    X = torch.zeros(2, 4, 8, device=gpu)
    y = torch.zeros(2, 4, dtype=torch.int64, device=gpu)
    with pytest.raises(ops.DolNativeError, match="multiple of 32"):
        ops.mlp_step(bank.buffer("x"), X, y, 8, 48, 3, grad=bank.buffer("grad"), update=False)


_FUSED_CHILD = r"""
import sys, torch
sys.path[:0] = sys.argv[1:3]
from dolhip.bank import AgentBank
from dolhip.mlp import BatchedMLP, mlp_layout
out = {}
for (n, B, d, h, c) in [(8, 32, 784, 128, 10), (3, 7, 100, 128, 5), (2, 32, 128, 128, 10), (5, 20, 800, 128, 3),
                        (4, 33, 100, 96, 17)]:
    for mom in (0.0, 0.5):
        torch.manual_seed(n * 1000 + d)
        bank = AgentBank(n, mlp_layout(d, h, c), "cuda:0")
        bank.rows().copy_(torch.randn(n, bank.P) * 0.05)
        mlp = BatchedMLP(bank, d, h, c)
        g = torch.Generator().manual_seed(d)
        for step in range(3):
            X = torch.randn(n, B, d, generator=g).cuda()
            y = torch.randint(0, c, (n, B), generator=g).cuda()
            loss = mlp.step(X, y, lr=0.1, momentum=mom, first_step=(step == 0), write_grad=(step == 2))
        torch.cuda.synchronize()
        k = f"{n},{B},{d},{h},{c},{mom}"
        out[k + ",x"] = bank.rows().cpu().clone()
        out[k + ",grad"] = bank.rows("grad").cpu().clone()
        out[k + ",loss"] = loss.cpu().clone()
        if mom:
            out[k + ",mom"] = bank.rows("mom").cpu().clone()
torch.save(out, sys.argv[3])
print("ok")
"""


_STEP_PATHS = {  # env of each alternative launch path (read once per process: run in children)
    "base": dict(DOL_MLP_FUSED="0", DOL_MLP_SPLIT_FWD="0", DOL_MLP_F1_TILES="0", DOL_MLP_F1_KW="32", DOL_MLP_TAIL_OCC="3",
                 DOL_MLP_DW1_OCC="3", DOL_MLP_DW1_CHAINS="2"),
    "fused": dict(DOL_MLP_FUSED="1"),
    "split": dict(DOL_MLP_SPLIT_FWD="1"),
    "f1tiles4": dict(DOL_MLP_F1_TILES="4"),
    "f1tiles5": dict(DOL_MLP_F1_TILES="5"),
    "f1tiles3kw64": dict(DOL_MLP_F1_TILES="3", DOL_MLP_F1_KW="64", DOL_MLP_TAIL_OCC="4"),
    "f1tiles4kw64": dict(DOL_MLP_F1_TILES="4", DOL_MLP_F1_KW="64"),
    "split_tail4": dict(DOL_MLP_SPLIT_FWD="1", DOL_MLP_TAIL_OCC="4"),
    "dw1occ4": dict(DOL_MLP_DW1_OCC="4"),
}


def _run_step_child(root, tmp_path, name):
    import os
    import subprocess
    import sys
    f = str(tmp_path / f"{name}.pt")
    env = dict(os.environ, **{k: "0" for k in _STEP_PATHS["base"]})
    env.update(_STEP_PATHS[name])
    r = subprocess.run([sys.executable, "-c", _FUSED_CHILD, root,
                        os.path.join(root, "distributed-optimization-and-learning_amd"), f],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
    return torch.load(f, weights_only=True)


@pytest.mark.parametrize("path", ["fused", "split", "f1tiles4", "f1tiles5", "f1tiles3kw64", "f1tiles4kw64", "split_tail4",
                                  "dw1occ4"])
def test_step_paths_bit_identical(path, gpu, tmp_path):
    """Each alternative launch path of the step gives the same parameters,
    momentum, gradients and losses as the default forward + dW1 kernels, bit
    for bit: the one-kernel step with W1 resident in registers
    (DOL_MLP_FUSED=1), F1 as its own per-agent kernel (DOL_MLP_SPLIT_FWD=1)
    and F1 per (agent, h-tile) single-wave workgroups (DOL_MLP_F1_TILES=NS,
    32- or 64-wide k chunks), each followed by the per-agent tail (at three or
    four waves per SIMD, DOL_MLP_TAIL_OCC).  Cases: d with and without a partial
    last chunk, B < 32, plain and momentum SGD, first steps, write_grad, and a
    shape outside the alternative path (B = 33: falls back)."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = _run_step_child(root, tmp_path, "base")
    alt = _run_step_child(root, tmp_path, path)
    assert base.keys() == alt.keys()
    for k, t in base.items():
        assert torch.equal(t, alt[k]), k
