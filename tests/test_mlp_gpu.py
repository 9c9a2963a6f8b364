"""Batched per-agent MLP local steps (dolhip.mlp) vs one nn.Module per agent
(the reference's per-agent loop structure, DIST/clients.py:34-59) on the GPU.
Tolerance: the batched GEMMs and the per-module GEMMs may pick different
hipBLASLt kernels, so gradients agree to fp32 rounding: rtol 1e-4, atol 1e-6."""
import numpy as np
import pytest
import torch

from dolhip.bank import AgentBank
from dolhip.mlp import BatchedMLP, mlp_layout

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,B,d,h,c", [(3, 7, 20, 16, 5), (8, 32, 784, 128, 10)])
def test_batched_mlp_matches_per_agent_modules(n, B, d, h, c, gpu):
    bank = AgentBank(n, mlp_layout(d, h, c), gpu)
    mlp = BatchedMLP(bank, d, h, c)
    torch.manual_seed(0)
    mods = [torch.nn.Sequential(torch.nn.Linear(d, h), torch.nn.ReLU(), torch.nn.Linear(h, c)).to(gpu) for _ in range(n)]
    for i, m in enumerate(mods):
        bank.load_module(i, m)
    X = torch.randn(n, B, d, device=gpu)
    y = torch.randint(0, c, (n, B), device=gpu)
    loss = mlp.forward_backward(X, y)
    for i, m in enumerate(mods):
        m.zero_grad()
        li = torch.nn.functional.cross_entropy(m(X[i]), y[i])
        li.backward()
        torch.testing.assert_close(loss[i], li.detach(), rtol=1e-5, atol=1e-6)
        want = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
        torch.testing.assert_close(bank.rows("grad")[i], want, rtol=1e-4, atol=1e-6)


def test_batched_mlp_sgd_step_matches_torch_sgd(gpu):
    n, B, d, h, c = 4, 16, 30, 12, 6
    bank = AgentBank(n, mlp_layout(d, h, c), gpu)
    mlp = BatchedMLP(bank, d, h, c)
    torch.manual_seed(1)
    mods = [torch.nn.Sequential(torch.nn.Linear(d, h), torch.nn.ReLU(), torch.nn.Linear(h, c)).to(gpu) for _ in range(n)]
    opts = [torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.5) for m in mods]
    for i, m in enumerate(mods):
        bank.load_module(i, m)
    for step in range(3):
        X = torch.randn(n, B, d, device=gpu)
        y = torch.randint(0, c, (n, B), device=gpu)
        mlp.step(X, y, lr=0.1, momentum=0.5, first_step=(step == 0))
        for i, (m, o) in enumerate(zip(mods, opts)):
            o.zero_grad()
            torch.nn.functional.cross_entropy(m(X[i]), y[i]).backward()
            o.step()
    for i, m in enumerate(mods):
        want = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        torch.testing.assert_close(bank.rows()[i], want, rtol=1e-4, atol=1e-5)
