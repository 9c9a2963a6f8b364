"""Batched per-agent MLP local steps (BASELINE config 5).

N agents each own a `nn.Sequential(Linear(d, h), ReLU(), Linear(h, c))`
whose parameters are rows of an AgentBank (state_dict order: 0.weight [h,d],
0.bias [h], 2.weight [c,h], 2.bias [c]).  One local step for ALL agents:

  Z1 = X W1^T + b1,  H = relu(Z1),  Z2 = H W2^T + b2,  loss = CE(Z2, y)  (mean over the batch)
  dZ2 = (softmax(Z2) - onehot(y)) / B
  dW2 = dZ2^T H,  db2 = sum_b dZ2,  dH = dZ2 W2,  dZ1 = dH * [Z1 > 0]
  dW1 = dZ1^T X,  db1 = sum_b dZ1
  then one fused SGD / prox / ADMM kernel over every row (dol_prox_admm_sgd_f32)

`step` runs the whole local iteration of every agent in ONE hand-written
kernel (dol_mlp_step_f32, csrc/mlp_step.hip): forward and backward GEMMs on
fp32 MFMA, softmax-CE, and the (prox/ADMM) momentum-SGD update applied to
each gradient tile in registers, so gradients never round-trip through HBM.
This is the per-agent loop of DIST/clients.py:34-59 (one nn.Module
forward/backward/step per agent) batched into one launch.

`forward_backward_torch` keeps the earlier strided-batched formulation
(torch.bmm over the bank rows) as a second implementation the tests compare
against; it is not used by `step`.
"""
from __future__ import annotations

from typing import Optional

import torch

from .bank import AgentBank


def mlp_layout(d: int, h: int, c: int):
    return [("0.weight", (h, d)), ("0.bias", (h,)), ("2.weight", (c, h)), ("2.bias", (c,))]


class BatchedMLP:
    def __init__(self, bank: AgentBank, d: int, h: int, c: int):
        if [k for k, *_ in bank.offsets] != ["0.weight", "0.bias", "2.weight", "2.bias"]:
            raise ValueError("bank layout must be mlp_layout(d, h, c)")
        self.bank, self.d, self.h, self.c = bank, d, h, c
        self.off = {k: o for k, o, _, _ in bank.offsets}

    def _views(self, name: str):
        t = self.bank.buffer(name, zero=(name == "grad"))
        n, d, h, c, o = self.bank.n, self.d, self.h, self.c, self.off
        W1 = t[:, o["0.weight"]:o["0.weight"] + h * d].view(n, h, d)
        b1 = t[:, o["0.bias"]:o["0.bias"] + h]
        W2 = t[:, o["2.weight"]:o["2.weight"] + c * h].view(n, c, h)
        b2 = t[:, o["2.bias"]:o["2.bias"] + c]
        return W1, b1, W2, b2

    def init_like_torch(self, seed: int = 0) -> None:
        """Default nn.Linear init per agent (same RNG order as constructing
        N modules one after another)."""
        g = torch.Generator().manual_seed(seed)
        for i in range(self.bank.n):
            torch.manual_seed(int(torch.randint(0, 2**31 - 1, (1,), generator=g)))
            m = torch.nn.Sequential(torch.nn.Linear(self.d, self.h), torch.nn.ReLU(), torch.nn.Linear(self.h, self.c))
            self.bank.load_module(i, m.to(self.bank.device))

    def forward_backward(self, X: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """X [N, B, d] fp32, y [N, B] int64 on the bank's device.  Writes every
        agent's gradient into the bank's grad rows (fused HIP kernel, no
        update); returns the per-agent mean cross-entropy [N]."""
        from . import ops
        loss = torch.empty(self.bank.n, dtype=torch.float32, device=self.bank.device)
        ops.mlp_step(self.bank.buffer("x"), X, y, self.d, self.h, self.c, grad=self.bank.buffer("grad"),
                     loss=loss, update=False)
        return loss

    def forward_backward_torch(self, X: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Same contract as forward_backward, via torch.bmm (library GEMMs)."""
        n, B = X.shape[0], X.shape[1]
        if n != self.bank.n or X.shape[2] != self.d:
            raise ValueError(f"X must be [{self.bank.n}, B, {self.d}]")
        W1, b1, W2, b2 = self._views("x")
        gW1, gb1, gW2, gb2 = self._views("grad")
        with torch.no_grad():
            Z1 = torch.baddbmm(b1.unsqueeze(1), X, W1.transpose(1, 2))        # [n, B, h]
            H = torch.relu(Z1)
            Z2 = torch.baddbmm(b2.unsqueeze(1), H, W2.transpose(1, 2))        # [n, B, c]
            logp = torch.log_softmax(Z2, dim=2)
            loss = -logp.gather(2, y.unsqueeze(2)).squeeze(2).mean(1)         # [n]
            dZ2 = torch.exp(logp)
            dZ2.scatter_add_(2, y.unsqueeze(2), torch.full_like(logp[..., :1], -1.0))
            dZ2.mul_(1.0 / B)
            torch.bmm(dZ2.transpose(1, 2), H, out=gW2)                        # [n, c, h] into grad rows
            torch.sum(dZ2, dim=1, out=gb2)
            dH = torch.bmm(dZ2, W2)                                           # [n, B, h]
            dZ1 = dH.mul_(Z1 > 0)
            torch.bmm(dZ1.transpose(1, 2), X, out=gW1)                        # [n, h, d] into grad rows
            torch.sum(dZ1, dim=1, out=gb1)
        return loss

    def step(self, X: torch.Tensor, y: torch.Tensor, lr: float, momentum: float, first_step: bool,
             theta: Optional[torch.Tensor] = None, rho: float = 0.0, admm: bool = False,
             write_grad: bool = False, rows: Optional[slice] = None,
             loss: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One fused local iteration for every agent (one kernel launch), or
        for the agents `rows` only (a contiguous slice; X / y / loss are then
        the full [n, ...] tensors and only those rows are read / written).
        Each agent's step is independent of the others, so stepping the bank
        slice by slice gives the same bits as one launch."""
        from . import ops
        b = self.bank
        sl = slice(0, b.n) if rows is None else slice(*rows.indices(b.n)[:2])
        if loss is None:
            loss = torch.empty(b.n, dtype=torch.float32, device=b.device)
        if sl.stop > sl.start:
            pick = (lambda t: t) if rows is None else (lambda t: t[sl])
            ops.mlp_step(pick(b.buffer("x")), pick(X), pick(y), self.d, self.h, self.c,
                         grad=pick(b.buffer("grad")) if write_grad else None,
                         mom=pick(b.buffer("mom", zero=True)) if momentum != 0.0 else None,
                         theta=theta, alpha=pick(b.buffer("alpha", zero=True)) if admm else None, loss=pick(loss),
                         lr=lr, momentum=momentum, rho=rho, first_step=first_step, update=True)
        if momentum != 0.0:
            b.mark_momentum_started(sl)
        return loss

    def step_unfused(self, X: torch.Tensor, y: torch.Tensor, lr: float, momentum: float, first_step: bool,
                     theta: Optional[torch.Tensor] = None, rho: float = 0.0, admm: bool = False) -> torch.Tensor:
        """forward_backward_torch + the fused SGD kernel (the pre-fusion path, for comparison)."""
        loss = self.forward_backward_torch(X, y)
        self.bank.local_step(lr=lr, momentum=momentum, first_step=first_step, theta=theta, rho=rho, admm=admm,
                             write_grad=False)
        return loss
