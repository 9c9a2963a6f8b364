"""Synthetic separable objectives for BASELINE config 3 (decentralised
gradient descent at 1024+ agents x 2^20 parameters, mixing-bound).

Agent i minimises f_i(x) over its own row of the bank; one round is the
reference's gossip round order (DIST/simulators.py:147-162: consensus with
W[t], then local_update = `local_steps` iterations of torch.optim.SGD(lr,
momentum), DIST/clients.py:43-49) with the local loss replaced by a
separable synthetic one, so the whole round fuses into one pass
(dol_dgd_ring_f32 / dol_dgd_csr_f32):

  least_squares  f_i(x) = 1/2 ||x - t_i||^2      (t_i = target row; optimum of
                                                  sum_i f_i is mean_i t_i)
  logistic       f_i(x) = sum_p log(1 + exp(-t_ip x_p))   (t = label * feature,
                                                  the diagonal-feature variant)

Not a reference model: the reference trains CNNs on MNIST (SURVEY §8d names
these objectives as the config-3 workload).  The momentum buffer persists
across rounds like the reference's optimizer state.
"""
from __future__ import annotations

from typing import Optional

import torch

from .bank import AgentBank
from .graph import MixingPlan


class SeparableDGD:
    def __init__(self, plan: MixingPlan, P: int, objective: str = "least_squares", lr: float = 0.01,
                 momentum: float = 0.0, local_steps: int = 1, seed: int = 2028, device=None,
                 bank: Optional[AgentBank] = None):
        self.plan = plan
        self.objective = objective
        self.lr, self.mu, self.local_steps = float(lr), float(momentum), int(local_steps)
        dev = plan.device if device is None else torch.device(device)
        self.bank = bank if bank is not None else AgentBank(plan.n_rows, P, dev)
        self.P = self.bank.P
        g = torch.Generator(device=dev).manual_seed(seed)
        self.bank.buffer("x").normal_(generator=g)
        t = self.bank.buffer("target")
        t.normal_(generator=g)
        if objective == "logistic":  # t = label (+-1) * feature
            t.copy_(torch.where(torch.rand(t.shape, generator=g, device=dev) < 0.5, -t, t))
        self.bank.buffer("y")
        if self.mu != 0.0:
            self.bank.buffer("mom", zero=True)
        self.first = True
        self.rounds = 0

    def params(self) -> torch.Tensor:
        return self.bank.rows("x")

    def targets(self) -> torch.Tensor:
        return self.bank.rows("target")

    def momentum_rows(self) -> Optional[torch.Tensor]:
        return self.bank.rows("mom") if self.mu != 0.0 else None

    def round(self) -> None:
        """X <- W X, then the local steps; swaps the Jacobi buffers (no copy)."""
        b = self.bank
        self.plan.apply_dgd(b.buffer("x"), b.buffer("y"), b.buffer("target"),
                            mom=b.buffer("mom") if self.mu != 0.0 else None, objective=self.objective,
                            steps=self.local_steps, lr=self.lr, momentum=self.mu, first_step=self.first,
                            P=self.P)
        b.swap("x", "y")
        self.first = False
        self.rounds += 1

    def loss(self) -> torch.Tensor:
        """Per-agent local loss f_i(x_i) (diagnostic, torch ops)."""
        x, t = self.params(), self.targets()
        if self.objective == "least_squares":
            return 0.5 * ((x - t) ** 2).sum(1)
        return torch.nn.functional.softplus(-t * x).sum(1)

    def consensus_error(self) -> float:
        x = self.params()
        return float((x - x.mean(0, keepdim=True)).norm() / max(1, x.shape[0]) ** 0.5)
