"""Agent plumbing shared by the drop-in `weighted_average` and `primal_dual`
packages: config dict, seeding, per-agent bank rows, and the bank-backed SGD
that replaces torch.optim.SGD (DIST/clients.py:17, DEC/clients.py:14).
"""
from __future__ import annotations

import random
from collections.abc import Mapping
from typing import Dict, Iterator, Optional

import numpy as np
import torch

from . import ops
from .bank import AgentBank, layout_of


class DotDict(dict):
    """Attribute access to a dict; a missing key reads as None (DIST/utils.py:10-23)."""

    def __getattr__(self, attr):
        return self.get(attr)

    __setattr__ = dict.__setitem__
    __delattr__ = dict.__delitem__

    def __getstate__(self):
        return self

    def __setstate__(self, state):
        self.update(state)
        self.__dict__ = self


def setup_seed(seed) -> None:
    """DIST/utils.py:51-56: torch (CPU + all GPUs), numpy, random; deterministic cuDNN/MIOpen."""
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.backends.cudnn.deterministic = True


def engine_device(args) -> torch.device:
    dev = torch.device(args.device) if args.device is not None else torch.device("cuda")
    if dev.type != "cuda":
        raise ops.DolNativeError(f"args.device={dev}: the HIP engine runs on a GPU (no CPU path)")
    return dev


class RowState(Mapping):
    """A live state_dict view of one bank row (what model.state_dict() returns
    when the module's parameters are bank views).  Servers average these
    without copies (bank rows are stable for the rest of the round)."""

    def __init__(self, bank: AgentBank, row: int, name: str = "x"):
        self.bank, self.row, self.name = bank, row, name

    def _views(self) -> Dict[str, torch.Tensor]:
        return self.bank.row_views(self.row, self.name)

    def __getitem__(self, k):
        return self._views()[k]

    def __iter__(self) -> Iterator[str]:
        return iter(k for k, *_ in self.bank.offsets)

    def __len__(self) -> int:
        return len(self.bank.offsets)

    def flat(self) -> torch.Tensor:
        return self.bank.buffer(self.name)[self.row, : self.bank.P]

    def __deepcopy__(self, memo):
        return {k: v.clone() for k, v in self._views().items()}


class BankSGD:
    """torch.optim.SGD(lr, momentum) over one bank row, as ONE fused HIP kernel
    (dol_prox_admm_sgd_f32 with theta = NULL): buf = g (first step) or
    buf*mu + g; w = fma(-lr, buf, w).  Momentum persists across rounds, as the
    reference's optimizer state does (it is never reset).  Whether a row's
    buffer has started lives in the bank (`AgentBank.mom_started`), so it
    moves with `attach` and survives `AgentBank.save/load`."""

    def __init__(self, agent: "BankAgent", lr: float, momentum: float = 0.0):
        self.agent = agent
        self.lr = float(lr)
        self.momentum = float(momentum or 0.0)
        self.steps = 0
        self.defaults = {"lr": self.lr, "momentum": self.momentum}

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.agent.zero_grad()

    def step(self, theta: Optional[torch.Tensor] = None, alpha: bool = False, rho: float = 0.0) -> None:
        a = self.agent
        a.sync_grads()
        b, i = a.bank, a.row
        ops.prox_admm_sgd(b.buffer("x")[i:i + 1], b.buffer("grad")[i:i + 1],
                          buf=b.buffer("mom")[i:i + 1] if self.momentum != 0.0 else None,
                          theta=theta, alpha=b.buffer("alpha", zero=True)[i:i + 1] if alpha else None,
                          rho=rho, lr=self.lr, momentum=self.momentum, first_step=not b.mom_started[i],
                          write_grad=True, P=b.P)
        if self.momentum != 0.0:
            b.mom_started[i] = True
        self.steps += 1


class BankAgent:
    """Mixin: the agent's nn.Module parameters (and grads) are views into row
    `row` of an AgentBank; a fresh agent owns a private 1-row bank until a
    simulator/server attaches it to the shared one."""

    def _init_bank(self, model: torch.nn.Module, device) -> None:
        self.model = model.to(device)
        self.bank = AgentBank(1, layout_of(self.model), device)
        self.row = 0
        self.bank.load_module(0, self.model)
        self.bank.buffer("grad", zero=True)
        self.bank.bind(0, self.model)

    def attach(self, bank: AgentBank, row: int) -> None:
        """Move this agent's state into row `row` of a shared bank."""
        old, oi = self.bank, self.row
        for name in ("x", "grad", "mom", "alpha"):
            if old.has(name):
                bank.buffer(name, zero=True)[row, : bank.P].copy_(old.buffer(name)[oi, : old.P])
        bank.mom_started[row] = old.mom_started[oi]
        self.bank, self.row = bank, row
        bank.buffer("grad", zero=True)
        bank.bind(row, self.model)

    def zero_grad(self) -> None:
        self.bank.buffer("grad")[self.row].zero_()
        self._ensure_grad_views()

    def _ensure_grad_views(self) -> None:
        views = self.bank.row_views(self.row, "grad")
        for k, p in self.model.named_parameters():
            v = views[k]
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def sync_grads(self) -> None:
        """If outside code replaced a param's .grad (e.g. model.zero_grad(set_to_none)),
        copy it into the bank row and restore the view."""
        views = self.bank.row_views(self.row, "grad")
        for k, p in self.model.named_parameters():
            v = views[k]
            if p.grad is None:
                v.zero_()
                p.grad = v
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v

    def flat_params(self) -> torch.Tensor:
        return self.bank.buffer("x")[self.row, : self.bank.P]

    def state_view(self) -> RowState:
        return RowState(self.bank, self.row)
