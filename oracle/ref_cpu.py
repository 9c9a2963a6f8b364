"""Reference-structured CPU consensus round — TEST/BENCH INFRASTRUCTURE.

bench.py's cpu_baseline leg times this on the GPU box's host cores.  It keeps
the reference's structure and torch CPU ops exactly:
  * Neighbors (DIST/simulators.py:91-97): scan j = 0..N-1 of W[i] (0-d tensor
    indexing), keep (W[i][j], agent j's state dict) when W[i][j] > 0;
  * consensus (DIST/clients.py:61-69): zeros_like + torch.mul(x_j, a) += ...;
  * synchronous write-back (DIST/simulators.py:151-152): load_state_dict,
    i.e. an in-place copy into each agent's tensors after all rows are mixed.
Agents here hold one flat tensor each (the synthetic workload has a single
parameter block of P floats).
"""
from __future__ import annotations

import time
from typing import Dict, List, Tuple

import torch


class Agent:
    def __init__(self, state: Dict[str, torch.Tensor]):
        self.state = state


def neighbors(i: int, W: torch.Tensor, agents: List[Agent]) -> List[Tuple[torch.Tensor, Dict[str, torch.Tensor]]]:
    out = []
    for j in range(len(agents)):
        a = W[i][j]
        if a > 0:
            out.append((a, agents[j].state))
    return out


def consensus(own: Dict[str, torch.Tensor], Ni) -> Dict[str, torch.Tensor]:
    acc = {k: torch.zeros_like(v) for k, v in own.items()}
    for a, sd in Ni:
        for k in sd:
            acc[k] += torch.mul(sd[k], a)
    return acc


def mixing_round(W: torch.Tensor, agents: List[Agent]) -> None:
    new = [consensus(ag.state, neighbors(i, W, agents)) for i, ag in enumerate(agents)]
    for ag, nw in zip(agents, new):
        for k, v in nw.items():
            ag.state[k].copy_(v)


def time_rounds(W: torch.Tensor, X: torch.Tensor, min_seconds: float = 10.0, max_rounds: int = 50,
                warmup: bool = True):
    """Run rounds on agents whose parameters are rows of X until min_seconds
    have elapsed (at least min(2, max_rounds) rounds).  Returns (rounds, seconds)."""
    agents = [Agent({"w": X[i]}) for i in range(X.shape[0])]
    if warmup:
        mixing_round(W, agents)  # allocator, thread pool
    t0 = time.perf_counter()
    r = 0
    while r < min(2, max_rounds) or (time.perf_counter() - t0 < min_seconds and r < max_rounds):
        mixing_round(W, agents)
        r += 1
    return r, time.perf_counter() - t0


def vectorized_ring_round(X: torch.Tensor, Y: torch.Tensor, w_prev: torch.Tensor, w_next: torch.Tensor) -> None:
    """The stronger CPU bar of SURVEY §8d(2): the same ring round with whole-
    matrix torch ops (no per-agent Python loop): Y = wp*X[i-1] + wn*X[i+1], the
    reference's rounding order without the +0 start (equal to the loop above
    except that a sum of two -0 products comes out -0 instead of +0).  A timing
    baseline only; parity is checked against dol_oracle.c."""
    torch.mul(torch.roll(X, 1, 0), w_prev[:, None], out=Y)
    Y.add_(torch.roll(X, -1, 0).mul_(w_next[:, None]))


def time_vectorized(X: torch.Tensor, w_prev: torch.Tensor, w_next: torch.Tensor, min_seconds: float = 5.0,
                    max_rounds: int = 200):
    Y = torch.empty_like(X)
    vectorized_ring_round(X, Y, w_prev, w_next)
    t0 = time.perf_counter()
    r = 0
    while r < 2 or (time.perf_counter() - t0 < min_seconds and r < max_rounds):
        vectorized_ring_round(X, Y, w_prev, w_next)
        X, Y = Y, X
        r += 1
    return r, time.perf_counter() - t0


# ---------------------------------------------------------------------------
# FedADMM round (BASELINE config 4's primal/dual side), reference-structured:
# FedAdmm_Client.update_weights (DEC/clients.py:36-53) with update_model's
# ADMM term (:125-139) and update_duals (:141-144), the server's deepcopy of
# every returned state dict and average_weights (DEC/servers.py:42-48), on the
# least-squares "model" f_k(w) = 1/2 ||w - t_k||^2 (autograd backward, as the
# reference's loss.backward()), torch.optim.SGD with momentum per client.
# ---------------------------------------------------------------------------
class _LSModel(torch.nn.Module):
    def __init__(self, P: int):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(P))


class AdmmClient:
    def __init__(self, target: torch.Tensor, rho: float, lr: float, momentum: float, local_ep: int):
        self.model = _LSModel(target.numel())
        self.target = target
        self.rho, self.local_ep = rho, local_ep
        self.alpha = {k: torch.zeros_like(v) for k, v in self.model.state_dict().items()}
        self.optimizer = torch.optim.SGD(self.model.parameters(), lr=lr, momentum=momentum)

    def update_model(self, theta):
        self.optimizer.zero_grad()
        self.model.zero_grad()
        loss = 0.5 * ((self.model.w - self.target) ** 2).sum()
        loss.backward()
        pre = self.model.state_dict()
        for name, param in self.model.named_parameters():
            param.grad = param.grad + (self.alpha[name] + self.rho * (pre[name] - theta[name]))
        return loss

    def update_weights(self, theta):
        self.model.load_state_dict(theta)
        for _ in range(self.local_ep):
            self.update_model(theta)
            self.optimizer.step()
        weights = self.model.state_dict()
        for k in self.alpha:
            self.alpha[k] = self.alpha[k] + self.rho * (weights[k] - theta[k])
        return self.model.state_dict()


def average_weights(w):
    import copy
    w_avg = copy.deepcopy(w[0])
    for key in w_avg.keys():
        for i in range(1, len(w)):
            w_avg[key] += w[i][key]
        w_avg[key] = torch.div(w_avg[key], len(w))
    return w_avg


def time_admm_rounds(n: int, P: int, local_ep: int = 10, rho: float = 0.1, lr: float = 0.1, momentum: float = 0.5,
                     rounds: int = 1, seed: int = 2028, warmup: bool = True):
    """One (or `rounds`) full-participation FedADMM rounds over n clients after a
    warm-up round; returns (rounds, seconds)."""
    import copy
    g = torch.Generator().manual_seed(seed)
    clients = [AdmmClient(torch.randn(P, generator=g), rho, lr, momentum, local_ep) for _ in range(n)]
    theta = {"w": torch.zeros(P)}

    def one(theta):
        local = [copy.deepcopy(c.update_weights(theta)) for c in clients]
        return average_weights(local)

    if warmup:
        theta = one(theta)  # warm-up (momentum buffers, allocator)
    t0 = time.perf_counter()
    for _ in range(rounds):
        theta = one(theta)
    return rounds, time.perf_counter() - t0


# ---------------------------------------------------------------------------
# Config 5 round, reference-structured: every agent's local step on its own
# nn.Module (DIST/clients.py:34-59: zero_grad, forward, CrossEntropyLoss,
# backward, SGD-with-momentum step) on a batch of B, then the synchronous
# consensus round with a new Erdos-Renyi W (Neighbors scan + consensus +
# load_state_dict, as mixing_round above).
# ---------------------------------------------------------------------------
def time_config5_rounds(n: int, d: int = 784, h: int = 128, c: int = 10, B: int = 32, p_edge: float = 0.1,
                        lr: float = 0.05, momentum: float = 0.5, rounds: int = 1, seed: int = 2028,
                        warmup: bool = True):
    from torch import nn
    torch.manual_seed(seed)
    models = [nn.Sequential(nn.Linear(d, h), nn.ReLU(), nn.Linear(h, c)) for _ in range(n)]
    opts = [torch.optim.SGD(m.parameters(), lr=lr, momentum=momentum) for m in models]
    crit = nn.CrossEntropyLoss()
    X = torch.randn(n, B, d)
    y = torch.randint(0, c, (n, B))

    class _A:
        def __init__(self, m):
            self.state = dict(m.state_dict())

    def er_w():
        A = (torch.rand(n, n) < p_edge).float()
        A.fill_diagonal_(0)
        Wt = torch.rand(n, n) * A
        s = Wt.sum(0)
        s[s == 0] = 1
        return (Wt / s).T

    def one():
        for k in range(n):
            opts[k].zero_grad()
            loss = crit(models[k](X[k]), y[k])
            loss.backward()
            opts[k].step()
        with torch.no_grad():
            mixing_round(er_w(), [_A(m) for m in models])

    if warmup:
        one()
    t0 = time.perf_counter()
    for _ in range(rounds):
        one()
    return rounds, time.perf_counter() - t0
