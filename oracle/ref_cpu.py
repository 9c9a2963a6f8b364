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
