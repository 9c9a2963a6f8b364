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


class SeparableADMM:
    """FedADMM on the separable least-squares objective f_k(w) = 1/2 ||w - t_k||^2
    over stacked agent rows (BASELINE config 4's primal/dual side).

    One round is the reference's Server.run body (DEC/servers.py:50-81) with
    the CNN loss replaced by least squares:
      m = max(int(frac * N), 1); order = np.random.choice(range(N), m, replace=False)
      every sampled client: FedAdmm_Client.update_weights(theta) (DEC/clients.py:36-53)
        = w <- theta, local_steps x (update_model :125-139 + SGD.step :44), update_duals :141-144
        -> one fused kernel over the sampled rows (dol_admm_ls_round_f32)
      theta <- average_weights(new w in sampled order) (DEC/servers.py:42-48)
        -> dol_ordered_mean_f32, or across ranks parallel.global_mean_exact
           ("exact", bit-identical to one process) / parallel.global_mean
           ("fast": local ordered sums + all_reduce(SUM), then / m).
    The reference's server averages the primal rows only (no alpha/rho term in
    theta, DEC/servers.py:42-48), so its iteration does NOT reach the optimum
    mean_k t_k of sum_k f_k: with every client sampled each round, sum_k alpha_k
    = rho*N*(theta - theta_0) holds after every round, and the fixed point
    (w_k = theta, grad = 0 => alpha_k = t_k - theta) is
        theta* = (mean_k t_k + rho*theta_0) / (1 + rho)          (fixed_point())
    which the engine reproduces, bias included.
    Each client's momentum buffer persists across rounds (the reference's
    per-client torch.optim.SGD is never reset); its first step ever sets
    buf = g'.  Metrics per round: sum over sampled clients of
    ||w_k - theta||^2 (primal residual, pre-round theta) and ||alpha_k||^2.

    Sharded (torch.distributed initialised), two ways:
      shard="agents": rank r owns the contiguous agent block
        parallel.shard_bounds(N, world, r); every rank draws the same order
        (same seed), runs its local sampled rows, and the mean is the only
        collective ("exact": parallel.global_mean_exact, "fast": all_reduce).
      shard="columns" (VERDICT r05 item 6): rank r owns EVERY
        agent x the parameter columns parallel.column_bounds(P, world, r).  The
        objective is separable per coordinate, so each rank runs the fused round
        + ordered mean (dol_admm_ls_round_mean_f32) over all sampled agents on
        its columns, in the global sampled order: theta's block is exactly
        DEC/servers.py:42-48's mean with NO collective on the round path.  The
        residual metrics are per-rank partials, summed across ranks when
        `history` is read (a collective: every rank reads it).
    `round_fn` / `ordered_sum` inject CPU checkers in tests.
    """

    def __init__(self, n_agents: int, P: int, rho: float = 0.1, lr: float = 0.1, momentum: float = 0.5,
                 local_steps: int = 1, frac: float = 1.0, seed: int = 2028, device=None, mean: str = "exact",
                 group=None, metrics: bool = True, round_fn=None, ordered_sum=None, fused: Optional[bool] = None,
                 shard: str = "agents"):
        import numpy as np
        import torch.distributed as dist

        from . import ops, parallel
        from .bank import row_stride
        if mean not in ("exact", "fast"):
            raise ValueError("mean must be 'exact' or 'fast'")
        if shard not in ("agents", "columns"):
            raise ValueError("shard must be 'agents' or 'columns'")
        self.shard = shard
        self.N, self.P = int(n_agents), int(P)
        self.rho, self.lr, self.mu, self.local_steps = float(rho), float(lr), float(momentum), int(local_steps)
        self.m = max(int(frac * self.N), 1)
        self.mean_mode, self.group, self.metrics = mean, group, metrics
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if shard == "columns":
            # every agent, this rank's parameter columns [c0, c1): the kernels see Pl columns
            self.lo, self.hi = 0, self.N
            self.c0, self.c1 = parallel.column_bounds(self.P, self.world, self.rank)
            mean = self.mean_mode = "exact"  # each column block's mean IS the reference's order
        else:
            self.lo, self.hi = parallel.shard_bounds(self.N, self.world, self.rank)
            self.c0, self.c1 = 0, self.P
        self.Pl = self.c1 - self.c0
        self.n = self.hi - self.lo
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self._round = round_fn if round_fn is not None else ops.admm_ls_round
        self._osum = ordered_sum if ordered_sum is not None else ops.ordered_sum
        # the client round and the mean in one pass (dol_admm_ls_round_mean_f32)
        # wherever the mean is this rank's ordered sum of its own rows: one
        # process, or the 'fast' mean's local part; off with injected checkers
        # or DOL_ADMM_FUSED_MEAN=0
        import os
        auto = fused is None
        if fused is None:
            fused = os.environ.get("DOL_ADMM_FUSED_MEAN", "1") != "0"
        self.fused = bool(fused) and round_fn is None and ordered_sum is None and \
            (self.world == 1 or mean == "fast" or shard == "columns")
        if auto and self.fused and shard == "columns" and self.world > 1 and self.device.type == "cuda":
            # the one-pass kernel's parallelism is its column strips: below ~1024 lanes
            # per CU the two-kernel round (row-major client round, then the ordered
            # sum) is faster -- 5.15 vs 7.4 ms at 8192 x 2^17, a rank's block at 8
            # ranks (profiles/r06c_admm_narrow_ab.jsonl); same bits either way
            n_cu = torch.cuda.get_device_properties(self.device).multi_processor_count
            self.fused = self.Pl >= 4 * 1024 * n_cu
        self._round_mean = ops.admm_ls_round_mean
        self._parallel = parallel
        self.rs = np.random.RandomState(seed)  # the reference's np.random.choice stream (setup_seed)
        ld = row_stride(max(self.Pl, 1))
        dev = self.device
        self.w = torch.zeros(max(self.n, 1), ld, dtype=torch.float32, device=dev)
        self.alpha = torch.zeros_like(self.w)
        self.target = torch.empty_like(self.w)
        self.mom = torch.zeros_like(self.w) if self.mu != 0.0 else None
        # per-row seeds over the whole row: identical rows (and column blocks) for every sharding
        full_row = torch.empty(self.P, dtype=torch.float32, device=dev) if shard == "columns" else None
        for k in range(self.lo, self.hi):
            g = torch.Generator(device=dev).manual_seed(seed * 1000003 + k + 1)
            if full_row is None:
                self.target[k - self.lo, :self.P].normal_(generator=g)
            else:
                full_row.normal_(generator=g)
                self.target[k - self.lo, :self.Pl].copy_(full_row[self.c0:self.c1])
        del full_row
        g = torch.Generator(device=dev).manual_seed(seed)
        self.theta = torch.zeros(ld, dtype=torch.float32, device=dev)
        th = torch.empty(self.P, dtype=torch.float32, device=dev).normal_(generator=g)
        self.theta[:self.Pl].copy_(th[self.c0:self.c1])
        del th
        self.theta0 = self.theta.clone()
        self._theta_next = torch.zeros_like(self.theta)
        self.mom_started = np.zeros(max(self.n, 1), dtype=bool)
        self.rounds = 0
        self._pending = []  # per-round device metrics, read lazily (no sync on the round path)
        self._history = []

    def sample(self):
        """The sampled clients of the next round, in the reference's order."""
        return self.rs.choice(range(self.N), self.m, replace=False)

    def round(self, order=None) -> None:
        import numpy as np
        order = np.asarray(self.sample() if order is None else order, dtype=np.int64)
        if order.size < 1 or order.min() < 0 or order.max() >= self.N or len(set(order.tolist())) != order.size:
            raise ValueError(f"order must be distinct agent ids in [0, {self.N})")
        local = [int(g) - self.lo for g in order if self.lo <= g < self.hi]
        dev = self.device
        ml = len(local)
        rw = ra = None
        if self.shard == "columns":
            return self._column_round(order)
        if self.fused:
            return self._fused_round(order, local)
        if ml:
            rows = torch.as_tensor(local, dtype=torch.int32, device=dev)
            first = None
            if self.mom is not None:
                first = torch.as_tensor(~self.mom_started[local], dtype=torch.int32, device=dev)
            if self.metrics:
                rw = torch.empty(ml, dtype=torch.float64, device=dev)
                ra = torch.empty(ml, dtype=torch.float64, device=dev)
            self._round(self.w, self.alpha, self.target, self.theta, agents=rows, first=first, buf=self.mom,
                        rho=self.rho, lr=self.lr, momentum=self.mu, local_steps=self.local_steps, resid_sq=rw,
                        alpha_sq=ra, P=self.P)
            if self.mom is not None and self.local_steps > 0:
                self.mom_started[local] = True
        par = self._parallel
        if self.mean_mode == "exact":
            par.global_mean_exact(self.w, self.lo, self.hi, [int(g) for g in order], self.P, group=self.group,
                                  out=self._theta_next, ordered_sum=self._osum)
        else:
            par.global_mean(self.w, local, self.m, self.P, group=self.group, out=self._theta_next,
                            ordered_sum=self._osum)
        self.theta, self._theta_next = self._theta_next, self.theta
        if self.metrics:
            s = torch.zeros(2, dtype=torch.float64, device=dev)
            if ml:
                s[0] = rw.sum()
                s[1] = ra.sum()
            if self.world > 1:
                self._all_reduce(s)
            self._pending.append((self.rounds, s))
        self.rounds += 1

    def _all_reduce(self, s: torch.Tensor) -> torch.Tensor:
        """all_reduce(SUM) in place (gloo: device tensors staged through host memory)."""
        import torch.distributed as dist
        if s.device.type == "cuda" and self._parallel._backend(self.group) == "gloo":
            h = s.cpu()
            dist.all_reduce(h, group=self.group)
            s.copy_(h)
        else:
            dist.all_reduce(s, group=self.group)
        return s

    def _column_round(self, order) -> None:
        """shard="columns": every sampled agent's client round and the server's
        ordered mean on this rank's parameter columns, in the global sampled
        order, with no collective (the round and the mean of DEC/servers.py:
        50-81 are per coordinate; theta's block is the reference's bits)."""
        dev = self.device
        m = int(order.size)
        s = torch.zeros(2, dtype=torch.float64, device=dev) if self.metrics else None
        if self.Pl > 0:
            rows = torch.as_tensor(order, dtype=torch.int32, device=dev)
            first = None
            if self.mom is not None:
                first = torch.as_tensor(~self.mom_started[order], dtype=torch.int32, device=dev)
            if self.fused:
                self._round_mean(self.w, self.alpha, self.target, self.theta, agents=rows, first=first, buf=self.mom,
                                 rho=self.rho, lr=self.lr, momentum=self.mu, local_steps=self.local_steps,
                                 out=self._theta_next, scale=float(m), resid_total=s, P=self.Pl, validate=False)
            else:  # two passes (injected checkers / DOL_ADMM_FUSED_MEAN=0): the client round, then the ordered mean
                rw = ra = None
                if self.metrics:
                    rw = torch.empty(m, dtype=torch.float64, device=dev)
                    ra = torch.empty(m, dtype=torch.float64, device=dev)
                self._round(self.w, self.alpha, self.target, self.theta, agents=rows, first=first, buf=self.mom,
                            rho=self.rho, lr=self.lr, momentum=self.mu, local_steps=self.local_steps, resid_sq=rw,
                            alpha_sq=ra, P=self.Pl)
                self._osum(self.w, rows, out=self._theta_next, scale=float(m), P=self.Pl)
                if self.metrics:
                    s[0] = rw.sum()
                    s[1] = ra.sum()
        if self.mom is not None and self.local_steps > 0:
            self.mom_started[order] = True
        self.theta, self._theta_next = self._theta_next, self.theta
        if self.metrics:
            self._pending.append((self.rounds, s))  # this rank's columns only: summed in `history`
        self.rounds += 1

    def full_theta(self) -> torch.Tensor:
        """theta over all P columns on every rank (shard="columns": one
        all_gather of the column blocks; diagnostics and checkpoints, not on the
        round path)."""
        if self.shard != "columns" or self.world == 1:
            return self.theta[:self.P]
        return self._gather_columns(self.theta[:self.Pl])

    def _gather_columns(self, v: torch.Tensor) -> torch.Tensor:
        par = self._parallel
        bounds = [par.column_bounds(self.P, self.world, q) for q in range(self.world)]
        width = max(max(b - a for a, b in bounds), 1)
        pad = torch.zeros(width, dtype=v.dtype, device=v.device)
        pad[:v.numel()] = v
        parts = par._all_gather(pad, self.group)
        return torch.cat([parts[q][:b - a] for q, (a, b) in enumerate(bounds)])

    def _fused_round(self, order, local) -> None:
        """round() on dol_admm_ls_round_mean_f32: the client round and this
        rank's ordered sum of its new rows in one pass (one process: the mean
        itself, bit-identical to the two-kernel round; 'fast' mean: the local
        sum, then all_reduce + / m).  The residual metrics come as the round's
        totals (fp64, another fixed summation order than the per-agent path's:
        equal to ~1e-15 relative)."""
        dev = self.device
        ml = len(local)
        s = torch.zeros(2, dtype=torch.float64, device=dev) if self.metrics else None
        if ml:
            rows = torch.as_tensor(local, dtype=torch.int32, device=dev)
            first = None
            if self.mom is not None:
                first = torch.as_tensor(~self.mom_started[local], dtype=torch.int32, device=dev)
            self._round_mean(self.w, self.alpha, self.target, self.theta, agents=rows, first=first, buf=self.mom,
                             rho=self.rho, lr=self.lr, momentum=self.mu, local_steps=self.local_steps,
                             out=self._theta_next, scale=float(self.m) if self.world == 1 else 1.0,
                             resid_total=s, P=self.P, validate=False)
            if self.mom is not None and self.local_steps > 0:
                self.mom_started[local] = True
        else:  # a rank without sampled rows ('fast' mean): contributes zeros
            self._theta_next.zero_()
        if self.world > 1:
            self._parallel.global_mean_finish(self._theta_next, self.m, self.P, group=self.group)
        self.theta, self._theta_next = self._theta_next, self.theta
        if self.metrics:
            if self.world > 1:
                self._all_reduce(s)
            self._pending.append((self.rounds, s))
        self.rounds += 1

    @property
    def history(self):
        """Per-round metrics: {"round", "primal_resid_sq", "dual_sq"} (sums over
        the sampled clients).  shard="columns" at world > 1: the pending
        per-rank partials are summed across ranks here, in one all_reduce --
        every rank must read `history` at the same point."""
        if self._pending:
            if self.shard == "columns" and self.world > 1:
                stacked = self._all_reduce(torch.stack([s for _, s in self._pending]))
                self._pending = [(r, stacked[i]) for i, (r, _) in enumerate(self._pending)]
            for r, s in self._pending:
                v = s.cpu().tolist()
                self._history.append({"round": r, "primal_resid_sq": v[0], "dual_sq": v[1]})
        self._pending = []
        return self._history

    def optimum(self) -> torch.Tensor:
        """mean_k t_k in fp64 (the minimiser of sum_k f_k); all ranks (diagnostic)."""
        if self.shard == "columns":
            s = self.target[:self.n, :self.Pl].double().sum(0)
            return (s if self.world == 1 else self._gather_columns(s)) / self.N
        s = self.target[:self.n, :self.P].double().sum(0)
        if self.world > 1:
            self._all_reduce(s)
        return s / self.N

    def distance_to_optimum(self) -> float:
        """||theta - mean_k t_k|| / sqrt(P)."""
        return float((self.full_theta().double() - self.optimum()).norm() / self.P ** 0.5)

    def fixed_point(self) -> torch.Tensor:
        """theta* = (mean_k t_k + rho*theta_0) / (1 + rho): where the reference's
        iteration settles under full participation (see the class docstring)."""
        theta0 = self.theta0[:self.P] if self.shard != "columns" or self.world == 1 else \
            self._gather_columns(self.theta0[:self.Pl])
        return (self.optimum() + self.rho * theta0.double()) / (1.0 + self.rho)

    def distance_to_fixed_point(self) -> float:
        """||theta - theta*|| / sqrt(P) (full participation)."""
        return float((self.full_theta().double() - self.fixed_point()).norm() / self.P ** 0.5)


class SeparableDGDPM:
    """Config 3 on the parameter-major bank: the round of SeparableDGD (same
    objectives, same round order, bit-identical values) with every state
    matrix stored transposed, XT[p][i] = agent i's parameter p ([P, ld], ld =
    round_up(N, 4)), so that any sparse W streams the bank once
    (dol_dgd_csr_pm_f32).  Build it from a SeparableDGD
    (`from_agent_major`, which transposes that problem's current state) or
    fresh (random init drawn directly in this layout).  At most
    ops.PM_DGD_MAX_AGENTS agents."""

    def __init__(self, plan: MixingPlan, P: int, objective: str = "least_squares", lr: float = 0.01,
                 momentum: float = 0.0, local_steps: int = 1, seed: int = 2028, _state=None):
        from . import ops
        if plan.n_rows > ops.PM_DGD_MAX_AGENTS:
            raise ValueError(f"the parameter-major round takes at most {ops.PM_DGD_MAX_AGENTS} agents")
        if plan.kind == "dense":
            raise ValueError("the parameter-major round mixes a sparse (CSR) W")
        self.plan, self.P, self.objective = plan, int(P), objective
        self.lr, self.mu, self.local_steps = float(lr), float(momentum), int(local_steps)
        self.N = plan.n_rows
        self.ld = (self.N + 3) // 4 * 4
        dev = plan.device
        shape = (self.P, self.ld)
        self.XT = torch.zeros(shape, dtype=torch.float32, device=dev)
        self.YT = torch.zeros_like(self.XT)
        self.TT = torch.zeros_like(self.XT)
        self.MT = torch.zeros_like(self.XT) if self.mu != 0.0 else None
        self.first, self.rounds = True, 0
        if _state is None:
            g = torch.Generator(device=dev).manual_seed(seed)
            self.XT[:, :self.N].normal_(generator=g)
            self.TT[:, :self.N].normal_(generator=g)
            if objective == "logistic":
                t = self.TT[:, :self.N]
                t.copy_(torch.where(torch.rand(t.shape, generator=g, device=dev) < 0.5, -t, t))

    @classmethod
    def from_agent_major(cls, prob: "SeparableDGD") -> "SeparableDGDPM":
        """Transpose prob's current state (x, targets, momentum, first-step flag)."""
        from . import ops
        self = cls(prob.plan, prob.P, prob.objective, prob.lr, prob.mu, prob.local_steps, _state=True)
        ops.transpose(prob.params(), self.XT, prob.plan.n_rows, prob.P)
        ops.transpose(prob.targets(), self.TT, prob.plan.n_rows, prob.P)
        if self.MT is not None:
            ops.transpose(prob.momentum_rows(), self.MT, prob.plan.n_rows, prob.P)
        self.first, self.rounds = prob.first, prob.rounds
        return self

    def round(self) -> None:
        """X <- W X, then the local steps (one kernel); swaps XT / YT."""
        from . import ops
        p = self.plan
        ops.dgd_csr_pm(self.XT, self.YT, p.rowptr, p.col, p.val, self.TT, self.MT, objective=self.objective,
                       steps=self.local_steps, lr=self.lr, momentum=self.mu, first_step=self.first, P=self.P)
        self.XT, self.YT = self.YT, self.XT
        self.first = False
        self.rounds += 1

    def params(self) -> torch.Tensor:
        """Agent-major copy [N, P] of the current parameters (diagnostic)."""
        return self.XT[:, :self.N].T.contiguous()

    def momentum_rows(self) -> Optional[torch.Tensor]:
        return None if self.MT is None else self.MT[:, :self.N].T.contiguous()

    def consensus_error(self) -> float:
        x = self.XT[:, :self.N]
        return float((x - x.mean(1, keepdim=True)).norm() / max(1, self.N) ** 0.5)


class TimeVaryingMLPGossip:
    """BASELINE config 5 as a first-class round: N agents, each an
    nn.Sequential(Linear(d, h), ReLU(), Linear(h, c)) row of the bank, a new
    Erdos-Renyi p W drawn every round ('stochastic' weighting,
    DIST/simulators.py:65-70), one local momentum-SGD step per agent on its
    batch (DIST/clients.py:34-59: forward, CrossEntropyLoss, backward, step;
    the fused dol_mlp_step_f32), then the synchronous consensus round with that
    W (DIST/clients.py:61-69, bit-exact: device Neighbors + the LDS-gather CSR
    kernel).  One process per GPU: with torch.distributed initialised, rank r
    owns the agent block shard_bounds(N, world, r) and the mix runs through
    parallel.AgentColumnTranspose (bit-identical to one GPU).  The round's W
    draw + CSR build runs on a side stream, overlapped with the local step.

    batch(X, y): per-agent batches for this rank's agents ([n_local, B, d] float32,
    [n_local, B] int64), kept until replaced."""

    def __init__(self, n_agents: int, d: int = 784, h: int = 128, c: int = 10, p_edge: float = 0.1,
                 lr: float = 0.05, momentum: float = 0.5, seed: int = 2028, device=None, group=None,
                 init_std: float = 0.05, overlap_chunks: int = 2):
        import torch.distributed as dist
        from . import parallel
        from .mlp import BatchedMLP, mlp_layout
        self.N, self.d, self.h, self.c = int(n_agents), d, h, c
        self.p_edge, self.lr, self.mu, self.seed = float(p_edge), float(lr), float(momentum), int(seed)
        self.device = torch.device("cuda" if device is None else device)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.lo, self.hi = parallel.shard_bounds(self.N, self.world, self.rank)
        self.n_local = self.hi - self.lo
        self.bank = AgentBank(self.n_local, mlp_layout(d, h, c), self.device)
        self.P = self.bank.P
        self.mlp = BatchedMLP(self.bank, d, h, c)
        # every agent's initial row from one global stream: the same model whatever the sharding
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        full = torch.empty(self.N, self.P, device=self.device).normal_(0, init_std, generator=g)
        self.bank.rows()[:] = full[self.lo:self.hi]
        del full
        self.bank.buffer("y").zero_()
        if self.mu != 0.0:
            self.bank.buffer("mom", zero=True)
        self.tr = parallel.AgentColumnTranspose(self.N, self.P, self.device, group) if self.world > 1 else None
        self.overlap_chunks = max(1, int(overlap_chunks))  # pieces of the local step overlapped with the exchange
        self._W = torch.empty(self.N, self.N, device=self.device)
        self._plan = None
        self._side = torch.cuda.Stream(self.device)
        self.X = self.y = None
        self.rounds = 0
        self.last_loss = None  # the latest round's per-agent losses (round() returns them too)

    def batch(self, X: torch.Tensor, y: torch.Tensor) -> None:
        if X.shape[:1] != (self.n_local,) or y.shape[:1] != (self.n_local,) or X.shape[-1] != self.d:
            raise ValueError(f"batch: expected X [{self.n_local}, B, {self.d}] and y [{self.n_local}, B]")
        self.X, self.y = X, y

    def round_seed(self, r: int) -> int:
        return self.seed * 1000003 + r + 1

    def round(self) -> torch.Tensor:
        """One round; returns this rank's per-agent losses (device tensor)."""
        from . import graph as G
        if self.X is None:
            raise RuntimeError("TimeVaryingMLPGossip.round: call batch() first")
        main = torch.cuda.current_stream(self.device)
        self._side.wait_stream(main)  # the previous round's mix has consumed the old plan
        with torch.cuda.stream(self._side):
            W = G.erdos_renyi_stochastic_hip(self.N, self.p_edge, self.round_seed(self.rounds), self.device,
                                             out=self._W)
            # balanced pack: it runs here, on the side stream, under the local step
            self._plan = G.MixingPlan.from_dense(W, dense_kernel="csr", reuse=self._plan, balance=True)
        if self.tr is None:
            loss = self.mlp.step(self.X, self.y, lr=self.lr, momentum=self.mu, first_step=(self.rounds == 0))
            self._plan_ready(main)
            self.bank.mix(self._plan)
        else:
            # the local steps in pieces, each piece's first exchange posted while
            # the next piece steps (parallel.AgentColumnTranspose.mix_with_local_steps)
            loss = torch.empty(self.n_local, dtype=torch.float32, device=self.device)

            def step_rows(a, b):
                self.mlp.step(self.X, self.y, lr=self.lr, momentum=self.mu, first_step=(self.rounds == 0),
                              rows=slice(a, b), loss=loss)

            def before_mix():
                self._plan_ready(main)
                self.tr.set_plan(self._plan)
            self.tr.mix_with_local_steps(self.bank.rows(), step_rows, chunks=self.overlap_chunks,
                                         before_mix=before_mix)
        self.rounds += 1
        self.last_loss = loss
        return loss

    def _plan_ready(self, main) -> None:
        """The compute stream waits for the side stream's W draw + plan build."""
        main.wait_stream(self._side)
        # the plan's buffers were allocated on the side stream and are read on the
        # main one: tell the caching allocator, so freeing them never races the mix
        for t in (self._plan.rowptr, self._plan.col, self._plan.val, self._plan.ent, self._plan.hdr):
            if t is not None:
                t.record_stream(main)

    def params(self) -> torch.Tensor:
        return self.bank.rows()
