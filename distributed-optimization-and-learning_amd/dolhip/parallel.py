"""Agent sharding across ranks (one process per GPU, torch.distributed).

The reference runs every agent in one process and "sends" a row by reading
another agent's state_dict (DIST/simulators.py:96); its server "all-reduce"
is a Python loop (DEC/servers.py:44-47).  Here agents are split into
contiguous blocks, one block per rank:

* ring mixing: the only cross-rank data are the two boundary rows.  Each round
  the interior rows are mixed on the compute stream while the halo rows travel
  (send/recv over RCCL/xGMI, or gloo on CPU), then the two boundary rows are
  mixed.  Results are bit-identical to the single-GPU mix for every world size
  (each output row sees the same two products added in the same order).
* parameter-dimension sharding (ColumnSharded): for graphs whose
  edges are not local in agent order (random-regular, Erdős–Rényi, dense W)
  an agent block would need most of X from other ranks every round; instead
  each rank owns ALL agents x a contiguous block of parameter columns, and
  Y[:, cols] = W X[:, cols] (also the fused config-3 DGD round, whose local
  steps are per-coordinate) needs no communication at all.  Bit-identical to
  one GPU: every column's arithmetic is unchanged.
* global mean (FedAvg / FedProx / FedADMM server average): each rank sums its
  local sampled rows in sampled order, then `all_reduce(SUM)` and a division
  by m ("fast", association order differs from the reference by rank), or
  ("exact": bit-identical to DEC/servers.py:42-48) one all_to_all of the
  sampled rows to parameter-column blocks, an ordered sum in the global
  sampled order per block, and one all_gather of theta.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import ops
from .bank import device_matrix, row_stride

# Fail fast instead of hanging: every collective of the engine's
# process groups is bounded by this timeout.  The reference has no collectives
# (its server loop, DEC/servers.py:44-47, and its neighbour reads,
# DIST/simulators.py:147-152, are in-process), so a stuck peer is a failure
# mode this engine adds and must surface as an error.
DEFAULT_TIMEOUT_S = float(os.environ.get("DOL_COLLECTIVE_TIMEOUT_S", "300"))


def init_process_group(backend: str, rank: Optional[int] = None, world_size: Optional[int] = None,
                       device=None, timeout_s: Optional[float] = None) -> None:
    """torch.distributed.init_process_group with a bounded timeout on every
    collective and RCCL's asynchronous error handling on: a rank that dies or
    stops participating makes the others raise (gloo) or abort their
    communicators (nccl = RCCL: the watchdog tears the process down) within
    `timeout_s` (DOL_COLLECTIVE_TIMEOUT_S, default 300 s) instead of hanging.
    The environment switch is set in-process before the group exists (no
    re-exec).  device: the rank's GPU for nccl (device_id, eager init)."""
    timeout = datetime.timedelta(seconds=float(DEFAULT_TIMEOUT_S if timeout_s is None else timeout_s))
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = {"timeout": timeout}
    if rank is not None:
        kw["rank"] = rank
    if world_size is not None:
        kw["world_size"] = world_size
    if backend == "nccl" and device is not None:
        kw["device_id"] = torch.device(device)
    dist.init_process_group(backend, **kw)


def _backend(group=None) -> str:
    """The group's backend.  Every backend-dependent branch of this module asks
    here (tests/test_parallel_gloo.py::test_every_rccl_line_runs_under_gloo
    answers "nccl" over a gloo group of CPU tensors, so the lines RCCL runs
    execute on the CPU tier)."""
    return dist.get_backend(group)


def _wait_all(reqs, group=None) -> None:
    """Wait for point-to-point requests.  gloo: bounded by DEFAULT_TIMEOUT_S on
    the host (a recv whose peer never sends raises instead of blocking
    forever).  nccl: a plain wait (the compute stream waits on the transfer,
    the host does not block; a timeout here would stall the host every round),
    with the hang bound by the group's timeout + RCCL's async error handling
    set up by init_process_group."""
    bounded = _backend(group) == "gloo"
    for r in reqs:
        if bounded:
            r.wait(datetime.timedelta(seconds=DEFAULT_TIMEOUT_S))  # gloo-only
        else:
            r.wait()


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of agent rows owned by `rank`."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


class ShardedRing:
    """Ring (circle) mixing of a globally N-agent system, sharded by rows.

    x/y: local [n_local, ld] buffers (allocated here; mapped as
    bank.device_matrix); w_prev/w_next: the GLOBAL ring weights [N] (host or
    device); the local slice is kept.
    """

    def __init__(self, n_agents: int, P: int, w_prev, w_next, device, ld: Optional[int] = None,
                 group=None, alloc: bool = True, mix_ring=None, dgd_ring=None, mix_edges=None, dgd_edges=None,
                 mapped: Optional[bool] = None, stage_sends: Optional[bool] = None):
        # mix_ring / dgd_ring / *_edges: kernel entries (default: the HIP ops); tests
        # inject CPU checkers.  The boundary rows go in ONE launch (dol_*_ring_edges_f32);
        # with an injected mix and no injected edge entry they go through the mix, one row each.
        self._mix = mix_ring if mix_ring is not None else ops.mix_ring
        self._dgd = dgd_ring if dgd_ring is not None else ops.dgd_ring
        self._mix_edges = mix_edges if mix_edges is not None else (ops.mix_ring_edges if mix_ring is None else None)
        self._dgd_edges = dgd_edges if dgd_edges is not None else (ops.dgd_ring_edges if dgd_ring is None else None)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if n_agents < max(3, 2 * self.world):
            raise ValueError("ring sharding needs >= 3 agents and >= 2 agents per rank")
        self.N, self.P = n_agents, P
        self.device = torch.device(device)
        self.lo, self.hi = shard_bounds(n_agents, self.world, self.rank)
        self.n_local = self.hi - self.lo
        self.ld = ld if ld is not None else row_stride(P)
        wp = torch.as_tensor(w_prev, dtype=torch.float32)
        wn = torch.as_tensor(w_next, dtype=torch.float32)
        self.w_prev = wp[self.lo:self.hi].contiguous().to(self.device)
        self.w_next = wn[self.lo:self.hi].contiguous().to(self.device)
        self.prev_rank = (self.rank - 1) % self.world
        self.next_rank = (self.rank + 1) % self.world
        if alloc:
            # x / y as bank matrices (mapped blocks of >= 1 GiB by default, the same
            # memory as at world 1); across ranks the two boundary rows are copied
            # into torch-allocated send buffers first (stage_sends), so RCCL only
            # ever sees the memory PyTorch RCCL users hand it
            self.x = device_matrix(self.n_local, self.ld, self.device, mapped=mapped)
            self.y = device_matrix(self.n_local, self.ld, self.device, mapped=mapped)
        self.halo_prev = torch.empty(self.ld, dtype=torch.float32, device=self.device)
        self.halo_next = torch.empty(self.ld, dtype=torch.float32, device=self.device)
        if stage_sends is None:
            stage_sends = self.world > 1 and self.device.type == "cuda"
        self.stage_sends = bool(stage_sends)
        self._send = torch.empty(2, self.ld, dtype=torch.float32, device=self.device) if self.stage_sends else None
        # optional (start, end) timing events recorded around the interior kernel
        self.kernel_events = None

    def _staged(self) -> bool:
        """gloo cannot send device tensors: stage the halo rows through host memory."""
        return self.device.type == "cuda" and _backend(self.group) == "gloo"

    def _exchange(self, x: torch.Tensor):
        """Post the halo send/recv pairs; returns the requests.

        Order is fixed so that world == 2 (prev == next) still pairs correctly:
        first the 'downstream' message (my last row -> next rank's halo_prev),
        then the 'upstream' one (my first row -> prev rank's halo_next)."""
        P = self.P
        first, last = x[0, :P], x[self.n_local - 1, :P]
        hp, hn = self.halo_prev[:P], self.halo_next[:P]
        if self.stage_sends:  # the boundary rows leave from torch-allocated buffers (x may be a mapped block)
            self._send[0, :P].copy_(first)
            self._send[1, :P].copy_(last)
            first, last = self._send[0, :P], self._send[1, :P]
        if self._staged():
            first, last = first.cpu(), last.cpu()  # staged
            self._host_halo = (torch.empty(P), torch.empty(P))  # staged
            hp, hn = self._host_halo  # staged
        ops_ = [
            dist.P2POp(dist.isend, last, self.next_rank, self.group, tag=0),
            dist.P2POp(dist.irecv, hp, self.prev_rank, self.group, tag=0),
            dist.P2POp(dist.isend, first, self.prev_rank, self.group, tag=1),
            dist.P2POp(dist.irecv, hn, self.next_rank, self.group, tag=1),
        ]
        return dist.batch_isend_irecv(ops_)

    def _finish_exchange(self, reqs) -> None:
        _wait_all(reqs, self.group)
        if self._staged():
            self.halo_prev[: self.P].copy_(self._host_halo[0])  # staged
            self.halo_next[: self.P].copy_(self._host_halo[1])  # staged

    def step(self, x: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None) -> None:
        """One Jacobi round Y = W X on the local block (then swap if using own buffers)."""
        own = x is None
        x = self.x if own else x
        y = self.y if own else y
        n, P = self.n_local, self.P
        if self.world == 1:
            self._mix(x, y, self.w_prev, self.w_next, P=P, n_rows=n)
        else:
            reqs = self._exchange(x)
            # interior rows 1..n-2: their neighbours are all local
            if n > 2:
                ev = self.kernel_events
                if ev:
                    ev[0].record()
                self._mix(x[1:], y[1:], self.w_prev[1:], self.w_next[1:], halo_prev=x[0],
                          halo_next=x[n - 1], P=P, n_rows=n - 2)
                if ev:
                    ev[1].record()
            self._finish_exchange(reqs)
            # boundary rows 0 and n-1
            if self._mix_edges is not None:
                self._mix_edges(x, y, self.w_prev, self.w_next, self.halo_prev, self.halo_next, P=P, n_rows=n)
            else:
                self._mix(x[0:1], y[0:1], self.w_prev[0:1], self.w_next[0:1], halo_prev=self.halo_prev,
                          halo_next=x[1], P=P, n_rows=1)
                self._mix(x[n - 1:n], y[n - 1:n], self.w_prev[n - 1:n], self.w_next[n - 1:n],
                          halo_prev=x[n - 2], halo_next=self.halo_next, P=P, n_rows=1)
        if own:
            self.x, self.y = self.y, self.x

    def dgd_step(self, target: torch.Tensor, mom: Optional[torch.Tensor] = None, **kw) -> None:
        """One fused config-3 round (mix + local steps, dol_dgd_ring_f32) on the
        local block; target / mom are the LOCAL [n_local, >=P] rows.  Same halo
        schedule as step(); bit-identical to the single-GPU round."""
        x, y = self.x, self.y
        n, P = self.n_local, self.P
        m = (lambda a, b: None) if mom is None else (lambda a, b: mom[a:b])
        if self.world == 1:
            self._dgd(x, y, self.w_prev, self.w_next, target, mom=mom, P=P, n_rows=n, **kw)
        else:
            reqs = self._exchange(x)
            if n > 2:
                ev = self.kernel_events
                if ev:
                    ev[0].record()
                self._dgd(x[1:], y[1:], self.w_prev[1:], self.w_next[1:], target[1:], mom=m(1, n - 1),
                          halo_prev=x[0], halo_next=x[n - 1], P=P, n_rows=n - 2, **kw)
                if ev:
                    ev[1].record()
            self._finish_exchange(reqs)
            if self._dgd_edges is not None:
                self._dgd_edges(x, y, self.w_prev, self.w_next, target, self.halo_prev, self.halo_next, mom=mom,
                                P=P, n_rows=n, **kw)
            else:
                self._dgd(x[0:1], y[0:1], self.w_prev[0:1], self.w_next[0:1], target[0:1], mom=m(0, 1),
                          halo_prev=self.halo_prev, halo_next=x[1], P=P, n_rows=1, **kw)
                self._dgd(x[n - 1:n], y[n - 1:n], self.w_prev[n - 1:n], self.w_next[n - 1:n], target[n - 1:n],
                          mom=m(n - 1, n), halo_prev=x[n - 2], halo_next=self.halo_next, P=P, n_rows=1, **kw)
        self.x, self.y = self.y, self.x


def column_bounds(P: int, world: int, rank: int, align: int = 64) -> Tuple[int, int]:
    """Contiguous block [c0, c1) of the parameter dimension owned by `rank`, cut
    on multiples of `align` floats (16-B lanes, whole 256-B tiles)."""
    units = (P + align - 1) // align
    lo, hi = shard_bounds(units, world, rank)
    return min(lo * align, P), min(hi * align, P)


class ColumnSharded:
    """Mixing with ANY W sharded over the parameter dimension (one process per
    GPU).  x / y: local [N, ld] buffers holding columns [c0, c1) of every agent.
    `step()` = one Jacobi round; `dgd_step()` = one fused config-3 round with
    the local `target` / `mom` blocks.  No collective on the data path."""

    def __init__(self, plan, P: int, device, group=None, alloc: bool = True, apply=None, apply_dgd=None):
        # apply / apply_dgd: kernel entries (default: the plan's HIP ops); tests inject a CPU checker
        self.plan = plan
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.N, self.P = plan.n_rows, P
        self.c0, self.c1 = column_bounds(P, self.world, self.rank)
        self.Pl = self.c1 - self.c0
        self.device = torch.device(device)
        self.ld = row_stride(max(self.Pl, 1))
        self._injected = (apply, apply_dgd)  # kept across set_plan (the tests' CPU checkers)
        self._apply = apply if apply is not None else plan.apply
        self._apply_dgd = apply_dgd if apply_dgd is not None else plan.apply_dgd
        if alloc:
            self.x = torch.empty(self.N, self.ld, dtype=torch.float32, device=self.device)
            self.y = torch.empty_like(self.x)

    def set_plan(self, plan, apply=None, apply_dgd=None) -> None:
        """A new W for the next rounds (time-varying graphs, BASELINE config 5:
        every rank draws the same W from the round's seed); same agent count.
        Entries injected at construction (or passed here) stay in use; the
        others follow the new plan's HIP ops."""
        if (plan.n_rows, plan.n_cols) != (self.N, self.plan.n_cols):
            raise ValueError("set_plan: the new W must have the same shape")
        self.plan = plan
        if apply is not None or apply_dgd is not None:
            self._injected = (apply if apply is not None else self._injected[0],
                              apply_dgd if apply_dgd is not None else self._injected[1])
        inj_apply, inj_dgd = self._injected
        self._apply = inj_apply if inj_apply is not None else plan.apply
        self._apply_dgd = inj_dgd if inj_dgd is not None else plan.apply_dgd

    def local_cols(self, full: torch.Tensor) -> torch.Tensor:
        """This rank's column block of a full [N, >=P] matrix."""
        return full[:, self.c0:self.c1]

    def step(self) -> None:
        if self.Pl > 0:
            self._apply(self.x, self.y, P=self.Pl)
        self.x, self.y = self.y, self.x

    def dgd_step(self, target: torch.Tensor, mom: Optional[torch.Tensor] = None, **kw) -> None:
        if self.Pl > 0:
            self._apply_dgd(self.x, self.y, target, mom=mom, P=self.Pl, **kw)
        self.x, self.y = self.y, self.x

    def gather(self, dst: int = 0) -> Optional[torch.Tensor]:
        """Full [N, P] on rank `dst` (checkpoints / tests; not on the round path)."""
        mine = self.x[:, :self.Pl].contiguous()
        if self.world == 1:
            return mine
        staged = mine.device.type == "cuda" and _backend(self.group) == "gloo"
        send = mine.cpu() if staged else mine
        if self.rank != dst:
            if self.Pl > 0:
                dist.send(send, dst=dst, group=self.group)
            return None
        parts = []
        for r in range(self.world):
            a, b = column_bounds(self.P, self.world, r)
            if r == self.rank:
                parts.append(send)
            elif b > a:  # uneven blocks: point-to-point with known shapes
                t = torch.empty(self.N, b - a, dtype=torch.float32, device=send.device)
                dist.recv(t, src=r, group=self.group)
                parts.append(t)
        return torch.cat(parts, dim=1)


class AgentColumnTranspose:
    """Config 5 across GPUs: per-agent nonlinear local steps AND a non-local W.

    The local step (`BatchedMLP.step`, DIST/clients.py:34-59) needs whole agent
    rows, so each rank r keeps its agents [lo_r, hi_r) agent-major (`rows`: an
    [n_local, >=P] bank view).  The mix with an Erdos-Renyi / dense W needs
    every agent, so `mix()` transposes the bank to parameter-column blocks with
    one all_to_all (rank r receives columns column_bounds(P, world, r) of all N
    agents, `cols`: [N, Pc_r]), mixes that block locally with the round's plan
    (the same W on every rank: drawn from the shared seed; exact slab kernel;
    no collective), and transposes back with a second all_to_all.  Per rank and
    round that moves 2 (world-1)/world of its own rows' bytes -- against
    (world-1) x that for an all_gather of X -- and every output element is the
    same computation as on one GPU (bit-identical).  NCCL (= RCCL) exchanges
    device tensors directly; gloo stages through host memory (rehearsal).

    apply(X, Y, P=...): the column-block mix (default: the plan's HIP op; tests
    inject a CPU checker)."""

    def __init__(self, n_agents: int, P: int, device, group=None, apply=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.N, self.P = n_agents, P
        self.device = torch.device(device)
        self.lo, self.hi = shard_bounds(n_agents, self.world, self.rank)
        self.n_local = self.hi - self.lo
        self.row_bounds = [shard_bounds(n_agents, self.world, q) for q in range(self.world)]
        self.col_bounds = [column_bounds(P, self.world, q) for q in range(self.world)]
        self.c0, self.c1 = self.col_bounds[self.rank]
        self.Pc = self.c1 - self.c0
        ldc = row_stride(max(self.Pc, 1))
        self.cols = torch.empty(self.N, ldc, dtype=torch.float32, device=self.device)
        self.cols_out = torch.empty_like(self.cols)
        self._apply = apply
        self.plan = None
        # exchange buffers, allocated once (the same sizes every round): rows ->
        # columns sends n_local x P and receives N x Pc floats, and back
        self._buf_rows = torch.empty(max(self.n_local * P, 1), dtype=torch.float32, device=self.device)
        self._buf_cols = torch.empty(max(self.N * self.Pc, 1), dtype=torch.float32, device=self.device)
        # r04: when the column block is a whole number of 16-B pieces, the mix reads
        # the received [N, Pc] block in place and writes the send buffer of the
        # way back (two staging copies fewer per round: direct=True)
        self.direct = self.world > 1 and self.Pc > 0 and self.Pc % 4 == 0
        self._buf_cols2 = (torch.empty(self.N * self.Pc, dtype=torch.float32, device=self.device)
                           if self.direct else None)
        self._stage = None  # mix_with_local_steps: the pieces' receive staging (allocated on first use)
        self._side = None

    def set_plan(self, plan) -> None:
        if (plan.n_rows, plan.n_cols) != (self.N, self.N):
            raise ValueError("AgentColumnTranspose.set_plan: W must be N x N")
        self.plan = plan

    def _staged(self) -> bool:
        return self.device.type == "cuda" and _backend(self.group) == "gloo"

    def _all_to_all(self, send: torch.Tensor, recv: torch.Tensor, send_splits, recv_splits) -> None:
        if self._staged():
            hs, hr = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)  # staged
            dist.all_to_all_single(hr, hs, recv_splits, send_splits, group=self.group)  # staged
            recv.copy_(hr)  # staged
        else:
            dist.all_to_all_single(recv, send, recv_splits, send_splits, group=self.group)

    def to_columns(self, rows: torch.Tensor) -> None:
        """rows [n_local, >=P] (this rank's agents) -> self.cols [N, Pc] (all agents, my columns)."""
        P, n = self.P, self.n_local
        if self.world == 1:
            self.cols[:, :P].copy_(rows[:, :P])
            return
        send = self._pack_rows(rows)
        recv = self._buf_cols[:self.N * self.Pc]
        self._all_to_all(send, recv, [n * (b - a) for a, b in self.col_bounds],
                         [(h - l) * self.Pc for l, h in self.row_bounds])
        # from rank q: its agents x my columns, in rank (= agent) order
        self.cols[:, :self.Pc].copy_(recv.view(self.N, self.Pc))

    def from_columns(self, rows: torch.Tensor) -> None:
        """self.cols_out [N, Pc] -> rows [n_local, >=P] (this rank's agents, every column)."""
        P, n = self.P, self.n_local
        if self.world == 1:
            rows[:, :P].copy_(self.cols_out[:, :P])
            return
        send = self._buf_cols[:self.N * self.Pc]
        send.view(self.N, self.Pc).copy_(self.cols_out[:, :self.Pc])  # to rank q: its agents x my columns
        recv = self._buf_rows[:n * P]
        self._all_to_all(send, recv, [(h - l) * self.Pc for l, h in self.row_bounds],
                         [n * (b - a) for a, b in self.col_bounds])
        self._unpack_rows(recv, rows)

    def _pack_rows(self, rows: torch.Tensor) -> torch.Tensor:
        P, n = self.P, self.n_local
        send = self._buf_rows[:n * P]
        off = 0
        for a, b in self.col_bounds:  # to rank q: my rows x its columns
            send[off:off + n * (b - a)].view(n, b - a).copy_(rows[:, a:b])
            off += n * (b - a)
        return send

    def _unpack_rows(self, recv: torch.Tensor, rows: torch.Tensor) -> None:
        n, off = self.n_local, 0
        for a, b in self.col_bounds:  # from rank q: my agents x its columns
            w = b - a
            rows[:, a:b].copy_(recv[off:off + n * w].view(n, w))
            off += n * w

    def _apply_block(self, X: torch.Tensor, Y: torch.Tensor) -> None:
        if self._apply is not None:
            self._apply(X, Y, P=self.Pc)
        else:
            if self.plan is None:
                raise RuntimeError("AgentColumnTranspose.mix: set_plan() first")
            self.plan.apply(X, Y, P=self.Pc)

    def _chunk_bounds(self, q: int, chunks: int) -> List[Tuple[int, int]]:
        """Rank q's local rows cut into `chunks` contiguous pieces (some may be empty)."""
        n_q = self.row_bounds[q][1] - self.row_bounds[q][0]
        return [shard_bounds(n_q, chunks, c) for c in range(chunks)]

    def mix_with_local_steps(self, rows: torch.Tensor, step_rows, chunks: int = 2,
                             out: Optional[torch.Tensor] = None, before_mix=None) -> torch.Tensor:
        """The round's local steps AND its mix, with the first exchange
        overlapped with the steps: this rank's agent rows
        are stepped in `chunks` contiguous pieces (step_rows(a, b): the local
        step of local rows [a, b), enqueued on the current stream); as soon as
        piece c is enqueued, piece c + 1 is enqueued too, and piece c is packed
        on a side stream and sent to the column blocks by its own all_to_all
        (NCCL: on RCCL's stream, behind the pack; the next piece's step runs
        meanwhile).  The side stream places each received piece at its agents'
        rows of the [N, Pc] block, the compute stream waits for all of them,
        and the mix and the way back are those of mix().  Every element is the
        same computation as step-all-then-mix() (bit-identical): the steps are
        per agent and the block is the same block.  before_mix(): called on the
        compute stream right before the mix (e.g. wait for the round's W)."""
        out = rows if out is None else out
        if self.world == 1:
            step_rows(0, self.n_local)
            if before_mix is not None:
                before_mix()
            return self.mix(rows, out)
        N, P, Pc, n = self.N, self.P, self.Pc, self.n_local
        dev = self.device
        main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        side = self._side_stream()
        mine = self._chunk_bounds(self.rank, chunks)
        block = self._buf_cols[:N * Pc].view(N, Pc) if Pc > 0 else None
        if self._stage is None or self._stage.numel() < max(N * Pc, 1):
            self._stage = torch.empty(max(N * Pc, 1), dtype=torch.float32, device=dev)
        posted = []
        stage_off = 0
        step_rows(*mine[0])
        for c in range(chunks):
            a, b = mine[c]
            ev = None
            if main is not None:
                ev = torch.cuda.Event()  # device-only
                ev.record(main)  # device-only
            if c + 1 < chunks:  # the next piece's step goes in before this piece's exchange
                step_rows(*mine[c + 1])
            src = [self._chunk_bounds(s, chunks)[c] for s in range(self.world)]
            m_src = [hi - lo for lo, hi in src]
            stage = self._stage[stage_off:stage_off + sum(m_src) * Pc]
            stage_off += sum(m_src) * Pc
            with self._on(side):
                if ev is not None:
                    side.wait_event(ev)  # device-only
                send = self._buf_rows[a * P:b * P]
                off = 0
                for qa, qb in self.col_bounds:  # to rank q: my piece's rows x its columns
                    if b > a and qb > qa:
                        send[off:off + (b - a) * (qb - qa)].view(b - a, qb - qa).copy_(rows[a:b, qa:qb])
                    off += (b - a) * (qb - qa)
                handle = self._post_all_to_all(stage, send, [m * Pc for m in m_src],
                                               [(b - a) * (qb - qa) for qa, qb in self.col_bounds])
            posted.append((handle, stage, src))
        with self._on(side):
            for handle, stage, src in posted:
                self._finish_all_to_all(handle, stage)
                off = 0
                for s, (lo, hi) in enumerate(src):
                    if hi > lo and Pc > 0:  # rank s's piece: its agents lo_s + [lo, hi)
                        g0 = self.row_bounds[s][0]
                        block[g0 + lo:g0 + hi].copy_(stage[off:off + (hi - lo) * Pc].view(hi - lo, Pc))
                    off += (hi - lo) * Pc
        if main is not None:
            main.wait_stream(side)  # device-only
        if before_mix is not None:
            before_mix()
        return self._mix_block_and_return(out)

    def _side_stream(self):
        if self.device.type != "cuda":
            return None
        if self._side is None:  # device-only
            self._side = torch.cuda.Stream(self.device)  # device-only
        return self._side  # device-only

    @staticmethod
    def _on(stream):
        import contextlib
        return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    def _post_all_to_all(self, recv: torch.Tensor, send: torch.Tensor, recv_splits, send_splits):
        """Start an all_to_all_single on the current stream's data; returns a handle."""
        if self._staged():
            hs, hr = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)  # staged
            return dist.all_to_all_single(hr, hs, recv_splits, send_splits, group=self.group, async_op=True), hr  # staged
        return dist.all_to_all_single(recv, send, recv_splits, send_splits, group=self.group, async_op=True), None

    def _finish_all_to_all(self, handle, recv: torch.Tensor) -> None:
        work, host = handle
        if host is not None:
            _wait_all([work], self.group)  # staged
            recv.copy_(host)  # staged
        else:
            work.wait()  # the current stream waits for the transfer (RCCL: stream-side)

    def _mix_block_and_return(self, out: torch.Tensor) -> torch.Tensor:
        """Mix the assembled [N, Pc] block (self._buf_cols) and send it back to the agent rows `out`."""
        n, N, Pc = self.n_local, self.N, self.Pc
        if not self.direct:
            if Pc > 0:
                self.cols[:, :Pc].copy_(self._buf_cols[:N * Pc].view(N, Pc))
                self._apply_block(self.cols, self.cols_out)
            self.from_columns(out)
            return out
        Y = self._buf_cols2[:N * Pc]
        self._apply_block(self._buf_cols[:N * Pc].view(N, Pc), Y.view(N, Pc))
        back = self._buf_rows[:n * self.P]
        self._all_to_all(Y, back, [(h - l) * Pc for l, h in self.row_bounds],
                         [n * (b - a) for a, b in self.col_bounds])
        self._unpack_rows(back, out)
        return out

    def mix(self, rows: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One Jacobi round Y = W X for this rank's agents (out may be rows' own
        storage: the column block is a separate buffer)."""
        out = rows if out is None else out
        if self.direct:
            # rows -> send (pack) -> all_to_all -> [N, Pc] block (agents in rank =
            # agent order) -> mix in place into the way-back send buffer ->
            # all_to_all -> unpack: the same elements and the same arithmetic as
            # the staged path below, without its two block copies
            n, N, Pc = self.n_local, self.N, self.Pc
            self._all_to_all(self._pack_rows(rows), self._buf_cols[:N * Pc], [n * (b - a) for a, b in self.col_bounds],
                             [(h - l) * Pc for l, h in self.row_bounds])
            return self._mix_block_and_return(out)
        self.to_columns(rows)
        if self.Pc > 0:
            self._apply_block(self.cols, self.cols_out)
        self.from_columns(out)
        return out


def global_mean(local_rows: torch.Tensor, local_order: Sequence[int], m_total: int, P: int,
                group=None, out: Optional[torch.Tensor] = None, ordered_sum=None) -> torch.Tensor:
    """'fast' global mean: local ordered partial sum, all_reduce(SUM), / m."""
    ordered_sum = ordered_sum if ordered_sum is not None else ops.ordered_sum
    device = local_rows.device
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=device)
    sharded = dist.is_initialized() and dist.get_world_size(group) > 1
    if not sharded and len(local_order):  # one pass: the sum, then / m in the same kernel
        idx = (local_order if isinstance(local_order, torch.Tensor) and local_order.device == device
               else torch.as_tensor(list(local_order), dtype=torch.int32, device=device))
        return ordered_sum(local_rows, idx, out=out, scale=float(m_total), P=P)
    if len(local_order):
        if isinstance(local_order, torch.Tensor) and local_order.device == device:
            idx = local_order
        else:
            idx = torch.as_tensor(list(local_order), dtype=torch.int32, device=device)
        ordered_sum(local_rows, idx, out=out, P=P)
    else:
        out.zero_()
    return global_mean_finish(out, m_total, P, group=group, ordered_sum=ordered_sum)


def global_mean_finish(out: torch.Tensor, m_total: int, P: int, group=None, ordered_sum=None) -> torch.Tensor:
    """The rest of `global_mean` once `out` holds this rank's local ordered
    sum (zeros without sampled rows): all_reduce(SUM), then / m in place."""
    ordered_sum = ordered_sum if ordered_sum is not None else ops.ordered_sum
    device = out.device
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        if out.device.type == "cuda" and _backend(group) == "gloo":
            host = out.cpu()  # staged
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)  # staged
            out.copy_(host)  # staged
        else:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
    zero = torch.empty(0, dtype=torch.int32, device=device)
    return ordered_sum(None, zero, acc_in=out, out=out, scale=float(m_total), P=P)


def exact_mean_plan(order: Sequence[int], bounds: Sequence[Tuple[int, int]], P: int, world: int, rank: int):
    """Host bookkeeping of global_mean_exact (pure numpy; the gloo tests and the
    GPU path share it).  Returns (mine, counts, perm, cols):
      mine   this rank's sampled rows (LOCAL indices) in global sampled order;
      counts sampled agents owned by each rank;
      perm   perm[k] = row of the k-th sampled agent in the received block
             (sources in rank order, each source's rows in global order);
      cols   the parameter-column blocks column_bounds(P, world, q)."""
    import numpy as np
    order = np.asarray(order, dtype=np.int64).reshape(-1)
    his = np.asarray([b for _, b in bounds], dtype=np.int64)
    los = np.asarray([a for a, _ in bounds], dtype=np.int64)
    owner = np.searchsorted(his, order, side="right")
    if order.size and (owner.max() >= world or np.any(order < los[np.minimum(owner, world - 1)])):
        raise ValueError("global_mean_exact: a sampled agent lies outside every rank's rows")
    counts = np.bincount(owner, minlength=world).astype(np.int64)
    within = np.empty(order.size, dtype=np.int64)
    for q in range(world):
        sel = np.nonzero(owner == q)[0]
        within[sel] = np.arange(sel.size)
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
    perm = (offs[owner] + within).astype(np.int32)
    mine = order[owner == rank] - bounds[rank][0]
    cols = [column_bounds(P, world, q) for q in range(world)]
    return mine, counts, perm, cols


def global_mean_exact(local_rows: torch.Tensor, lo: int, hi: int, order: Sequence[int], P: int,
                      group=None, out: Optional[torch.Tensor] = None, ordered_sum=None) -> torch.Tensor:
    """Bit-exact DEC/servers.py:42-48 across ranks with O(1) collectives.

    average_weights adds the sampled clients' rows one after another in the
    sampled order, then divides by m, and each column's sum is independent of
    every other column.  So the sampled rows move once, to parameter-column
    blocks: one all_to_all sends rank q the columns column_bounds(P, world, q)
    of this rank's sampled rows, each rank adds its column block's m rows in
    the GLOBAL sampled order (ops.ordered_sum over a permutation of the
    received block: the reference's association order, + then / m in one
    pass), and one all_gather assembles theta on every rank.  Every element of
    theta is the same fp32 computation as on one GPU, whatever the world size.
    Traffic per rank: its own sampled rows once (an all_reduce would move the
    [P] sum twice, but in a rank-dependent association order: `global_mean`).
    `order` holds GLOBAL agent ids; rows [lo, hi) are local."""
    ordered_sum = ordered_sum if ordered_sum is not None else ops.ordered_sum
    device = local_rows.device
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    m = len(order)
    if m < 1:
        raise ValueError("need at least one sampled agent")
    acc = out if out is not None else torch.empty(P, dtype=torch.float32, device=device)
    if world == 1:
        if min(order) < lo or max(order) >= hi:
            raise ValueError("global_mean_exact: a sampled agent lies outside the local rows")
        idx = torch.as_tensor([int(g) - lo for g in order], dtype=torch.int32, device=device)
        return ordered_sum(local_rows, idx, out=acc, scale=float(m), P=P)
    bounds = _all_bounds(lo, hi, device, group)
    mine, counts, perm, cols = exact_mean_plan(order, bounds, P, world, rank)
    c0, c1 = cols[rank]
    Pc, m_me = c1 - c0, int(mine.size)
    # pack: to rank q, my sampled rows (global order) x q's columns, contiguous
    send = torch.empty(max(m_me * P, 1), dtype=torch.float32, device=device)
    if m_me:
        sel = torch.as_tensor(mine, dtype=torch.int64, device=device)
        off = 0
        for a, b in cols:
            if b > a:
                torch.index_select(local_rows[:, a:b], 0, sel, out=send[off:off + m_me * (b - a)].view(m_me, b - a))
            off += m_me * (b - a)
    recv = torch.empty(max(m * Pc, 1), dtype=torch.float32, device=device)
    _all_to_all(recv, send, [int(counts[s]) * Pc for s in range(world)], [m_me * (b - a) for a, b in cols], group)
    pmax = max(b - a for a, b in cols)
    part = torch.zeros(max(pmax, 1), dtype=torch.float32, device=device)
    if Pc > 0:
        idx = torch.as_tensor(perm, dtype=torch.int32, device=device)
        ordered_sum(recv[:m * Pc].view(m, Pc), idx, out=part, scale=float(m), P=Pc)
    parts = _all_gather(part, group)
    for q, (a, b) in enumerate(cols):
        if b > a:
            acc[a:b].copy_(parts[q][:b - a])
    return acc


def _all_to_all(recv: torch.Tensor, send: torch.Tensor, recv_splits, send_splits, group) -> None:
    """all_to_all_single over the first sum(splits) elements (gloo: staged through host memory)."""
    ns, nr = int(sum(send_splits)), int(sum(recv_splits))
    if _gloo_staged(send, group):
        hs, hr = send[:ns].cpu(), torch.empty(nr, dtype=recv.dtype)  # staged
        dist.all_to_all_single(hr, hs, list(recv_splits), list(send_splits), group=group)  # staged
        recv[:nr].copy_(hr)  # staged
    else:
        dist.all_to_all_single(recv[:nr], send[:ns], list(recv_splits), list(send_splits), group=group)


def _all_gather(t: torch.Tensor, group) -> List[torch.Tensor]:
    """Every rank's `t` (equal sizes), in rank order: one all_gather_into_tensor
    into a [world, numel] block on every backend (gloo: device tensors staged
    through host memory)."""
    world = dist.get_world_size(group)
    staged = _gloo_staged(t, group)
    src = t.contiguous()
    if staged:
        src = src.cpu()  # staged
    flat = torch.empty(world * t.numel(), dtype=t.dtype, device=src.device)
    dist.all_gather_into_tensor(flat, src, group=group)
    if staged:
        flat = flat.to(t.device)  # staged
    return list(flat.view(world, t.numel()))


def _gloo_staged(t: torch.Tensor, group) -> bool:
    """gloo reads raw host pointers: device tensors go through host memory."""
    return t.device.type == "cuda" and _backend(group) == "gloo"


def _all_bounds(lo: int, hi: int, device, group=None) -> List[Tuple[int, int]]:
    world = dist.get_world_size(group)
    mine = torch.tensor([lo, hi], dtype=torch.int64)  # host: tiny, and valid for gloo and RCCL via .to()
    if not (torch.device(device).type == "cuda" and _backend(group) == "gloo"):
        mine = mine.to(device)
    allb = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allb, mine, group=group)
    return [(int(t[0]), int(t[1])) for t in allb]
