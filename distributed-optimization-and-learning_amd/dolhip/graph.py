"""Mixing-matrix construction and its device form (CSR / ring plan).

`communication_graph` reproduces Simulator.communication_graph
(DIST/simulators.py:40-86) value-for-value, including how much of the global
torch RNG it consumes (one torch.rand(n, n) for either weighted mode, drawn
after model init in Simulator.__init__, :19-22), so seeded runs build the
same W as the reference.  Differences, all opt-in or failure-only:
  * the Sinkhorn loop of "double_stochastic" (:80-84) is bounded: it raises
    SinkhornNotConverged after `sinkhorn_max_iters` sweeps instead of hanging
    (SURVEY.md section 7 lists seeds/sizes where the reference never returns),
    and `sinkhorn_tol` > 0 accepts max|sum-1| <= tol;
  * "complete" is accepted as an alias of the reference's spelling "compelete".

`csr_from_dense` is Simulator.Neighbors (:91-97) for every row at once:
ascending j, keep W[i][j] > 0 (so NaN and non-positive weights drop out).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Union

import numpy as np
import torch

Graph = Union[torch.Tensor, np.ndarray]

TOPOLOGIES = ("circle", "star", "compelete", "dynamic")


class SinkhornNotConverged(RuntimeError):
    pass


def adjacency(topology: str, n: int) -> List[np.ndarray]:
    """0/1 float64 adjacency list (one entry, or n for 'dynamic')."""
    topology = "compelete" if topology == "complete" else topology
    if topology == "circle":
        a = np.zeros((n, n))
        idx = np.arange(n)
        a[idx, (idx + 1) % n] = 1.0
        a[(idx + 1) % n, idx] = 1.0
        return [a]
    if topology == "star":
        a = np.zeros((n, n))
        a[1:, 0] = 1.0
        a[0, 1:] = 1.0
        return [a]
    if topology == "compelete":
        a = np.ones((n, n))
        np.fill_diagonal(a, 0.0)
        return [a]
    if topology == "dynamic":
        out = []
        for t in range(n):
            a = np.zeros((n, n))
            a[t, (t + 1) % n] = 1.0
            a[(t + 1) % n, t] = 1.0
            out.append(a)
        return out
    return []  # the reference silently builds no graph for an unknown topology


def _column_stochastic_T(rand: torch.Tensor, a: np.ndarray) -> torch.Tensor:
    # G = R o A; normalise columns; W = G^T, so row i holds agent i's weights
    g = rand * torch.tensor(a).int().float()
    g /= g.sum(0)
    return g.T


def _sinkhorn(g: np.ndarray, max_iters: int, tol: float) -> np.ndarray:
    def done(x):
        r, c = x.sum(1), x.sum(0)
        if tol > 0:
            return max(np.max(np.abs(r - 1)), np.max(np.abs(c - 1))) <= tol
        return not ((np.any(r != 1)) | (np.any(c != 1)))

    it = 0
    while not done(g):
        if it >= max_iters:
            raise SinkhornNotConverged(
                f"double_stochastic: row/column sums not exactly 1 after {max_iters} sweeps "
                "(the reference loops forever here); pass sinkhorn_tol > 0 to accept a tolerance")
        g /= g.sum(0)
        g = g / g.sum(1)[:, np.newaxis]
        it += 1
    return g


def communication_graph(topology: str, mode: str, n: int, sinkhorn_max_iters: int = 100_000,
                        sinkhorn_tol: float = 0.0, verbose: bool = False) -> List[Graph]:
    """Mixing matrices W[t] (row i = weights agent i puts on its neighbours).

    stochastic         -> list of fp32 torch tensors (rows sum to 1)
    double_stochastic  -> list of fp32 torch tensors (Sinkhorn, bounded)
    anything else      -> list of raw 0/1 float64 numpy adjacencies
    """
    graphs: List[Graph] = list(adjacency(topology, n))
    if mode == "stochastic":
        rand = torch.rand(n, n)
        graphs = [_column_stochastic_T(rand, a) for a in graphs]
    elif mode == "double_stochastic":
        rand = torch.rand(n, n)
        if topology == "star":
            rand = torch.ones(n, n) / n
        out = []
        for a in graphs:
            g = (rand * torch.tensor(a).int().float()).numpy().copy()
            if verbose:
                print(g.sum(1), g.sum(0))
            out.append(torch.tensor(_sinkhorn(g, sinkhorn_max_iters, sinkhorn_tol)).T)
        graphs = out
    return graphs


def communication_csr(topology: str, mode: str, n: int, **kw) -> List["CSR"]:
    """communication_graph(...) as CSRs (Neighbors' selection applied),
    without materialising a dense N x N matrix per time step.

    circle / dynamic with mode 'stochastic' or a raw mode are built straight
    from the ONE torch.rand(n, n) draw the reference makes (so the global RNG
    advances identically): every column of R o A has at most two nonzeros, so
    its sum — and therefore every W entry — is the same whatever order torch's
    column reduction uses.  The reference's 'dynamic' list would be n dense
    n x n matrices (2 TB at n = 8192); here it is n CSRs of 2 entries.
    Other topologies/modes go through the dense construction."""
    topo = "compelete" if topology == "complete" else topology
    weighted = mode == "stochastic"
    raw = mode not in ("stochastic", "double_stochastic")
    if topo not in ("circle", "dynamic") or not (weighted or raw):
        return [csr_from_dense(g) for g in communication_graph(topology, mode, n, **kw)]
    R = torch.rand(n, n).numpy() if weighted else None

    def build(edges):
        # edges: undirected pairs (a, b); A[a][b] = A[b][a] = 1
        A = {}
        for a, b in edges:
            A[(a, b)] = 1.0
            A[(b, a)] = 1.0
        if raw:
            vals = {(i, j): np.float32(1.0) for (i, j) in A}
        else:
            colsum = {}
            for (i, j) in A:  # G[i][j] = R[i][j]; W[j][i] = G[i][j] / colsum_j
                colsum[j] = np.float32(colsum.get(j, np.float32(0.0)) + np.float32(R[i, j]))
            with np.errstate(invalid="ignore", divide="ignore"):
                vals = {(j, i): np.float32(np.float32(R[i, j]) / colsum[j]) for (i, j) in A}
        rows = {}
        for (i, j), v in vals.items():
            if v > 0:  # Neighbors keeps W[i][j] > 0 (NaN and 0 drop out)
                rows.setdefault(i, []).append((j, v))
        rowptr = np.zeros(n + 1, np.int64)
        cols, vv = [], []
        for i in range(n):
            for j, v in sorted(rows.get(i, [])):
                cols.append(j)
                vv.append(v)
            rowptr[i + 1] = len(cols)
        return CSR(n, n, rowptr.astype(np.int32), np.asarray(cols, np.int32), np.asarray(vv, np.float32))

    if topo == "circle":
        if n == 1:
            return [csr_from_dense(g) for g in _graphs_from_rand(topology, mode, n, R)]
        return [build([(i, (i + 1) % n) for i in range(n)])]
    return [build([(t, (t + 1) % n)]) for t in range(n)]


def _graphs_from_rand(topology, mode, n, R):
    """Dense fallback that reuses an already drawn R (keeps the RNG stream)."""
    graphs = list(adjacency(topology, n))
    if mode == "stochastic":
        rand = torch.from_numpy(R)
        return [_column_stochastic_T(rand, a) for a in graphs]
    return graphs


@dataclass
class CSR:
    """Host CSR of a mixing matrix (int32 rowptr/col, fp32 val)."""

    n_rows: int
    n_cols: int
    rowptr: np.ndarray
    col: np.ndarray
    val: np.ndarray

    @property
    def nnz(self) -> int:
        return int(self.col.size)

    def validate(self) -> "CSR":
        """Raise ValueError unless the arrays form a well-formed CSR: rowptr has
        n_rows + 1 entries, starts at 0, never decreases and ends at nnz; every
        column index is in [0, n_cols); one value per entry.  MixingPlan runs
        this once per graph; the raw ops (ops.mix_csr, dol_mix_csr_f32) trust
        their inputs and would read out of bounds on a malformed CSR."""
        rp, col = np.asarray(self.rowptr), np.asarray(self.col)
        if rp.ndim != 1 or rp.size != self.n_rows + 1:
            raise ValueError(f"rowptr has {rp.size} entries, expected n_rows + 1 = {self.n_rows + 1}")
        if rp[0] != 0 or rp[-1] != col.size:
            raise ValueError(f"rowptr must start at 0 and end at nnz = {col.size} (got {rp[0]} .. {rp[-1]})")
        if np.any(np.diff(rp.astype(np.int64)) < 0):
            raise ValueError("rowptr decreases")
        if np.asarray(self.val).size != col.size:
            raise ValueError("col and val lengths differ")
        if col.size and (col.min() < 0 or col.max() >= self.n_cols):
            raise ValueError(f"column index out of [0, {self.n_cols})")
        return self

    def ring_weights(self):
        """(w_prev, w_next) if every row i is exactly {i-1, i+1} (mod n), n >= 3."""
        n = self.n_rows
        if n < 3 or self.n_cols != n or self.nnz != 2 * n:
            return None
        if not np.all(np.diff(self.rowptr) == 2):
            return None
        i = np.arange(n)
        prev, nxt = (i - 1) % n, (i + 1) % n
        c0, c1 = self.col[0::2], self.col[1::2]
        lo, hi = np.minimum(prev, nxt), np.maximum(prev, nxt)
        if not (np.array_equal(c0, lo) and np.array_equal(c1, hi)):
            return None
        v0, v1 = self.val[0::2], self.val[1::2]
        w_prev = np.where(prev < nxt, v0, v1).astype(np.float32)
        w_next = np.where(prev < nxt, v1, v0).astype(np.float32)
        return w_prev, w_next

    def dense(self) -> np.ndarray:
        d = np.zeros((self.n_rows, self.n_cols), np.float32)
        rows = np.repeat(np.arange(self.n_rows), np.diff(self.rowptr))
        d[rows, self.col] = self.val
        return d


def csr_from_dense(W: Graph) -> CSR:
    """Neighbors (DIST/simulators.py:91-97) for all rows: j ascending, W[i][j] > 0."""
    Wn = W.detach().cpu().numpy() if isinstance(W, torch.Tensor) else np.asarray(W)
    if Wn.ndim != 2:
        raise ValueError("W must be 2-D")
    n, m = Wn.shape
    with np.errstate(invalid="ignore"):
        mask = Wn > 0
    rows, cols = np.nonzero(mask)  # row-major: ascending j within each row
    counts = np.bincount(rows, minlength=n)
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    if rowptr[-1] > np.iinfo(np.int32).max:
        raise ValueError("too many nonzeros for int32 CSR")
    return CSR(n, m, rowptr.astype(np.int32), cols.astype(np.int32),
               Wn[rows, cols].astype(np.float32))


def random_regular_csr(n: int, degree: int = 4, seed: int = 2028) -> CSR:
    """Seeded simple random d-regular graph with the reference's 'stochastic'
    weight rule (G = R o A, columns normalised, W = G^T).  Construction: the
    circulant C_n(1..d/2) under a random relabelling, then n*d degree-
    preserving double-edge swaps (rejecting self-loops and multi-edges).
    Not in the reference: the synthetic mixing workload of BASELINE config 3."""
    if degree % 2 or degree < 2 or n <= degree:
        raise ValueError("need an even degree 2 <= d < n")
    gen = torch.Generator().manual_seed(seed)
    perm = torch.randperm(n, generator=gen).numpy()
    elist = []
    for k in range(1, degree // 2 + 1):
        for i in range(n):
            a, b = int(perm[i]), int(perm[(i + k) % n])
            elist.append((min(a, b), max(a, b)))
    edges = set(elist)
    if len(edges) != len(elist):
        raise RuntimeError("circulant seed graph is not simple")
    picks = torch.randint(0, len(elist), (2 * n * degree, 2), generator=gen).numpy()
    flips = torch.randint(0, 2, (n * degree,), generator=gen).numpy()
    for s_ in range(n * degree):
        i, j = picks[s_]
        if i == j:
            continue
        (a, b), (c, d) = elist[i], elist[j]
        if flips[s_]:
            c, d = d, c
        e1, e2 = (min(a, d), max(a, d)), (min(c, b), max(c, b))
        if a == d or c == b or e1 in edges or e2 in edges:
            continue
        edges.discard(elist[i])
        edges.discard(elist[j])
        edges.add(e1)
        edges.add(e2)
        elist[i], elist[j] = e1, e2
    e = np.array(sorted(edges), np.int64)
    r = np.concatenate([e[:, 0], e[:, 1]])
    c = np.concatenate([e[:, 1], e[:, 0]])
    u = torch.rand(r.size, generator=gen).numpy().astype(np.float32)  # G[r, c]
    # column sums of G in ascending-row order (fp32)
    order = np.lexsort((r, c))
    colsum = np.zeros(n, np.float32)
    for idx in order:
        colsum[c[idx]] = np.float32(colsum[c[idx]] + u[idx])
    wval = (u / colsum[c]).astype(np.float32)
    # W = G^T: W[c, r] = G[r, c] / colsum[c]; rows of W are columns of G
    key = np.lexsort((r, c))  # sort by W row (= c), then W col (= r)
    rows_w, cols_w, vals_w = c[key], r[key], wval[key]
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(rows_w, minlength=n), out=rowptr[1:])
    keep = vals_w > 0
    if not keep.all():  # the >0 selection rule of Neighbors
        return csr_from_dense(CSR(n, n, rowptr.astype(np.int32), cols_w.astype(np.int32),
                                  vals_w).dense())
    return CSR(n, n, rowptr.astype(np.int32), cols_w.astype(np.int32), vals_w)


def erdos_renyi_stochastic(n: int, p: float, generator: torch.Generator, device=None) -> torch.Tensor:
    """Dense W of a seeded undirected Erdős–Rényi G(n, p) graph under the
    reference's 'stochastic' weighting (DIST/simulators.py:65-70: G = R o A,
    G /= colsum(G), W = G^T), built on the generator's device (no host round
    trip, so a new W every round is cheap: BASELINE config 5's time-varying
    dense W; not a reference topology).  Zero diagonal like every reference
    adjacency; entries Neighbors would drop (NaN from an empty column, <= 0)
    are 0, so the dense MFMA mix equals the CSR selection."""
    dev = generator.device if device is None else torch.device(device)
    up = torch.rand(n, n, generator=generator, device=dev) < p
    A = torch.triu(up, diagonal=1)
    A = (A | A.T).to(torch.float32)
    g = torch.rand(n, n, generator=generator, device=dev) * A
    g = g / g.sum(0)
    W = g.T.contiguous()
    return torch.where(W > 0, W, torch.zeros((), dtype=W.dtype, device=dev))


def erdos_renyi_stochastic_hip(n: int, p: float, seed: int, device, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The same kind of W as erdos_renyi_stochastic (undirected G(n, p), zero
    diagonal, 'stochastic' weighting, rows summing to 1), drawn by ONE HIP
    kernel from a counter-based hash keyed by `seed` (dol_er_stochastic_f32)
    instead of nine torch kernels: config 5's per-round W draw.  Not the
    torch generator's stream."""
    from . import ops
    W = out if out is not None else torch.empty(n, n, dtype=torch.float32, device=device)
    return ops.er_stochastic(W, p, seed)


class MixingPlan:
    """Device form of one W: CSR tensors plus the ring specialisation if it applies."""

    DENSE_KERNELS = ("split3", "f32")
    SLAB_MIN_DEGREE = 16  # mean neighbours per row from which the LDS-gather CSR kernel takes over

    def __init__(self, csr: CSR, device, allow_ring: bool = True, dense: bool = False,
                 dense_kernel: str = "split3", slab: Optional[bool] = None):
        """kind: 'ring' (bit-exact, ring kernel), 'csr' (bit-exact, any W), or
        'dense' (opt-in tolerance path: a GEMM over the dense W on the matrix
        cores; dense_kernel 'split3' = three-piece bf16 split at fp32 accuracy,
        'f32' = exact-f32 MFMA fma chain).  A 'csr' plan whose rows average at
        least SLAB_MIN_DEGREE neighbours (or slab=True) also packs the CSR for
        the LDS-gather kernel (dol_mix_csr_slab_f32, same bits), used whenever
        the matrices' layout allows it."""
        if dense_kernel not in self.DENSE_KERNELS:
            raise ValueError(f"dense_kernel must be one of {self.DENSE_KERNELS}")
        self.dense_kernel = dense_kernel
        self._work, self._work_key = None, None
        self.csr = csr.validate()
        self.device = torch.device(device)
        self.n_rows = csr.n_rows
        self.n_cols = csr.n_cols
        self.rowptr = torch.from_numpy(csr.rowptr).to(self.device)
        self.col = torch.from_numpy(csr.col).to(self.device)
        self.val = torch.from_numpy(csr.val).to(self.device)
        ring = csr.ring_weights() if (allow_ring and not dense) else None
        self.kind = "dense" if dense else ("ring" if ring is not None else "csr")
        if ring is not None:
            self.w_prev = torch.from_numpy(ring[0]).to(self.device)
            self.w_next = torch.from_numpy(ring[1]).to(self.device)
        if dense:
            # the CSR's selection (W_ij > 0 kept, NaN/negatives dropped) densified
            self.W = torch.from_numpy(csr.dense()).to(self.device)
        self.ent = self.hdr = None
        if slab is None:
            slab = csr.nnz >= self.SLAB_MIN_DEGREE * max(1, csr.n_rows)
        if self.kind == "csr" and slab and csr.n_rows > 0:
            from . import ops
            self.ent, self.hdr = ops.csr_slab_pack(self.rowptr, self.col, self.val, self.n_cols, balance=True)

    @property
    def density(self) -> float:
        if self.csr is None:
            return float((self.W > 0).sum().item()) / max(1, self.W.numel())
        return self.csr.nnz / max(1, self.csr.n_rows * self.csr.n_cols)

    # from_dense(csr, balance=True) deals rows to the slab kernel's waves by their
    # per-chunk loads (csr_slab_pack balance=True) up to this many X rows (64
    # chunks: the register-resident packing kernel, ~0.04 ms at 1024 agents,
    # where the balanced mix runs ~2-3 % faster; beyond, the LDS kernel costs
    # more than it saves).  Worth it where the pack overlaps other work (the
    # config-5 round builds the next plan on a side stream during the local
    # step); a plan built and mixed back to back is faster unbalanced.
    BALANCE_MAX_X_ROWS = 4096

    @classmethod
    def from_dense(cls, W: torch.Tensor, dense_kernel: str = "split3",
                   reuse: Optional["MixingPlan"] = None, balance: bool = False) -> "MixingPlan":
        """A plan straight from a device W (no host round trip; e.g. a per-round
        erdos_renyi_stochastic_hip draw).  dense_kernel 'split3' / 'f32': a
        'dense' plan on the matrix cores (tolerance path).  dense_kernel 'csr':
        the Neighbors selection runs on the device (dol_dense_to_csr_f32) and
        the plan mixes bit-exactly with the LDS-gather CSR kernel; `reuse` (a
        previous 'csr' plan of the same shape) lends its buffers and is retired
        (mixing with it afterwards raises).  The lent col / val buffers are sized
        n_rows * n_cols (a dense W's worst case), so a reused plan never
        reallocates whatever the round's W.  balance: the wave-balanced packing
        (same bits) when n_cols <= BALANCE_MAX_X_ROWS."""
        if W.device.type != "cuda" or W.dtype != torch.float32 or W.dim() != 2:
            raise ValueError("from_dense: expected a 2-D float32 CUDA tensor")
        if dense_kernel not in cls.DENSE_KERNELS + ("csr",):
            raise ValueError(f"dense_kernel must be one of {cls.DENSE_KERNELS + ('csr',)}")
        plan = cls.__new__(cls)
        plan.dense_kernel = dense_kernel
        plan._work, plan._work_key = None, None
        plan.csr = None
        plan.device = W.device
        plan.n_rows, plan.n_cols = W.shape
        plan.W = W.contiguous()
        plan.ent = plan.hdr = None
        if dense_kernel != "csr":
            plan.kind = "dense"
            return plan
        from . import ops
        plan.kind = "csr"
        same = (reuse is not None and reuse.kind == "csr" and reuse.csr is None and reuse.device == W.device
                and (reuse.n_rows, reuse.n_cols) == (plan.n_rows, plan.n_cols))
        bufs = (reuse.rowptr, reuse.col, reuse.val) if same else (None, None, None)
        plan.rowptr, plan.col, plan.val = ops.dense_to_csr(plan.W, *bufs)
        balance = bool(balance) and plan.n_cols <= cls.BALANCE_MAX_X_ROWS
        plan.ent, plan.hdr = ops.csr_slab_pack(plan.rowptr, plan.col, plan.val, plan.n_cols,
                                               *((reuse.ent, reuse.hdr) if same else (None, None)),
                                               balance=bool(balance))
        if same:  # the lender's buffers now hold this W: it must not mix again
            reuse._retire()
        return plan

    def _retire(self) -> None:
        self.kind = "stale"
        self.rowptr = self.col = self.val = self.ent = self.hdr = self.W = None

    def _check_live(self) -> None:
        if self.kind == "stale":
            raise RuntimeError("this MixingPlan lent its buffers to a newer from_dense(..., reuse=plan) plan "
                               "and no longer holds its W")

    @classmethod
    def from_graph(cls, W: Graph, device, allow_ring: bool = True, dense: bool = False,
                   dense_kernel: str = "split3") -> "MixingPlan":
        return cls(csr_from_dense(W), device, allow_ring, dense, dense_kernel)

    def _mix_dense(self, X: torch.Tensor, Y: torch.Tensor, P: Optional[int]) -> torch.Tensor:
        from . import ops
        if self.dense_kernel == "f32":
            return ops.mix_dense(self.W, X, Y, P=P)
        P = X.shape[1] if P is None else P
        M, K = self.W.shape
        need = ops.dense_split3_workspace_bytes(M, K, P, 0)
        key = (M, K, X.device)
        ready = self._work_key == key and self._work.numel() >= need  # W already split into the workspace
        if not ready:
            self._work = torch.empty(max(need, 1), dtype=torch.uint8, device=X.device)
        ops.mix_dense_split3(self.W, X, Y, P=P, work=self._work, w_ready=ready)
        self._work_key = key
        return Y

    MAX_FUSED_STEPS = 8

    def apply_steps(self, X: torch.Tensor, Y: torch.Tensor, steps: int, P: Optional[int] = None) -> int:
        """Apply up to `steps` synchronous rounds in one pass when the plan and
        layout allow (ring, P % 4 == 0, 16-B aligned rows); returns how many
        rounds were applied (>= 1).  Bit-identical to single rounds."""
        P = X.shape[1] if P is None else P
        self._check_x(X)
        k = min(int(steps), self.MAX_FUSED_STEPS)
        if (k > 1 and self.kind == "ring" and P % 4 == 0 and X.data_ptr() % 16 == 0 and Y.data_ptr() % 16 == 0
                and X.stride(0) % 4 == 0 and Y.stride(0) % 4 == 0):
            from . import ops
            ops.mix_ring_steps(X, Y, self.w_prev, self.w_next, k, P=P, n_rows=self.n_rows)
            return k
        self.apply(X, Y, P=P)
        return 1

    def _check_x(self, X: torch.Tensor) -> None:
        self._check_live()
        need = self.n_cols
        if X.shape[0] < need:
            raise ValueError(f"X has {X.shape[0]} rows; W has {need} columns")

    def apply(self, X: torch.Tensor, Y: torch.Tensor, P: Optional[int] = None) -> torch.Tensor:
        from . import ops
        self._check_x(X)
        if self.kind == "ring":
            return ops.mix_ring(X, Y, self.w_prev, self.w_next, P=P, n_rows=self.n_rows)
        if self.kind == "dense":
            return self._mix_dense(X, Y, P)
        P_ = X.shape[1] if P is None else P
        if self.ent is not None and ops.slab_layout_ok(X, Y, P_):
            return ops.mix_csr_slab(X, Y, self.ent, self.hdr, self.n_rows, x_rows=self.n_cols, P=P_)
        return ops.mix_csr(X, Y, self.rowptr, self.col, self.val, P=P)


    def apply_dgd(self, X: torch.Tensor, Y: torch.Tensor, target: torch.Tensor, mom: Optional[torch.Tensor] = None,
                  objective: str = "least_squares", steps: int = 1, lr: float = 0.01, momentum: float = 0.0,
                  first_step: bool = False, P: Optional[int] = None) -> torch.Tensor:
        """One fused DGD round (mix + local steps, BASELINE config 3); ring or CSR."""
        from . import ops
        self._check_x(X)
        kw = dict(mom=mom, objective=objective, steps=steps, lr=lr, momentum=momentum, first_step=first_step, P=P)
        if self.kind == "ring":
            return ops.dgd_ring(X, Y, self.w_prev, self.w_next, target, n_rows=self.n_rows, **kw)
        if self.kind == "dense":
            raise NotImplementedError("DGD rounds are fused into the sparse mixes; use a ring/CSR plan")
        return ops.dgd_csr(X, Y, self.rowptr, self.col, self.val, target, **kw)


def plans_for(graphs: Sequence[Graph], device, allow_ring: bool = True) -> List[MixingPlan]:
    return [MixingPlan.from_graph(g, device, allow_ring) for g in graphs]
