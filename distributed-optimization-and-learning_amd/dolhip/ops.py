"""Tensor-level wrappers over the C-ABI (include/dol_hip.h).

Every function takes CUDA(HIP) fp32 tensors, validates shapes/strides on the
host (the kernels trust their arguments), and enqueues on the current torch
stream.  There is deliberately no CPU path: a CPU tensor raises.
"""
from __future__ import annotations

import os as _os
from typing import Optional

import torch

from . import _native
from ._native import DolNativeError

__all__ = [
    "DolNativeError", "pm_stage_order", "tune_pm_stage_order", "ring_steps_variant", "tune_ring_steps_variant",
    "RING_STEPS_VARIANTS", "PM_STAGE_ORDERS", "tuned_choices", "autotune_enabled", "ring_steps_choice",
    "pm_stage_order_choice", "mix_csr", "mix_ring", "mix_dense", "mix_dense_split3", "dense_split3_workspace_bytes", "split3_x_flags", "er_stochastic",
    "mix_ring_steps", "mix_ring_edges", "dgd_ring_edges", "prox_admm_sgd", "admm_dual", "ordered_mean",
    "ordered_sum", "stream_copy", "dual_workspace_bytes", "prox_grad", "admm_step_dual", "mlp_step",
    "dgd_ring", "dgd_csr", "OBJECTIVES", "admm_ls_round", "admm_ls_round_workspace_bytes", "mix_csr_pm",
    "transpose", "PM_MAX_AGENTS", "stream_copy_rows", "dgd_csr_pm", "PM_DGD_MAX_AGENTS",
    "SLAB_CHUNK", "SLAB_ROWS", "csr_slab_pack", "mix_csr_slab", "slab_layout_ok", "dense_to_csr",
]

PM_MAX_AGENTS = 8192  # dol_mix_csr_pm_f32: one p-row image (<= 32 KiB) per LDS stage
PM_DGD_MAX_AGENTS = 4096  # dol_dgd_csr_pm_f32: X, target and momentum p-rows share a 64 KiB stage


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check_rows(name: str, t: torch.Tensor, P: Optional[int] = None) -> int:
    """Validate a stacked [rows, >=P] fp32 device matrix; return its ld."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise DolNativeError(f"{name}: tensor is on {t.device}; the HIP engine has no CPU path")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    if t.dim() != 2:
        raise ValueError(f"{name}: expected a 2-D [rows, P] tensor, got shape {tuple(t.shape)}")
    if t.shape[1] > 1 and t.stride(1) != 1:
        raise ValueError(f"{name}: rows must be contiguous (stride(1) == 1)")
    ld = t.stride(0) if t.shape[0] > 1 else max(t.shape[1], 1)
    if P is not None and t.shape[1] < P:
        raise ValueError(f"{name}: has {t.shape[1]} columns < P={P}")
    return int(ld)


def _check_vec(name: str, t: Optional[torch.Tensor], P: int, device) -> None:
    if t is None:
        return
    if t.device != device:
        raise DolNativeError(f"{name}: on {t.device}, expected {device}")
    if t.dtype != torch.float32 or t.dim() != 1 or t.shape[0] < P or (t.shape[0] > 1 and t.stride(0) != 1):
        raise ValueError(f"{name}: expected a contiguous float32 vector of >= {P} elements")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def mix_csr(X: torch.Tensor, Y: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor,
            val: torch.Tensor, P: Optional[int] = None) -> torch.Tensor:
    """Y[i] = sum_e val[e] * X[col[e]] (ascending e, +0 start, no FMA).

    Reference: DIST/simulators.py:91-97 + DIST/clients.py:61-69."""
    P = X.shape[1] if P is None else P
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    n = rowptr.shape[0] - 1
    if Y.shape[0] < n:
        raise ValueError(f"Y has {Y.shape[0]} rows < {n}")
    for nm, t, dt in (("rowptr", rowptr, torch.int32), ("col", col, torch.int32), ("val", val, torch.float32)):
        if t.device != X.device or t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous {dt} on {X.device}")
    if col.numel() != val.numel():
        raise ValueError("col and val lengths differ")
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias: the Jacobi mix needs two buffers")
    _native.call("dol_mix_csr_f32", X.data_ptr(), ldx, X.shape[0], Y.data_ptr(), ldy, n, P,
                 rowptr.data_ptr(), col.data_ptr() if col.numel() else None,
                 val.data_ptr() if val.numel() else None, _stream(X))
    return Y


def mix_csr_pm(XT: torch.Tensor, YT: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor,
               x_agents: Optional[int] = None, P: Optional[int] = None, nseg: Optional[int] = None) -> torch.Tensor:
    """The gossip mix on the parameter-major bank: YT[p, i] = sum_e val[e] *
    XT[p, col[e]] for every parameter row p (bit-identical to mix_csr on the
    transposed matrices).  XT [P, >= x_agents], YT [P, >= n] (n = rowptr
    length - 1), row strides multiples of 4, 16-B aligned; at most
    PM_MAX_AGENTS agents.  nseg: the stage order (None = tuned for these
    buffers on first use, 0 = the process setting).  Reference:
    DIST/simulators.py:91-97 + DIST/clients.py:61-69."""
    P = XT.shape[0] if P is None else P
    n = rowptr.shape[0] - 1
    x_agents = n if x_agents is None else int(x_agents)
    ldx = _check_rows("XT", XT)
    ldy = _check_rows("YT", YT)
    if XT.shape[0] < P or YT.shape[0] < P:
        raise ValueError(f"XT/YT need >= {P} parameter rows")
    if XT.shape[1] < x_agents or YT.shape[1] < n:
        raise ValueError(f"XT needs >= {x_agents} agent columns, YT >= {n}")
    for nm, t, dt in (("rowptr", rowptr, torch.int32), ("col", col, torch.int32), ("val", val, torch.float32)):
        if t.device != XT.device or t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous {dt} on {XT.device}")
    if XT.data_ptr() == YT.data_ptr():
        raise ValueError("XT and YT alias: the Jacobi mix needs two buffers")

    def launch(ns):
        _native.call("dol_mix_csr_pm_ex_f32", XT.data_ptr(), ldx, x_agents, YT.data_ptr(), ldy, n, P,
                     rowptr.data_ptr(), col.data_ptr() if col.numel() else None,
                     val.data_ptr() if val.numel() else None, int(ns), _stream(XT))
    if nseg is None:
        nseg = _pm_auto(XT, YT, ldx, ldy, x_agents, n, P, launch)
    launch(nseg)
    return YT


def _pm_auto(XT, YT, ldx, ldy, x_agents, n, P, launch) -> int:
    key = _pair_key("pm", XT, YT, ldx, ldy, x_agents, n, P)
    return _auto_choice(key, launch, PM_STAGE_ORDERS, (x_agents + n) * P * 4, XT.device)


def pm_stage_order(nseg: int) -> int:
    """Set the parameter-major kernels' stage order for this process (nseg
    regions streamed at once; 0 = the default) and return the previous setting
    (dol_pm_set_stage_order).  Same bits for every order."""
    rc = _native.lib().dol_pm_set_stage_order(int(nseg))
    if rc < 0:
        raise DolNativeError("dol_pm_set_stage_order: " + _native.lib().dol_last_error().decode(errors="replace"))
    return rc


def tune_pm_stage_order(run, candidates=(8, 16, 32), reps: int = 3) -> dict:
    """Time `run()` (a parameter-major mix on the buffers it will keep using)
    under each stage order and keep the fastest for this process: which order
    balances the HBM channels best depends on where those buffers' pages
    landed (profiles/r03_pm_stage_order.txt).  Returns {"nseg": best, "ms":
    {nseg: ms}}.  Setup-time only; results are bit-identical under every order."""
    best, times = _tune(pm_stage_order, run, candidates, reps)
    return {"nseg": best, "ms": times}


def ring_steps_variant(variant: int) -> int:
    """Kernel of mix_ring_steps for this process: 1 register tiles, 2 streaming,
    3 / 4 / 5 streaming by LDS-DMA (plain / block-synchronised / 64-row sweep),
    0 default; returns the previous setting (dol_ring_steps_set_variant)."""
    rc = _native.lib().dol_ring_steps_set_variant(int(variant))
    if rc < 0:
        raise DolNativeError("dol_ring_steps_set_variant: " + _native.lib().dol_last_error().decode(errors="replace"))
    return rc


def _time_each(run_with, candidates, reps, device=None):
    """{candidate: mean ms of `reps` calls of run_with(candidate)} on the
    current stream of `device` (default: the current device) -- the stream the
    ops launch on for tensors there.  Events bracket the calls on that stream
    and the host waits on the closing event only: no device-wide
    synchronisation, so work on other streams (a side stream's W draw, another
    rank's buffers) is neither waited for nor serialised."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    times = {}
    with torch.cuda.device(device):
        stream = torch.cuda.current_stream(device)
        for c in candidates:
            run_with(c)  # warm (first launch of this variant on these buffers)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(reps):
                run_with(c)
            e.record(stream)
            e.synchronize()
            times[c] = s.elapsed_time(e) / reps
    return times


def _tune(setter, run, candidates, reps):
    def run_with(c):
        setter(c)
        run()
    times = _time_each(run_with, candidates, reps)
    best = min(times, key=times.get)
    setter(best)
    return best, times


def tune_ring_steps_variant(run, reps: int = 3) -> dict:
    """Time `run()` (a mix_ring_steps call on the buffers it will keep using)
    with the register-tile and the streaming kernel and keep the faster for
    this process; which wins depends on where the buffers' pages landed.
    Returns {"variant": 1 | 2, "ms": {variant: ms}}.  Same bits either way."""
    best, times = _tune(ring_steps_variant, run, RING_STEPS_VARIANTS, reps)
    return {"variant": best, "ms": times}


# ---------------------------------------------------------------------------
# Launch choices tuned on the product path.  Which ring-steps kernel / which
# parameter-major stage order is fastest follows where a bank's pages landed
# (DESIGN.md §4.1, §4.4), so the first large call on a pair of buffers times
# every candidate on THOSE buffers (the calls are pure X -> Y mixes: re-running
# them only rewrites Y) and caches the winner for that (buffer pair, geometry);
# later calls pass it per call (the _ex entry points), so nothing process-wide
# changes and the results are the same bits whatever is picked.  A stale entry
# after the memory is reused can only cost speed.  DOL_AUTOTUNE=0 turns it off
# (every call then takes the library default).
# ---------------------------------------------------------------------------
RING_STEPS_VARIANTS = (1, 2, 3, 4, 5)
PM_STAGE_ORDERS = (8, 16, 32)
AUTOTUNE_MIN_BYTES = 1 << 30  # below this one pass is too short to be worth timing
AUTOTUNE_REPS = 3
_TUNED: dict = {}


def autotune_enabled() -> bool:
    return _os.environ.get("DOL_AUTOTUNE", "1") != "0"


def tuned_choices() -> dict:
    """{key: {"choice": c, "ms": {candidate: ms}}} of every launch choice this process tuned."""
    return {repr(k): dict(v) for k, v in _TUNED.items()}


def _auto_choice(key, run_with, candidates, nbytes: int, device) -> int:
    """The cached pick for `key`, or time every candidate on `device`'s current
    stream (where the buffers live and the ops launch), cache and return the
    fastest; 0 (the library default) when tuning is off, the buffers are small
    or that stream is being captured into a graph."""
    if not autotune_enabled() or nbytes < AUTOTUNE_MIN_BYTES:
        return 0
    hit = _TUNED.get(key)
    if hit is not None:
        return hit["choice"]
    with torch.cuda.device(device):
        if torch.cuda.is_current_stream_capturing():  # no timing inside a graph capture
            return 0
    times = _time_each(run_with, candidates, AUTOTUNE_REPS, device=device)
    best = min(times, key=times.get)
    _TUNED[key] = {"choice": best, "ms": times}
    return best


def _pair_key(kind, A: torch.Tensor, B: torch.Tensor, *geometry):
    return (kind, A.device.index, frozenset((A.data_ptr(), B.data_ptr())), *geometry)


def _ld(t: torch.Tensor) -> int:
    return int(t.stride(0) if t.shape[0] > 1 else max(t.shape[1], 1))


def ring_steps_choice(X: torch.Tensor, Y: torch.Tensor, steps: int, P: Optional[int] = None,
                      n_rows: Optional[int] = None) -> Optional[dict]:
    """The tuned mix_ring_steps entry ({"choice", "ms"}) for this buffer pair, or None."""
    P = X.shape[1] if P is None else P
    n = X.shape[0] if n_rows is None else n_rows
    return _TUNED.get(_pair_key("ring_steps", X, Y, _ld(X), _ld(Y), n, P, int(steps)))


def pm_stage_order_choice(XT: torch.Tensor, YT: torch.Tensor, n: int, x_agents: Optional[int] = None,
                          P: Optional[int] = None) -> Optional[dict]:
    """The tuned mix_csr_pm / dgd_csr_pm entry ({"choice", "ms"}) for this buffer pair, or None."""
    P = XT.shape[0] if P is None else P
    x_agents = n if x_agents is None else int(x_agents)
    return _TUNED.get(_pair_key("pm", XT, YT, _ld(XT), _ld(YT), x_agents, n, P))


SLAB_CHUNK = 64  # DOL_SLAB_CHUNK: agents per LDS chunk of dol_mix_csr_slab_f32


def _check_csr(rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, device) -> None:
    for nm, t, dt in (("rowptr", rowptr, torch.int32), ("col", col, torch.int32), ("val", val, torch.float32)):
        if t.device != device or t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous {dt} on {device}")
    if col.numel() != val.numel():
        raise ValueError("col and val lengths differ")


SLAB_ROWS = 128  # DOL_SLAB_ROWS: rows per row group of the chunk-major packing


def csr_slab_pack(rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, x_rows: int,
                  ent: Optional[torch.Tensor] = None, hdr: Optional[torch.Tensor] = None, balance: bool = False):
    """(ent, hdr) of a device CSR for mix_csr_slab (dol_csr_slab_pack): the
    rows of each group of SLAB_ROWS dealt to slots (balanced per-chunk wave
    loads), the entries re-packed chunk-major as (weight bits, LDS byte offset)
    pairs, every (slot, chunk) segment padded to an even length; hdr[g][k][s] =
    first entry of slot s in chunk k, bit 0 = the segment ends in a pad, then
    perm[g][s] = row and inv[row] = slot (include/dol_hip.h).  col/val may be
    longer than nnz (a capacity); ent is sized from it.  balance: deal the
    rows to the kernel's waves by greedy packing of their per-chunk loads
    (same bits; worth it when one W is mixed many times)."""
    n = rowptr.numel() - 1
    _check_csr(rowptr, col, val, rowptr.device)
    L = _native.lib()
    need_e = int(L.dol_csr_slab_ent_len(col.numel(), n, int(x_rows)))
    need_h = int(L.dol_csr_slab_hdr_len(n, int(x_rows)))
    if ent is None or ent.numel() < need_e:
        ent = torch.empty(max(need_e, 4), dtype=torch.int32, device=rowptr.device)
    if hdr is None or hdr.numel() < need_h:
        hdr = torch.empty(max(need_h, 4), dtype=torch.int32, device=rowptr.device)
    _native.call("dol_csr_slab_pack", rowptr.data_ptr(), col.data_ptr() if col.numel() else None,
                 val.data_ptr() if val.numel() else None, n, int(x_rows), int(bool(balance)), ent.data_ptr(),
                 hdr.data_ptr(), _stream(rowptr))
    return ent, hdr


SLAB_VARIANTS = (1, 2, 3)  # 1: a loop per (row, chunk) segment (r03); 2: the wave's pairs as one pipelined stream (r06); 3: that stream hand-scheduled (asm)


def slab_variant(variant: int) -> int:
    """Kernel of mix_csr_slab for this process (dol_slab_set_variant; 0 =
    the default).  Same bits for every variant.  Returns the previous setting."""
    return int(_native.lib().dol_slab_set_variant(int(variant)))


def slab_layout_ok(X: torch.Tensor, Y: torch.Tensor, P: int) -> bool:
    """Whether mix_csr_slab accepts these matrices: 16-B aligned rows, row
    strides multiples of 4, X rows readable up to round_up(P, 4) floats."""
    if X.dim() != 2 or Y.dim() != 2 or X.data_ptr() % 16 or Y.data_ptr() % 16:
        return False
    ldx = X.stride(0) if X.shape[0] > 1 else X.shape[1]
    ldy = Y.stride(0) if Y.shape[0] > 1 else Y.shape[1]
    p4 = -(-P // 4) * 4
    if ldx % 4 or ldy % 4 or ldx < p4:
        return False
    need = X.storage_offset() + (X.shape[0] - 1) * ldx + p4
    return need * 4 <= X.untyped_storage().nbytes()


def mix_csr_slab(X: torch.Tensor, Y: torch.Tensor, ent: torch.Tensor, hdr: torch.Tensor, n_rows: int,
                 x_rows: Optional[int] = None, P: Optional[int] = None) -> torch.Tensor:
    """mix_csr for high-degree graphs (dol_mix_csr_slab_f32): the same sum in
    the same order, bit-identical, with X's columns staged through LDS.
    (ent, hdr) from csr_slab_pack.  Reference: DIST/simulators.py:91-97 +
    DIST/clients.py:61-69."""
    P = X.shape[1] if P is None else P
    x_rows = X.shape[0] if x_rows is None else int(x_rows)
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    if Y.shape[0] < n_rows or X.shape[0] < x_rows:
        raise ValueError(f"X has {X.shape[0]} rows (need {x_rows}), Y {Y.shape[0]} (need {n_rows})")
    if not slab_layout_ok(X, Y, P):
        raise ValueError("mix_csr_slab: X, Y need 16-B aligned rows with strides % 4 == 0 and X readable to "
                         "round_up(P, 4) floats per row")
    for nm, t in (("ent", ent), ("hdr", hdr)):
        if t.device != X.device or t.dtype != torch.int32 or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous int32 on {X.device}")
    if hdr.numel() < int(_native.lib().dol_csr_slab_hdr_len(int(n_rows), x_rows)):
        raise ValueError("hdr too short for these row counts (rebuild with csr_slab_pack)")
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias: the Jacobi mix needs two buffers")
    _native.call("dol_mix_csr_slab_f32", X.data_ptr(), ldx, x_rows, Y.data_ptr(), ldy, int(n_rows), P,
                 ent.data_ptr(), hdr.data_ptr(), _stream(X))
    return Y


def dense_to_csr(W: torch.Tensor, rowptr: Optional[torch.Tensor] = None, col: Optional[torch.Tensor] = None,
                 val: Optional[torch.Tensor] = None):
    """Neighbors (DIST/simulators.py:91-97) of every row of a dense device W, on
    the device (dol_dense_to_csr_f32): (rowptr, col, val) with col/val of
    capacity n*m (nnz = rowptr[-1], not synchronised to the host)."""
    ld = _check_rows("W", W)
    n, m = W.shape
    cap = n * m
    if rowptr is None or rowptr.numel() < n + 1:
        rowptr = torch.empty(n + 1, dtype=torch.int32, device=W.device)
    if col is None or col.numel() < cap:
        col = torch.empty(max(cap, 1), dtype=torch.int32, device=W.device)
    if val is None or val.numel() < cap:
        val = torch.empty(max(cap, 1), dtype=torch.float32, device=W.device)
    _native.call("dol_dense_to_csr_f32", W.data_ptr(), ld, n, m, rowptr.data_ptr(), col.data_ptr(), val.data_ptr(),
                 col.numel() if val.numel() >= col.numel() else val.numel(), _stream(W))
    return rowptr, col, val


def transpose(A: torch.Tensor, B: torch.Tensor, rows: Optional[int] = None, cols: Optional[int] = None) -> torch.Tensor:
    """B[c, r] = A[r, c] for r < rows, c < cols (tiled through LDS): converts the
    agent-major bank [N, ld] to the parameter-major one [P, ldt] and back."""
    rows = A.shape[0] if rows is None else rows
    cols = A.shape[1] if cols is None else cols
    lda = _check_rows("A", A, cols)
    ldb = _check_rows("B", B, rows)
    if A.shape[0] < rows or B.shape[0] < cols:
        raise ValueError(f"shapes: A {tuple(A.shape)}, B {tuple(B.shape)}, rows {rows}, cols {cols}")
    if A.device != B.device:
        raise ValueError("A and B on different devices")
    _native.call("dol_transpose_f32", A.data_ptr(), lda, B.data_ptr(), ldb, rows, cols, _stream(A))
    return B


def mix_ring_steps(X: torch.Tensor, Y: torch.Tensor, w_prev: torch.Tensor, w_next: torch.Tensor, steps: int,
                   P: Optional[int] = None, n_rows: Optional[int] = None,
                   variant: Optional[int] = None) -> torch.Tensor:
    """Y = W^steps X for the wrap-around ring in one HBM pass (bit-identical to
    `steps` mix_ring calls).  Needs P % 4 == 0 and 16-B aligned rows.
    variant: the kernel (RING_STEPS_VARIANTS; None = tuned for these buffers
    on first use, 0 = the process setting)."""
    P = X.shape[1] if P is None else P
    n = X.shape[0] if n_rows is None else n_rows
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    for nm, t in (("w_prev", w_prev), ("w_next", w_next)):
        if t.device != X.device or t.dtype != torch.float32 or t.numel() < n or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous float32 [{n}] on {X.device}")
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias")

    def launch(v):
        _native.call("dol_mix_ring_steps_ex_f32", X.data_ptr(), ldx, Y.data_ptr(), ldy, n, P, int(steps),
                     w_prev.data_ptr(), w_next.data_ptr(), int(v), _stream(X))
    if variant is None:
        variant = _auto_choice(_pair_key("ring_steps", X, Y, ldx, ldy, n, P, int(steps)), launch,
                               RING_STEPS_VARIANTS, 2 * n * P * 4, X.device) if steps > 1 else 0
    launch(variant)
    return Y


OBJECTIVES = {"least_squares": 0, "logistic": 1}


def _dgd_args(X, target, mom, objective, steps, momentum, P, n):
    if objective not in OBJECTIVES:
        raise ValueError(f"objective must be one of {sorted(OBJECTIVES)}")
    if int(steps) < 1:
        raise ValueError("local steps must be >= 1")
    ldt = _check_rows("target", target, P)
    if target.shape[0] < n or target.device != X.device:
        raise ValueError(f"target: expected >= {n} rows on {X.device}")
    ldm = 0
    if momentum != 0.0:
        if mom is None:
            raise ValueError("momentum != 0 needs mom")
        ldm = _check_rows("mom", mom, P)
        if mom.shape[0] < n or mom.device != X.device:
            raise ValueError(f"mom: expected >= {n} rows on {X.device}")
    return ldt, ldm


def dgd_ring(X: torch.Tensor, Y: torch.Tensor, w_prev: torch.Tensor, w_next: torch.Tensor, target: torch.Tensor,
             mom: Optional[torch.Tensor] = None, objective: str = "least_squares", steps: int = 1, lr: float = 0.01,
             momentum: float = 0.0, first_step: bool = False, halo_prev: Optional[torch.Tensor] = None,
             halo_next: Optional[torch.Tensor] = None, P: Optional[int] = None,
             n_rows: Optional[int] = None) -> torch.Tensor:
    """One fused DGD round on a ring: Y = W X (bit-exact mix), then `steps` local
    momentum-SGD iterations per row on a separable loss (BASELINE config 3;
    round order of DIST/simulators.py:147-162)."""
    P = X.shape[1] if P is None else P
    n = X.shape[0] if n_rows is None else n_rows
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    if X.shape[0] < n or Y.shape[0] < n:
        raise ValueError("X/Y have fewer rows than n_rows")
    for nm, t in (("w_prev", w_prev), ("w_next", w_next)):
        if t.device != X.device or t.dtype != torch.float32 or t.numel() < n or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous float32 [{n}] on {X.device}")
    if (halo_prev is None) != (halo_next is None):
        raise ValueError("pass both halos or neither")
    if halo_prev is None and n < 3:
        raise ValueError("a wrap-around ring needs >= 3 rows (use dgd_csr)")
    _check_vec("halo_prev", halo_prev, P, X.device)
    _check_vec("halo_next", halo_next, P, X.device)
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias: the Jacobi mix needs two buffers")
    ldt, ldm = _dgd_args(X, target, mom, objective, steps, momentum, P, n)
    _native.call("dol_dgd_ring_f32", X.data_ptr(), ldx, Y.data_ptr(), ldy, n, P, _ptr(halo_prev), _ptr(halo_next),
                 w_prev.data_ptr(), w_next.data_ptr(), target.data_ptr(), ldt, _ptr(mom) if ldm else None, ldm,
                 OBJECTIVES[objective], int(steps), float(lr), float(momentum), int(bool(first_step)), _stream(X))
    return Y


def dgd_csr(X: torch.Tensor, Y: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor,
            target: torch.Tensor, mom: Optional[torch.Tensor] = None, objective: str = "least_squares",
            steps: int = 1, lr: float = 0.01, momentum: float = 0.0, first_step: bool = False,
            P: Optional[int] = None) -> torch.Tensor:
    """dgd_ring for any W (CSR mix, bit-exact), then the same local steps."""
    P = X.shape[1] if P is None else P
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    n = rowptr.shape[0] - 1
    if Y.shape[0] < n:
        raise ValueError(f"Y has {Y.shape[0]} rows < {n}")
    for nm, t, dt in (("rowptr", rowptr, torch.int32), ("col", col, torch.int32), ("val", val, torch.float32)):
        if t.device != X.device or t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous {dt} on {X.device}")
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias: the Jacobi mix needs two buffers")
    ldt, ldm = _dgd_args(X, target, mom, objective, steps, momentum, P, n)
    _native.call("dol_dgd_csr_f32", X.data_ptr(), ldx, X.shape[0], Y.data_ptr(), ldy, n, P, rowptr.data_ptr(),
                 col.data_ptr() if col.numel() else None, val.data_ptr() if val.numel() else None,
                 target.data_ptr(), ldt, _ptr(mom) if ldm else None, ldm, OBJECTIVES[objective], int(steps),
                 float(lr), float(momentum), int(bool(first_step)), _stream(X))
    return Y


def dgd_csr_pm(XT: torch.Tensor, YT: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor,
               TT: torch.Tensor, MT: Optional[torch.Tensor] = None, objective: str = "least_squares",
               steps: int = 1, lr: float = 0.01, momentum: float = 0.0, first_step: bool = False,
               x_agents: Optional[int] = None, P: Optional[int] = None, nseg: Optional[int] = None) -> torch.Tensor:
    """dgd_csr on the parameter-major bank: XT/YT as mix_csr_pm, TT [P, >= n]
    the targets and MT [P, >= n] the momentum (transposed like XT); the same
    mix and local steps, bit-identical to dgd_csr on the transposed matrices.
    At most PM_DGD_MAX_AGENTS agents.  nseg as mix_csr_pm (None: the order
    tuned for XT / YT, timed on the plain mix, which only writes YT)."""
    P = XT.shape[0] if P is None else P
    n = rowptr.shape[0] - 1
    x_agents = n if x_agents is None else int(x_agents)
    ldx = _check_rows("XT", XT)
    ldy = _check_rows("YT", YT)
    if XT.shape[0] < P or YT.shape[0] < P:
        raise ValueError(f"XT/YT need >= {P} parameter rows")
    if XT.shape[1] < x_agents or YT.shape[1] < n:
        raise ValueError(f"XT needs >= {x_agents} agent columns, YT >= {n}")
    for nm, t, dt in (("rowptr", rowptr, torch.int32), ("col", col, torch.int32), ("val", val, torch.float32)):
        if t.device != XT.device or t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous {dt} on {XT.device}")
    if XT.data_ptr() == YT.data_ptr():
        raise ValueError("XT and YT alias: the Jacobi mix needs two buffers")
    if objective not in OBJECTIVES:
        raise ValueError(f"objective must be one of {sorted(OBJECTIVES)}")
    if int(steps) < 1:
        raise ValueError("local steps must be >= 1")
    ldt = _check_rows("TT", TT)
    if TT.shape[0] < P or TT.shape[1] < n or TT.device != XT.device:
        raise ValueError(f"TT: expected [>= {P}, >= {n}] on {XT.device}")
    ldm = 0
    if momentum != 0.0:
        if MT is None:
            raise ValueError("momentum != 0 needs MT")
        ldm = _check_rows("MT", MT)
        if MT.shape[0] < P or MT.shape[1] < n or MT.device != XT.device:
            raise ValueError(f"MT: expected [>= {P}, >= {n}] on {XT.device}")
    if nseg is None:
        def mix(ns):
            _native.call("dol_mix_csr_pm_ex_f32", XT.data_ptr(), ldx, x_agents, YT.data_ptr(), ldy, n, P,
                         rowptr.data_ptr(), col.data_ptr() if col.numel() else None,
                         val.data_ptr() if val.numel() else None, int(ns), _stream(XT))
        nseg = _pm_auto(XT, YT, ldx, ldy, x_agents, n, P, mix)
    _native.call("dol_dgd_csr_pm_ex_f32", XT.data_ptr(), ldx, x_agents, YT.data_ptr(), ldy, n, P, rowptr.data_ptr(),
                 col.data_ptr() if col.numel() else None, val.data_ptr() if val.numel() else None, TT.data_ptr(),
                 ldt, _ptr(MT) if ldm else None, ldm, OBJECTIVES[objective], int(steps), float(lr), float(momentum),
                 int(bool(first_step)), int(nseg), _stream(XT))
    return YT


def mix_dense(W: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, P: Optional[int] = None) -> torch.Tensor:
    """Y = W X on fp32 MFMA (fma chain over k; tolerance path, see dol_hip.h)."""
    P = X.shape[1] if P is None else P
    ldw = _check_rows("W", W)
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    M, K = W.shape
    if X.shape[0] < K or Y.shape[0] < M:
        raise ValueError(f"shapes: W {tuple(W.shape)}, X {tuple(X.shape)}, Y {tuple(Y.shape)}")
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias")
    _native.call("dol_mix_dense_f32", W.data_ptr(), ldw, X.data_ptr(), ldx, Y.data_ptr(), ldy, M, K, P, _stream(X))
    return Y


SPLIT3_W_READY, SPLIT3_X_ROWS_PADDED, SPLIT3_FUSE_X = 1, 2, 4  # dol_hip.h flags


def split3_x_flags(X: torch.Tensor, P: int) -> int:
    """DOL_SPLIT3_X_ROWS_PADDED when the GEMM may read X's rows in whole 16-B
    pieces up to round_up(P, 4) floats (aligned rows, ld % 4 == 0, storage
    present): X is then split in registers, with no split pass."""
    if X.data_ptr() % 16 or X.dim() != 2 or (X.shape[0] > 1 and X.stride(0) % 4):
        return 0
    ld = X.stride(0) if X.shape[0] > 1 else X.shape[1]
    p4 = -(-P // 4) * 4
    if ld < p4:
        return 0
    need = X.storage_offset() + (X.shape[0] - 1) * ld + p4
    return SPLIT3_X_ROWS_PADDED if need * 4 <= X.untyped_storage().nbytes() else 0


def dense_split3_workspace_bytes(M: int, K: int, P: int, flags: int = 0) -> int:
    return int(_native.lib().dol_mix_dense_split3_workspace_bytes(int(M), int(K), int(P), int(flags)))


SPLIT3_FUSE_MAX_M = 2048  # auto-fused X split up to this many output rows (agents)


def mix_dense_split3(W: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, P: Optional[int] = None,
                     work: Optional[torch.Tensor] = None, w_ready: bool = False,
                     fuse: Optional[bool] = None) -> torch.Tensor:
    """Y = W X on the bf16 matrix cores at fp32 accuracy (dol_mix_dense_split3_f32:
    three-piece bf16 split of both operands, six piece products per term).
    fuse (None = when X's rows allow it, split3_x_flags, and M <=
    SPLIT3_FUSE_MAX_M): X is split inside the GEMM (dense_split3_fx8_kernel:
    no split pass, no X workspace; same bits) instead of by a split pass.  Its
    GEMM runs ~6-8 % slower than the record-staged one, so it pays where the
    pass is a large share of the round, i.e. few output rows per X value:
    1024 x 1024 x 101,770 0.94-0.95 vs 1.04 ms, 8192 x 8192 x 101,770 56.2
    vs 53.1 ms (tools/split3_ab.py, profiles/r05m_split3_ab.jsonl,
    r05n_split3_ab_8192.jsonl).  fuse=False forces the split pass.  `work`: a uint8 device
    buffer of >= dense_split3_workspace_bytes(M, K, P, flags) bytes (allocated
    per call when None); w_ready=True reuses the split W that a previous call
    with the same W left in `work`."""
    P = X.shape[1] if P is None else P
    ldw = _check_rows("W", W)
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    M, K = W.shape
    if X.shape[0] < K or Y.shape[0] < M:
        raise ValueError(f"shapes: W {tuple(W.shape)}, X {tuple(X.shape)}, Y {tuple(Y.shape)}")
    if Y.data_ptr() in (X.data_ptr(), W.data_ptr()):
        raise ValueError("Y aliases an input")
    if fuse is None:
        fuse = None if W.shape[0] <= SPLIT3_FUSE_MAX_M else False
    xf = split3_x_flags(X, P) if fuse is not False else 0
    fused = bool(xf) or (fuse is True and P % 4 == 0)
    flags = ((SPLIT3_FUSE_X | xf) if fused else 0) | (SPLIT3_W_READY if w_ready else 0)
    need = dense_split3_workspace_bytes(M, K, P, flags)
    if work is None:
        if w_ready:
            raise ValueError("w_ready needs the workspace of the call that split W")
        work = torch.empty(max(need, 1), dtype=torch.uint8, device=X.device)
    elif work.device != X.device or work.dtype != torch.uint8 or work.numel() < need:
        raise ValueError(f"work: need a uint8 tensor of >= {need} bytes on {X.device}")
    _native.call("dol_mix_dense_split3_f32", W.data_ptr(), ldw, X.data_ptr(), ldx, Y.data_ptr(), ldy, M, K, P,
                 work.data_ptr(), work.numel(), flags, _stream(X))
    return Y


def er_stochastic(W: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """W[n, >=n] <- a fresh Erdos-Renyi G(n, p) mixing matrix under the
    reference's 'stochastic' weighting, in one kernel (dol_er_stochastic_f32)."""
    ld = _check_rows("W", W)
    n = W.shape[0]
    if W.shape[1] < n:
        raise ValueError(f"W: expected [n, >= n], got {tuple(W.shape)}")
    _native.call("dol_er_stochastic_f32", W.data_ptr(), ld, n, float(p), int(seed) & (2**64 - 1), _stream(W))
    return W


def mix_ring(X: torch.Tensor, Y: torch.Tensor, w_prev: torch.Tensor, w_next: torch.Tensor,
             halo_prev: Optional[torch.Tensor] = None, halo_next: Optional[torch.Tensor] = None,
             P: Optional[int] = None, n_rows: Optional[int] = None) -> torch.Tensor:
    """Ring (circle topology) mix; halos are the rows before/after the local block."""
    P = X.shape[1] if P is None else P
    n = X.shape[0] if n_rows is None else n_rows
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    if X.shape[0] < n or Y.shape[0] < n:
        raise ValueError("X/Y have fewer rows than n_rows")
    for nm, t in (("w_prev", w_prev), ("w_next", w_next)):
        if t.device != X.device or t.dtype != torch.float32 or t.numel() < n or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous float32 [{n}] on {X.device}")
    if (halo_prev is None) != (halo_next is None):
        raise ValueError("pass both halos or neither")
    if halo_prev is None and n < 3:
        raise ValueError("a wrap-around ring needs >= 3 rows (use mix_csr)")
    _check_vec("halo_prev", halo_prev, P, X.device)
    _check_vec("halo_next", halo_next, P, X.device)
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias: the Jacobi mix needs two buffers")
    _native.call("dol_mix_ring_f32", X.data_ptr(), ldx, Y.data_ptr(), ldy, n, P, _ptr(halo_prev),
                 _ptr(halo_next), w_prev.data_ptr(), w_next.data_ptr(), _stream(X))
    return Y


def mix_ring_edges(X: torch.Tensor, Y: torch.Tensor, w_prev: torch.Tensor, w_next: torch.Tensor,
                   halo_prev: torch.Tensor, halo_next: torch.Tensor, P: Optional[int] = None,
                   n_rows: Optional[int] = None) -> torch.Tensor:
    """Rows 0 and n_rows-1 of mix_ring with halos, in one launch (the second
    half of a sharded ring round; dol_mix_ring_edges_f32)."""
    P = X.shape[1] if P is None else P
    n = X.shape[0] if n_rows is None else n_rows
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    if X.shape[0] < n or Y.shape[0] < n:
        raise ValueError("X/Y have fewer rows than n_rows")
    for nm, t in (("w_prev", w_prev), ("w_next", w_next)):
        if t.device != X.device or t.dtype != torch.float32 or t.numel() < n or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous float32 [{n}] on {X.device}")
    if halo_prev is None or halo_next is None:
        raise ValueError("mix_ring_edges needs both halos")
    _check_vec("halo_prev", halo_prev, P, X.device)
    _check_vec("halo_next", halo_next, P, X.device)
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias: the Jacobi mix needs two buffers")
    _native.call("dol_mix_ring_edges_f32", X.data_ptr(), ldx, Y.data_ptr(), ldy, n, P, halo_prev.data_ptr(),
                 halo_next.data_ptr(), w_prev.data_ptr(), w_next.data_ptr(), _stream(X))
    return Y


def dgd_ring_edges(X: torch.Tensor, Y: torch.Tensor, w_prev: torch.Tensor, w_next: torch.Tensor,
                   target: torch.Tensor, halo_prev: torch.Tensor, halo_next: torch.Tensor,
                   mom: Optional[torch.Tensor] = None, objective: str = "least_squares", steps: int = 1,
                   lr: float = 0.01, momentum: float = 0.0, first_step: bool = False, P: Optional[int] = None,
                   n_rows: Optional[int] = None) -> torch.Tensor:
    """Rows 0 and n_rows-1 of dgd_ring with halos, in one launch (dol_dgd_ring_edges_f32)."""
    P = X.shape[1] if P is None else P
    n = X.shape[0] if n_rows is None else n_rows
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    if X.shape[0] < n or Y.shape[0] < n:
        raise ValueError("X/Y have fewer rows than n_rows")
    for nm, t in (("w_prev", w_prev), ("w_next", w_next)):
        if t.device != X.device or t.dtype != torch.float32 or t.numel() < n or not t.is_contiguous():
            raise ValueError(f"{nm}: expected contiguous float32 [{n}] on {X.device}")
    if halo_prev is None or halo_next is None:
        raise ValueError("dgd_ring_edges needs both halos")
    _check_vec("halo_prev", halo_prev, P, X.device)
    _check_vec("halo_next", halo_next, P, X.device)
    if X.data_ptr() == Y.data_ptr():
        raise ValueError("X and Y alias: the Jacobi mix needs two buffers")
    ldt, ldm = _dgd_args(X, target, mom, objective, steps, momentum, P, n)
    _native.call("dol_dgd_ring_edges_f32", X.data_ptr(), ldx, Y.data_ptr(), ldy, n, P, halo_prev.data_ptr(),
                 halo_next.data_ptr(), w_prev.data_ptr(), w_next.data_ptr(), target.data_ptr(), ldt,
                 _ptr(mom) if ldm else None, ldm, OBJECTIVES[objective], int(steps), float(lr), float(momentum),
                 int(bool(first_step)), _stream(X))
    return Y


def prox_admm_sgd(w: torch.Tensor, g: torch.Tensor, buf: Optional[torch.Tensor] = None,
                  theta: Optional[torch.Tensor] = None, alpha: Optional[torch.Tensor] = None,
                  rho: float = 0.0, lr: float = 0.01, momentum: float = 0.0, first_step: bool = False,
                  write_grad: bool = True, P: Optional[int] = None) -> None:
    """Fused FedProx/FedADMM gradient term + torch.optim.SGD(momentum) step, in place.

    Reference: DEC/clients.py:101-115, :125-139 and SGD.step (:44)."""
    P = w.shape[1] if P is None else P
    n = w.shape[0]
    ldw = _check_rows("w", w, P)
    ldg = _check_rows("g", g, P)
    if g.shape[0] < n:
        raise ValueError("g has fewer rows than w")
    ldb = 0
    if momentum != 0.0:
        if buf is None:
            raise ValueError("momentum != 0 needs buf")
        ldb = _check_rows("buf", buf, P)
        if buf.shape[0] < n:
            raise ValueError("buf has fewer rows than w")
    lda = 0
    if alpha is not None:
        if theta is None:
            raise ValueError("alpha needs theta")
        lda = _check_rows("alpha", alpha, P)
        if alpha.shape[0] < n:
            raise ValueError("alpha has fewer rows than w")
    _check_vec("theta", theta, P, w.device)
    _native.call("dol_prox_admm_sgd_f32", w.data_ptr(), ldw, _ptr(buf) if momentum != 0.0 else None, ldb,
                 g.data_ptr(), ldg, _ptr(theta), _ptr(alpha), lda, float(rho), float(lr), float(momentum),
                 int(bool(first_step)), int(bool(write_grad)), n, P, _stream(w))


def admm_step_dual(w: torch.Tensor, g: torch.Tensor, theta: torch.Tensor, alpha: torch.Tensor,
                   buf: Optional[torch.Tensor] = None, rho: float = 0.0, lr: float = 0.01, momentum: float = 0.0,
                   first_step: bool = False, write_grad: bool = True, P: Optional[int] = None) -> None:
    """Last FedADMM local step + dual ascent in one pass (bit-identical to
    prox_admm_sgd(theta, alpha) followed by admm_dual)."""
    P = w.shape[1] if P is None else P
    n = w.shape[0]
    ldw = _check_rows("w", w, P)
    ldg = _check_rows("g", g, P)
    lda = _check_rows("alpha", alpha, P)
    if g.shape[0] < n or alpha.shape[0] < n:
        raise ValueError("g/alpha have fewer rows than w")
    ldb = 0
    if momentum != 0.0:
        if buf is None:
            raise ValueError("momentum != 0 needs buf")
        ldb = _check_rows("buf", buf, P)
    _check_vec("theta", theta, P, w.device)
    _native.call("dol_admm_step_dual_f32", w.data_ptr(), ldw, _ptr(buf) if momentum != 0.0 else None, ldb,
                 g.data_ptr(), ldg, theta.data_ptr(), alpha.data_ptr(), lda, float(rho), float(lr), float(momentum),
                 int(bool(first_step)), int(bool(write_grad)), n, P, _stream(w))


def prox_grad(g: torch.Tensor, w: torch.Tensor, theta: torch.Tensor, rho: float,
              alpha: Optional[torch.Tensor] = None, P: Optional[int] = None) -> None:
    """g += rho*(w - theta) (+ alpha), in place: the update_model gradient term alone
    (DEC/clients.py:108-111, :132-135)."""
    P = g.shape[1] if P is None else P
    n = g.shape[0]
    ldg = _check_rows("g", g, P)
    ldw = _check_rows("w", w, P)
    if w.shape[0] < n:
        raise ValueError("w has fewer rows than g")
    lda = 0
    if alpha is not None:
        lda = _check_rows("alpha", alpha, P)
        if alpha.shape[0] < n:
            raise ValueError("alpha has fewer rows than g")
    _check_vec("theta", theta, P, g.device)
    _native.call("dol_prox_grad_f32", g.data_ptr(), ldg, w.data_ptr(), ldw, theta.data_ptr(), _ptr(alpha), lda,
                 float(rho), n, P, _stream(g))


def dual_workspace_bytes(n_agents: int, P: int) -> int:
    return int(_native.lib().dol_admm_dual_workspace_bytes(n_agents, P))


def admm_dual(alpha: torch.Tensor, w: torch.Tensor, theta: torch.Tensor, rho: float,
              resid_sq: Optional[torch.Tensor] = None, work: Optional[torch.Tensor] = None,
              P: Optional[int] = None) -> None:
    """alpha += rho*(w - theta) for every row (DEC/clients.py:141-144), in place."""
    P = alpha.shape[1] if P is None else P
    n = alpha.shape[0]
    lda = _check_rows("alpha", alpha, P)
    ldw = _check_rows("w", w, P)
    if w.shape[0] < n:
        raise ValueError("w has fewer rows than alpha")
    _check_vec("theta", theta, P, alpha.device)
    if resid_sq is not None:
        if resid_sq.dtype != torch.float64 or resid_sq.numel() < n or resid_sq.device != alpha.device:
            raise ValueError("resid_sq: expected float64 [n_agents] on the same device")
        need = dual_workspace_bytes(n, P)
        if work is None:
            work = torch.empty(max(need, 8), dtype=torch.uint8, device=alpha.device)
        elif work.numel() * work.element_size() < need:
            raise ValueError(f"work: need {need} bytes")
    _native.call("dol_admm_dual_f32", alpha.data_ptr(), lda, w.data_ptr(), ldw, theta.data_ptr(), float(rho),
                 n, P, _ptr(resid_sq), _ptr(work) if resid_sq is not None else None, _stream(alpha))


def admm_ls_round_workspace_bytes(m: int, P: int) -> int:
    return int(_native.lib().dol_admm_ls_round_workspace_bytes(int(m), int(P)))


def admm_ls_round(w: torch.Tensor, alpha: torch.Tensor, target: torch.Tensor, theta: torch.Tensor,
                  agents: Optional[torch.Tensor] = None, first: Optional[torch.Tensor] = None,
                  buf: Optional[torch.Tensor] = None, rho: float = 0.1, lr: float = 0.1, momentum: float = 0.0,
                  local_steps: int = 1, resid_sq: Optional[torch.Tensor] = None,
                  alpha_sq: Optional[torch.Tensor] = None, work: Optional[torch.Tensor] = None,
                  P: Optional[int] = None) -> None:
    """One FedADMM client round on f_a(w) = 1/2 ||w - t_a||^2 for the sampled
    rows `agents` (int32 device [m]; None = rows 0..n-1), fused per row
    (dol_admm_ls_round_f32): w = theta, `local_steps` x (LS gradient + ADMM
    term + momentum SGD), then the dual ascent.  first: int32 device [m],
    nonzero where that agent's optimizer takes its first step ever.
    resid_sq / alpha_sq: float64 [m] outputs (||w - theta||^2, ||alpha||^2).
    Reference: DEC/clients.py:36-53, :125-144 (update_weights, update_model,
    update_duals) with the CNN loss replaced by least squares."""
    P = w.shape[1] if P is None else P
    ldw = _check_rows("w", w, P)
    lda = _check_rows("alpha", alpha, P)
    ldt = _check_rows("target", target, P)
    n = w.shape[0]
    if alpha.shape[0] < n or target.shape[0] < n:
        raise ValueError("alpha/target have fewer rows than w")
    _check_vec("theta", theta, P, w.device)
    if int(local_steps) < 0:
        raise ValueError("local_steps must be >= 0")
    ldb = 0
    if momentum != 0.0:
        if buf is None:
            raise ValueError("momentum != 0 needs buf")
        ldb = _check_rows("buf", buf, P)
        if buf.shape[0] < n:
            raise ValueError("buf has fewer rows than w")
    m = n
    if agents is not None:
        _check_order(agents, w.device, n)
        m = agents.numel()
    if first is not None and (first.device != w.device or first.dtype != torch.int32 or not first.is_contiguous()
                              or first.numel() < m):
        raise ValueError(f"first: expected contiguous int32 [{m}] on {w.device}")
    if (resid_sq is None) != (alpha_sq is None):
        raise ValueError("pass both resid_sq and alpha_sq or neither")
    if resid_sq is not None:
        for nm, t in (("resid_sq", resid_sq), ("alpha_sq", alpha_sq)):
            if t.dtype != torch.float64 or t.numel() < m or t.device != w.device or not t.is_contiguous():
                raise ValueError(f"{nm}: expected contiguous float64 [{m}] on {w.device}")
        need = admm_ls_round_workspace_bytes(m, P)
        if work is None:
            work = _workspace(w.device, need)
        elif work.device != w.device or work.numel() * work.element_size() < need:
            raise ValueError(f"work: need {need} bytes on {w.device}")
    _native.call("dol_admm_ls_round_f32", w.data_ptr(), ldw, _ptr(buf) if ldb else None, ldb, alpha.data_ptr(), lda,
                 target.data_ptr(), ldt, theta.data_ptr(), _ptr(agents), _ptr(first), m, P, float(rho), float(lr),
                 float(momentum), int(local_steps), _ptr(resid_sq), _ptr(alpha_sq),
                 _ptr(work) if resid_sq is not None else None, _stream(w))


def admm_ls_round_mean(w: torch.Tensor, alpha: torch.Tensor, target: torch.Tensor, theta: torch.Tensor,
                       agents: Optional[torch.Tensor] = None, first: Optional[torch.Tensor] = None,
                       buf: Optional[torch.Tensor] = None, rho: float = 0.1, lr: float = 0.1, momentum: float = 0.0,
                       local_steps: int = 1, out: Optional[torch.Tensor] = None, scale: Optional[float] = None,
                       resid_total: Optional[torch.Tensor] = None, work: Optional[torch.Tensor] = None,
                       P: Optional[int] = None, validate: bool = True) -> torch.Tensor:
    """admm_ls_round + the server's ordered average in ONE pass
    (dol_admm_ls_round_mean_f32): the rows come out as admm_ls_round leaves
    them and `out` = ordered_sum(w, agents, scale=scale) of the new rows, the
    same bits, without reading w back.  scale None = m (the mean,
    DEC/servers.py:42-48); 1.0 = the raw ordered sum.  agents: DISTINCT rows in
    the sampled order (None = 0..n-1).  resid_total: float64 [2] output, the
    round's sums over the agents of ||w - theta||^2 and ||alpha||^2.
    validate (default): check on the host that `agents` are distinct rows of w
    (one device-to-host copy of m ids).  The kernel loads the next agents'
    rows before it stores the current ones, so a repeated id would read a
    stale row, and an out-of-range id would read and write out of bounds
    (ADVICE r05).  Callers that drew the ids themselves on the host and
    checked them (SeparableADMM.round) pass validate=False.
    Reference: DEC/servers.py:50-81 (Server.run's round) on least squares."""
    P = w.shape[1] if P is None else P
    ldw = _check_rows("w", w, P)
    lda = _check_rows("alpha", alpha, P)
    ldt = _check_rows("target", target, P)
    n = w.shape[0]
    if alpha.shape[0] < n or target.shape[0] < n:
        raise ValueError("alpha/target have fewer rows than w")
    _check_vec("theta", theta, P, w.device)
    if int(local_steps) < 0:
        raise ValueError("local_steps must be >= 0")
    ldb = 0
    if momentum != 0.0:
        if buf is None:
            raise ValueError("momentum != 0 needs buf")
        ldb = _check_rows("buf", buf, P)
        if buf.shape[0] < n:
            raise ValueError("buf has fewer rows than w")
    m = n
    if agents is not None:
        _check_order(agents, w.device, n)
        m = agents.numel()
        if m > n:
            raise ValueError(f"admm_ls_round_mean: {m} agents but w has {n} rows (agents must be distinct)")
        if validate and m:
            ids = agents.cpu()
            if int(ids.min()) < 0 or int(ids.max()) >= n or torch.unique(ids).numel() != m:
                raise ValueError(f"admm_ls_round_mean: agents must be distinct rows in [0, {n})")
    if m < 1:
        raise ValueError("admm_ls_round_mean needs at least one agent (the average indexes w[0])")
    if first is not None and (first.device != w.device or first.dtype != torch.int32 or not first.is_contiguous()
                              or first.numel() < m):
        raise ValueError(f"first: expected contiguous int32 [{m}] on {w.device}")
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=w.device)
    _check_vec("out", out, P, w.device)
    if resid_total is not None:
        if (resid_total.dtype != torch.float64 or resid_total.numel() < 2 or resid_total.device != w.device
                or not resid_total.is_contiguous()):
            raise ValueError(f"resid_total: expected contiguous float64 [2] on {w.device}")
        need = int(_native.lib().dol_admm_ls_round_mean_workspace_bytes(int(P)))
        if work is None:
            work = _workspace(w.device, need)
        elif work.device != w.device or work.numel() * work.element_size() < need:
            raise ValueError(f"work: need {need} bytes on {w.device}")
    _native.call("dol_admm_ls_round_mean_f32", w.data_ptr(), ldw, _ptr(buf) if ldb else None, ldb, alpha.data_ptr(),
                 lda, target.data_ptr(), ldt, theta.data_ptr(), _ptr(agents), _ptr(first), m, P, float(rho), float(lr),
                 float(momentum), int(local_steps), out.data_ptr(), float(m if scale is None else scale),
                 _ptr(resid_total), _ptr(work) if resid_total is not None else None, _stream(w))
    return out


def _check_order(order: torch.Tensor, device, n_rows: int) -> None:
    if order.device != device or order.dtype != torch.int32 or not order.is_contiguous():
        raise ValueError("order: expected contiguous int32 on the rows' device")


def ordered_mean(W: torch.Tensor, order: torch.Tensor, out: Optional[torch.Tensor] = None,
                 P: Optional[int] = None) -> torch.Tensor:
    """theta = (((w[o0] + w[o1]) + ...) / m (DEC/servers.py:42-48)."""
    P = W.shape[1] if P is None else P
    ldw = _check_rows("W", W, P)
    _check_order(order, W.device, W.shape[0])
    m = order.numel()
    if m < 1:
        raise ValueError("ordered_mean needs at least one row (the reference indexes w[0])")
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=W.device)
    _check_vec("out", out, P, W.device)
    _native.call("dol_ordered_mean_f32", W.data_ptr(), ldw, order.data_ptr(), m, P, out.data_ptr(), _stream(W))
    return out


def ordered_sum(W: torch.Tensor, order: torch.Tensor, acc_in: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, scale: float = 1.0, P: Optional[int] = None) -> torch.Tensor:
    P = (W.shape[1] if W is not None else acc_in.shape[0]) if P is None else P
    device = W.device if W is not None else acc_in.device
    ldw = _check_rows("W", W, P) if W is not None else P
    m = 0 if order is None else order.numel()
    if m:
        _check_order(order, device, W.shape[0])
    _check_vec("acc_in", acc_in, P, device)
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=device)
    _check_vec("out", out, P, device)
    _native.call("dol_ordered_sum_f32", _ptr(W) if m else None, ldw, _ptr(order) if m else None, m, P,
                 _ptr(acc_in), out.data_ptr(), float(scale), torch.cuda.current_stream(device).cuda_stream)
    return out


def stream_copy(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    if src.device.type != "cuda" or dst.device != src.device:
        raise DolNativeError("stream_copy: device tensors required")
    if not (src.is_contiguous() and dst.is_contiguous()) or src.numel() != dst.numel():
        raise ValueError("stream_copy: contiguous tensors of equal size required")
    _native.call("dol_stream_copy_f32", src.data_ptr(), dst.data_ptr(), src.numel(), _stream(src))
    return dst


def stream_copy_rows(X: torch.Tensor, Y: torch.Tensor, P: Optional[int] = None) -> torch.Tensor:
    """Y[:, :P] = X[:, :P] in the ring mix's tile geometry (roofline calibration)."""
    P = X.shape[1] if P is None else P
    ldx = _check_rows("X", X, P)
    ldy = _check_rows("Y", Y, P)
    if Y.shape[0] < X.shape[0]:
        raise ValueError("Y has fewer rows than X")
    _native.call("dol_stream_copy_rows_f32", X.data_ptr(), ldx, Y.data_ptr(), ldy, X.shape[0], P, _stream(X))
    return Y


def mlp_step(w: torch.Tensor, X: torch.Tensor, y: torch.Tensor, d: int, h: int, c: int,
             grad: Optional[torch.Tensor] = None, mom: Optional[torch.Tensor] = None,
             theta: Optional[torch.Tensor] = None, alpha: Optional[torch.Tensor] = None,
             loss: Optional[torch.Tensor] = None, lr: float = 0.01, momentum: float = 0.0, rho: float = 0.0,
             first_step: bool = False, update: bool = True,
             work: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Fused forward + CE + backward + (prox/ADMM) momentum-SGD step of every
    agent's MLP Linear(d,h)-ReLU-Linear(h,c) (rows of w, state_dict order).

    X [n, B, d] fp32, y [n, B] int64.  update=False only writes the raw
    gradients into grad.  Reference: DIST/clients.py:34-59 (one local
    iteration per agent), DEC/clients.py:101-139 (prox / ADMM terms)."""
    P = h * d + h + c * h + c
    n = w.shape[0]
    ldw = _check_rows("w", w, P)
    if X.device != w.device or X.dtype != torch.float32 or X.dim() != 3 or X.shape[0] != n or X.shape[2] != d:
        raise ValueError(f"X: expected float32 [{n}, B, {d}] on {w.device}")
    if X.stride(2) != 1:
        raise ValueError("X: samples must be contiguous")
    B = X.shape[1]
    if y.device != w.device or y.dtype != torch.int64 or tuple(y.shape) != (n, B) or (B > 1 and y.stride(1) != 1):
        raise ValueError(f"y: expected int64 [{n}, {B}] on {w.device}")
    ldg = _check_rows("grad", grad, P) if grad is not None else 0
    ldm = 0
    if update and momentum != 0.0:
        if mom is None:
            raise ValueError("momentum != 0 needs mom")
        ldm = _check_rows("mom", mom, P)
    lda = 0
    if alpha is not None:
        if theta is None:
            raise ValueError("alpha needs theta")
        lda = _check_rows("alpha", alpha, P)
    _check_vec("theta", theta, P, w.device)
    for nm, t in (("grad", grad), ("mom", mom if ldm else None), ("alpha", alpha)):
        if t is not None and t.shape[0] < n:
            raise ValueError(f"{nm} has fewer rows than w")
    if loss is not None and (loss.device != w.device or loss.dtype != torch.float32 or loss.numel() < n
                             or not loss.is_contiguous()):
        raise ValueError(f"loss: expected a contiguous float32 [{n}] on {w.device}")
    wbytes = int(_native.lib().dol_mlp_step_workspace_bytes(n, B, h))
    if work is None:
        work = _workspace(w.device, wbytes)
    elif work.device != w.device or work.numel() * work.element_size() < wbytes:
        raise ValueError(f"work: need {wbytes} bytes on {w.device}")
    ldxa = X.stride(0) if n > 1 else B * X.stride(1)
    ldxb = X.stride(1) if B > 1 else d
    _native.call("dol_mlp_step_f32", w.data_ptr(), ldw, _ptr(grad), ldg, _ptr(mom) if ldm else None, ldm,
                 _ptr(theta), _ptr(alpha), lda, X.data_ptr(), ldxa, ldxb, y.data_ptr(),
                 y.stride(0) if n > 1 else B, _ptr(loss), n, B, d, h, c, float(lr), float(momentum), float(rho),
                 int(bool(first_step)), int(bool(update)), work.data_ptr(), _stream(w))
    return loss


_WORK = {}


def _workspace(device, nbytes: int) -> torch.Tensor:
    """Per-device scratch, grown on demand and reused (stream-ordered on the
    current stream like every other op)."""
    t = _WORK.get(device)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _WORK[device] = t
    return t
