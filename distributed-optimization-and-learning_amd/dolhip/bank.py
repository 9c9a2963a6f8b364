"""AgentBank: the stacked, HBM-resident state of N agents.

The reference keeps one nn.Module per agent and "communicates" by reading
other agents' state_dict() (DIST/simulators.py:91-97, DEC/servers.py:60-64).
Here agent k's flattened parameters are row k of one [N, ld] fp32 matrix
(flattening order = state_dict key order, ld = P rounded up to 64 floats so
every row starts 256-B aligned and streams as 16-B lanes).  Each agent's
nn.Module parameters are *views* into its row, so PyTorch-ROCm forward/
backward and the HIP kernels see the same memory without copies.

Buffers (allocated on demand):
  x      parameters (the mixing input)          [N, ld]
  y      mixing output (Jacobi double buffer)   [N, ld]
  grad   per-agent gradients                    [N, ld]
  mom    SGD momentum buffers                   [N, ld]
  alpha  ADMM duals                             [N, ld]
A mixing round writes y from x and then swaps the two (no copy, matching the
reference's synchronous load_state_dict write-back, DIST/simulators.py:151-152).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import ctypes
import os

import torch

from . import _native, ops

Layout = List[Tuple[str, Tuple[int, ...]]]

ROW_ALIGN = 64  # floats (256 B)


def layout_of(module: torch.nn.Module) -> Layout:
    return [(k, tuple(v.shape)) for k, v in module.state_dict().items()]


def layout_size(layout: Layout) -> int:
    n = 0
    for _, shape in layout:
        c = 1
        for s in shape:
            c *= int(s)
        n += c
    return n


def round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


LONG_ROW = 1 << 18  # floats (1 MiB rows)


def row_stride(P: int) -> int:
    """Leading dimension for P-float agent rows: 256-B aligned, and never a
    multiple of 8 KiB — power-of-two row strides put the rows a tile walks on
    the same HBM channels (ring mix at 8192 x 2^20 on MI355X: 5.57 TB/s with
    ld = 2^20, 6.14 TB/s with ld = 2^20 + 1024, tools/membench5.hip).  Rows of
    >= 1 MiB (r04): an odd multiple of 8 KiB, ld = 2048 (mod 4096) floats.  The
    ring round at 8192 x 2^20, strides alternating in one process on two boxes
    (tools/ring_ld_probe.py, profiles/r04q_ring_ld_probe.jsonl): 2^20 + 1024
    10.94 ms (6.28 TB/s), + 2048 10.64-10.66 ms (6.45), + 3072 11.05-11.08,
    + 4096 11.9, + 6144 10.65-10.69; the eps = 5 pass over the same rows runs
    2-3 % slower at + 2048 (10.59 -> 10.87 ms best kernel on one box,
    12.66 -> 12.86 on the other, profiles/r04q_eps_ld_probe.jsonl)."""
    ld = round_up(max(P, 1), ROW_ALIGN)
    if ld >= LONG_ROW:
        return ld + (2048 - ld % 4096) % 4096
    if ld % 2048 == 0:
        ld += 1024
    return ld


class _MappedBlock:
    """Owner of one dol_bank_alloc block, exposed to torch through
    __cuda_array_interface__ (the tensor's storage keeps this object alive and
    frees the block with it)."""

    def __init__(self, rows: int, cols: int, device: torch.device):
        self.device = device
        nbytes = max(rows * cols, 1) * 4
        ptr, mapped = ctypes.c_void_p(), ctypes.c_int64()
        with torch.cuda.device(device):
            _native.call("dol_bank_alloc", nbytes, ctypes.addressof(ptr), ctypes.addressof(mapped))
        self.ptr, self.mapped = int(ptr.value), int(mapped.value)
        self.__cuda_array_interface__ = {"shape": (rows, cols), "typestr": "<f4", "data": (self.ptr, False),
                                         "version": 2, "strides": None}

    def release(self) -> None:
        """Wait for the device, then unmap and release the block; raises
        DolNativeError (with dol_last_error) if a step fails -- the block then
        stays registered and release() can be called again."""
        if not getattr(self, "ptr", 0):
            return
        torch.cuda.synchronize(self.device)  # no kernel may still use the block
        _native.call("dol_bank_free", self.ptr, self.mapped)
        self.ptr = 0

    def __del__(self):
        if not getattr(self, "ptr", 0):
            return
        try:
            self.release()
        except Exception as e:  # noqa: BLE001 - a destructor cannot raise; say so instead of leaking silently
            import sys
            import warnings
            if sys is not None and not sys.is_finalizing():
                warnings.warn(f"dolhip: a mapped bank block of {self.mapped} bytes at {self.ptr:#x} was not "
                              f"released ({type(e).__name__}: {e}); it stays allocated", ResourceWarning,
                              stacklevel=2)
            _LEAKED.append(self)  # keep the registration reachable for a later retry (release_leaked)


_LEAKED: List["_MappedBlock"] = []


def release_leaked() -> int:
    """Retry the release of mapped blocks whose destructor failed; returns how
    many are still held."""
    keep = []
    for blk in _LEAKED:
        try:
            blk.release()
        except Exception:  # noqa: BLE001 - still failing: keep it
            keep.append(blk)
    _LEAKED[:] = keep
    return len(keep)


MAPPED_MIN_BYTES = 1 << 30
_CAP_WARNED = []


def retired_va() -> dict:
    """Address space retired by dol_bank_free (freed mapped blocks keep their
    virtual range reserved) and its cap (dol_bank_alloc refuses
    new mapped blocks past it)."""
    L = _native.lib()
    return {"bytes": int(L.dol_bank_retired_bytes()), "blocks": int(L.dol_bank_retired_blocks()),
            "cap_bytes": int(L.dol_bank_retired_cap_bytes())}


def device_matrix(rows: int, cols: int, device, zero: bool = False, mapped: Optional[bool] = None) -> torch.Tensor:
    """A [rows, cols] fp32 device matrix for bank state.  Matrices of >= 1 GiB
    are ONE mapped physical allocation (dol_bank_alloc: hipMemCreate +
    hipMemMap) by default; DOL_BANK_ALLOC=torch (or mapped=False) takes
    torch's caching allocator instead.  In one process, both pairs held at
    once and alternated (tools/alloc_ab.py, profiles/r05d_alloc_ab.jsonl), the
    8192 x 2^20 ring round ran 10.69 ms on mapped buffers against 10.90 on
    torch-allocated ones, and FedLCon's eps = 5 pass 12.79 against 13.30-13.39.
    r04 made this opt-in after a GPU memory fault in a process that had mapped
    and freed many blocks (profiles/r04k_vmm_fault.txt); r05 found the cause:
    a block mapped at a virtual range a freed block used is read and written
    through stale translations of the old block (7 of 11 re-mapped cycles
    wrong, profiles/r05c_vmm_remap_probe.jsonl).  dol_bank_free now retires
    the range instead of freeing it, and twelve map/free cycles are bit-exact
    (tests/test_bank_alloc_gpu.py::test_mapped_blocks_survive_map_free_remap_cycles).
    mapped=True / False decides for this matrix regardless of the environment.
    Retired address space is counted and capped (retired_va()): past the cap
    a default (mapped=None) matrix falls back to torch's allocator with a
    warning; mapped=True raises."""
    device = torch.device(device)
    want = os.environ.get("DOL_BANK_ALLOC", "vmm") == "vmm" if mapped is None else bool(mapped)
    if want and device.type == "cuda" and rows * cols * 4 >= MAPPED_MIN_BYTES:
        try:
            blk = _MappedBlock(rows, cols, device)
        except _native.DolNativeError as e:
            if mapped is not None or "DOL_BANK_RETIRED_VA_CAP_GIB" not in str(e):
                raise
            if not _CAP_WARNED:
                import warnings
                warnings.warn(f"dolhip: {e}; bank matrices now come from torch's allocator", ResourceWarning,
                              stacklevel=2)
                _CAP_WARNED.append(True)
            blk = None
        if blk is not None:
            t = torch.as_tensor(blk, device=device)
            if zero:
                t.zero_()
            return t
    alloc = torch.zeros if zero else torch.empty
    return alloc(rows, cols, dtype=torch.float32, device=device)


# Destination check of fused ring passes (r05): on some pairs of
# large allocations the eps pass's column-strip read + write stream runs ~20 %
# slower than on others (13.1-13.5 vs 11.0-11.4 ms at 8192 x 2^20, while the
# ring round is 10.6-10.9 ms on every pair; which pairs is random per
# allocation, any allocator).  Before a bank's fused pass first writes a
# buffer from a given source, a PAIR_PROBE_STEPS-round pass and one ring round
# are timed on that (source, destination) pair; when the pass is slower than
# PAIR_RATIO x the round, the destination -- whose contents the pass is about
# to overwrite -- is replaced by a fresh allocation (up to PAIR_TRIES times,
# keeping the fastest).  The probe's step count is fixed at the one PAIR_RATIO
# was calibrated on (eps = 5, 8192 x 2^20): the slowness belongs to the pair of
# allocations, not to the step count, and a longer pass carries more
# arithmetic per byte.  At most ONE candidate besides the
# current best is held at a time (the loser is dropped before the next
# allocation); a candidate at an address already probed (torch's caching
# allocator hands a dropped block straight back) ends the search; buffers the
# caller adopted are not replaced unless adopted with replaceable=True.
# DOL_BANK_PAIR_PROBE=0 turns it off.
PAIR_PROBE_MIN_BYTES = 4 << 30
PAIR_RATIO = 1.12
PAIR_TRIES = 3
PAIR_PROBE_STEPS = 5


def _pair_probe_ms(x: torch.Tensor, y: torch.Tensor, plan, steps: int, P: int, reps: int = 2) -> Tuple[float, float]:
    """(ms of the fused `steps`-round pass x -> y, ms of one ring round x -> y) on
    the current stream; y is overwritten, x is only read."""
    def one_pass():
        ops.mix_ring_steps(x, y, plan.w_prev, plan.w_next, steps, P=P, n_rows=plan.n_rows, variant=3)

    def one_round():
        ops.mix_ring(x, y, plan.w_prev, plan.w_next, P=P, n_rows=plan.n_rows)
    t = ops._time_each(lambda f: f(), [one_pass, one_round], reps, device=x.device)
    return t[one_pass], t[one_round]


class AgentBank:
    def __init__(self, n_agents: int, layout_or_P, device, ld: Optional[int] = None):
        self.device = torch.device(device)
        # (source ptr, destination ptr) pairs whose fused-pass rate was checked; the probe log
        self._pair_checked: set = set()
        self.pair_probes: List[dict] = []
        self._pair_timer = _pair_probe_ms  # tests inject a timer
        self._pinned: set = set()  # names of adopted buffers the destination check must not replace
        if isinstance(layout_or_P, int):
            self.layout: Layout = [("w", (int(layout_or_P),))]
        else:
            self.layout = [(k, tuple(s)) for k, s in layout_or_P]
        self.n = int(n_agents)
        self.P = layout_size(self.layout)
        self.ld = int(ld) if ld is not None else row_stride(self.P)
        self._buf: Dict[str, torch.Tensor] = {}
        self._modules: List[Optional[torch.nn.Module]] = [None] * self.n
        # per row: has the SGD momentum buffer been written yet?  torch.optim.SGD
        # takes buf = g on a parameter's first step and buf*mu + g after; the
        # flag is saved with the checkpoint so a resumed run keeps its momentum.
        self.mom_started: List[bool] = [False] * self.n
        self.offsets = []
        off = 0
        for k, shape in self.layout:
            c = 1
            for s in shape:
                c *= int(s)
            self.offsets.append((k, off, c, shape))
            off += c

    # ------------------------------------------------------------------ buffers
    def buffer(self, name: str, zero: bool = False) -> torch.Tensor:
        t = self._buf.get(name)
        if t is None:
            t = device_matrix(self.n, self.ld, self.device, zero=zero)
            self._buf[name] = t
        return t

    def adopt(self, name: str, t: torch.Tensor, replaceable: bool = False) -> None:
        """Use an existing [N, ld] fp32 device matrix as buffer `name` (e.g. a
        bank over state that was allocated elsewhere).  replaceable: the fused
        ring pass's destination check may swap it for a fresh allocation (its
        contents are dead when replaced); otherwise it stays the caller's."""
        if (t.device != self.device or t.dtype != torch.float32 or tuple(t.shape) != (self.n, self.ld)
                or t.stride(1) != 1 or (self.n > 1 and t.stride(0) != self.ld)):
            raise ValueError(f"adopt({name!r}): expected a float32 [{self.n}, {self.ld}] row-major matrix on "
                             f"{self.device}")
        self._buf[name] = t
        if replaceable:
            self._pinned.discard(name)
        else:
            self._pinned.add(name)
        if name == "x":
            self.rebind_all()

    @property
    def x(self) -> torch.Tensor:
        return self.buffer("x")

    def has(self, name: str) -> bool:
        return name in self._buf

    def rows(self, name: str = "x") -> torch.Tensor:
        """[N, P] view (without the alignment padding)."""
        return self.buffer(name)[:, : self.P]

    def row_views(self, i: int, name: str = "x") -> Dict[str, torch.Tensor]:
        r = self.buffer(name)[i]
        return {k: r[o:o + c].view(shape) for k, o, c, shape in self.offsets}

    # ------------------------------------------------------------------ modules
    def load_module(self, i: int, module: torch.nn.Module, name: str = "x") -> None:
        sd = module.state_dict()
        r = self.buffer(name)[i]
        with torch.no_grad():
            for k, o, c, _ in self.offsets:
                r[o:o + c].copy_(sd[k].reshape(-1))

    def bind(self, i: int, module: torch.nn.Module, grads: bool = True) -> None:
        """Make module's parameters (and .grad) views into row i of x (grad)."""
        self._modules[i] = module
        self._rebind(i, grads)

    def _rebind(self, i: int, grads: bool = True) -> None:
        module = self._modules[i]
        if module is None:
            return
        xv = self.row_views(i, "x")
        gv = self.row_views(i, "grad") if grads else None
        params = dict(module.named_parameters())
        for k, t in module.state_dict(keep_vars=True).items():
            if k in params:
                p = params[k]
                p.data = xv[k]
                if gv is not None:
                    p.grad = gv[k]
            else:  # buffers (none in the reference models) are copied, not bound
                with torch.no_grad():
                    xv[k].copy_(t)

    def rebind_all(self) -> None:
        for i in range(self.n):
            if self._modules[i] is not None:
                self._rebind(i, self.has("grad"))

    def state_dict(self, i: int, name: str = "x", clone: bool = True) -> Dict[str, torch.Tensor]:
        v = self.row_views(i, name)
        return {k: t.clone() for k, t in v.items()} if clone else v

    # ------------------------------------------------------------------ mixing
    def swap(self, a: str = "x", b: str = "y") -> None:
        self._buf[a], self._buf[b] = self._buf[b], self._buf[a]
        pa, pb = a in self._pinned, b in self._pinned  # pinning follows the tensor
        self._pinned.discard(a)
        self._pinned.discard(b)
        if pa:
            self._pinned.add(b)
        if pb:
            self._pinned.add(a)
        if a == "x" or b == "x":
            self.rebind_all()

    def mix(self, plan, steps: int = 1, fuse: bool = True) -> None:
        """X <- W X, `steps` times (synchronous / Jacobi rounds).  With `fuse`,
        ring plans apply up to 8 rounds per HBM pass (temporal blocking,
        bit-identical to single rounds)."""
        y = self.buffer("y")
        done = 0
        while done < steps:
            if fuse:
                if steps - done > 1:
                    y = self._check_destination(plan, min(steps - done, plan.MAX_FUSED_STEPS))
                done += plan.apply_steps(self.buffer("x"), y, steps - done, P=self.P)
            else:
                plan.apply(self.buffer("x"), y, P=self.P)
                done += 1
            self.swap_xy_nobind()
            y = self._buf["y"]
        self.rebind_all()

    def swap_xy_nobind(self) -> None:
        self._buf["x"], self._buf["y"] = self._buf["y"], self._buf["x"]
        px, py = "x" in self._pinned, "y" in self._pinned
        self._pinned.difference_update(("x", "y"))
        self._pinned.update(n for n, p in (("y", px), ("x", py)) if p)

    def _check_destination(self, plan, steps: int) -> torch.Tensor:
        """The buffer the next fused ring pass writes ("y"), replaced first if
        its pair with "x" is one of the slow ones (see PAIR_RATIO above).  Only
        for ring plans on large CUDA banks, once per (x, y) pair; y's contents
        are dead (the pass overwrites them) and x is only read."""
        y = self.buffer("y")
        x = self.buffer("x")
        if (getattr(plan, "kind", None) != "ring" or self.device.type != "cuda" or self.P % 4
                or self.n * self.ld * 4 < PAIR_PROBE_MIN_BYTES or os.environ.get("DOL_BANK_PAIR_PROBE", "1") == "0"):
            return y
        if (x.data_ptr(), y.data_ptr()) in self._pair_checked:
            return y
        with torch.cuda.device(self.device):
            if torch.cuda.is_current_stream_capturing():  # no timing inside a graph capture
                return y
        replace = "y" not in self._pinned
        best = (float("inf"), y)
        probed = set()
        del self._buf["y"]  # held in y / best only: a losing candidate is dropped before the next allocation
        try:
            for attempt in range(PAIR_TRIES):
                probed.add(y.data_ptr())
                pass_ms, round_ms = self._pair_timer(x, y, plan, PAIR_PROBE_STEPS, self.P)
                self.pair_probes.append({"attempt": attempt, "steps": PAIR_PROBE_STEPS, "pass_ms": pass_ms,
                                         "round_ms": round_ms,
                                         "ratio": pass_ms / round_ms if round_ms > 0 else float("inf")})
                if pass_ms < best[0]:
                    best = (pass_ms, y)
                if pass_ms <= PAIR_RATIO * round_ms or attempt + 1 == PAIR_TRIES:
                    break
                if not replace:
                    self.pair_probes[-1]["kept_adopted"] = True
                    break
                y = None  # the loser (unless it is the best) goes before the next allocation
                try:  # a fresh allocation for the destination; no memory for one: keep the best so far
                    y = device_matrix(self.n, self.ld, self.device)
                except RuntimeError:  # torch's OOM and DolNativeError alike
                    self.pair_probes[-1]["realloc_failed"] = True
                    break
                if y.data_ptr() in probed:  # the allocator handed back a block already measured
                    self.pair_probes[-1]["same_block"] = True
                    y = None
                    break
        finally:
            y = best[1]
            self._buf["y"] = y
        self._pair_checked.add((x.data_ptr(), y.data_ptr()))
        return y

    # ------------------------------------------------------------------ primal / dual
    def local_step(self, lr: float, momentum: float, first_step: bool, theta: Optional[torch.Tensor] = None,
                   rho: float = 0.0, admm: bool = False, write_grad: bool = True,
                   agents: Optional[slice] = None) -> None:
        """Fused gradient term + momentum SGD on rows `agents` (default all)."""
        sl = agents if agents is not None else slice(0, self.n)
        x, g = self.buffer("x")[sl], self.buffer("grad")[sl]
        buf = self.buffer("mom")[sl] if momentum != 0.0 else None
        alpha = self.buffer("alpha", zero=True)[sl] if admm else None
        ops.prox_admm_sgd(x, g, buf=buf, theta=theta, alpha=alpha, rho=rho, lr=lr, momentum=momentum,
                          first_step=first_step, write_grad=write_grad, P=self.P)
        if momentum != 0.0:
            self.mark_momentum_started(sl)

    def mark_momentum_started(self, agents: slice) -> None:
        """Record that rows `agents` have taken a momentum step (the batched
        paths bypass the per-row optimizer, so they set the flags here)."""
        a, b, st = agents.indices(self.n)
        if st == 1 and not all(self.mom_started[a:b]):
            self.mom_started[a:b] = [True] * max(0, b - a)
        elif st != 1:
            for i in range(a, b, st):
                self.mom_started[i] = True

    def dual_update(self, theta: torch.Tensor, rho: float, resid_sq: Optional[torch.Tensor] = None,
                    agents: Optional[slice] = None) -> None:
        sl = agents if agents is not None else slice(0, self.n)
        ops.admm_dual(self.buffer("alpha", zero=True)[sl], self.buffer("x")[sl], theta, rho,
                      resid_sq=resid_sq, P=self.P)

    def ordered_mean(self, order: Sequence[int], out: Optional[torch.Tensor] = None,
                     name: str = "x") -> torch.Tensor:
        idx = torch.as_tensor(list(order), dtype=torch.int32, device=self.device)
        return ops.ordered_mean(self.buffer(name), idx, out=out, P=self.P)

    # ------------------------------------------------------------------ checkpoint / resume
    def save(self, path: str, names: Iterable[str] = ("x", "mom", "alpha")) -> None:
        """Write the stacked state (unpadded [N, P] per buffer) with safetensors
        (no pickles).  The reference keeps no model checkpoints."""
        from safetensors.torch import save_file
        tensors = {n: self.rows(n).contiguous().cpu() for n in names if self.has(n)}
        meta = {"P": str(self.P), "n": str(self.n), "layout": repr(self.layout),
                "mom_started": "".join("1" if f else "0" for f in self.mom_started)}
        save_file(tensors, path, metadata=meta)

    def load(self, path: str) -> None:
        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
            if int(meta.get("P", self.P)) != self.P or int(meta.get("n", self.n)) != self.n:
                raise ValueError(f"checkpoint is [{meta.get('n')}, {meta.get('P')}], bank is [{self.n}, {self.P}]")
            for name in f.keys():
                self.buffer(name, zero=True)[:, : self.P].copy_(f.get_tensor(name))
            flags = meta.get("mom_started")
            if flags is not None and len(flags) == self.n:
                self.mom_started = [c == "1" for c in flags]
            elif "mom" in f.keys():  # older checkpoint: a saved momentum buffer is a started one
                self.mom_started = [True] * self.n
        self.rebind_all()

    def unflatten(self, vec: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {k: vec[o:o + c].view(shape) for k, o, c, shape in self.offsets}

    def flatten(self, sd: Dict[str, torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(self.P, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for k, o, c, _ in self.offsets:
                out[o:o + c].copy_(sd[k].reshape(-1))
        return out
