"""ctypes binding of libdol_hip.so (the C-ABI declared in include/dol_hip.h).

The library is built in-tree (csrc/Makefile -> dolhip/libdol_hip.so) and is
the only compute path: there is no CPU fallback.  If the library is missing
every op raises DolNativeError.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(_HERE, "libdol_hip.so")
CSRC = os.path.join(PKG_ROOT, "csrc")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "dol_hip.h")


class DolNativeError(RuntimeError):
    """Raised when the HIP library is missing or a C-ABI call fails."""


_c_f32p = ctypes.c_void_p  # device pointers travel as integers
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f32 = ctypes.c_float
_ptr = ctypes.c_void_p

# name -> argtypes (restype int unless listed in _RESTYPES)
SIGNATURES = {
    "dol_version": [],
    "dol_last_error": [],
    "dol_mix_csr_f32": [_ptr, _i64, _i32, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr],
    "dol_mix_ring_steps_f32": [_ptr, _i64, _ptr, _i64, _i32, _i64, _i32, _ptr, _ptr, _ptr],
    "dol_mix_ring_steps_ex_f32": [_ptr, _i64, _ptr, _i64, _i32, _i64, _i32, _ptr, _ptr, _i32, _ptr],
    "dol_mix_dense_f32": [_ptr, _i64, _ptr, _i64, _ptr, _i64, _i32, _i32, _i64, _ptr],
    "dol_mix_ring_f32": [_ptr, _i64, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr, _ptr],
    "dol_mix_ring_edges_f32": [_ptr, _i64, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr, _ptr],
    "dol_dgd_ring_edges_f32": [_ptr, _i64, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr, _ptr, _i64, _ptr, _i64,
                               _i32, _i32, _f32, _f32, ctypes.c_int, _ptr],
    "dol_prox_admm_sgd_f32": [_ptr, _i64, _ptr, _i64, _ptr, _i64, _ptr, _ptr, _i64, _f32, _f32, _f32,
                              ctypes.c_int, ctypes.c_int, _i32, _i64, _ptr],
    "dol_admm_step_dual_f32": [_ptr, _i64, _ptr, _i64, _ptr, _i64, _ptr, _ptr, _i64, _f32, _f32, _f32,
                               ctypes.c_int, ctypes.c_int, _i32, _i64, _ptr],
    "dol_prox_grad_f32": [_ptr, _i64, _ptr, _i64, _ptr, _ptr, _i64, _f32, _i32, _i64, _ptr],
    "dol_admm_dual_f32": [_ptr, _i64, _ptr, _i64, _ptr, _f32, _i32, _i64, _ptr, _ptr, _ptr],
    "dol_admm_dual_workspace_bytes": [_i32, _i64],
    "dol_admm_ls_round_f32": [_ptr, _i64, _ptr, _i64, _ptr, _i64, _ptr, _i64, _ptr, _ptr, _ptr, _i32, _i64, _f32, _f32,
                              _f32, _i32, _ptr, _ptr, _ptr, _ptr],
    "dol_admm_ls_round_workspace_bytes": [_i32, _i64],
    "dol_admm_ls_round_mean_f32": [_ptr, _i64, _ptr, _i64, _ptr, _i64, _ptr, _i64, _ptr, _ptr, _ptr, _i32, _i64, _f32,
                                   _f32, _f32, _i32, _ptr, _f32, _ptr, _ptr, _ptr],
    "dol_admm_ls_round_mean_workspace_bytes": [_i64],
    "dol_ordered_mean_f32": [_ptr, _i64, _ptr, _i32, _i64, _ptr, _ptr],
    "dol_ordered_sum_f32": [_ptr, _i64, _ptr, _i32, _i64, _ptr, _ptr, _f32, _ptr],
    "dol_stream_copy_f32": [_ptr, _ptr, _i64, _ptr],
    "dol_stream_copy_rows_f32": [_ptr, _i64, _ptr, _i64, _i32, _i64, _ptr],
    "dol_mlp_step_f32": [_ptr, _i64, _ptr, _i64, _ptr, _i64, _ptr, _ptr, _i64, _ptr, _i64, _i64, _ptr, _i64, _ptr,
                         _i32, _i32, _i32, _i32, _i32, _f32, _f32, _f32, ctypes.c_int, ctypes.c_int, _ptr, _ptr],
    "dol_mlp_step_workspace_bytes": [_i32, _i32, _i32],
    "dol_dgd_ring_f32": [_ptr, _i64, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr, _ptr, _i64, _ptr, _i64, _i32, _i32,
                         _f32, _f32, ctypes.c_int, _ptr],
    "dol_dgd_csr_f32": [_ptr, _i64, _i32, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr, _i64, _ptr, _i64, _i32, _i32,
                        _f32, _f32, ctypes.c_int, _ptr],
    "dol_mlp_step_lds_bytes": [_i32, _i32, _i32],
    "dol_mix_dense_split3_f32": [_ptr, _i64, _ptr, _i64, _ptr, _i64, _i32, _i32, _i64, _ptr, _i64, ctypes.c_int, _ptr],
    "dol_mix_dense_split3_workspace_bytes": [_i32, _i32, _i64, ctypes.c_int],
    "dol_er_stochastic_f32": [_ptr, _i64, _i32, _f32, ctypes.c_uint64, _ptr],
    "dol_mix_csr_pm_f32": [_ptr, _i64, _i32, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr],
    "dol_mix_csr_pm_ex_f32": [_ptr, _i64, _i32, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _i32, _ptr],
    "dol_pm_set_stage_order": [_i32],
    "dol_ring_steps_set_variant": [_i32],
    "dol_dgd_csr_pm_f32": [_ptr, _i64, _i32, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr, _i64, _ptr, _i64, _i32,
                           _i32, _f32, _f32, ctypes.c_int, _ptr],
    "dol_dgd_csr_pm_ex_f32": [_ptr, _i64, _i32, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr, _ptr, _i64, _ptr, _i64,
                              _i32, _i32, _f32, _f32, ctypes.c_int, _i32, _ptr],
    "dol_transpose_f32": [_ptr, _i64, _ptr, _i64, _i64, _i64, _ptr],
    "dol_csr_slab_nk": [_i32],
    "dol_csr_slab_hdr_len": [_i32, _i32],
    "dol_csr_slab_ent_len": [_i64, _i32, _i32],
    "dol_mix_csr_slab_f32": [_ptr, _i64, _i32, _ptr, _i64, _i32, _i64, _ptr, _ptr, _ptr],
    "dol_csr_slab_pack": [_ptr, _ptr, _ptr, _i32, _i32, _i32, _ptr, _ptr, _ptr],
    "dol_slab_set_variant": [_i32],
    "dol_dense_to_csr_f32": [_ptr, _i64, _i32, _i32, _ptr, _ptr, _ptr, _i64, _ptr],
    "dol_bank_alloc": [_i64, _ptr, _ptr],  # (bytes, void** out, int64_t* out): addresses of host words
    "dol_bank_free": [_ptr, _i64],
    "dol_bank_retired_bytes": [],
    "dol_bank_retired_blocks": [],
    "dol_bank_retired_cap_bytes": [],
}
_RESTYPES = {"dol_last_error": ctypes.c_char_p, "dol_admm_dual_workspace_bytes": ctypes.c_int64,
             "dol_admm_ls_round_workspace_bytes": ctypes.c_int64,
             "dol_admm_ls_round_mean_workspace_bytes": ctypes.c_int64,
             "dol_mlp_step_lds_bytes": ctypes.c_int64, "dol_mlp_step_workspace_bytes": ctypes.c_int64,
             "dol_mix_dense_split3_workspace_bytes": ctypes.c_int64, "dol_csr_slab_hdr_len": ctypes.c_int64,
             "dol_csr_slab_ent_len": ctypes.c_int64, "dol_bank_retired_bytes": ctypes.c_int64,
             "dol_bank_retired_blocks": ctypes.c_int64, "dol_bank_retired_cap_bytes": ctypes.c_int64}

_lib = None


def build(force: bool = False) -> str:
    """Compile libdol_hip.so for gfx950 with hipcc (works without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", CSRC], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DolNativeError(
                f"{LIB_PATH} is missing: build it with `make -C {CSRC}` (or __graft_entry__.build()); "
                "dolhip has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
    return _lib


_TRACE = os.environ.get("DOL_TRACE", "") not in ("", "0")


def call(name: str, *args) -> None:
    if _TRACE:  # roctx range per C-ABI call (visible in rocprofv3 --marker-trace)
        import torch
        torch.cuda.nvtx.range_push(name)
        try:
            rc = getattr(lib(), name)(*args)
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().dol_last_error().decode(errors="replace")
        raise DolNativeError(f"{name} returned {rc}: {msg}")
