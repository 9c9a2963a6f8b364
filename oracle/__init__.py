"""CPU oracle for the consensus / primal-dual hot path — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this package, and only as the checker (or the timed CPU baseline); the product
(`dolhip`) never imports it and has no CPU fallback.

Two restatements live here:
  * liboracle.so (dol_oracle.c): scalar C, the reference's exact rounding
    sequence; pinned by tests/golden/*.npz generated from the reference itself.
  * ref_cpu.py: the reference-structured torch-CPU round (per-agent dict loop
    with the O(N^2) neighbour scan), used as bench.py's CPU baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


def build():
    """Compile liboracle.so (gcc) in place."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_mix_csr_f32.argtypes = [_f32p, _i64, _f32p, _i64, _i32, _i64, _i32p, _i32p, _f32p]
        L.oracle_mix_ring_f32.argtypes = [_f32p, _i64, _f32p, _i64, _i32, _i64, _f32p, _f32p, _f32p, _f32p]
        L.oracle_prox_admm_sgd_f32.argtypes = [_f32p, _i64, _f32p, _i64, _f32p, _i64, _f32p, _f32p, _i64,
                                               ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                               ctypes.c_int, ctypes.c_int, _i32, _i64]
        L.oracle_prox_grad_f32.argtypes = [_f32p, _i64, _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_float, _i32, _i64]
        L.oracle_prox_grad_f32.restype = None
        L.oracle_admm_dual_f32.argtypes = [_f32p, _i64, _f32p, _i64, _f32p, ctypes.c_float, _i32, _i64, _f64p]
        L.oracle_ordered_mean_f32.argtypes = [_f32p, _i64, _i32p, _i32, _i64, _f32p]
        L.oracle_ordered_sum_f32.argtypes = [_f32p, _i64, _i32p, _i32, _i64, _f32p, _f32p, ctypes.c_float]
        L.oracle_dgd_local_f32.argtypes = [_f32p, _i64, _f32p, _i64, _f32p, _i64, _i32, _i64, _i32, _i32,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.oracle_dgd_local_f32.restype = None
        L.oracle_admm_ls_round_f32.argtypes = [_f32p, _i64, _f32p, _i64, _f32p, _i64, _f32p, _i64, _f32p, _i32p, _i32p,
                                               _i32, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_float, _i32,
                                               _f64p, _f64p]
        L.oracle_admm_ls_round_f32.restype = None
        for f in (L.oracle_mix_csr_f32, L.oracle_mix_ring_f32, L.oracle_prox_admm_sgd_f32,
                  L.oracle_admm_dual_f32, L.oracle_ordered_mean_f32, L.oracle_ordered_sum_f32):
            f.restype = None
        _lib = L
    return _lib


def _p(a, t=_f32p):
    return None if a is None else a.ctypes.data_as(t)


def _f32c(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


def mix_csr(X, rowptr, col, val, n_rows=None):
    """Y = W X for a CSR W (ascending columns, W_ij > 0 kept)."""
    X = _f32c(X)
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    n = len(rowptr) - 1 if n_rows is None else n_rows
    P = X.shape[1]
    Y = np.empty((n, P), np.float32)
    lib().oracle_mix_csr_f32(_p(X), P, _p(Y), P, n, P, _p(rowptr, _i32p), _p(col, _i32p), _p(val))
    return Y


def mix_ring(X, w_prev, w_next, halo_prev=None, halo_next=None):
    X = _f32c(X)
    n, P = X.shape
    Y = np.empty_like(X)
    hp = None if halo_prev is None else _f32c(halo_prev)
    hn = None if halo_next is None else _f32c(halo_next)
    lib().oracle_mix_ring_f32(_p(X), P, _p(Y), P, n, P, _p(hp), _p(hn), _p(_f32c(w_prev)), _p(_f32c(w_next)))
    return Y


def prox_admm_sgd(w, buf, g, theta, alpha, rho, lr, momentum, first_step, write_grad=True):
    """In-place on copies; returns (w', buf', g')."""
    w = _f32c(w).copy()
    g = _f32c(g).copy()
    n, P = w.shape
    buf = None if buf is None else _f32c(buf).copy()
    th = None if theta is None else _f32c(theta)
    al = None if alpha is None else _f32c(alpha)
    lib().oracle_prox_admm_sgd_f32(_p(w), P, _p(buf), P, _p(g), P, _p(th), _p(al), P,
                                   rho, lr, momentum, int(first_step), int(write_grad), n, P)
    return w, buf, g


def prox_grad(g, w, theta, alpha, rho):
    g = _f32c(g).copy()
    w = _f32c(w)
    n, P = g.shape
    al = None if alpha is None else _f32c(alpha)
    lib().oracle_prox_grad_f32(_p(g), P, _p(w), P, _p(_f32c(theta)), _p(al), P, rho, n, P)
    return g


def admm_dual(alpha, w, theta, rho):
    a = _f32c(alpha).copy()
    w = _f32c(w)
    n, P = a.shape
    r = np.zeros(n, np.float64)
    lib().oracle_admm_dual_f32(_p(a), P, _p(w), P, _p(_f32c(theta)), rho, n, P, _p(r, _f64p))
    return a, r


def ordered_mean(W, order):
    W = _f32c(W)
    order = np.ascontiguousarray(order, np.int32)
    P = W.shape[1]
    out = np.empty(P, np.float32)
    lib().oracle_ordered_mean_f32(_p(W), P, _p(order, _i32p), len(order), P, _p(out))
    return out


def ordered_sum(W, order, acc_in=None, scale=1.0):
    W = _f32c(W)
    order = np.ascontiguousarray(order, np.int32)
    P = W.shape[1]
    out = np.empty(P, np.float32)
    ai = None if acc_in is None else _f32c(acc_in)
    lib().oracle_ordered_sum_f32(_p(W), P, _p(order, _i32p), len(order), P, _p(ai), _p(out), scale)
    return out


OBJECTIVES = {"least_squares": 0, "logistic": 1}


def dgd_local(Y, T, M, objective, steps, lr, momentum, first_step):
    """Local steps after the mix (config 3); returns (Y', M') (M' None without momentum)."""
    Y = _f32c(Y).copy()
    T = _f32c(T)
    n, P = Y.shape
    M = None if M is None else _f32c(M).copy()
    lib().oracle_dgd_local_f32(_p(Y), P, _p(T), P, _p(M), P, n, P, OBJECTIVES[objective], int(steps), lr,
                               momentum, int(first_step))
    return Y, M


def admm_ls_round(w, buf, alpha, target, theta, agents, first, rho, lr, momentum, local_steps):
    """One FedADMM least-squares client round for the sampled rows `agents`
    (config 4); returns (w', buf', alpha', resid_sq[m], alpha_sq[m]) on copies."""
    w = _f32c(w).copy()
    alpha = _f32c(alpha).copy()
    n, P = w.shape
    buf = None if buf is None else _f32c(buf).copy()
    T = _f32c(target)
    ag = np.ascontiguousarray(agents, np.int32)
    m = len(ag)
    fs = None if first is None else np.ascontiguousarray(first, np.int32)
    rw = np.zeros(m, np.float64)
    ra = np.zeros(m, np.float64)
    lib().oracle_admm_ls_round_f32(_p(w), P, _p(buf), P, _p(alpha), P, _p(T), P, _p(_f32c(theta)), _p(ag, _i32p),
                                   _p(fs, _i32p), m, P, rho, lr, momentum, int(local_steps), _p(rw, _f64p),
                                   _p(ra, _f64p))
    return w, buf, alpha, rw, ra


def bits_equal(a, b):
    """Bitwise equality, treating any two NaNs as equal (payloads may differ)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all((a.view(np.uint32) == b.view(np.uint32)) | both_nan))
