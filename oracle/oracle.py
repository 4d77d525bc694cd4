"""ctypes front-end of the CPU ORACLE (oracle/ldpc_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module — as the checker
and as the CPU comparator, never as a product code path.  See ldpc_oracle.c for the reference citations
(bp/bp.py:43-51, bp/bp_vc.py:16-27, bp/bp_cv.py:22-50, ofdm/ofdm_functions.py:161).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ldpc-sims_amd"))
from ldpc_amd.codes import Graph  # noqa: E402

_lib = None


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "ldpc_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        vp = ctypes.c_void_p
        garg = [ctypes.c_int, ctypes.c_int, ctypes.c_int, i32p, i32p, i32p, i32p]
        L.oracle_sp_f32.argtypes = garg + [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_float, vp, vp, vp, vp,
                                           ctypes.c_int, vp] + [vp] * 4 + [ctypes.c_int]
        L.oracle_sp_f64.argtypes = garg + [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_double, vp, vp, vp] + [vp] * 4
        L.oracle_sp_f64_pmax.argtypes = garg + [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                                vp, vp, vp] + [vp] * 4
        L.oracle_ms_f32.argtypes = garg + [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_int, vp, vp, vp, vp]
        L.oracle_qms.argtypes = garg + [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, vp, vp, vp]
        for f in (L.oracle_sp_f32, L.oracle_sp_f64, L.oracle_sp_f64_pmax, L.oracle_ms_f32, L.oracle_qms):
            f.restype = ctypes.c_int
        L.oracle_num_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _graph(H_or_graph) -> Graph:
    return H_or_graph if isinstance(H_or_graph, Graph) else Graph.from_H(H_or_graph)


def _gargs(g: Graph):
    return (g.m, g.n, g.E, g.row_ptr, g.col_idx, g.var_ptr, g.var_edges)


def _weights(weights, dtype):
    """weights: None or dict(vn=[iters][W], llr=[iters][n], fin=[E], fin_llr=[n]) in the compact layout of
    ldpc_oracle.c (any key may be missing = all ones).  Returns the 4 pointers and the arrays to keep alive."""
    if not weights:
        return [None] * 4, []
    arrs = [None if weights.get(k) is None else np.ascontiguousarray(weights[k], dtype=dtype)
            for k in ("vn", "llr", "fin", "fin_llr")]
    return [_ptr(a) for a in arrs], arrs


def sp_f32(H, llr, iters, clamp, trace=False, early_stop=False, weights=None, stable=False):
    """tanh sum-product in fp32. Returns dict(p1, z, bits, iters_used[, trace[iters,B,E]]).

    stable=False: the reference's own fp32 operations (bp_vc.py:27, bp_cv.py:38-50); stable=True: the same
    function in the (D, S) form the GPU kernels compute (ldpc_oracle.c cn_stable_f32)."""
    g = _graph(H)
    wp, _keep = _weights(weights, np.float32)
    llr = np.ascontiguousarray(llr, dtype=np.float32)
    B = llr.shape[0]
    p1 = np.empty((B, g.n), np.float32)
    z = np.empty((B, g.n), np.float32)
    bits = np.empty((B, g.n), np.uint8)
    tr = np.empty((iters, B, g.E), np.float32) if trace else None
    used = np.empty(B, np.int32)
    lib().oracle_sp_f32(*_gargs(g), _ptr(llr), B, int(iters), float(clamp), _ptr(p1), _ptr(z), _ptr(bits), _ptr(tr),
                        int(bool(early_stop)), _ptr(used), *wp, int(bool(stable)))
    out = dict(p1=p1, z=z, bits=bits, iters_used=used)
    if trace:
        out["trace"] = tr
    return out


def sp_f64(H, llr, iters, clamp, weights=None, ceiling="f64"):
    """tanh sum-product in fp64.  ceiling="f64": the reference's .double() module (p clamped to 1-1e-7, messages
    <= log(19999999) = 16.8112); ceiling="f32": the same fp64 arithmetic with the fp32 module's bound
    (float)(1-1e-7) (messages <= log(16777215) = 16.6355, bp_cv.py:44-47 as torch evaluates it in fp32)."""
    g = _graph(H)
    wp, _keep = _weights(weights, np.float64)
    llr = np.ascontiguousarray(llr, dtype=np.float64)
    B = llr.shape[0]
    p1 = np.empty((B, g.n), np.float64)
    z = np.empty((B, g.n), np.float64)
    bits = np.empty((B, g.n), np.uint8)
    pmax = {"f64": 1.0 - 1e-7, "f32": float(np.float32(1.0 - 1e-7))}[ceiling]
    lib().oracle_sp_f64_pmax(*_gargs(g), _ptr(llr), B, int(iters), float(clamp), pmax, _ptr(p1), _ptr(z), _ptr(bits),
                             *wp)
    return dict(p1=p1, z=z, bits=bits)


def ms_f32(H, llr, iters, clamp, alpha=1.0, beta=0.0, early_stop=False):
    g = _graph(H)
    llr = np.ascontiguousarray(llr, dtype=np.float32)
    B = llr.shape[0]
    p1 = np.empty((B, g.n), np.float32)
    z = np.empty((B, g.n), np.float32)
    bits = np.empty((B, g.n), np.uint8)
    used = np.empty(B, np.int32)
    lib().oracle_ms_f32(*_gargs(g), _ptr(llr), B, int(iters), float(clamp), float(alpha), float(beta),
                        int(bool(early_stop)), _ptr(p1), _ptr(z), _ptr(bits), _ptr(used))
    return dict(p1=p1, z=z, bits=bits, iters_used=used)


def qms(H, qllr, iters, qmax=15, app_max=127, beta=0, early_stop=False):
    g = _graph(H)
    qllr = np.ascontiguousarray(qllr, dtype=np.int8)
    B = qllr.shape[0]
    app = np.empty((B, g.n), np.int16)
    bits = np.empty((B, g.n), np.uint8)
    used = np.empty(B, np.int32)
    lib().oracle_qms(*_gargs(g), _ptr(qllr), B, int(iters), int(qmax), int(app_max), int(beta),
                     int(bool(early_stop)), _ptr(app), _ptr(bits), _ptr(used))
    return dict(app=app, bits=bits, iters_used=used)


def num_threads() -> int:
    return int(lib().oracle_num_threads())
