"""ctypes wrapper of oracle/liboracle.so -- the CPU parity ORACLE.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, and only as the checker / reported baseline.
The product (sparsematrixmultiplicationmpi_amd, libsmfv.so) never imports it.
See oracle/smfv_oracle.c for the reference file:line each function follows.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, byref, c_double, c_int, c_int64

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_DRIVER = os.path.join(HERE, "_ref", "ref_driver")

VARIANTS = ("sequential", "rowwise", "columnwise", "nonzero")


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def _load():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    P, PD = POINTER(c_int), POINTER(c_double)
    for name in ("oracle_spmm_rowwise", "oracle_spmm_columnwise", "oracle_spmm_nonzero"):
        getattr(lib, name).argtypes = [c_int, c_int, P, P, PD, PD, c_int, PD]
        getattr(lib, name).restype = c_int
    lib.oracle_spmm_sequential.argtypes = [c_int, P, P, PD, PD, c_int, PD]
    lib.oracle_spmm_sequential.restype = c_int
    lib.oracle_partition_rows.argtypes = [c_int, c_int, c_int, P, P]
    lib.oracle_partition_cols.argtypes = [c_int, c_int, c_int, P, P]
    lib.oracle_partition_nnz.argtypes = [c_int64, c_int, c_int, POINTER(c_int64), POINTER(c_int64)]
    lib.oracle_max_abs_diff.argtypes = [PD, PD, c_int64]
    lib.oracle_max_abs_diff.restype = c_double
    lib.oracle_fatvector_rand.argtypes = [c_int, c_int, PD]
    lib.oracle_mtx_read.argtypes = [ctypes.c_char_p, P, P, POINTER(c_int64), POINTER(P), POINTER(P),
                                    POINTER(PD)]
    lib.oracle_mtx_read.restype = c_int
    lib.oracle_free.argtypes = [ctypes.c_void_p]
    return lib


_lib = _load()


def _ip(a):
    return a.ctypes.data_as(POINTER(c_int))


def _dp(a):
    return a.ctypes.data_as(POINTER(c_double))


def spmm(variant: str, row_ptr, col_idx, values, X, p: int = 1) -> np.ndarray:
    """Y = A*X by the restated reference algorithm `variant` with p simulated ranks."""
    rp = np.ascontiguousarray(row_ptr, dtype=np.int32)
    ci = np.ascontiguousarray(col_idx, dtype=np.int32)
    va = np.ascontiguousarray(values, dtype=np.float64)
    X = np.ascontiguousarray(X, dtype=np.float64)
    m = len(rp) - 1
    K = X.shape[1]
    Y = np.empty((m, K), dtype=np.float64)
    if variant == "sequential":
        rc = _lib.oracle_spmm_sequential(m, _ip(rp), _ip(ci), _dp(va), _dp(X), K, _dp(Y))
    else:
        fn = getattr(_lib, f"oracle_spmm_{variant}")
        rc = fn(p, m, _ip(rp), _ip(ci), _dp(va), _dp(X), K, _dp(Y))
    if rc != 0:
        raise RuntimeError(f"oracle {variant} failed: {rc}")
    return Y


def partition_rows(m, p, r):
    s, e = c_int(), c_int()
    _lib.oracle_partition_rows(m, p, r, byref(s), byref(e))
    return s.value, e.value


def partition_cols(K, p, r):
    s, e = c_int(), c_int()
    _lib.oracle_partition_cols(K, p, r, byref(s), byref(e))
    return s.value, e.value


def partition_nnz(nnz, p, r):
    s, e = c_int64(), c_int64()
    _lib.oracle_partition_nnz(nnz, p, r, byref(s), byref(e))
    return s.value, e.value


def fatvector_rand(n: int, K: int) -> np.ndarray:
    X = np.empty((n, K), dtype=np.float64)
    _lib.oracle_fatvector_rand(n, K, _dp(X))
    return X


def mtx_read(path: str):
    """(m, n, row_ptr, col_idx, values) or raises ValueError."""
    m, n, nnz = c_int(), c_int(), c_int64()
    rp, ci, va = POINTER(c_int)(), POINTER(c_int)(), POINTER(c_double)()
    rc = _lib.oracle_mtx_read(str(path).encode(), byref(m), byref(n), byref(nnz), byref(rp),
                              byref(ci), byref(va))
    if rc != 0:
        raise ValueError(f"oracle_mtx_read({path}) failed: {rc}")
    k = nnz.value
    out = (m.value, n.value,
           np.ctypeslib.as_array(rp, (m.value + 1,)).copy(),
           np.ctypeslib.as_array(ci, (k,)).copy() if k else np.empty(0, np.int32),
           np.ctypeslib.as_array(va, (k,)).copy() if k else np.empty(0, np.float64))
    for ptr in (rp, ci, va):
        _lib.oracle_free(ctypes.cast(ptr, ctypes.c_void_p))
    return out


def max_rel_err(Y: np.ndarray, Yref: np.ndarray, A_abs_X_abs: np.ndarray | None = None) -> float:
    """max |Y - Yref| / max(|A||X| row scale, tiny): the tolerance measure used
    for results that differ from the sequential association (NONZERO)."""
    d = np.abs(Y - Yref)
    den = np.abs(Yref) if A_abs_X_abs is None else A_abs_X_abs
    den = np.maximum(den, 1e-300)
    return float(np.max(d / den)) if d.size else 0.0
