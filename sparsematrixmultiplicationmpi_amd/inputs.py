"""Host-side inputs: the reference's data model and its input functions.

Python mirror of SC/MatrixDefinitions.h:14-22 and SC/utils.{h,cpp}; every
function here calls the native host code in libsmfv.so (include/smfv_host.h):

    SparseMatrix                 SC/MatrixDefinitions.h:14-19 (+ numRows/numCols)
    readMatrixMarketFile         SC/utils.cpp:70-185
    generateLargeFatVector       SC/utils.cpp:193-209
    serialize / deserialize      SC/utils.cpp:216-253
    areMatricesEqual             SC/utils.cpp:38-63

plus the synthetic generators used where no input file exists offline
(cop20k_A surrogate, BASELINE configs 4-5).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, byref, c_double, c_int, c_int64
from dataclasses import dataclass

import numpy as np

from ._lib import call, lib

# SuiteSparse cop20k_A (report/425500_Report.tex:687): the size the
# surrogate reproduces
COP20K_M = 121192
COP20K_NNZ = 2624331


@dataclass
class SparseMatrix:
    """CSR matrix, 0-based; same fields as SC/MatrixDefinitions.h:14-19 plus
    the numRows/numCols every reference source uses."""

    values: np.ndarray      # float64[nnz]
    colIndices: np.ndarray  # int32[nnz]
    rowPtr: np.ndarray      # int32[numRows + 1]
    numRows: int
    numCols: int

    @property
    def nnz(self) -> int:
        return int(self.rowPtr[-1]) if len(self.rowPtr) else 0

    def validate(self) -> None:
        rp = self.rowPtr
        if len(rp) != self.numRows + 1 or rp[0] != 0 or np.any(np.diff(rp) < 0):
            raise ValueError("malformed rowPtr")
        if len(self.colIndices) != self.nnz or len(self.values) != self.nnz:
            raise ValueError("colIndices/values length != nnz")
        if self.nnz and (self.colIndices.min() < 0 or self.colIndices.max() >= self.numCols):
            raise ValueError("column index out of range")


def _take(ptr, count, dtype) -> np.ndarray:
    """Copy a library-malloc'd array into numpy and free it."""
    if count == 0:
        arr = np.empty(0, dtype=dtype)
    else:
        arr = np.ctypeslib.as_array(ptr, shape=(count,)).copy().astype(dtype, copy=False)
    lib.smfv_free(ctypes.cast(ptr, ctypes.c_void_p))
    return arr


def _csr_out(fn_name, *args, m=None, n=None) -> SparseMatrix:
    pm, pn, pnnz = c_int(0), c_int(0), c_int64(0)
    rp, ci, va = POINTER(c_int)(), POINTER(c_int)(), POINTER(c_double)()
    if m is None:
        call(fn_name, *args, byref(pm), byref(pn), byref(pnnz), byref(rp), byref(ci), byref(va))
        m, n = pm.value, pn.value
    else:
        call(fn_name, *args, byref(pnnz), byref(rp), byref(ci), byref(va))
    nnz = pnnz.value
    return SparseMatrix(values=_take(va, nnz, np.float64), colIndices=_take(ci, nnz, np.int32),
                        rowPtr=_take(rp, m + 1, np.int32), numRows=m, numCols=n)


def _ip(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_int))


def _dp(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_double))


def readMatrixMarketFile(filename: str) -> SparseMatrix:
    """SC/utils.cpp:70-185.  Raises SmfvError (the reference throws
    std::runtime_error) on an unreadable or malformed file."""
    return _csr_out("smfv_mtx_read", str(filename).encode())


def writeMatrixMarketFile(filename: str, A: SparseMatrix, symmetric: bool = False) -> None:
    call("smfv_mtx_write", str(filename).encode(), A.numRows, A.numCols, _ip(A.rowPtr),
         _ip(A.colIndices), _dp(A.values), int(symmetric))


def generateLargeFatVector(n: int, k: int) -> np.ndarray:
    """SC/utils.cpp:193-209: X[i][j] = rand()%100+1 from glibc's default-seed
    stream, returned as the flat row-major (n, k) array (serialize layout)."""
    X = np.empty((n, k), dtype=np.float64)
    lib.smfv_fatvector_rand(n, k, _dp(X))
    return X


def serialize(fat) -> np.ndarray:
    """SC/utils.cpp:216-228: FatVector (list of rows) -> flat row-major."""
    return np.ascontiguousarray(np.asarray(fat, dtype=np.float64)).reshape(-1)


def deserialize(flat: np.ndarray, rows: int, cols: int) -> np.ndarray:
    """SC/utils.cpp:237-253: flat row-major -> (rows, cols)."""
    return np.asarray(flat, dtype=np.float64)[: rows * cols].reshape(rows, cols).copy()


def areMatricesEqual(mat1, mat2, tolerance: float) -> bool:
    """SC/utils.cpp:38-63: same shape and max |a-b| <= tolerance (absolute).
    One deliberate difference: a NaN difference counts as unequal here (and in
    the device compare, smfv_compare_f64), where the reference's
    `fabs(a - b) > tolerance` is false for NaN and calls the matrices equal;
    the C++ drop-in's areMatricesEqual keeps the reference's behaviour."""
    a, b = np.asarray(mat1, dtype=np.float64), np.asarray(mat2, dtype=np.float64)
    if a.shape != b.shape:
        return False
    if a.size == 0:
        return True
    d = np.abs(a - b)
    return not bool(np.any(d > tolerance) or np.any(np.isnan(d)))


def read_csr_bin(path: str) -> SparseMatrix:
    return _csr_out("smfv_csr_read_bin", str(path).encode())


def write_csr_bin(path: str, A: SparseMatrix) -> None:
    call("smfv_csr_write_bin", str(path).encode(), A.numRows, A.numCols, _ip(A.rowPtr),
         _ip(A.colIndices), _dp(A.values))


def write_dense_bin(path: str, X: np.ndarray) -> None:
    X = np.ascontiguousarray(X, dtype=np.float64)
    call("smfv_dense_write_bin", str(path).encode(), X.shape[0], X.shape[1], _dp(X))


def read_dense_bin(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        if f.read(8) != b"SMFVDNS1":
            raise ValueError(f"{path}: not an SMFV dense file")
        rows, cols = np.frombuffer(f.read(16), dtype=np.int64)
        data = np.frombuffer(f.read(int(rows * cols) * 8), dtype=np.float64)
    return data.reshape(int(rows), int(cols)).copy()


def gen_fem27(m: int, nx: int = 50, ny: int = 50, keep: float = 0.8, seed: int = 20) -> SparseMatrix:
    """Symmetric 27-point-stencil surrogate (see smfv_host.h)."""
    return _csr_out("smfv_gen_fem27", m, nx, ny, float(keep), seed, m=m, n=m)


def gen_random_rows(m: int, n: int, mean: float, alpha: float, cap: int, seed: int,
                    row_begin: int = 0, row_end: int | None = None) -> SparseMatrix:
    """Row block [row_begin, row_end) of a random matrix (power-law row
    lengths for alpha > 1, fixed round(mean) for alpha <= 0)."""
    row_end = m if row_end is None else row_end
    return _csr_out("smfv_gen_random_rows", m, n, row_begin, row_end, float(mean), float(alpha),
                    int(cap), seed, m=row_end - row_begin, n=n)


# keep probability that gives the cop20k_A nnz (2,624,331) on a 50x50 grid
# truncated to 121,192 points: see cop20k_surrogate()
COP20K_KEEP = 0.82834


def cop20k_surrogate(seed: int = 20) -> SparseMatrix:
    """Labelled stand-in for SuiteSparse cop20k_A (not available offline):
    symmetric 27-point-stencil pattern on a 50x50x49 grid truncated to
    m = 121,192 rows, pair keep-probability tuned so nnz ~ 2,624,331."""
    return gen_fem27(COP20K_M, 50, 50, COP20K_KEEP, seed)


def gen_knn3d(m: int, target_nnz: int, seed: int = 7) -> SparseMatrix:
    """Irregular FEM-like matrix: symmetrised variable-k nearest-neighbour
    graph of clustered 3-D points, Morton-numbered (see smfv_host.h)."""
    return _csr_out("smfv_gen_knn3d", m, int(target_nnz), seed, m=m, n=m)


def cop20k_irregular_surrogate(seed: int = 7) -> SparseMatrix:
    """A second labelled stand-in for cop20k_A with its m and nnz but an
    unstructured pattern: row degrees spread ~5..80 (cop20k_A is an FEM
    matrix with variable row lengths; the 27-point stencil of
    cop20k_surrogate() is regular)."""
    return gen_knn3d(COP20K_M, COP20K_NNZ, seed)


def permute_symmetric(A: SparseMatrix, perm: np.ndarray) -> SparseMatrix:
    """P A P^T for a square A: new row i is old row perm[i], old column c
    becomes inv[c] (inv = perm^-1), each row sorted by column.  The same
    matrix under another numbering (the ordering-robustness variant of the
    cop20k_A surrogate)."""
    perm = np.asarray(perm, dtype=np.int64)
    m = A.numRows
    if A.numCols != m or len(perm) != m:
        raise ValueError("permute_symmetric needs a square matrix and a permutation of its rows")
    inv = np.empty(m, np.int64)
    inv[perm] = np.arange(m)
    rp = np.asarray(A.rowPtr, np.int64)
    lens = rp[perm + 1] - rp[perm]
    nrp = np.zeros(m + 1, np.int64)
    np.cumsum(lens, out=nrp[1:])
    src = np.repeat(rp[perm] - nrp[:-1], lens) + np.arange(nrp[-1])
    rows = np.repeat(np.arange(m), lens)
    cols = inv[np.asarray(A.colIndices)[src]]
    order = np.lexsort((cols, rows))
    return SparseMatrix(values=np.asarray(A.values)[src][order], colIndices=cols[order].astype(np.int32),
                        rowPtr=nrp.astype(np.int32), numRows=m, numCols=m)
