"""Device-side SpMM: Y = A_csr * X on an MI355X through the libsmfv C ABI.

Python mirror of the reference's hot-path call surface
(SC = /root/reference/Source Code):

    sparseMatrixFatVectorMultiply              SC/SparseMatrixFatVectorMultiply.h:14-15
    sparseMatrixFatVectorMultiplyRowWise       SC/SparseMatrixFatVectorMultiplyRowWise.h:15-17
    sparseMatrixFatVectorMultiplyColumnWise    SC/SparseMatrixFatVectorMultiplyColumnWise.h:15
    sparseMatrixFatVectorMultiplyNonZeroElement SC/SparseMatrixFatVectorMultiplyNonZeroElement.h:15

Same arguments (A, fat vector, vecCols) and result (m x K, row-major).  The
MPI variants are collective over a Communicator (dist.py) when one is given
and return the result on rank 0 only (an empty (0, K) array elsewhere), as
SC/...RowWise.cpp:125 does; without one they run on the local GPU.

torch is used only for device memory and the current HIP stream.  Every
compute call goes to the HIP kernels; there is no CPU path.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_size_t
from enum import IntEnum

import numpy as np
import torch

from ._lib import call
from .inputs import SparseMatrix


class Variant(IntEnum):
    SEQUENTIAL = 0   # SC/SparseMatrixFatVectorMultiply.cpp:11-31
    ROWWISE = 1      # SC/SparseMatrixFatVectorMultiplyRowWise.cpp:12-126
    COLUMNWISE = 2   # SC/SparseMatrixFatVectorMultiplyColumnWise.cpp:13-131
    NONZERO = 3      # SC/SparseMatrixFatVectorMultiplyNonZeroElement.cpp:12-120


def _require_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("smfv: no HIP device visible; the SpMM engine has no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def stream_handle(stream: torch.cuda.Stream | None = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class DeviceCSR:
    """A CSR matrix resident in HBM (int32 row_ptr / col_idx, f64 values)
    plus the host copy of the pattern the plans analyse.

    spmm() keeps one plan per (variant, K) on the matrix (analysed once).  A
    tiled plan computes with a snapshot of the values taken when it was bound
    (include/smfv.h, values contract).  The cached plans re-bind by
    themselves when `values` has changed since their bind -- a new tensor, or
    an in-place change (torch's version counter of the tensor) -- and
    values_changed() re-binds them explicitly (e.g. after a write torch did
    not see, such as a kernel of another library)."""

    def __init__(self, A: SparseMatrix, device: torch.device | None = None):
        device = device or _require_device()
        A.validate()
        self.m, self.n, self.nnz = A.numRows, A.numCols, A.nnz
        self.h_row_ptr = np.ascontiguousarray(A.rowPtr, dtype=np.int32)
        self.h_col_idx = np.ascontiguousarray(A.colIndices, dtype=np.int32)  # plan analysis
        self.row_ptr = torch.from_numpy(self.h_row_ptr).to(device)
        self.col_idx = torch.from_numpy(self.h_col_idx).to(device)
        self.values = torch.from_numpy(np.ascontiguousarray(A.values, dtype=np.float64)).to(device)
        self.device = device
        self._plans: dict = {}

    @property
    def nbytes(self) -> int:
        return 4 * (self.m + 1) + 12 * self.nnz

    def ptrs(self):
        return self.row_ptr.data_ptr(), self.col_idx.data_ptr(), self.values.data_ptr()

    def plan(self, variant: int, K: int, stream: torch.cuda.Stream | None = None) -> "SpmmPlan":
        """The cached plan of (variant, K), created (and bound on `stream`) on first use."""
        key = (int(variant), int(K))
        p = self._plans.get(key)
        if p is None:
            p = self._plans[key] = SpmmPlan(variant, self, K, stream=stream)
        elif p.bound_version != self.values_version():
            p.bind_values(stream)  # values changed since the bind: snapshot them again
        return p

    def values_version(self) -> tuple[int, int]:
        """(address, torch version counter) of `values`: changes with every
        in-place write torch performs and with a new tensor."""
        return self.values.data_ptr(), self.values._version

    def values_changed(self, stream: torch.cuda.Stream | None = None) -> None:
        """Re-bind every cached plan after `values` changed in place."""
        for p in self._plans.values():
            p.bind_values(stream)


def workspace_bytes(variant: int, m: int, nnz: int, K: int) -> int:
    b = c_size_t(0)
    call("smfv_spmm_workspace_bytes", int(variant), m, nnz, K, byref(b))
    return b.value


def _check_dense(T: torch.Tensor, rows: int, K: int, name: str) -> int:
    if not T.is_cuda or T.dtype != torch.float64:
        raise TypeError(f"{name} must be a float64 HIP tensor")
    if T.dim() != 2 or T.shape[0] != rows or T.shape[1] != K:
        raise ValueError(f"{name} must have shape ({rows}, {K}), got {tuple(T.shape)}")
    if K > 0 and T.stride(1) != 1:
        raise ValueError(f"{name} must be row-major (unit column stride)")
    return max(int(T.stride(0)), K)


PLAN_NO_TILES, PLAN_FORCE_TILES, PLAN_FMA, PLAN_NATURAL_SEEDS, PLAN_MFMA, PLAN_SPLIT_ENDS = 1, 2, 4, 8, 16, 32
PLAN_ONE_WAVEFRONT, PLAN_SIMPLE_ROWS, PLAN_CS, PLAN_WS = 64, 128, 256, 512
PLAN_WS_GEOM1, PLAN_WS_GEOM2, PLAN_WS_GEOM3 = 1024, 2048, 4096
PLAN_LIVE_VALUES = 8192  # (r5) the tiled kernel reads the live CSR values (no snapshot, no bind)
PLAN_SINGLE_ROWS = 16384  # (r5) one row per k_rows_ws team (no row pairs; A/B)
PLAN_ROW_PAIRS = 32768  # (r5) row pairs forced (without either: the plan with fewer rounds)
PLAN_STATS = 18  # SMFV_PLAN_STATS
PLAN_KERNELS = {0: None, 1: "k_rows_ws", 2: "k_rows_mfma", 3: "k_spmv_chunks", 5: "k_rows_wsn"}


class SpmmPlan:
    """One variant of Y = A*X analysed once for (A, K) (smfv_plan_create):
    device workspace allocated up front and, for K % 32 == 0 or K = 4 / 8 /
    16 (one narrow column window), the row-tile analysis that lets the kernel
    stage re-used X rows in LDS.  run() is a pure asynchronous launch
    sequence (capturable into a hipGraph).

    tiles: "auto" (stage when re-use >= 3), "off", or "force".  fma: opt-in
    fused multiply-add in the tiled kernel (SMFV_PLAN_FMA).  rows=(begin,
    end): plan of that row block only (smfv_plan_create_rows; run() writes
    the block's rows to Y[0:end-begin]).  xcd_parts: "auto" (one row range
    per XCD when their X footprints allow it) or "one" (one wavefront cut in
    8 shares; SMFV_PLAN_ONE_WAVEFRONT, A/B).  The values snapshot of a tiled plan
    is gathered on `stream`; a run() on another stream waits for it."""

    def __init__(self, variant: int, A: DeviceCSR, K: int, tiles: str = "auto", fma: bool = False,
                 stream: torch.cuda.Stream | None = None, rows: tuple[int, int] | None = None,
                 seeds: str = "frontier", mfma: bool = False, split_ends: bool = False,
                 xcd_parts: str = "auto", tiled_kernel: str = "auto", live_values: bool = False,
                 row_pairs: str = "auto"):
        self.variant, self.A, self.K = Variant(variant), A, K
        self.rows = rows
        flags = {"auto": 0, "off": PLAN_NO_TILES, "force": PLAN_FORCE_TILES}[tiles]
        if live_values:  # (r5) SMFV_PLAN_LIVE_VALUES: value pairs DMA'd from the CSR values, bind a no-op
            flags |= PLAN_LIVE_VALUES
        # (r5) row pairs in k_rows_ws tiles: "auto" (the plan whose busiest
        # block runs fewer tiles), "off" (SMFV_PLAN_SINGLE_ROWS), "on" (SMFV_PLAN_ROW_PAIRS)
        flags |= {"auto": 0, "off": PLAN_SINGLE_ROWS, "on": PLAN_ROW_PAIRS}[row_pairs]
        if fma:  # opt-in fused multiply-add in the tiled kernel: within tolerance, not bit-identical
            flags |= PLAN_FMA
        if seeds == "natural":  # tiles seeded in row order (A/B of the wavefront seeding)
            flags |= PLAN_NATURAL_SEEDS
        if mfma:  # opt-in dense-block MFMA tile kernel: within tolerance, not bit-identical
            flags |= PLAN_MFMA
        if split_ends:  # opt-in: half tiles first and last in every block (A/B; measured slower)
            flags |= PLAN_SPLIT_ENDS
        if {"auto": False, "one": True}[xcd_parts]:
            flags |= PLAN_ONE_WAVEFRONT
        # which tiled kernel for K % 32 == 0: the library's choice, or k_rows_ws
        # (SMFV_PLAN_WS) for A/B; "ws1" / "ws2" / "ws3": k_rows_ws with one
        # 1024-lane / two 512-lane / one 768-lane pipeline(s) per CU
        # (SMFV_PLAN_WS_GEOM1 / 2 / 3)
        flags |= {"auto": 0, "ws": PLAN_WS, "ws1": PLAN_WS | PLAN_WS_GEOM1,
                  "ws2": PLAN_WS | PLAN_WS_GEOM2, "ws3": PLAN_WS | PLAN_WS_GEOM3}[tiled_kernel]
        self._plan = ctypes.c_void_p()
        ip = ctypes.POINTER(ctypes.c_int)
        if rows is None:
            call("smfv_plan_create", byref(self._plan), int(variant), A.m, A.n, A.nnz,
                 A.h_row_ptr.ctypes.data_as(ip), A.h_col_idx.ctypes.data_as(ip), K, flags)
            self.m_out = A.m
        else:
            r0, r1 = int(rows[0]), int(rows[1])
            call("smfv_plan_create_rows", byref(self._plan), int(variant), r0, r1, A.n,
                 A.h_row_ptr.ctypes.data_as(ip), A.h_col_idx.ctypes.data_as(ip), K, flags)
            self.m_out = r1 - r0
        self.bind_values(stream)

    def bind_values(self, stream: torch.cuda.Stream | None = None) -> None:
        """(Re)bind a tiled plan to A's current device values (after they change)."""
        call("smfv_plan_bind_values", self._plan, self.A.values.data_ptr(), stream_handle(stream))
        self.bound_version = self.A.values_version()

    def stats(self) -> dict:
        out = (ctypes.c_double * PLAN_STATS)()
        call("smfv_plan_stats", self._plan, out)
        return {"tiled": bool(out[0]), "tiles": int(out[1]), "staged_rows": int(out[2]),
                "reuse": float(out[3]), "plan_bytes": int(out[4]), "direct_rows": int(out[5]),
                "row_begin": int(out[6]), "est_reuse": float(out[7]), "analysis_ms": float(out[8]),
                "snapshot_entries": int(out[9]), "mfma": bool(out[10]), "xcd_parts": int(out[11]),
                "footprint": float(out[12]), "kernel": PLAN_KERNELS.get(int(out[13])), "live_values": bool(out[14]),
                "ws_geom": int(out[15]), "bind_descriptors": bool(out[16]),
                "paired_rows": int(out[17])}

    def run(self, X: torch.Tensor, Y: torch.Tensor, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
        A, K = self.A, self.K
        ldx = _check_dense(X, A.n, K, "X")
        ldy = _check_dense(Y, self.m_out, K, "Y")
        rp, ci, va = A.ptrs()
        call("smfv_plan_execute", self._plan, rp, ci, va, X.data_ptr(), ldx, Y.data_ptr(), ldy,
             stream_handle(stream))
        return Y

    def __del__(self):
        try:
            if self._plan:
                call("smfv_plan_destroy", self._plan)
                self._plan = ctypes.c_void_p()
        except Exception:
            pass


def spmm(variant: int, A: DeviceCSR, X: torch.Tensor, Y: torch.Tensor | None = None,
         stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Y = A * X on the device (asynchronous on `stream`), through A's cached
    plan for (variant, K)."""
    K = X.shape[1]
    if Y is None:
        Y = torch.empty((A.m, K), dtype=torch.float64, device=A.device)
    return A.plan(variant, K, stream).run(X, Y, stream)


def spmm_rowblock(A: DeviceCSR, row_begin: int, row_end: int, X: torch.Tensor, Yblock: torch.Tensor,
                  stream=None) -> torch.Tensor:
    K = X.shape[1]
    ldx = _check_dense(X, A.n, K, "X")
    ldy = _check_dense(Yblock, row_end - row_begin, K, "Yblock")
    rp, ci, va = A.ptrs()
    call("smfv_spmm_rowblock_f64", row_begin, row_end, A.n, rp, ci, va, X.data_ptr(), ldx, K,
         Yblock.data_ptr(), ldy, stream_handle(stream))
    return Yblock


def spmm_colpanel(A: DeviceCSR, col_begin: int, col_end: int, X: torch.Tensor, panel: torch.Tensor,
                  stream=None) -> torch.Tensor:
    K = X.shape[1]
    ldx = _check_dense(X, A.n, K, "X")
    ldp = _check_dense(panel, A.m, col_end - col_begin, "panel")
    rp, ci, va = A.ptrs()
    call("smfv_spmm_colpanel_f64", A.m, A.n, col_begin, col_end, rp, ci, va, X.data_ptr(), ldx,
         panel.data_ptr(), max(ldp, 1), stream_handle(stream))
    return panel


def nnz_range_rows(A_host_row_ptr: np.ndarray, nnz_begin: int, nnz_end: int) -> tuple[int, int]:
    rp = np.ascontiguousarray(A_host_row_ptr, dtype=np.int32)
    rf, rl = ctypes.c_int(0), ctypes.c_int(0)
    call("smfv_nnz_range_rows", len(rp) - 1, rp.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
         nnz_begin, nnz_end, byref(rf), byref(rl))
    return rf.value, rl.value


def spmm_nnzrange(A: DeviceCSR, nnz_begin: int, nnz_end: int, X: torch.Tensor, stream=None):
    """Partial rows of the nnz range (SC/...NonZeroElement.cpp:56-67):
    returns (row_first, row_last, Ypart[(row_last-row_first+1) x K])."""
    K = X.shape[1]
    ldx = _check_dense(X, A.n, K, "X")
    rf, rl = nnz_range_rows(A.h_row_ptr, nnz_begin, nnz_end)
    nr = max(0, rl - rf + 1)
    Yp = torch.empty((nr, K), dtype=torch.float64, device=A.device)
    b = c_size_t(0)
    call("smfv_spmm_nnzrange_workspace_bytes", nr, nnz_end - nnz_begin, K, byref(b))
    ws = torch.empty(max(b.value, 1), dtype=torch.uint8, device=A.device)
    rp, ci, va = A.ptrs()
    call("smfv_spmm_nnzrange_f64", rf, rl, nnz_begin, nnz_end, A.n, rp, ci, va, X.data_ptr(), ldx, K,
         Yp.data_ptr(), max(K, 1), ws.data_ptr(), b.value, stream_handle(stream))
    return rf, rl, Yp


def compare(A: torch.Tensor, B: torch.Tensor, stream=None) -> tuple[float, float]:
    """Device areMatricesEqual (SC/utils.cpp:38-63): (max abs diff, max rel diff)."""
    m, K = A.shape
    lda = _check_dense(A, m, K, "A")
    ldb = _check_dense(B, m, K, "B")
    out = (ctypes.c_double * 2)()
    call("smfv_compare_f64", m, K, A.data_ptr(), lda, B.data_ptr(), ldb, out, stream_handle(stream))
    return out[0], out[1]


def fill_x_hash(X: torch.Tensor, seed: int, stream=None) -> torch.Tensor:
    n, K = X.shape
    ldx = _check_dense(X, n, K, "X")
    call("smfv_fill_x_hash_f64", n, K, seed, X.data_ptr(), ldx, stream_handle(stream))
    return X


# ---------------------------------------------------------------------------
# the reference's four functions (host arrays in, host array out)
# ---------------------------------------------------------------------------
def _run_host(variant: Variant, A: SparseMatrix, fatVector, vecCols: int) -> np.ndarray:
    X = np.ascontiguousarray(np.asarray(fatVector, dtype=np.float64).reshape(A.numCols, vecCols))
    dA = DeviceCSR(A)
    dX = torch.from_numpy(X).to(dA.device)
    Y = spmm(variant, dA, dX)
    return Y.cpu().numpy()


def sparseMatrixFatVectorMultiply(sparseMatrix: SparseMatrix, fatVector, vecCols: int) -> np.ndarray:
    return _run_host(Variant.SEQUENTIAL, sparseMatrix, fatVector, vecCols)


def _collective(variant: Variant, A: SparseMatrix, fatVector, vecCols: int, comm) -> np.ndarray:
    if comm is None or comm.size == 1:
        return _run_host(variant, A, fatVector, vecCols)
    from .dist import dist_spmm
    dA = DeviceCSR(A)
    X = np.ascontiguousarray(np.asarray(fatVector, dtype=np.float64).reshape(A.numCols, vecCols))
    dX = torch.from_numpy(X).to(dA.device)
    Y = dist_spmm(comm, variant, dA, dX, to_all=False, root=0)
    torch.cuda.synchronize()
    return Y.cpu().numpy() if comm.rank == 0 else np.empty((0, vecCols))


def sparseMatrixFatVectorMultiplyRowWise(sparseMatrix: SparseMatrix, fatVector, vecCols: int,
                                         comm=None) -> np.ndarray:
    return _collective(Variant.ROWWISE, sparseMatrix, fatVector, vecCols, comm)


def sparseMatrixFatVectorMultiplyColumnWise(sparseMatrix: SparseMatrix, fatVector, vecCols: int,
                                            comm=None) -> np.ndarray:
    return _collective(Variant.COLUMNWISE, sparseMatrix, fatVector, vecCols, comm)


def sparseMatrixFatVectorMultiplyNonZeroElement(sparseMatrix: SparseMatrix, fatVector, vecCols: int,
                                                comm=None) -> np.ndarray:
    return _collective(Variant.NONZERO, sparseMatrix, fatVector, vecCols, comm)


class VendorSpmm:
    """rocSPARSE generic SpMM on the same device operands (smfv_vendor_spmm_*):
    the vendor-library comparator, the analogue of the reference's PETSc
    MatMatMult block (SC/main.cpp:289-402).  Not the product path.
    alg: 0 rocSPARSE default, 1 CSR row split, 2 CSR merge path."""

    def __init__(self, A: DeviceCSR, X: torch.Tensor, Y: torch.Tensor, alg: int = 0,
                 stream: torch.cuda.Stream | None = None):
        K = X.shape[1]
        ldx = _check_dense(X, A.n, K, "X")
        ldy = _check_dense(Y, A.m, K, "Y")
        self.A, self.X, self.Y = A, X, Y  # keep the bound operands alive
        self._h = ctypes.c_void_p()
        rp, ci, va = A.ptrs()
        call("smfv_vendor_spmm_create", byref(self._h), alg, A.m, A.n, A.nnz, rp, ci, va, X.data_ptr(), ldx, K,
             Y.data_ptr(), ldy, stream_handle(stream))

    def run(self) -> torch.Tensor:
        call("smfv_vendor_spmm_execute", self._h)
        return self.Y

    def __del__(self):
        try:
            if self._h:
                call("smfv_vendor_spmm_destroy", self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass
