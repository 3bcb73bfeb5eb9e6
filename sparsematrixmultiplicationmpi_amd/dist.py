"""Multi-GPU variants: one process per GPU, RCCL over xGMI.

The reference's three MPI decompositions (SC/...RowWise.cpp:26-29,
SC/...ColumnWise.cpp:25-28, SC/...NonZeroElement.cpp:24-39) run in the
native library (csrc/smfv_dist.cpp): rank-local HIP kernel + one RCCL
exchange (gather-to-root, or all-gatherv).  torch.distributed is used only to
hand the RCCL unique id from rank 0 to the other ranks (MPI_COMM_WORLD's
role in the reference) and for host-side barriers.

`exchange_plan` exposes the native plan function (who owns which rows /
columns / nnz, and where each block sits in the exchange buffer) so the
exchange logic can be exercised with gloo on CPU-only hosts.
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, byref, c_int, c_int64, c_size_t, c_void_p

import numpy as np
import torch

from ._lib import call, lib
from .engine import DeviceCSR, Variant, stream_handle

UNIQUE_ID_BYTES = 128
TO_ROOT, TO_ALL = 0, 1


def exchange_plan(variant: int, m: int, nnz: int, row_ptr: np.ndarray | None, K: int, p: int):
    """Native smfv_dist_plan: per-rank (first, last, offset, count) arrays."""
    first = np.zeros(p, dtype=np.int32)
    last = np.zeros(p, dtype=np.int32)
    offset = np.zeros(p, dtype=np.int64)
    count = np.zeros(p, dtype=np.int64)
    rp = None
    if row_ptr is not None:
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
        rp = row_ptr.ctypes.data_as(POINTER(c_int))
    call("smfv_dist_plan", int(variant), m, nnz, rp, K, p,
         first.ctypes.data_as(POINTER(c_int)), last.ctypes.data_as(POINTER(c_int)),
         offset.ctypes.data_as(POINTER(c_int64)), count.ctypes.data_as(POINTER(c_int64)))
    return first, last, offset, count


class Communicator:
    """An RCCL communicator over the ranks of the default torch.distributed
    process group (rank 0 creates the unique id)."""

    def __init__(self, rank: int, size: int, unique_id: bytes):
        if len(unique_id) != UNIQUE_ID_BYTES:
            raise ValueError("bad RCCL unique id")
        self.rank, self.size = rank, size
        self._handle = c_void_p()
        buf = ctypes.create_string_buffer(unique_id, UNIQUE_ID_BYTES)
        call("smfv_comm_init", byref(self._handle), size, rank, buf)

    @staticmethod
    def new_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        call("smfv_comm_unique_id", buf)
        return buf.raw

    @classmethod
    def from_torch_distributed(cls) -> "Communicator":
        import torch.distributed as dist
        if not dist.is_initialized():
            return cls(0, 1, cls.new_unique_id())
        rank, size = dist.get_rank(), dist.get_world_size()
        obj = [cls.new_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(rank, size, obj[0])

    @property
    def handle(self) -> c_void_p:
        return self._handle

    def close(self) -> None:
        if self._handle:
            call("smfv_comm_destroy", self._handle)
            self._handle = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dist_workspace_bytes(comm: Communicator, variant: int, A: DeviceCSR, K: int) -> int:
    b = c_size_t(0)
    call("smfv_dist_workspace_bytes", comm.handle, int(variant), A.m, A.nnz,
         A.h_row_ptr.ctypes.data_as(POINTER(c_int)), K, byref(b))
    return b.value


class DistPlan:
    """Pre-sized distributed execution (workspace allocated once)."""

    def __init__(self, comm: Communicator, variant: int, A: DeviceCSR, K: int, to_all: bool,
                 root: int = 0):
        self.comm, self.variant, self.A, self.K = comm, Variant(variant), A, K
        self.mode = TO_ALL if to_all else TO_ROOT
        self.root = root
        nb = dist_workspace_bytes(comm, variant, A, K)
        self.ws_bytes = nb
        self.workspace = torch.empty(max(nb, 1), dtype=torch.uint8, device=A.device)

    def run(self, X: torch.Tensor, Y: torch.Tensor, stream=None) -> torch.Tensor:
        A = self.A
        if X.shape != (A.n, self.K) or not X.is_contiguous() or X.dtype != torch.float64:
            raise ValueError("X must be a contiguous float64 (n, K) device tensor")
        if Y.shape != (A.m, self.K) or not Y.is_contiguous() or Y.dtype != torch.float64:
            raise ValueError("Y must be a contiguous float64 (m, K) device tensor")
        rp, ci, va = A.ptrs()
        call("smfv_dist_spmm_f64", self.comm.handle, int(self.variant), self.mode, self.root, A.m,
             A.n, A.nnz, A.h_row_ptr.ctypes.data_as(POINTER(c_int)), rp, ci, va, X.data_ptr(),
             self.K, Y.data_ptr(), self.workspace.data_ptr(), self.ws_bytes, stream_handle(stream))
        return Y


def dist_spmm(comm: Communicator, variant: int, A: DeviceCSR, X: torch.Tensor, to_all: bool = False,
              root: int = 0, Y: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Collective SpMM; Y (m x K, on every rank) holds the result on `root`
    (to_all=False, the reference's semantics) or on every rank (to_all)."""
    K = X.shape[1]
    if Y is None:
        Y = torch.zeros((A.m, K), dtype=torch.float64, device=A.device)
    return DistPlan(comm, variant, A, K, to_all, root).run(X, Y, stream)


def dist_rowpart_spmm(comm: Communicator, m: int, A_local: DeviceCSR, X: torch.Tensor, Y: torch.Tensor,
                      to_all: bool = True, root: int = 0, stream=None) -> torch.Tensor:
    """Row-partitioned ROWWISE (smfv_dist_rowpart_spmm_f64): A_local holds only
    this rank's rows of the RowWise partition of an m-row matrix (local
    row_ptr, global column ids); X (n x K) replicated; Y (m x K) receives
    the full result on every rank (to_all) or on root."""
    K = X.shape[1]
    if X.shape != (A_local.n, K) or not X.is_contiguous() or X.dtype != torch.float64:
        raise ValueError("X must be a contiguous float64 (n, K) device tensor")
    if Y.shape != (m, K) or not Y.is_contiguous() or Y.dtype != torch.float64:
        raise ValueError("Y must be a contiguous float64 (m, K) device tensor")
    first, last, _, _ = exchange_plan(Variant.ROWWISE, m, 0, None, K, comm.size)
    if A_local.m != last[comm.rank] - first[comm.rank] + 1:
        raise ValueError(f"rank {comm.rank}: A_local has {A_local.m} rows, its partition "
                         f"[{first[comm.rank]}, {last[comm.rank]}] has {last[comm.rank] - first[comm.rank] + 1}")
    rp, ci, va = A_local.ptrs()
    call("smfv_dist_rowpart_spmm_f64", comm.handle, TO_ALL if to_all else TO_ROOT, root, m, A_local.n,
         rp, ci, va, X.data_ptr(), K, Y.data_ptr(), stream_handle(stream))
    return Y
