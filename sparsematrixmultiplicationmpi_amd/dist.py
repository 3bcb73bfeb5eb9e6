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
# (r5) distribution options (include/smfv.h SMFV_DIST_*), the high byte of a
# distributed plan's flags
BALANCED_ROWS = 1 << 24


def dist_opts(partition: str = "reference", chunks: int = 1) -> int:
    """SMFV_DIST_* bits: ROWWISE row blocks by the reference's equal row
    counts ("reference", SC/...RowWise.cpp:26-29, the default) or of equal
    work ("balanced", SMFV_DIST_BALANCED_ROWS); `chunks` row chunks per
    rank, each exchanged as soon as it is computed (SMFV_DIST_CHUNKS)."""
    if partition not in ("balanced", "reference") or not 1 <= chunks <= 7:
        raise ValueError(f"partition {partition!r}, chunks {chunks}")
    return (BALANCED_ROWS if partition == "balanced" else 0) | ((chunks & 7) << 25 if chunks > 1 else 0)


def _rp(row_ptr):
    if row_ptr is None:
        return None, None
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
    return row_ptr, row_ptr.ctypes.data_as(POINTER(c_int))


def exchange_plan(variant: int, m: int, nnz: int, row_ptr: np.ndarray | None, K: int, p: int,
                  dopts: int = 0):
    """Native smfv_dist_plan_opts: per-rank (first, last, offset, count)
    arrays; by default the reference's partition (smfv_dist_plan)."""
    first = np.zeros(p, dtype=np.int32)
    last = np.zeros(p, dtype=np.int32)
    offset = np.zeros(p, dtype=np.int64)
    count = np.zeros(p, dtype=np.int64)
    keep, rp = _rp(row_ptr)
    call("smfv_dist_plan_opts", int(variant), int(dopts), m, nnz, rp, K, p,
         first.ctypes.data_as(POINTER(c_int)), last.ctypes.data_as(POINTER(c_int)),
         offset.ctypes.data_as(POINTER(c_int64)), count.ctypes.data_as(POINTER(c_int64)))
    return first, last, offset, count


def chunk_rows(variant: int, dopts: int, m: int, nnz: int, row_ptr: np.ndarray | None, K: int, p: int,
               rank: int) -> list[int]:
    """Native smfv_dist_chunk_rows: rank's chunk boundaries (chunk j = rows
    [b[j], b[j + 1]))."""
    b = np.zeros(8, dtype=np.int32)
    n = c_int(0)
    keep, rp = _rp(row_ptr)
    call("smfv_dist_chunk_rows", int(variant), int(dopts), m, nnz, rp, K, p, rank,
         b.ctypes.data_as(POINTER(c_int)), byref(n))
    return [int(v) for v in b[:n.value + 1]]


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

    def nranks(self) -> int:
        """The ranks RCCL itself counts in this communicator (ncclCommCount)."""
        n = c_int(0)
        call("smfv_comm_count", self._handle, byref(n))
        return n.value

    def close(self) -> None:
        if self._handle:
            call("smfv_comm_destroy", self._handle)
            self._handle = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


EX_ALLGATHER, EX_BCAST, EX_SEND, EX_RECV = 1, 2, 3, 4  # SMFV_EX_*


def exchange_ops(variant: int, mode: int, root: int, m: int, nnz: int, row_ptr: np.ndarray | None, K: int,
                 p: int, rank: int, dopts: int = 0, chunk: int = 0) -> list[tuple[int, int, int, int]]:
    """Native smfv_dist_exchange_ops_opts: the exchange step of `rank` (of
    chunk `chunk` under SMFV_DIST_CHUNKS) as a list of (kind, peer, offset,
    count) -- the schedule the RCCL path runs, in one group."""
    cap = 2 * p + 2
    kinds = np.zeros(cap, np.int32)
    peers = np.zeros(cap, np.int32)
    offs = np.zeros(cap, np.int64)
    cnts = np.zeros(cap, np.int64)
    n = c_int(0)
    keep, rp = _rp(row_ptr)
    call("smfv_dist_exchange_ops_opts", int(variant), int(dopts), int(mode), int(root), m, nnz, rp, K, p, rank,
         int(chunk), kinds.ctypes.data_as(POINTER(c_int)), peers.ctypes.data_as(POINTER(c_int)),
         offs.ctypes.data_as(POINTER(c_int64)), cnts.ctypes.data_as(POINTER(c_int64)), byref(n))
    return [(int(kinds[i]), int(peers[i]), int(offs[i]), int(cnts[i])) for i in range(n.value)]


def dist_workspace_bytes(comm: Communicator, variant: int, A: DeviceCSR, K: int) -> int:
    b = c_size_t(0)
    call("smfv_dist_workspace_bytes", comm.handle, int(variant), A.m, A.nnz,
         A.h_row_ptr.ctypes.data_as(POINTER(c_int)), K, byref(b))
    return b.value


class DistPlan:
    """A distributed variant analysed once (smfv_dist_plan_create): this
    rank's share (RowWise row block, ColumnWise K-column window,
    NonZeroElement nnz range) as a single-device plan -- the tiled kernel
    where it pays -- plus the exchange buffers and schedule.

    rowpart=True: A holds only this rank's rows of the RowWise partition of
    an m-row matrix (smfv_dist_plan_create_rowpart; `m` required).

    comm=None with rank=(r, p): the plan of rank r of p alone, no
    communicator (smfv_dist_plan_create_rank): run_local() computes what that
    rank of the reference's variant computes, into Y (ROWWISE) or the plan's
    exchange buffer (exchange_buffer()); exchange() is refused.

    Values: a tiled share (and every K = 1 chunk plan) computes with the
    snapshot of A's values taken by the last bind; run() / run_local() bind
    again by themselves when A's values tensor changed in place since (its
    version counter), as SpmmPlan does through DeviceCSR.plan()."""

    def __init__(self, comm: Communicator | None, variant: int, A: DeviceCSR, K: int, to_all: bool,
                 root: int = 0, tiles: str = "auto", rowpart: bool = False, m: int | None = None,
                 stream=None, rank: tuple[int, int] | None = None, fma: bool = False, tiled_kernel: str = "auto",
                 partition: str = "reference", chunks: int = 1, live_values: bool = False):
        self.comm, self.variant, self.A, self.K = comm, Variant(variant), A, K
        self.mode = TO_ALL if to_all else TO_ROOT
        self.root = root
        self.m = A.m if not rowpart else int(m)
        from .engine import PLAN_LIVE_VALUES, PLAN_WS, PLAN_WS_GEOM1, PLAN_WS_GEOM2, PLAN_WS_GEOM3
        flags = {"auto": 0, "off": 1, "force": 2}[tiles] | (4 if fma else 0) | (PLAN_LIVE_VALUES if live_values else 0)
        # the rank share's tiled-kernel geometry (SpmmPlan's tiled_kernel; A/B)
        flags |= {"auto": 0, "ws1": PLAN_WS | PLAN_WS_GEOM1, "ws2": PLAN_WS | PLAN_WS_GEOM2,
                  "ws3": PLAN_WS | PLAN_WS_GEOM3}[tiled_kernel]
        # (r5) ROWWISE: the reference's equal rows by default, "balanced": blocks
        # of equal work; chunks > 1: per-chunk exchanges overlapped with the
        # next chunk's compute
        flags |= dist_opts(partition, chunks)
        ip = POINTER(c_int)
        self._h = c_void_p()
        if comm is None:
            r, p = rank
            call("smfv_dist_plan_create_rank", byref(self._h), int(p), int(r), int(variant), self.mode, root, A.m,
                 A.n, A.nnz, A.h_row_ptr.ctypes.data_as(ip), A.h_col_idx.ctypes.data_as(ip), K, flags)
        elif rowpart:
            call("smfv_dist_plan_create_rowpart", byref(self._h), comm.handle, self.mode, root, self.m, A.n,
                 A.h_row_ptr.ctypes.data_as(ip), A.h_col_idx.ctypes.data_as(ip), K, flags)
        else:
            call("smfv_dist_plan_create", byref(self._h), comm.handle, int(variant), self.mode, root, A.m, A.n,
                 A.nnz, A.h_row_ptr.ctypes.data_as(ip), A.h_col_idx.ctypes.data_as(ip), K, flags)
        self.bind_values(stream)

    def bind_values(self, stream=None) -> None:
        call("smfv_dist_plan_bind_values", self._h, self.A.values.data_ptr(), stream_handle(stream))
        self.bound_version = self.A.values_version()

    def _rebind_if_changed(self, stream) -> None:
        if self.A.values_version() != self.bound_version:
            self.bind_values(stream)

    def _check(self, X: torch.Tensor, Y: torch.Tensor) -> None:
        if X.shape != (self.A.n, self.K) or not X.is_contiguous() or X.dtype != torch.float64:
            raise ValueError("X must be a contiguous float64 (n, K) device tensor")
        if Y.shape != (self.m, self.K) or not Y.is_contiguous() or Y.dtype != torch.float64:
            raise ValueError("Y must be a contiguous float64 (m, K) device tensor")

    def run(self, X: torch.Tensor, Y: torch.Tensor, stream=None) -> torch.Tensor:
        self._check(X, Y)
        self._rebind_if_changed(stream)
        rp, ci, va = self.A.ptrs()
        call("smfv_dist_plan_execute", self._h, rp, ci, va, X.data_ptr(), Y.data_ptr(), stream_handle(stream))
        return Y

    def run_local(self, X: torch.Tensor, Y: torch.Tensor, stream=None) -> torch.Tensor:
        """The rank-local compute alone (no exchange)."""
        self._check(X, Y)
        self._rebind_if_changed(stream)
        rp, ci, va = self.A.ptrs()
        call("smfv_dist_plan_execute_local", self._h, rp, ci, va, X.data_ptr(), Y.data_ptr(),
             stream_handle(stream))
        return Y

    def exchange(self, Y: torch.Tensor, stream=None) -> torch.Tensor:
        """The exchange step alone (after run_local)."""
        call("smfv_dist_plan_exchange", self._h, Y.data_ptr(), stream_handle(stream))
        return Y

    def exchange_buffer(self) -> torch.Tensor | None:
        """The plan's exchange buffer as a (device) tensor view: rank-major
        COLUMNWISE panels / NONZERO compact row blocks, laid out as
        exchange_plan's offset / count say; None for ROWWISE (Y itself)."""
        ptr, n = ctypes.POINTER(ctypes.c_double)(), c_int64(0)
        call("smfv_dist_plan_exchange_buffer", self._h, byref(ptr), byref(n))
        if not n.value:
            return None
        addr = ctypes.cast(ptr, c_void_p).value
        # a non-owning view of the plan's device buffer (the plan outlives it)
        return _device_view(addr, n.value, self.A.device, owner=self)

    def partition(self):
        """(first, last, offset, count) per rank: the partition this plan was
        created with (smfv_dist_plan_partition)."""
        p, r, c = self.shape()
        first = np.zeros(p, dtype=np.int32)
        last = np.zeros(p, dtype=np.int32)
        offset = np.zeros(p, dtype=np.int64)
        count = np.zeros(p, dtype=np.int64)
        call("smfv_dist_plan_partition", self._h, first.ctypes.data_as(POINTER(c_int)),
             last.ctypes.data_as(POINTER(c_int)), offset.ctypes.data_as(POINTER(c_int64)),
             count.ctypes.data_as(POINTER(c_int64)))
        return first, last, offset, count

    def shape(self) -> tuple[int, int, int]:
        """(p, rank, chunks per rank) of the plan."""
        p, r, c = c_int(0), c_int(0), c_int(0)
        call("smfv_dist_plan_shape", self._h, byref(p), byref(r), byref(c))
        return p.value, r.value, c.value

    def stats(self) -> dict:
        from .engine import PLAN_STATS
        out = (ctypes.c_double * PLAN_STATS)()
        call("smfv_dist_plan_stats", self._h, out)
        return {"tiled": bool(out[0]), "tiles": int(out[1]), "reuse": float(out[3]),
                "row_begin": int(out[6]), "analysis_ms": float(out[8]), "xcd_parts": int(out[11]),
                "footprint": float(out[12]), "ws_geom": int(out[15])}

    def __del__(self):
        try:
            if self._h:
                call("smfv_dist_plan_destroy", self._h)
                self._h = c_void_p()
        except Exception:
            pass


def _device_view(addr: int, count: int, device: torch.device, owner) -> torch.Tensor:
    """A float64 tensor over `count` doubles of device memory at `addr` that
    the library owns (kept alive by `owner`)."""
    class _Holder:
        def __init__(self):
            self.owner = owner
            self.__cuda_array_interface__ = {"shape": (count,), "typestr": "<f8", "data": (addr, False),
                                             "version": 3, "strides": None, "stream": None}
    return torch.as_tensor(_Holder(), device=device)


def dist_spmm(comm: Communicator, variant: int, A: DeviceCSR, X: torch.Tensor, to_all: bool = False,
              root: int = 0, Y: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Collective SpMM; Y (m x K, on every rank) holds the result on `root`
    (to_all=False, the reference's semantics) or on every rank (to_all)."""
    K = X.shape[1]
    if Y is None:
        Y = torch.zeros((A.m, K), dtype=torch.float64, device=A.device)
    return DistPlan(comm, variant, A, K, to_all, root, stream=stream).run(X, Y, stream)


def dist_spmm_oneshot(comm: Communicator, variant: int, A: DeviceCSR, X: torch.Tensor, to_all: bool = False,
                      root: int = 0, Y: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """The same through smfv_dist_spmm_f64 (no plan: workspace per call, row kernel)."""
    K = X.shape[1]
    if Y is None:
        Y = torch.zeros((A.m, K), dtype=torch.float64, device=A.device)
    nb = dist_workspace_bytes(comm, variant, A, K)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=A.device)
    rp, ci, va = A.ptrs()
    call("smfv_dist_spmm_f64", comm.handle, int(variant), TO_ALL if to_all else TO_ROOT, root, A.m,
         A.n, A.nnz, A.h_row_ptr.ctypes.data_as(POINTER(c_int)), rp, ci, va, X.data_ptr(),
         K, Y.data_ptr(), ws.data_ptr(), nb, stream_handle(stream))
    return Y


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
