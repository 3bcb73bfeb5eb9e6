"""ctypes binding of libsmfv.so (include/smfv.h, include/smfv_host.h).

The shared library is the product: HIP kernels for gfx950 plus the C ABI.
There is no Python or CPU fallback for any compute entry point -- if the
library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char, c_char_p, c_double, c_int, c_int64, c_size_t, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
# The product is libsmfv.so.  SMFV_LIB=<file name in this directory> loads
# another build of the same sources instead -- for A/B runs only, e.g. a copy
# of the previous build (scripts/ab_lib.sh); the driver never sets it.
LIB_PATH = os.path.join(HERE, os.path.basename(os.environ.get("SMFV_LIB") or "libsmfv.so"))

SMFV_OK = 0
STATUS_NAMES = {
    -1: "SMFV_ERR_INVALID",
    -2: "SMFV_ERR_WORKSPACE",
    -3: "SMFV_ERR_HIP",
    -4: "SMFV_ERR_COMM",
    -5: "SMFV_ERR_HOST",
}


class SmfvError(RuntimeError):
    """A C-ABI call returned a non-zero smfv_status."""

    def __init__(self, fn: str, status: int, message: str):
        super().__init__(f"{fn}: {STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


_PI = POINTER(c_int)
_PD = POINTER(c_double)
_PI64 = POINTER(c_int64)

# name -> (restype, argtypes)
_SIGS = {
    "smfv_last_error": (c_char_p, []),
    "smfv_version": (c_char_p, []),
    "smfv_device_init": (c_int, [c_void_p]),
    "smfv_partition_rows": (None, [c_int, c_int, c_int, _PI, _PI]),
    "smfv_partition_cols": (None, [c_int, c_int, c_int, _PI, _PI]),
    "smfv_partition_nnz": (None, [c_int64, c_int, c_int, _PI64, _PI64]),
    "smfv_merge_geometry": (c_int, [c_int, c_int64, c_int, _PI64]),
    "smfv_spmm_workspace_bytes": (c_int, [c_int, c_int, c_int64, c_int, POINTER(c_size_t)]),
    "smfv_spmm_csr_f64": (c_int, [c_int, c_int, c_int, c_int64, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_int64, c_int, c_void_p, c_int64, c_void_p, c_size_t,
                                  c_void_p]),
    "smfv_plan_create": (c_int, [POINTER(c_void_p), c_int, c_int, c_int, c_int64, _PI, _PI, c_int,
                                 c_int]),
    "smfv_plan_create_rows": (c_int, [POINTER(c_void_p), c_int, c_int, c_int, c_int, _PI, _PI, c_int,
                                      c_int]),
    "smfv_plan_analyse": (c_int, [c_int, c_int, _PI, _PI, _PD]),
    "smfv_plan_analyse_rows": (c_int, [c_int, c_int, c_int, _PI, _PI, c_int, _PD]),
    "smfv_wsn_plan_analyse": (c_int, [c_int, c_int, c_int, _PI, _PI, c_int, _PD]),
    "smfv_spmv_chunks_analyse": (c_int, [c_int, c_int, c_int, _PI, _PI, c_int, _PD]),
    "smfv_set_analysis_threads": (None, [c_int]),
    "smfv_plan_bind_values": (c_int, [c_void_p, c_void_p, c_void_p]),
    "smfv_plan_execute": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                  c_void_p, c_int64, c_void_p]),
    "smfv_plan_stats": (c_int, [c_void_p, _PD]),
    "smfv_plan_destroy": (c_int, [c_void_p]),
    "smfv_spmm_rowblock_f64": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int64, c_int, c_void_p, c_int64, c_void_p]),
    "smfv_spmm_colpanel_f64": (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_int64, c_void_p, c_int64, c_void_p]),
    "smfv_nnz_range_rows": (c_int, [c_int, _PI, c_int64, c_int64, _PI, _PI]),
    "smfv_spmm_nnzrange_workspace_bytes": (c_int, [c_int, c_int64, c_int, POINTER(c_size_t)]),
    "smfv_spmm_nnzrange_f64": (c_int, [c_int, c_int, c_int64, c_int64, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int64,
                                       c_void_p, c_size_t, c_void_p]),
    "smfv_panels_to_rowmajor_f64": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int64,
                                            c_void_p]),
    "smfv_combine_row_blocks_f64": (c_int, [c_int, c_int, c_int, _PI, _PI, c_void_p, c_void_p,
                                            c_int64, c_void_p]),
    "smfv_compare_f64": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, _PD,
                                 c_void_p]),
    "smfv_fill_x_hash_f64": (c_int, [c_int64, c_int, c_uint64, c_void_p, c_int64, c_void_p]),
    "smfv_comm_unique_id": (c_int, [POINTER(c_char)]),
    "smfv_comm_init": (c_int, [POINTER(c_void_p), c_int, c_int, POINTER(c_char)]),
    "smfv_comm_destroy": (c_int, [c_void_p]),
    "smfv_comm_rank": (c_int, [c_void_p]),
    "smfv_comm_size": (c_int, [c_void_p]),
    "smfv_comm_count": (c_int, [c_void_p, _PI]),
    "smfv_comm_bcast": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "smfv_dist_workspace_bytes": (c_int, [c_void_p, c_int, c_int, c_int64, _PI, c_int,
                                          POINTER(c_size_t)]),
    "smfv_dist_plan": (c_int, [c_int, c_int, c_int64, _PI, c_int, c_int, _PI, _PI, _PI64,
                               _PI64]),
    "smfv_dist_spmm_f64": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int64, _PI,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "smfv_dist_rowpart_spmm_f64": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "smfv_dist_exchange_ops": (c_int, [c_int, c_int, c_int, c_int, c_int64, _PI, c_int, c_int, c_int, _PI, _PI,
                                       _PI64, _PI64, _PI]),
    "smfv_dist_plan_opts": (c_int, [c_int, c_int, c_int, c_int64, _PI, c_int, c_int, _PI, _PI, _PI64, _PI64]),
    "smfv_dist_chunk_rows": (c_int, [c_int, c_int, c_int, c_int64, _PI, c_int, c_int, c_int, _PI, _PI]),
    "smfv_dist_exchange_ops_opts": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int64, _PI, c_int, c_int, c_int,
                                            c_int, _PI, _PI, _PI64, _PI64, _PI]),
    "smfv_dist_plan_partition": (c_int, [c_void_p, _PI, _PI, _PI64, _PI64]),
    "smfv_dist_plan_shape": (c_int, [c_void_p, _PI, _PI, _PI]),
    "smfv_dist_plan_create": (c_int, [POINTER(c_void_p), c_void_p, c_int, c_int, c_int, c_int, c_int, c_int64,
                                      _PI, _PI, c_int, c_int]),
    "smfv_dist_plan_create_rowpart": (c_int, [POINTER(c_void_p), c_void_p, c_int, c_int, c_int, c_int, _PI, _PI,
                                              c_int, c_int]),
    "smfv_dist_plan_create_rank": (c_int, [POINTER(c_void_p), c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                           c_int64, _PI, _PI, c_int, c_int]),
    "smfv_dist_plan_exchange_buffer": (c_int, [c_void_p, POINTER(_PD), _PI64]),
    "smfv_comm_exchange_f64": (c_int, [c_void_p, _PI, _PI, _PI64, _PI64, c_int, c_void_p, c_void_p]),
    "smfv_test_fail_exchange": (None, [c_int]),
    "smfv_dist_plan_bind_values": (c_int, [c_void_p, c_void_p, c_void_p]),
    "smfv_dist_plan_execute": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "smfv_dist_plan_execute_local": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p]),
    "smfv_dist_plan_exchange": (c_int, [c_void_p, c_void_p, c_void_p]),
    "smfv_dist_plan_stats": (c_int, [c_void_p, _PD]),
    "smfv_dist_plan_destroy": (c_int, [c_void_p]),
    "smfv_stream_copy": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "smfv_stream_mix": (c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_int, c_void_p]),
    "smfv_vendor_spmm_create": (c_int, [c_void_p, c_int, c_int, c_int, c_int64, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int64, c_void_p]),
    "smfv_vendor_spmm_execute": (c_int, [c_void_p]),
    "smfv_vendor_spmm_destroy": (c_int, [c_void_p]),
    # smfv_host.h
    "smfv_free": (None, [c_void_p]),
    "smfv_mtx_read": (c_int, [c_char_p, _PI, _PI, _PI64, POINTER(_PI), POINTER(_PI),
                              POINTER(_PD)]),
    "smfv_mtx_write": (c_int, [c_char_p, c_int, c_int, _PI, _PI, _PD, c_int]),
    "smfv_fatvector_rand": (None, [c_int64, c_int, _PD]),
    "smfv_csr_write_bin": (c_int, [c_char_p, c_int, c_int, _PI, _PI, _PD]),
    "smfv_csr_read_bin": (c_int, [c_char_p, _PI, _PI, _PI64, POINTER(_PI), POINTER(_PI),
                                  POINTER(_PD)]),
    "smfv_dense_write_bin": (c_int, [c_char_p, c_int64, c_int64, _PD]),
    "smfv_gen_fem27": (c_int, [c_int, c_int, c_int, c_double, c_uint64, _PI64, POINTER(_PI),
                               POINTER(_PI), POINTER(_PD)]),
    "smfv_gen_knn3d": (c_int, [c_int, c_int64, c_uint64, _PI64, POINTER(_PI), POINTER(_PI), POINTER(_PD)]),
    "smfv_gen_random_rows": (c_int, [c_int64, c_int64, c_int64, c_int64, c_double, c_double,
                                     c_int, c_uint64, _PI64, POINTER(_PI), POINTER(_PI),
                                     POINTER(_PD)]),
}


def _load() -> ctypes.CDLL:
    # torch bundles its own ROCm runtime (libamdhip64.so.7, librccl.so.1,
    # libhsa-runtime64.so.1).  Importing it FIRST makes libsmfv.so's NEEDED
    # sonames bind to those already-loaded copies, so the process has one HIP
    # runtime and one RCCL (two copies corrupt the heap at exit).
    import torch  # noqa: F401

    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C sparsematrixmultiplicationmpi_amd/csrc). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None and os.environ.get("SMFV_LIB"):
            continue  # an older build loaded for an A/B run lacks newer entry points
        if fn is None:
            raise ImportError(f"{LIB_PATH} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    msg = lib.smfv_last_error()
    return msg.decode() if msg else ""


def check(fn_name: str, status: int) -> None:
    if status != SMFV_OK:
        raise SmfvError(fn_name, status, last_error())


def call(fn_name: str, *args) -> None:
    check(fn_name, getattr(lib, fn_name)(*args))


def exported_symbols() -> list[str]:
    return list(_SIGS)
