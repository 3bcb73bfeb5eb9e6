"""Row samples for checking full-size results (BASELINE configs 4-5) where
the whole reference result is too large to compute on the host.

Pure index selection over a CSR row_ptr -- no arithmetic on values: the
tests pass the sampled rows to their CPU checker, bench.py to its own
small checker.  The sample holds the rows where the kernels' edge cases live:

  * the longest rows (a power-law row is split across many merge-path teams),
  * every row open at a merge-path team boundary (its sum is finished by the
    carry fix-up: k_merge_flat / k_carry_fixup, SC/...NonZeroElement.cpp:88's
    role), from the library's own merge geometry (smfv_merge_geometry),
  * empty rows, the first and last rows, and uniformly random rows.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import call


def merge_geometry(nrows: int, nnz: int, K: int) -> tuple[int, int, int]:
    out = (ctypes.c_int64 * 3)()
    call("smfv_merge_geometry", nrows, nnz, K, out)
    return int(out[0]), int(out[1]), int(out[2])


def merge_boundary_rows(row_ptr: np.ndarray, K: int) -> np.ndarray:
    """Rows open at a merge-path team boundary (diagonal t * ipt): row i is
    at diagonal d when end(i) + i >= d > end(i - 1) + i - 1."""
    rp = np.asarray(row_ptr, dtype=np.int64)
    m = len(rp) - 1
    items, ipt, nteams = merge_geometry(m, int(rp[-1]), K)
    d = np.arange(1, nteams, dtype=np.int64) * ipt
    key = rp[1:] + np.arange(m, dtype=np.int64)  # end(i) + i, strictly increasing
    rows = np.searchsorted(key, d, side="left")
    return np.unique(rows[rows < m])


def sample_rows(row_ptr: np.ndarray, K: int, n_random: int = 2000, n_longest: int = 200,
                max_boundary: int = 4000, seed: int = 0) -> np.ndarray:
    rp = np.asarray(row_ptr, dtype=np.int64)
    m = len(rp) - 1
    if m == 0:
        return np.zeros(0, np.int64)
    lens = np.diff(rp)
    rng = np.random.default_rng(seed)
    parts = [np.array([0, m - 1]),
             np.argsort(lens, kind="stable")[-n_longest:],
             np.flatnonzero(lens == 0)[:200],
             rng.integers(0, m, n_random)]
    b = merge_boundary_rows(rp, K)
    if len(b) > max_boundary:
        b = np.concatenate([b[:max_boundary // 2], rng.choice(b, max_boundary // 2, replace=False)])
    parts.append(b)
    return np.unique(np.concatenate(parts).astype(np.int64))


def sub_csr(row_ptr: np.ndarray, col_idx: np.ndarray, values: np.ndarray, rows: np.ndarray):
    """The sampled rows as a compact CSR over the columns they touch:
    (row_ptr, local col ids, values, the global columns)."""
    rp = np.asarray(row_ptr, dtype=np.int64)
    lens = rp[rows + 1] - rp[rows]
    srp = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=srp[1:])
    idx = np.repeat(rp[rows] - srp[:-1], lens) + np.arange(srp[-1])
    cols = np.asarray(col_idx)[idx]
    ucols, local = np.unique(cols, return_inverse=True)
    return srp.astype(np.int32), local.astype(np.int32), np.asarray(values)[idx], ucols
