#!/usr/bin/env python3
"""Kernel lab: time the shipped kernels on ablated inputs to locate the
bottleneck (not part of the product or the bench).

Cases (all m = 121,192, ~21.65 nnz/row, K = 32 unless noted):
  surrogate      cop20k_A surrogate as benched
  diag_cols      same row lengths, every column index = the row itself
                 (X gather always hits one L1-resident row: CSR/Y/issue floor)
  uniform_cols   same row lengths, uniform random columns (no locality)
  rcm_shuffle    surrogate with rows/cols randomly permuted
Prints median kernel time (HIP events around each launch, warm and rotated).
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sparsematrixmultiplicationmpi_amd as smfv  # noqa: E402


def timeit(plan, X, Y, reps=100, copies=None):
    st = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for i in range(10):
        plan.run(X, Y)
    torch.cuda.synchronize()
    for i in range(reps):
        evs[2 * i].record(st)
        if copies:
            p, x, y = copies[i % len(copies)]
            p.run(x, y)
        else:
            plan.run(X, Y)
        evs[2 * i + 1].record(st)
    torch.cuda.synchronize()
    t = sorted(evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(reps))
    return t[len(t) // 2] * 1e3  # us


def variants(A, K, dev, variant=smfv.Variant.ROWWISE, ncopies=8):
    X = torch.from_numpy(smfv.generateLargeFatVector(A.numCols, K)).to(dev)
    copies = []
    for _ in range(ncopies):
        dA = smfv.DeviceCSR(A, dev)
        copies.append((smfv.SpmmPlan(variant, dA, K, tiles=os.environ.get("LAB_TILES", "auto")), X.clone(), torch.empty((A.numRows, K), dtype=torch.float64, device=dev)))
    p, x, y = copies[0]
    warm = timeit(p, x, y)
    cold = timeit(p, x, y, copies=copies)
    return warm, cold


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    A = smfv.cop20k_surrogate()
    m, nnz = A.numRows, A.nnz
    rng = np.random.default_rng(0)
    rows = np.repeat(np.arange(m, dtype=np.int32), np.diff(A.rowPtr))
    res = {}

    def rec(name, B, K=32, variant=smfv.Variant.ROWWISE):
        w, c = variants(B, K, dev, variant)
        alg = 12 * B.nnz + 4 * (B.numRows + 1) + 8 * B.numCols * K + 8 * B.numRows * K
        res[name] = {"warm_us": round(w, 2), "cold_us": round(c, 2),
                     "cold_GBps": round(alg / (c * 1e-6) / 1e9, 1), "warm_GBps": round(alg / (w * 1e-6) / 1e9, 1)}
        print(name, res[name], flush=True)

    rec("surrogate_k32", A)
    D = smfv.SparseMatrix(A.values, rows.copy(), A.rowPtr, m, m)
    rec("diag_cols_k32", D)
    U = smfv.SparseMatrix(A.values, np.sort(rng.integers(0, m, nnz).astype(np.int32)), A.rowPtr, m, m)
    # sort within rows
    ci = U.colIndices.copy()
    for_sort = np.lexsort((rng.integers(0, m, nnz), rows))
    ci = rng.integers(0, m, nnz).astype(np.int32)
    order = np.lexsort((ci, rows))
    U = smfv.SparseMatrix(A.values, ci[order], A.rowPtr, m, m)
    rec("uniform_cols_k32", U)
    rec("surrogate_k128", A, 128)
    rec("surrogate_k1", A, 1)
    rec("surrogate_k32_nonzero", A, 32, smfv.Variant.NONZERO)
    rec("surrogate_k32_columnwise", A, 32, smfv.Variant.COLUMNWISE)
    # column-window: colIdx confined to a 2048-row window around the row
    W = np.clip(rows + (A.colIndices - rows) // 4, 0, m - 1).astype(np.int32)
    order = np.lexsort((W, rows))
    rec("narrow_band_k32", smfv.SparseMatrix(A.values, W[order], A.rowPtr, m, m))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
