"""(r4) Golden fixtures at SURVEY.md 8(c)'s sizes, from the REFERENCE itself.

Two patterns, each run through the reference's four kernels compiled
unmodified (oracle/_ref/ref_driver, oracle/Makefile target `ref`) under
MPICH's mpiexec at p in {1, 2, 3, 8} and K in {1, 3, 32, 128}, X = the
reference driver's own fat vector (glibc rand()%100+1, seed 1):

  sym2k    2,048 x 2,048 random symmetric (a banded random pattern plus its
           transpose, diagonal added), values k / 7, k = 1..9
  plaw20k  20,000 x 20,000, power-law row lengths (alpha 2, 8..600, mean
           ~16) with columns drawn in a window of +-max(40, L/2 + 1) around
           the row: short rows re-use X rows (the tiled plan takes them, in
           several XCD parts) and rows with more than 239 distinct columns
           are the plan's direct rows; values k / 7, k = +-1..9

The results are too large to store whole under ~1 MB, so a fixture holds
the inputs (compactly: row lengths, int16 column offsets from the row,
int8 values) and, per K, the sha256 of the reference's Y bytes:
  sha_seq_k{K}                  its sequential result
  sha_row_k{K}_p{p}, sha_col... its RowWise / ColumnWise result at p ranks
                                (asserted here equal to sha_seq_k{K})
  nnzx_idx_k{K}_p{p}, nnzx_xor  its NonZeroElement result at p ranks, as
                                the 64-bit XOR with the sequential result
                                at the flat indices where they differ
                                (the reference's Y_nnz = Y_seq ^ mask, exact)
Re-run with:

    make -C oracle all ref && python tests/golden/make_golden_large.py
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402  (checker-side code only)
from sparsematrixmultiplicationmpi_amd import inputs  # noqa: E402  (input synthesis only)

MPIEXEC = "/opt/conda/bin/mpiexec"
KS = (1, 3, 32, 128)
PS = (1, 2, 3, 8)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def sym2k(rng):
    m = 2048
    rows, cols = [], []
    for i in range(m):
        k = rng.integers(2, 9)
        c = np.clip(i + rng.integers(-64, 65, k), 0, m - 1)
        rows += [i] * len(c)
        cols += list(c)
    r = np.array(rows + cols + list(range(m)))
    c = np.array(cols + rows + list(range(m)))
    key = np.unique(r.astype(np.int64) * m + c)
    r, c = key // m, key % m
    lens = np.bincount(r, minlength=m)
    off = (c - r).astype(np.int16)
    vals = rng.integers(1, 10, key.size).astype(np.int8)
    return m, m, lens.astype(np.int16), off, vals


def plaw20k(rng):
    m = 20000
    u = rng.random(m)
    L = np.minimum(600, np.floor(8 / np.sqrt(1 - u))).astype(np.int64)  # alpha 2 tail from 8
    lens, offs = [], []
    for i in range(m):
        w = max(40, (int(L[i]) + 1) // 2 + 1)  # a window the row's columns fill, at least +-40
        lo, hi = max(0, i - w), min(m, i + w + 1)
        k = min(int(L[i]), hi - lo)
        c = np.sort(rng.choice(np.arange(lo, hi), k, replace=False))
        lens.append(k)
        offs.append((c - i).astype(np.int16))
    off = np.concatenate(offs)
    vals = rng.integers(1, 10, off.size) * rng.choice([-1, 1], off.size)
    return m, m, np.array(lens, np.int16), off, vals.astype(np.int8)


def expand(m, n, lens, off, vals):
    """The CSR a fixture's compact inputs stand for (tests/conftest.load_golden_large)."""
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum(lens.astype(np.int64))
    row = np.repeat(np.arange(m, dtype=np.int64), lens.astype(np.int64))
    ci = (row + off.astype(np.int64)).astype(np.int32)
    # values k / 7 (k = the stored int8): not dyadic, so products and sums
    # round and NonZeroElement's reassociation shows in the last bits
    return inputs.SparseMatrix(vals.astype(np.float64) / 7.0, ci, rp, m, n)


def run_ref(tmp, A, K, p):
    csr = os.path.join(tmp, "a.bin")
    inputs.write_csr_bin(csr, A)
    subprocess.run([MPIEXEC, "-n", str(p), oracle.REF_DRIVER, csr, str(K), "--out", os.path.join(tmp, "y")],
                   check=True, capture_output=True, text=True)
    return {k: inputs.read_dense_bin(os.path.join(tmp, f"y.{k}.bin")) for k in ("seq", "row", "col", "nnz")}


def case(name, gen, rng, manifest):
    m, n, lens, off, vals = gen(rng)
    A = expand(m, n, lens, off, vals)
    data = dict(m=np.int64(m), n=np.int64(n), lens=lens, off=off, vals=vals)
    info = {"m": m, "n": n, "nnz": int(A.rowPtr[-1]), "K": list(KS), "p": list(PS),
            "x": "glibc rand()%100+1 (reference driver)",
            "a_sha": hashlib.sha256(A.rowPtr.tobytes() + A.colIndices.tobytes() + A.values.tobytes()).hexdigest(),
            "max_row": int(lens.max())}
    with tempfile.TemporaryDirectory() as tmp:
        for K in KS:
            y_seq = None
            for p in PS:
                res = run_ref(tmp, A, K, p)
                if y_seq is None:
                    y_seq = res["seq"]
                    data[f"sha_seq_k{K}"] = np.array(sha(y_seq))
                    info[f"x_sha_k{K}"] = sha(oracle.fatvector_rand(n, K))
                assert np.array_equal(res["seq"].view(np.uint64), y_seq.view(np.uint64))
                assert sha(res["row"]) == sha(y_seq) and sha(res["col"]) == sha(y_seq), (name, K, p)
                data[f"sha_row_k{K}_p{p}"] = np.array(sha(res["row"]))
                data[f"sha_col_k{K}_p{p}"] = np.array(sha(res["col"]))
                x = (res["nnz"].view(np.uint64) ^ y_seq.view(np.uint64)).reshape(-1)
                idx = np.flatnonzero(x)
                data[f"nnzx_idx_k{K}_p{p}"] = idx.astype(np.int64)
                data[f"nnzx_xor_k{K}_p{p}"] = x[idx]
                info[f"nnz_rows_differing_k{K}_p{p}"] = int(np.unique(idx // K).size)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **data)
    with open(path, "rb") as f:
        info["sha256"] = hashlib.sha256(f.read()).hexdigest()
    info["bytes"] = os.path.getsize(path)
    manifest[name] = info
    print(name, {k: v for k, v in info.items() if not k.startswith("nnz_rows")})


def main():
    if not os.path.exists(oracle.REF_DRIVER):
        raise SystemExit("build the reference driver first: make -C oracle ref")
    manifest = {}
    case("sym2k", sym2k, np.random.default_rng(2048), manifest)
    case("plaw20k", plaw20k, np.random.default_rng(20000), manifest)
    with open(os.path.join(HERE, "manifest_large.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
