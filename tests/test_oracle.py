"""Pin the CPU oracle against the REFERENCE's own outputs (tests/golden,
produced by the reference's kernel sources compiled unmodified; see
tests/golden/make_golden.py) and against known-answer Matrix Market reads."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_cases, load_golden
from oracle import oracle

CASES = sorted(golden_cases())


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def test_manifest_hashes():
    for name, info in golden_cases().items():
        with open(os.path.join(GOLDEN, f"{name}.npz"), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == info["sha256"], name


@pytest.mark.parametrize("name", CASES)
def test_oracle_sequential_bitwise(name):
    g = load_golden(name)
    Y = oracle.spmm("sequential", g["row_ptr"], g["col_idx"], g["values"], g["X"])
    assert np.array_equal(Y.view(np.uint64), g["Y_seq"].view(np.uint64))


@pytest.mark.parametrize("name", CASES)
def test_oracle_rowwise_columnwise_bitwise(name):
    g = load_golden(name)
    info = golden_cases()[name]
    for p in info["p"]:
        Yr = oracle.spmm("rowwise", g["row_ptr"], g["col_idx"], g["values"], g["X"], p)
        Yc = oracle.spmm("columnwise", g["row_ptr"], g["col_idx"], g["values"], g["X"], p)
        assert sha(Yr) == str(g[f"sha_row_p{p}"]), (name, p)
        assert sha(Yc) == str(g[f"sha_col_p{p}"]), (name, p)


@pytest.mark.parametrize("name", CASES)
def test_oracle_nonzero(name):
    """NonZeroElement: bitwise at p = 1 and p = 2 (a two-operand sum has one
    association); for p > 2 the reference's MPICH reduce association is not
    restated, so compare within 1e-12 relative to sum |a||x|."""
    g = load_golden(name)
    info = golden_cases()[name]
    absY = oracle.spmm("sequential", g["row_ptr"], g["col_idx"], np.abs(g["values"]), np.abs(g["X"]))
    for p in info["p"]:
        Yz = oracle.spmm("nonzero", g["row_ptr"], g["col_idx"], g["values"], g["X"], p)
        ref = g[f"Y_nnz_p{p}"]
        if p <= 2:
            assert np.array_equal(Yz.view(np.uint64), ref.view(np.uint64)), (name, p)
        else:
            assert oracle.max_rel_err(Yz, ref, absY) <= 1e-12, (name, p)


def test_fatvector_rand_matches_reference_driver():
    # cases whose X came from the reference driver's rand()%100+1
    for name, info in golden_cases().items():
        if info["x"].startswith("glibc"):
            g = load_golden(name)
            X = oracle.fatvector_rand(int(g["n"]), int(g["X"].shape[1]))
            assert np.array_equal(X, g["X"]), name
    assert oracle.fatvector_rand(1, 2).tolist() == [[84.0, 87.0]]


def test_partitions_match_reference_formulas():
    # RowWise.cpp:26-29, ColumnWise.cpp:25-28, NonZeroElement.cpp:24-39
    for m in (0, 1, 5, 7, 121192):
        for p in (1, 2, 3, 8, 9):
            got = [oracle.partition_rows(m, p, r) for r in range(p)]
            q, ex = divmod(m, p)
            exp = [(r * q + min(r, ex), r * q + min(r, ex) + q + (r < ex)) for r in range(p)]
            assert got == exp
            assert got[0][0] == 0 and got[-1][1] == m
    assert [oracle.partition_cols(3, 8, r) for r in range(8)] == [(0, 0)] * 7 + [(0, 3)]
    assert [oracle.partition_cols(32, 3, r) for r in range(3)] == [(0, 10), (10, 20), (20, 32)]
    assert [oracle.partition_nnz(10, 3, r) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]


# ---- Matrix Market reader known answers (SC/utils.cpp:70-185) ----------
def test_mtx_symmetric_known_answer():
    m, n, rp, ci, va = oracle.mtx_read(os.path.join(GOLDEN, "sym5.mtx"))
    assert (m, n) == (5, 5)
    assert rp.tolist() == [0, 3, 6, 7, 9, 11]
    assert ci.tolist() == [0, 1, 4, 0, 1, 3, 2, 1, 3, 0, 4]
    assert va.tolist() == [4.0, -1.5, 1e-3, -1.5, 3.25, 0.5, 2.0, 0.5, -7.0, 1e-3, 6.5]


def test_mtx_pattern_duplicates_known_answer():
    m, n, rp, ci, va = oracle.mtx_read(os.path.join(GOLDEN, "pat4x6.mtx"))
    assert (m, n) == (4, 6)
    assert rp.tolist() == [0, 2, 5, 5, 7]          # row 3 empty
    assert ci.tolist() == [0, 5, 1, 2, 2, 0, 4]    # duplicate (2,3) kept, rows sorted
    assert va.tolist() == [1.0] * 7


def test_mtx_general_unsorted_known_answer():
    m, n, rp, ci, va = oracle.mtx_read(os.path.join(GOLDEN, "empty7x5.mtx"))
    assert (m, n) == (7, 5)
    assert rp.tolist() == [0, 0, 2, 3, 3, 4, 6, 6]
    assert ci.tolist() == [0, 4, 2, 1, 0, 3]
    assert va.tolist() == [-2.0, 0.25, 1.5, 8.0, 3.0, -0.125]


def test_mtx_errors(tmp_path):
    with pytest.raises(ValueError):
        oracle.mtx_read(str(tmp_path / "missing.mtx"))
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1.0\n")
    with pytest.raises(ValueError):
        oracle.mtx_read(str(bad))


# ---- (r4) fixtures at SURVEY 8(c)'s sizes (tests/golden/make_golden_large.py) ----
from conftest import golden_large_cases, golden_large_nnz, load_golden_large, sha_f64  # noqa: E402

LARGE = sorted(golden_large_cases())


def test_large_manifest_hashes_and_sizes():
    for name, info in golden_large_cases().items():
        with open(os.path.join(GOLDEN, f"{name}.npz"), "rb") as f:
            b = f.read()
        assert hashlib.sha256(b).hexdigest() == info["sha256"], name
        assert len(b) < 1 << 20, name  # each under 1 MB
        A = load_golden_large(name)["A"]
        assert hashlib.sha256(A.rowPtr.tobytes() + A.colIndices.tobytes() + A.values.tobytes()).hexdigest() == \
            info["a_sha"], name


@pytest.mark.parametrize("name", LARGE)
def test_large_oracle_vs_reference(name):
    """The oracle against the reference's own results at 2k / 20k rows, K in
    {1, 3, 32, 128}, p in {1, 2, 3, 8}: sequential / RowWise / ColumnWise by
    the sha256 of the reference's bytes; NonZeroElement bitwise at p <= 2 and
    within 1e-12 x sum|a||x| beyond (the MPICH reduce association)."""
    g = load_golden_large(name)
    info = golden_large_cases()[name]
    A = g["A"]
    for K in info["K"]:
        X = oracle.fatvector_rand(A.numCols, K)  # the reference driver's X
        assert sha_f64(X) == info[f"x_sha_k{K}"]
        Y = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
        assert sha_f64(Y) == str(g[f"sha_seq_k{K}"]), (name, K)
        absY = oracle.spmm("sequential", A.rowPtr, A.colIndices, np.abs(A.values), X)
        for p in info["p"]:
            assert sha_f64(oracle.spmm("rowwise", A.rowPtr, A.colIndices, A.values, X, p)) == \
                str(g[f"sha_row_k{K}_p{p}"]), (name, K, p)
            assert sha_f64(oracle.spmm("columnwise", A.rowPtr, A.colIndices, A.values, X, p)) == \
                str(g[f"sha_col_k{K}_p{p}"]), (name, K, p)
            ref = golden_large_nnz(g, K, p, Y)
            Yz = oracle.spmm("nonzero", A.rowPtr, A.colIndices, A.values, X, p)
            if p <= 2:
                assert np.array_equal(Yz.view(np.uint64), ref.view(np.uint64)), (name, K, p)
            else:
                assert oracle.max_rel_err(Yz, ref, absY) <= 1e-12, (name, K, p)
