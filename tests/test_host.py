"""CPU-only tests of the product's host side: the C ABI library loads and
exports every symbol the headers declare, partitions / plans / reader /
fat-vector / generators agree with the oracle and the reference fixtures.
No device calls here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden_cases, load_golden
from oracle import oracle

import sparsematrixmultiplicationmpi_amd as smfv
from sparsematrixmultiplicationmpi_amd import _lib, inputs
from sparsematrixmultiplicationmpi_amd.dist import exchange_plan

INCLUDE = os.path.join(ROOT, "include")
PKG = os.path.join(ROOT, "sparsematrixmultiplicationmpi_amd")


def header_symbols(header):
    src = open(os.path.join(INCLUDE, header)).read()
    return set(re.findall(r"SMFV_API\s+[\w\s\*]+?\b(smfv_\w+)\s*\(", src))


def test_c_abi_exports_every_declared_symbol():
    declared = header_symbols("smfv.h") | header_symbols("smfv_host.h")
    assert len(declared) >= 30
    nm = subprocess.run(["nm", "-D", "--defined-only", os.path.join(PKG, "libsmfv.so")],
                        capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (smfv_\w+)", nm))
    assert declared <= exported, declared - exported
    # and the ctypes binding covers all of them
    assert declared <= set(_lib.exported_symbols())
    assert _lib.lib.smfv_version().decode().startswith("smfv")


def test_dropin_library_exports_reference_surface():
    nm = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(PKG, "libsmfv_mpi.so")],
                        capture_output=True, text=True, check=True).stdout
    for sym in ("sparseMatrixFatVectorMultiply(SparseMatrix const&",
                "sparseMatrixFatVectorMultiplyRowWise(SparseMatrix const&",
                "sparseMatrixFatVectorMultiplyColumnWise(SparseMatrix const&",
                "sparseMatrixFatVectorMultiplyNonZeroElement(SparseMatrix const&",
                "readMatrixMarketFile(", "generateLargeFatVector(int, int)", "areMatricesEqual(",
                "serialize(", "deserialize("):
        assert sym in nm, sym
    assert os.access(os.path.join(PKG, "smfv_main"), os.X_OK)


def _part(fn, *args):
    a, b = (ctypes.c_int64(), ctypes.c_int64()) if fn == "smfv_partition_nnz" else (ctypes.c_int(), ctypes.c_int())
    getattr(_lib.lib, fn)(*args, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def test_partitions_equal_oracle():
    for m in (0, 1, 3, 8, 100, 121192):
        for p in (1, 2, 3, 7, 8, 64):
            for r in range(p):
                assert _part("smfv_partition_rows", m, p, r) == oracle.partition_rows(m, p, r)
                assert _part("smfv_partition_cols", m, p, r) == oracle.partition_cols(m, p, r)
                assert _part("smfv_partition_nnz", m * 7, p, r) == oracle.partition_nnz(m * 7, p, r)


@pytest.mark.parametrize("variant", [1, 2, 3])
@pytest.mark.parametrize("p", [1, 2, 3, 8, 13])
def test_exchange_plan_covers_output(variant, p):
    A = smfv.gen_random_rows(700, 500, 6, 2.0, 200, 5)
    # add empty rows at both ends and in the middle
    lens = np.diff(A.rowPtr)
    lens[[0, 1, 350, 699]] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    K = 5
    first, last, off, cnt = exchange_plan(variant, 700, int(rp[-1]), rp, K, p)
    if variant == 1:   # rows tile [0, m)
        assert first[0] == 0 and last[-1] == 699
        assert np.all(first[1:] == last[:-1] + 1)
        assert np.all(off == first * K) and np.all(cnt == (last - first + 1) * K)
    elif variant == 2:  # columns tile [0, K), panels back to back
        assert first[0] == 0 and last[-1] == K - 1
        assert np.all(off == 700 * first)
        assert cnt.sum() == 700 * K
    else:              # nnz ranges: touched rows, consecutive compact blocks
        nnz = int(rp[-1])
        for r in range(p):
            s, e = oracle.partition_nnz(nnz, p, r)
            if e > s:
                assert rp[first[r]] <= s < rp[first[r] + 1]
                assert rp[last[r]] <= e - 1 < rp[last[r] + 1]
            else:
                assert cnt[r] == 0
        assert np.all(off[1:] == off[:-1] + cnt[:-1])
        # every non-empty row is covered by some rank
        covered = np.zeros(700, bool)
        for r in range(p):
            covered[first[r]:last[r] + 1] = True
        assert np.all(covered[lens > 0])


def test_host_reader_matches_oracle_and_golden():
    for f in ("sym5.mtx", "pat4x6.mtx", "empty7x5.mtx"):
        A = smfv.readMatrixMarketFile(os.path.join(GOLDEN, f))
        m, n, rp, ci, va = oracle.mtx_read(os.path.join(GOLDEN, f))
        assert (A.numRows, A.numCols) == (m, n)
        assert np.array_equal(A.rowPtr, rp) and np.array_equal(A.colIndices, ci)
        assert np.array_equal(A.values, va)


def test_host_reader_roundtrip_and_errors(tmp_path):
    A = smfv.gen_fem27(500, 8, 8, 0.8, 3)
    p = tmp_path / "a.mtx"
    smfv.writeMatrixMarketFile(str(p), A, symmetric=True)
    B = smfv.readMatrixMarketFile(str(p))
    assert np.array_equal(A.rowPtr, B.rowPtr) and np.array_equal(A.colIndices, B.colIndices)
    assert np.array_equal(A.values, B.values)
    m, n, rp, ci, va = oracle.mtx_read(str(p))
    assert np.array_equal(rp, B.rowPtr) and np.array_equal(va, B.values)
    with pytest.raises(smfv.SmfvError):
        smfv.readMatrixMarketFile(str(tmp_path / "missing.mtx"))
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix coordinate real general\n\n2 2 1\n1 1 1\n")
    with pytest.raises(smfv.SmfvError):   # blank size line: UB in the reference, error here
        smfv.readMatrixMarketFile(str(bad))


def test_fatvector_matches_reference_rand():
    for name, info in golden_cases().items():
        if info["x"].startswith("glibc"):
            g = load_golden(name)
            assert np.array_equal(smfv.generateLargeFatVector(int(g["n"]), g["X"].shape[1]), g["X"])
    X = smfv.generateLargeFatVector(3000, 7)
    assert np.array_equal(X, oracle.fatvector_rand(3000, 7))


def test_serialize_roundtrip():
    fat = [[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]]
    flat = smfv.serialize(fat)
    assert flat.tolist() == [1, 2, 3, 4, 5, 6]
    assert smfv.deserialize(flat, 2, 3).tolist() == fat
    assert smfv.areMatricesEqual(fat, [[1.0, 2.0, 3.0], [4.0, 5.0, 6.0 + 1e-7]], 1e-6)
    assert not smfv.areMatricesEqual(fat, [[1.0, 2.0, 3.0], [4.0, 5.0, 6.1]], 1e-6)
    assert not smfv.areMatricesEqual(fat, [[1.0, 2.0, 3.0]], 1e-6)


def test_generators():
    A = smfv.cop20k_surrogate()
    A.validate()
    assert A.numRows == smfv.COP20K_M and abs(A.nnz - smfv.COP20K_NNZ) < 100
    # exactly symmetric
    import scipy.sparse as sp
    M = sp.csr_matrix((A.values, A.colIndices, A.rowPtr), shape=(A.numRows, A.numCols))
    assert (M != M.T).nnz == 0
    # sorted, distinct columns per row; deterministic
    B = smfv.gen_random_rows(20000, 30000, 16, 2.0, 4096, 9)
    B.validate()
    d = np.diff(B.colIndices)
    starts = B.rowPtr[1:-1]
    mask = np.ones(len(d), bool)
    mask[starts[starts < len(d) + 1] - 1] = False
    assert np.all(d[mask] > 0)
    C = smfv.gen_random_rows(20000, 30000, 16, 2.0, 4096, 9)
    assert np.array_equal(B.colIndices, C.colIndices) and np.array_equal(B.values, C.values)
    assert 14 < B.nnz / B.numRows < 18
    # a row block equals the same rows of the whole matrix
    blk = smfv.gen_random_rows(20000, 30000, 16, 2.0, 4096, 9, 5000, 6000)
    assert np.array_equal(blk.colIndices, B.colIndices[B.rowPtr[5000]:B.rowPtr[6000]])
    U = smfv.gen_random_rows(1000, 1000, 16, 0.0, 16, 1)
    assert np.all(np.diff(U.rowPtr) == 16)


def test_csr_bin_roundtrip(tmp_path):
    A = smfv.gen_fem27(300, 7, 7, 0.7, 2)
    p = str(tmp_path / "a.bin")
    inputs.write_csr_bin(p, A)
    B = inputs.read_csr_bin(p)
    assert np.array_equal(A.rowPtr, B.rowPtr) and np.array_equal(A.values, B.values)


def test_product_has_no_oracle_dependency():
    """The product never imports, links or calls the oracle."""
    for dirpath, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", "Makefile")):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.lower().replace("oracle_", ""), f
    nm = subprocess.run(["nm", "-D", os.path.join(PKG, "libsmfv.so")], capture_output=True, text=True).stdout
    assert "oracle_" not in nm


def _analyse(A):
    out = (ctypes.c_double * 6)()
    ip = ctypes.POINTER(ctypes.c_int)
    _lib.call("smfv_plan_analyse", A.numRows, A.numCols, A.rowPtr.ctypes.data_as(ip),
              A.colIndices.ctypes.data_as(ip), out)
    return list(out)


def test_tile_analysis_invariants_and_reuse():
    """Clustered row tiles: the native analysis verifies its own invariants
    (every row in one tile, caps, CSR order, union positions) and reports
    re-use; adjacency clustering must beat runs of consecutive rows."""
    tiles, staged, reuse, direct, padded, tiled_nnz = _analyse(smfv.cop20k_surrogate())
    assert reuse > 4.0 and direct == 0 and padded % 8 == 0
    # wide rows become direct tiles, random patterns have no re-use
    B = smfv.gen_random_rows(20000, 20000, 16, 2.0, 4096, 42)
    tiles, staged, reuse, direct, padded, tiled_nnz = _analyse(B)
    assert direct > 0 and reuse < 1.5
    # empty rows, rectangular, duplicates
    A = smfv.readMatrixMarketFile(os.path.join(GOLDEN, "pat4x6.mtx"))
    assert _analyse(A)[0] >= 1
    A = smfv.readMatrixMarketFile(os.path.join(GOLDEN, "empty7x5.mtx"))
    assert _analyse(A)[0] >= 1


def _analyse_rows(A, r0, r1, flags=0):
    out = (ctypes.c_double * 9)()
    ip = ctypes.POINTER(ctypes.c_int)
    _lib.call("smfv_plan_analyse_rows", r0, r1, A.numCols, A.rowPtr.ctypes.data_as(ip),
              A.colIndices.ctypes.data_as(ip), flags, out)
    return {"tiles": out[0], "reuse": out[2], "direct": out[3], "parts": int(out[6]),
            "footprint": out[7], "xcd_footprint": out[8]}


def test_ws_plan_tiny_and_empty_rows():
    """The headline kernel's tile plan (built and verified natively) on tiny
    and empty-row patterns: a tile of empty rows stages no values (a quad's
    last batch stores only the value pairs its rows sum), and the value
    entries never exceed 8 per non-zero rounded up per batch."""
    for name in ("empty7x5.mtx", "pat4x6.mtx"):
        A = smfv.readMatrixMarketFile(os.path.join(GOLDEN, name))
        out = (ctypes.c_double * 9)()
        ip = ctypes.POINTER(ctypes.c_int)
        _lib.call("smfv_plan_analyse_rows", 0, A.numRows, A.numCols, A.rowPtr.ctypes.data_as(ip),
                  A.colIndices.ctypes.data_as(ip), 0, out)
        assert out[0] >= 1, name
        nnz = int(A.rowPtr[-1])
        assert out[5] == nnz and out[4] % 8 == 0 and nnz <= out[4] <= 32 * A.numRows, (name, list(out))


def test_ws_geometry2_plans_verify():
    """(r4) Geometry 2 of k_rows_ws (two 512-lane pipelines per CU,
    SMFV_PLAN_WS_GEOM2): tiles of <= 32 rows and <= 125 staged X rows, built
    and verified natively (the replay of the kernel's reads, with its 32-slot
    record and 4 loader waves) on the stand-ins and on tiny, empty-row and
    unsorted patterns.  Geometry 1 stays what it was."""
    G1, G2 = 1024, 2048  # SMFV_PLAN_WS_GEOM1 / GEOM2
    A = smfv.cop20k_surrogate()
    g1, g2 = _analyse_rows(A, 0, A.numRows, G1), _analyse_rows(A, 0, A.numRows, G2)
    assert g1 == _analyse_rows(A, 0, A.numRows)  # the default is geometry 1
    # (r5) row pairs: 1906 tiles, 8 rounds per block as 2011 tiles of one row
    # per team, so the automatic choice keeps one row per team
    assert _analyse_rows(A, 0, A.numRows, G1 | ROW_PAIRS)["tiles"] == 1906
    assert g1["tiles"] == 2011 == _analyse_rows(A, 0, A.numRows, G1 | SINGLE_ROWS)["tiles"] and g2["direct"] == 0
    assert 2.4 * g1["tiles"] < g2["tiles"] < 2.7 * g1["tiles"] and g2["reuse"] > 4.0
    for name in ("empty7x5.mtx", "pat4x6.mtx"):
        B = smfv.readMatrixMarketFile(os.path.join(GOLDEN, name))
        assert _analyse_rows(B, 0, B.numRows, G2)["tiles"] >= 1, name
    # a row block starting mid-matrix (a rank's share)
    assert _analyse_rows(A, 50_000, 70_000, G2)["tiles"] >= 20_000 / 32


SINGLE_ROWS, ROW_PAIRS = 16384, 32768  # SMFV_PLAN_SINGLE_ROWS / SMFV_PLAN_ROW_PAIRS


def test_row_pair_tiles_on_host():
    """(r5) Row pairs (SMFV_PLAN_ROW_PAIRS; SMFV_PLAN_SINGLE_ROWS one row
    per team; neither: the plan whose busiest block runs fewer tiles): a
    k_rows_ws tile holds up to twice its teams in rows, the shortest riding
    as second rows, and the native replay of the kernel's reads verifies
    every plan (a failed check fails the call).  Short-row patterns stop at
    the X-row cap instead of the row count: about half the tiles on a
    0-7-entry band, 19 % fewer on the irregular cop20k_A stand-in (10 -> 8
    rounds: the automatic choice pairs); geometries 1 / 2 / 3, a row block
    starting mid-matrix, tiny patterns."""
    from conftest import short_rows_band
    A = short_rows_band(20000, 3)
    for g in (1024, 2048, 4096):
        pr, one = _analyse_rows(A, 0, A.numRows, g | ROW_PAIRS), _analyse_rows(A, 0, A.numRows, g | SINGLE_ROWS)
        assert pr["direct"] == one["direct"] == 0
        assert pr["tiles"] <= 0.55 * one["tiles"] and pr["reuse"] > one["reuse"], (g, pr, one)
        assert _analyse_rows(A, 0, A.numRows, g) == pr  # fewer rounds: the automatic choice pairs
    pr, one = _analyse_rows(A, 777, 15000, ROW_PAIRS), _analyse_rows(A, 777, 15000, SINGLE_ROWS)
    assert pr["tiles"] <= 0.55 * one["tiles"]
    B = smfv.inputs.cop20k_irregular_surrogate()
    pr, one = _analyse_rows(B, 0, B.numRows, ROW_PAIRS), _analyse_rows(B, 0, B.numRows, SINGLE_ROWS)
    assert one["tiles"] == 2441 and pr["tiles"] <= 0.85 * one["tiles"] and pr["direct"] == 0, (pr, one)
    assert _analyse_rows(B, 0, B.numRows) == pr
    # live-values plans pair rows too (the second row's odd-length flag and
    # value slots replayed): the same tiles as the snapshot plan
    LIVE = 8192  # SMFV_PLAN_LIVE_VALUES
    for M, r0, r1 in ((A, 0, A.numRows), (A, 777, 15000), (B, 0, B.numRows)):
        assert _analyse_rows(M, r0, r1, LIVE | ROW_PAIRS)["tiles"] == _analyse_rows(M, r0, r1, ROW_PAIRS)["tiles"]
    for name in ("empty7x5.mtx", "pat4x6.mtx", "sym5.mtx"):
        C = smfv.readMatrixMarketFile(os.path.join(GOLDEN, name))
        assert _analyse_rows(C, 0, C.numRows)["tiles"] >= 1, name
        assert _analyse_rows(C, 0, C.numRows, LIVE | ROW_PAIRS)["tiles"] >= 1, name


def test_tile_analysis_unsorted_rows_with_repeats():
    """a row whose repeated column is not adjacent (unsorted CSR
    rows) must not undercount the tile's union; the plan still verifies
    (every row's entries in CSR order) in both geometries."""
    rng = np.random.default_rng(5)
    m = 3000
    rows = []
    for r in range(m):
        cols = [(r + d) % m for d in (-2, -1, 0, 1, 2)] + [(r + 1) % m, (r - 2) % m]  # repeats, unsorted
        rng.shuffle(cols)
        rows.append(cols)
    rp = np.zeros(m + 1, dtype=np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    ci = np.concatenate(rows).astype(np.int32)
    out = (ctypes.c_double * 9)()
    ip = ctypes.POINTER(ctypes.c_int)
    for flags in (1024, 2048):
        _lib.call("smfv_plan_analyse_rows", 0, m, m, rp.ctypes.data_as(ip), ci.ctypes.data_as(ip), flags, out)
        assert out[0] >= 1 and out[5] == len(ci), (flags, list(out))


def test_xcd_parts_cut_compulsory_x_traffic():
    """Each XCD has its own L2: the plan splits the rows into 8 parts (row
    ranges or breadth-first shares, whichever reads fewer X rows) and runs
    part x on XCD x, so the X rows the 8 XCDs read, summed, drop from 1.69x
    to 1.30x X on the mesh-numbered surrogate (ranges) and from 2.06x to
    1.62x on its random renumbering (breadth-first shares), at about the same
    re-use.  The native check replays the kernel's reads of every plan."""
    A = smfv.cop20k_surrogate()
    m = A.numRows
    auto = _analyse_rows(A, 0, m)
    one = _analyse_rows(A, 0, m, 64)  # SMFV_PLAN_ONE_WAVEFRONT
    assert auto["parts"] == 8 and one["parts"] == 1
    assert auto["xcd_footprint"] == pytest.approx(auto["footprint"], rel=0.01)  # (a few edge tiles rebalanced)
    assert auto["xcd_footprint"] < 1.35 < 1.6 < one["xcd_footprint"]
    assert auto["reuse"] > 0.98 * one["reuse"] and auto["direct"] == 0
    # no XCD runs more rounds of 32 tiles than the tile count needs
    P = inputs.permute_symmetric(A, np.random.default_rng(7).permutation(m))
    pa, po = _analyse_rows(P, 0, m), _analyse_rows(P, 0, m, 64)
    assert pa["parts"] == 8 and pa["xcd_footprint"] < 1.7 < 2.0 < po["xcd_footprint"]
    assert pa["reuse"] > 0.97 * po["reuse"]


def test_row_block_tiles_grow_by_the_blocks_own_neighbours():
    """A row block's tiles (one rank of the decomposition) are grown through
    its rows' neighbours -- column c is the block's row c - row_begin -- so a
    middle block reaches the whole matrix's re-use."""
    A = smfv.cop20k_surrogate()
    m = A.numRows
    whole = _analyse_rows(A, 0, m, 64)
    mid = _analyse_rows(A, m // 4, 3 * m // 4, 64)
    assert mid["reuse"] > 0.97 * whole["reuse"]


def test_mtx_reader_parallel_and_fallback(tmp_path):
    """The parallel Matrix Market parse (one entry per line, files > 64 KiB)
    gives the same CSR as the sequential token reader, and files it cannot
    cut by lines (an entry split over lines, extra trailing entries) fall
    back to the sequential reader's semantics (SC/utils.cpp:116-153)."""
    A = smfv.gen_random_rows(3000, 2500, 6, 2.0, 200, 9)
    p1 = tmp_path / "a.mtx"
    smfv.writeMatrixMarketFile(str(p1), A)
    assert p1.stat().st_size > 65536
    B = smfv.readMatrixMarketFile(str(p1))
    assert np.array_equal(A.rowPtr, B.rowPtr) and np.array_equal(A.colIndices, B.colIndices)
    assert np.array_equal(A.values.view(np.uint64), B.values.view(np.uint64))
    lines = p1.read_text().splitlines()
    hdr, body = lines[:2], lines[2:]
    # first entry split over two lines + two junk entries past nz
    r, c, v = body[0].split()
    odd = hdr + [f"{r} {c}", v] + body[1:] + ["1 1 5.0", "2 2 6.0"]
    p2 = tmp_path / "b.mtx"
    p2.write_text("\n".join(odd) + "\n")
    C = smfv.readMatrixMarketFile(str(p2))
    assert np.array_equal(A.rowPtr, C.rowPtr) and np.array_equal(A.colIndices, C.colIndices)
    assert np.array_equal(A.values.view(np.uint64), C.values.view(np.uint64))


REF_SC = "/root/reference/Source Code"


def test_relink_recipe(tmp_path):
    """a caller compiled against the reference's own
    headers (quoted includes resolved in the reference's directory, as
    SC/main.cpp's are) with the drop-in struct force-included, linked to
    libsmfv_mpi.so.  Compile + link only (running needs a GPU)."""
    if not os.path.isdir(REF_SC):
        pytest.skip("reference sources not present (container only)")
    src = os.path.join(ROOT, "tests", "cpp", "relink_caller.cpp")
    inc = os.path.join(ROOT, "include")
    out = str(tmp_path / "caller")
    cmd = ["g++", "-std=c++17", "-include", os.path.join(inc, "MatrixDefinitions.h"), f"-I{REF_SC}", src,
           f"-L{PKG}", "-lsmfv_mpi", "-lsmfv", "-Wl,--allow-shlib-undefined", "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # without the force-include the reference's own struct is used and the
    # caller's numRows does not exist: the recipe's -include is what makes it work
    r2 = subprocess.run([c for c in cmd if c not in ("-include", os.path.join(inc, "MatrixDefinitions.h"))],
                        capture_output=True, text=True)
    assert r2.returncode != 0 and "numRows" in r2.stderr


@pytest.mark.parametrize("p", [1, 2, 4, 7, 8])
@pytest.mark.parametrize("variant", [1, 2, 3])
@pytest.mark.parametrize("mode", [0, 1])
def test_exchange_schedule_delivers_every_block(p, variant, mode):
    """The native exchange schedule (smfv_dist_exchange_ops) simulated for
    all p ranks at once (p up to 8, the driver's node): sends pair with
    receives, every broadcast is issued by every rank in the same order, an
    all-gather is issued by all ranks with equal counts, and afterwards the
    root (TO_ROOT) or every rank (TO_ALL) holds every rank's block."""
    from sparsematrixmultiplicationmpi_amd.dist import EX_ALLGATHER, EX_BCAST, EX_RECV, EX_SEND, exchange_ops, exchange_plan
    A = smfv.gen_random_rows(1203, 900, 7, 2.0, 200, 5)
    K, root = 12, p - 1
    first, last, off, cnt = exchange_plan(variant, A.numRows, A.nnz, A.rowPtr, K, p)
    ops = [exchange_ops(variant, mode, root, A.numRows, A.nnz, A.rowPtr, K, p, r) for r in range(p)]
    have = [{r} for r in range(p)]  # blocks (by owner rank) each rank holds
    block_at = {int(off[r]): r for r in range(p) if cnt[r] > 0}
    if p == 1:
        assert ops == [[]]
        return
    if any(o and o[0][0] == EX_ALLGATHER for o in ops):
        assert all(len(o) == 1 and o[0][0] == EX_ALLGATHER and o[0][3] == cnt[0] for o in ops)
        assert all(o[0][2] == off[r] for r, o in enumerate(ops))
        have = [set(range(p)) for _ in range(p)]
    else:
        bc = [[(k, pe, of, c) for k, pe, of, c in o if k == EX_BCAST] for o in ops]
        assert all(b == bc[0] for b in bc)  # same broadcasts, same order, on every rank
        for k, pe, of, c in bc[0]:
            assert block_at[of] == pe and c == cnt[pe]
            for r in range(p):
                have[r].add(pe)
        sends = sorted((r, pe, of, c) for r, o in enumerate(ops) for k, pe, of, c in o if k == EX_SEND)
        recvs = sorted((pe, r, of, c) for r, o in enumerate(ops) for k, pe, of, c in o if k == EX_RECV)
        assert sends == recvs  # (sender, receiver, offset, count) pair up
        for s_, r_, of, c in sends:
            assert block_at[of] == s_ and c == cnt[s_]
            have[r_].add(s_)
    owners = {r for r in range(p) if cnt[r] > 0}
    targets = range(p) if mode == 1 else [root]
    for t in targets:
        assert owners <= have[t], (t, owners - have[t])


def _both_readers(path):
    A = smfv.readMatrixMarketFile(str(path))
    m, n, rp, ci, va = oracle.mtx_read(str(path))
    assert (A.numRows, A.numCols) == (m, n)
    assert np.array_equal(A.rowPtr, rp) and np.array_equal(A.colIndices, ci) and np.array_equal(A.values, va)
    return A


def test_mtx_reader_reference_quirks(tmp_path):
    """Known answers for what SC/utils.cpp:70-185 does beyond the Matrix
    Market spec, on the product reader and the oracle alike: the
    symmetric / pattern flags come from ANY comment line containing the word
    (:84-105), so "skew-symmetric" mirrors like "symmetric" and its mirror is
    NOT negated (:149-152); duplicates stay, and std::sort on (col, value)
    pairs orders a row's duplicates by value (:157-160); an "integer" field is
    read as a double; entries past the header's count are ignored (:124)."""
    p = tmp_path / "skew.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real skew-symmetric\n3 3 2\n2 1 -4.5\n3 2 2.0\n")
    A = _both_readers(p)
    assert A.rowPtr.tolist() == [0, 1, 3, 4]
    assert A.colIndices.tolist() == [1, 0, 2, 1]
    assert A.values.tolist() == [-4.5, -4.5, 2.0, 2.0]  # mirrored, not negated
    p = tmp_path / "later.mtx"  # the flag words in a later comment line count
    p.write_text("%%MatrixMarket matrix coordinate real general\n% not symmetric, no pattern\n2 2 1\n2 1\n")
    A = _both_readers(p)
    assert A.rowPtr.tolist() == [0, 1, 2] and A.colIndices.tolist() == [1, 0] and A.values.tolist() == [1.0, 1.0]
    p = tmp_path / "dups.mtx"  # duplicates ordered by value; integer field
    p.write_text("%%MatrixMarket matrix coordinate integer general\n2 3 5\n1 2 7\n1 2 -3\n1 1 9\n2 3 1\n1 2 5\n"
                 "2 2 99\n")
    A = _both_readers(p)
    assert A.rowPtr.tolist() == [0, 4, 5]
    assert A.colIndices.tolist() == [0, 1, 1, 1, 2]
    assert A.values.tolist() == [9.0, -3.0, 5.0, 7.0, 1.0]  # the sixth entry (2 2 99) is past the count


def test_mtx_reader_reference_quirks_parallel_parse(tmp_path):
    """The same quirks through the parallel parse (files over 64 KiB): a
    skew-symmetric banner, an integer field, duplicates with distinct
    values, against the oracle's sequential restatement."""
    rng = np.random.default_rng(5)
    m = 3000
    r = rng.integers(1, m + 1, 20000)
    c = rng.integers(1, m + 1, 20000)
    keep = r >= c  # lower triangle, as a symmetric file stores it
    r, c = r[keep], c[keep]
    r = np.concatenate([r, r[:500]])  # duplicates of the first 500 entries, other values
    c = np.concatenate([c, c[:500]])
    v = rng.integers(-50, 50, r.size)
    p = tmp_path / "big_skew.mtx"
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix coordinate integer skew-symmetric\n%\n")
        f.write(f"{m} {m} {r.size}\n")
        f.writelines(f"{a} {b} {x}\n" for a, b, x in zip(r, c, v))
    assert p.stat().st_size > 64 * 1024
    A = _both_readers(p)
    assert A.nnz == 2 * r.size - int(np.sum(r == c))


def test_are_matrices_equal_nan_policy():
    """The Python mirror (and the device compare) treat a NaN difference as
    unequal; the reference's fabs(NaN) > tol is false (SC/utils.cpp:55), which
    the C++ drop-in keeps -- documented in inputs.areMatricesEqual."""
    assert not smfv.areMatricesEqual([[1.0, float("nan")]], [[1.0, 2.0]], 1e-6)
    assert smfv.areMatricesEqual([[1.0, 2.0]], [[1.0, 2.0 + 5e-7]], 1e-6)


def test_knn3d_irregular_surrogate():
    """The second cop20k_A stand-in: same m, nnz within a few of 2,624,331,
    exactly symmetric (pattern and values), diagonal present, rows sorted,
    degrees spread 4..85 (the stencil surrogate's are 8..27), deterministic;
    the tile analysis still tiles it (re-use >= 3)."""
    import ctypes
    import sparsematrixmultiplicationmpi_amd as smfv
    from sparsematrixmultiplicationmpi_amd._lib import call
    A = smfv.inputs.cop20k_irregular_surrogate()
    A.validate()
    assert A.numRows == smfv.COP20K_M and abs(A.nnz - smfv.COP20K_NNZ) <= 10
    rp, ci, va = np.asarray(A.rowPtr), np.asarray(A.colIndices), np.asarray(A.values)
    d = np.diff(rp)
    assert d.min() <= 5 and d.max() >= 70 and np.percentile(d, 99) > 2 * np.median(d)
    rows = np.repeat(np.arange(A.numRows), d)
    assert np.all(np.diff(ci)[np.diff(rows) == 0] > 0)  # sorted, no duplicates
    assert np.sum(rows == ci) == A.numRows  # diagonal
    import scipy.sparse as sp
    M = sp.csr_matrix((va, ci, rp), shape=(A.numRows, A.numCols))
    assert abs(M - M.T).max() == 0.0
    B = smfv.inputs.cop20k_irregular_surrogate()
    assert np.array_equal(B.colIndices, A.colIndices) and np.array_equal(B.values, A.values)
    out = (ctypes.c_double * 9)()
    ip = ctypes.POINTER(ctypes.c_int)
    rp32, ci32 = np.ascontiguousarray(rp, np.int32), np.ascontiguousarray(ci, np.int32)
    call("smfv_plan_analyse_rows", 0, A.numRows, A.numCols, rp32.ctypes.data_as(ip), ci32.ctypes.data_as(ip), 0, out)
    assert out[2] >= 3.0 and out[3] == 0  # re-use, direct rows


def _chunks(A, r0=0, r1=None, cap=0):
    out = (ctypes.c_double * 6)()
    ip = ctypes.POINTER(ctypes.c_int)
    r1 = A.numRows if r1 is None else r1
    _lib.call("smfv_spmv_chunks_analyse", r0, r1, A.numCols, A.rowPtr.ctypes.data_as(ip),
              A.colIndices.ctypes.data_as(ip), cap, out)
    return {"fits": bool(out[0]), "chunks": int(out[1]), "entries": int(out[2]), "most_rows": int(out[3]),
            "fill": out[4], "wide": bool(out[5])}


def test_spmv_chunk_layout():
    """The K = 1 chunk layout (k_spmv_chunks), built and verified natively as a
    K = 1 plan builds it: every non-zero placed once, chunks full to > 95 % on
    the cop20k stand-ins, at most 256 rows per chunk (one lane per row), a
    row block's layout covers only its non-zeros; 16-bit column offsets on
    the stencil, 32-bit columns where a row spans more than 2^16 columns (the
    Morton-numbered k-NN stand-in); rows longer than a chunk leave the
    pattern on the CSR kernel."""
    for A, wide in ((smfv.cop20k_surrogate(), False), (smfv.inputs.cop20k_irregular_surrogate(), True)):
        for cap in (1024, 2048):
            c = _chunks(A, cap=cap)
            assert c["fits"] and c["entries"] == A.nnz and c["fill"] > 0.95, (cap, c)
            assert c["chunks"] >= A.nnz // cap and c["most_rows"] <= 256 and c["wide"] == wide
    A = smfv.cop20k_surrogate()
    c = _chunks(A, 1000, 50000)
    assert c["fits"] and c["entries"] == int(A.rowPtr[50000] - A.rowPtr[1000])
    # short rows: the 256-row cap ends chunks, not the entries
    S = smfv.gen_random_rows(20000, 20000, 2.0, 0.0, 2, 5)
    c = _chunks(S)
    assert c["fits"] and c["most_rows"] == 256 and c["chunks"] == -(-20000 // 256) and not c["wide"]
    # empty blocks and empty matrices
    assert _chunks(A, 7, 7)["chunks"] == 0
    E = smfv.readMatrixMarketFile(os.path.join(GOLDEN, "empty7x5.mtx"))
    assert _chunks(E)["fits"]
    # random columns over 10M: the wide layout; a row of 4,096 (> 2,048 slots): no chunk plan
    assert _chunks(smfv.gen_random_rows(2000, 10_000_000, 16.0, 0.0, 16, 7))["wide"]
    P = smfv.gen_random_rows(20000, 20000, 16, 2.0, 4096, 42)
    assert np.diff(P.rowPtr).max() > 2048 and not _chunks(P, cap=2048)["fits"]


def test_no_lab_code_in_the_product():
    """(r5) The r2-r4 lab build (ablation copies of the kernels, environment
    overrides, k_rows_cs) is retired: no source of the product mentions it
    and libsmfv.so exports no k_rows_cs / smfv_cs_plan_analyse.  A/B runs
    load another build of the same sources (SMFV_LIB), never an ifdef path."""
    nm = subprocess.run(["nm", "-D", "-C", os.path.join(PKG, "libsmfv.so")], capture_output=True, text=True).stdout
    assert "smfv_cs_plan_analyse" not in nm and "k_rows_cs" not in nm
    csrc = os.path.join(PKG, "csrc")
    assert not os.path.exists(os.path.join(csrc, "lab"))
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h", ".inc")):
            assert "SMFV_LAB" not in open(os.path.join(csrc, f)).read(), f


def test_balanced_row_partition():
    """(r5) SMFV_DIST_BALANCED_ROWS cuts a distributed ROWWISE plan's rows
    into blocks of equal work (12 B per non-zero + 8K + 4 B per row); without
    it the blocks are the reference's equal row counts (SC/...RowWise.cpp:26-29,
    = smfv_dist_plan).  Blocks tile [0, m) in rank order; on a skewed
    pattern the balanced blocks' work is within one row of the mean, and
    chunk boundaries tile each block."""
    from sparsematrixmultiplicationmpi_amd import dist as D
    A = smfv.gen_random_rows(20000, 20000, 16.0, 2.0, 2000, 77)
    rp = A.rowPtr.astype(np.int64)
    K = 32
    m = A.numRows
    work = lambda s, e: 12 * (rp[e] - rp[s]) + (8 * K + 4) * (e - s)  # noqa: E731
    maxrow = int(12 * np.diff(rp).max() + 8 * K + 4)
    for p in (2, 3, 8, 13):
        ref = exchange_plan(1, m, A.nnz, A.rowPtr, K, p)
        assert all(np.array_equal(a, b) for a, b in zip(ref, D.exchange_plan(1, m, A.nnz, A.rowPtr, K, p,
                                                                             D.dist_opts("reference"))))
        first, last, off, cnt = D.exchange_plan(1, m, A.nnz, A.rowPtr, K, p, D.dist_opts("balanced"))
        assert first[0] == 0 and last[-1] == m - 1 and np.all(first[1:] == last[:-1] + 1)
        assert np.all(off == first.astype(np.int64) * K) and np.all(cnt == (last - first + 1).astype(np.int64) * K)
        wb = [work(int(first[r]), int(last[r]) + 1) for r in range(p)]
        wr = [work(int(ref[0][r]), int(ref[1][r]) + 1) for r in range(p)]
        mean = work(0, m) / p
        assert max(wb) - mean <= maxrow, (p, max(wb) / mean)
        assert max(wb) <= max(wr), p
        for chunks in (2, 5):
            dopts = D.dist_opts("balanced", chunks)
            for r in range(p):
                b = D.chunk_rows(1, dopts, m, A.nnz, A.rowPtr, K, p, r)
                assert len(b) == chunks + 1 and b[0] == first[r] and b[-1] == last[r] + 1 and b == sorted(b)
    # the power-law pattern is imbalanced under equal rows
    p = 8
    ref = exchange_plan(1, m, A.nnz, A.rowPtr, K, p)
    wr = [work(int(ref[0][r]), int(ref[1][r]) + 1) for r in range(p)]
    assert max(wr) / (work(0, m) / p) > 1.02


def test_ws_kernels_register_budget(tmp_path):
    """(r5) Every k_rows_ws instance in libsmfv.so fits the waves
    per SIMD its geometry runs: one 1024-lane block (geometry 1) or two
    512-lane blocks (geometry 2) per CU = 4 waves per SIMD -> <= 128 VGPRs;
    a 768-lane block (geometry 3) = 3 waves -> <= 168.  No spills.  Read from
    the code object's metadata (llvm-objdump --offloading, llvm-readelf
    --notes), so a compiler change that breaks the budget fails here."""
    import re
    import shutil
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-readelf")):
        pytest.skip("no ROCm llvm tools")
    so = tmp_path / "libsmfv.so"
    shutil.copy(os.path.join(PKG, "libsmfv.so"), so)
    subprocess.run([os.path.join(llvm, "llvm-objdump"), "--offloading", str(so)], cwd=tmp_path, capture_output=True,
                   check=True)
    co = [f for f in os.listdir(tmp_path) if "gfx950" in f]
    assert co, os.listdir(tmp_path)
    notes = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--notes", str(tmp_path / co[0])],
                           capture_output=True, text=True, check=True).stdout
    seen = 0
    for blk in notes.split("  - .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        if "k_rows_ws" not in name:
            continue
        vgpr = int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1))
        spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1))
        geo = re.search(r"k_rows_ws(?:_live)?ILi(\d+)ELi(\d+)E", name)
        if geo is None:  # (r5) k_rows_wsn: one 1024-lane block per CU
            assert "k_rows_wsn" in name and vgpr <= 128 and spill == 0, (name, vgpr, spill)
            continue
        cw, lw = map(int, geo.groups())
        waves_per_simd = 4 if (cw, lw) in ((8, 8), (4, 4)) else 3
        assert vgpr <= 512 // waves_per_simd and spill == 0, (name, vgpr, spill)
        seen += 1
    assert seen >= 24, seen


def test_narrow_team_plan_on_host():
    """(r5) The k_rows_wsn plan of a 4 / 8-column window (a ColumnWise rank's
    panel) is built and verified on the host (its reads replayed): every row
    once, in CSR order, pads on the zero image row; on the cop20k stand-in it
    runs well under half the units of k_rows_ws's 2,011 tiles with < 8 %
    padded entries, and a row too long for a tile becomes direct."""
    ip = ctypes.POINTER(ctypes.c_int)

    def wsn(A, kw, r0=0, r1=None):
        out = (ctypes.c_double * 9)()
        _lib.call("smfv_wsn_plan_analyse", r0, A.numRows if r1 is None else r1, A.numCols,
                  A.rowPtr.ctypes.data_as(ip), A.colIndices.ctypes.data_as(ip), kw, out)
        # (r6) the X reads' modelled LDS cycles: conflict-free count <= the
        # plan's bank-coloured slots < first-use slots (58 -> 45 % conflict
        # cycles at K/p = 4 on the stencil stand-in)
        groups, coloured, plain = out[6], out[7], out[8]
        assert 0 < groups <= coloured <= plain, (kw, groups, coloured, plain)
        if A.numRows == 121192:
            assert (coloured - groups) / coloured < 0.9 * (plain - groups) / plain, (kw, coloured, plain)
        return [float(v) for v in out[:6]]
    A = smfv.inputs.cop20k_surrogate()
    for kw, rows in ((4, 256), (8, 128)):
        tiles, union, reuse, direct, most, entries = wsn(A, kw)
        assert 0 < tiles < 2011 * 0.6 and direct == 0 and most <= rows and reuse > 6.0, (kw, tiles, reuse)
        # (r5) batches of 4 trimmed to the running teams: 2.80 M entries for
        # 2.62 M non-zeros (3.54 M with untrimmed batches of 8)
        assert A.nnz <= entries <= 1.08 * A.nnz, (kw, entries)
        # (r5) the plan is picked by rounds of units on the busiest blocks
        # (32 per XCD): 3 at K/p = 4 (<= 768 tiles), 4 at K/p = 8 (<= 1,024)
        assert tiles <= {4: 768, 8: 1024}[kw], (kw, tiles)
    P = smfv.gen_random_rows(5000, 5000, 12, 2.0, 5000, 3)  # a few very long rows
    tiles, union, reuse, direct, most, entries = wsn(P, 4)
    assert tiles > 0 and direct >= 1
    tiles_b, *_ = wsn(A, 8, 30000, 90000)  # a row block (columns shifted by its first row)
    assert tiles_b > 0
    with pytest.raises(RuntimeError):
        wsn(A, 16)
