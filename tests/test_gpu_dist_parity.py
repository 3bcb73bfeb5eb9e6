"""The distributed variants' rank-local path against the reference's own
outputs at the rank counts its fixtures hold (tests/golden: p in {1, 2, 3,
8}), all on one device.

Every rank r of p is computed by the product's own pieces -- the rank plan
(smfv_dist_plan_create_rank: the same partition and single-device plan a
rank of smfv_dist_plan_create runs, tiled where it pays) and the plain
building blocks (smfv_spmm_rowblock / colpanel / nnzrange) -- on the
partition smfv_dist_plan gives.  The blocks are then moved as the exchange
schedule (smfv_dist_exchange_ops) says and assembled by the device kernels
(panels_to_rowmajor, combine_row_blocks).  Compared with:
  ROWWISE / COLUMNWISE  Y_seq bit for bit (the reference's RowWise and
                        ColumnWise are bitwise equal to its serial result:
                        sha_row_p{p} / sha_col_p{p} in the fixtures)
  NONZERO               the reference's own NonZeroElement result at that p
                        (Y_nnz_p{p}) within 1e-12 x sum|a||x|.
The degenerate partitions the reference produces are all here: pat4x6_k3
at p = 8 has K < p (ColumnWise ranks 0-6 own no column, SC/...ColumnWise.cpp
:25-28), m < p (RowWise ranks 4-7 own no row, SC/...RowWise.cpp:26-29) and
nnz < p (NonZeroElement rank 7 owns no non-zero, SC/...NonZeroElement.cpp
:24-39); empty7x5 has empty rows at every p.
"""
import ctypes
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden_cases, load_golden
from oracle import oracle

import sparsematrixmultiplicationmpi_amd as smfv
from sparsematrixmultiplicationmpi_amd import dist as D
from sparsematrixmultiplicationmpi_amd import engine as S

pytestmark = pytest.mark.gpu
NNZ_TOL = 1e-12
CASES = [(name, p) for name, meta in sorted(golden_cases().items()) for p in meta["p"]]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def golden_problem(name, gpu):
    g = load_golden(name)
    A = smfv.SparseMatrix(np.asarray(g["values"], np.float64), np.asarray(g["col_idx"], np.int32),
                          np.asarray(g["row_ptr"], np.int32), int(g["m"]), int(g["n"]))
    X = np.ascontiguousarray(g["X"], dtype=np.float64)
    return g, A, smfv.DeviceCSR(A, gpu), torch.from_numpy(X).to(gpu)


def assemble(variant, A, K, p, xbuf, Y, first, last):
    """The root's assembly step of the exchange (device kernels)."""
    if variant == smfv.Variant.COLUMNWISE:
        smfv._lib.call("smfv_panels_to_rowmajor_f64", A.numRows, K, p, xbuf.data_ptr(), Y.data_ptr(), K,
                       S.stream_handle())
    elif variant == smfv.Variant.NONZERO:
        rfa = (ctypes.c_int * p)(*[int(v) for v in first])
        rla = (ctypes.c_int * p)(*[int(v) for v in last])
        smfv._lib.call("smfv_combine_row_blocks_f64", A.numRows, K, p, rfa, rla, xbuf.data_ptr(), Y.data_ptr(), K,
                       S.stream_handle())


def replay_exchange(variant, A, K, p, root, blocks, xbuf):
    """Every rank's exchange ops (the native schedule, gather-to-root) moved
    by device copies: what the root holds after RCCL ran them."""
    moved = 0
    for r in range(p):
        for kind, peer, off, cnt in D.exchange_ops(variant, D.TO_ROOT, root, A.numRows, A.nnz, A.rowPtr, K, p, r):
            if kind == D.EX_SEND:  # rank r's block lands at the root
                assert peer == root
                xbuf[off:off + cnt] = blocks[r][off:off + cnt]
                moved += 1
    # the root's own block needs no op
    fr, lr, off, cnt = D.exchange_plan(variant, A.numRows, A.nnz, A.rowPtr, K, p)
    xbuf[off[root]:off[root] + cnt[root]] = blocks[root][off[root]:off[root] + cnt[root]]
    return moved


def check(variant, g, p, Y):
    Yh = Y.cpu().numpy()
    if variant == smfv.Variant.NONZERO:
        absY = oracle.spmm("sequential", g["row_ptr"], g["col_idx"], np.abs(g["values"]), np.abs(g["X"]))
        Yz = g[f"Y_nnz_p{p}"]
        err = float(np.max(np.abs(Yh - Yz) / np.maximum(absY, 1e-300))) if Yh.size else 0.0
        assert err <= NNZ_TOL, (p, err)
        assert smfv.areMatricesEqual(Yh, Yz, 1e-6)  # the reference's own check (SC/utils.cpp:55)
    else:
        assert np.array_equal(bits(Yh), bits(g["Y_seq"])), p
        # the fixture's hash of the reference's own RowWise / ColumnWise output at this p
        key = f"sha_row_p{p}" if variant == smfv.Variant.ROWWISE else f"sha_col_p{p}"
        if key in g:
            assert hashlib.sha256(bits(Yh).tobytes()).hexdigest() == str(g[key]), key


@pytest.mark.parametrize("name,p", CASES)
@pytest.mark.parametrize("variant,partition", [(smfv.Variant.ROWWISE, "reference"), (smfv.Variant.ROWWISE, "balanced"),
                                               (smfv.Variant.COLUMNWISE, "balanced"),
                                               (smfv.Variant.NONZERO, "balanced")])
@pytest.mark.parametrize("tiles", ["auto", "force", "off"])
def test_rank_plans_vs_reference(gpu, name, p, variant, partition, tiles):
    """Every rank's plan (smfv_dist_plan_create_rank) + the native exchange
    schedule replayed on the device = the reference's result at p ranks.
    (r5) ROWWISE under both row partitions: the reference's equal rows (the
    default) and the opt-in equal-work blocks, SMFV_DIST_BALANCED_ROWS (same
    bytes: a row is summed by one rank in CSR order either way)."""
    g, A, dA, dX = golden_problem(name, gpu)
    K = dX.shape[1]
    root = p - 1  # a root other than 0 where p > 1
    first, last, off, cnt = D.exchange_plan(variant, A.numRows, A.nnz, A.rowPtr, K, p, D.dist_opts(partition))
    Y = torch.full((A.numRows, K), float("nan"), dtype=torch.float64, device=gpu)
    blocks, plans = [], []
    for r in range(p):
        P = D.DistPlan(None, variant, dA, K, to_all=False, root=root, tiles=tiles, rank=(r, p), partition=partition)
        plans.append(P)
        P.run_local(dX, Y)
        buf = P.exchange_buffer()
        assert (buf is None) == (variant == smfv.Variant.ROWWISE)
        blocks.append(buf)
        if tiles == "force" and variant == smfv.Variant.ROWWISE and K % 32 == 0 and last[r] >= first[r]:
            assert P.stats()["tiled"]
    if variant != smfv.Variant.ROWWISE:
        xbuf = torch.full((max(int((off + cnt).max()), 1),), float("nan"), dtype=torch.float64, device=gpu)
        replay_exchange(variant, A, K, p, root, blocks, xbuf)
        Y.fill_(float("nan"))
        assemble(variant, A, K, p, xbuf, Y, first, last)
    torch.cuda.synchronize()
    check(variant, g, p, Y)
    if p > 1 and len(D.exchange_ops(variant, D.TO_ROOT, root, A.numRows, A.nnz, A.rowPtr, K, p, 0)):
        with pytest.raises(smfv.SmfvError):  # a rank plan has no communicator to exchange over
            plans[0].exchange(Y)


@pytest.mark.parametrize("name,p", CASES)
def test_building_blocks_vs_reference(gpu, name, p):
    """The plain rank-local building blocks (no plan) on smfv_dist_plan's
    partitions: rowblock / colpanel / nnzrange + panels_to_rowmajor /
    combine_row_blocks."""
    g, A, dA, dX = golden_problem(name, gpu)
    K = dX.shape[1]
    m = A.numRows
    # RowWise row blocks
    first, last, off, cnt = D.exchange_plan(smfv.Variant.ROWWISE, m, A.nnz, A.rowPtr, K, p)
    Y = torch.full((m, K), float("nan"), dtype=torch.float64, device=gpu)
    for r in range(p):
        if last[r] >= first[r]:
            S.spmm_rowblock(dA, int(first[r]), int(last[r]) + 1, dX, Y[first[r]:last[r] + 1])
    torch.cuda.synchronize()
    check(smfv.Variant.ROWWISE, g, p, Y)
    # ColumnWise panels -> rank-major buffer -> device rebuild
    first, last, off, cnt = D.exchange_plan(smfv.Variant.COLUMNWISE, m, A.nnz, A.rowPtr, K, p)
    panels = torch.full((max(m * K, 1),), float("nan"), dtype=torch.float64, device=gpu)
    for r in range(p):
        kc = int(last[r] - first[r] + 1)
        if kc > 0:
            S.spmm_colpanel(dA, int(first[r]), int(last[r]) + 1, dX, panels[off[r]:off[r] + cnt[r]].view(m, kc))
    Y.fill_(float("nan"))
    assemble(smfv.Variant.COLUMNWISE, A, K, p, panels, Y, first, last)
    torch.cuda.synchronize()
    check(smfv.Variant.COLUMNWISE, g, p, Y)
    # NonZeroElement nnz ranges -> compact row blocks -> combine
    first, last, off, cnt = D.exchange_plan(smfv.Variant.NONZERO, m, A.nnz, A.rowPtr, K, p)
    xbuf = torch.full((max(int((off + cnt).max()), 1),), float("nan"), dtype=torch.float64, device=gpu)
    for r in range(p):
        s, e = oracle.partition_nnz(A.nnz, p, r)
        rf, rl, Yp = S.spmm_nnzrange(dA, s, e, dX)
        assert (rf, rl) == ((int(first[r]), int(last[r])) if e > s else (0, -1))
        if rl >= rf:
            xbuf[off[r]:off[r] + cnt[r]] = Yp.reshape(-1)
    Y.fill_(float("nan"))
    assemble(smfv.Variant.NONZERO, A, K, p, xbuf, Y, first, last)
    torch.cuda.synchronize()
    check(smfv.Variant.NONZERO, g, p, Y)


def test_exchange_error_closes_group(gpu):
    """An RCCL failure inside the exchange's group (injected by the test hook
    smfv_test_fail_exchange) closes the group before the error returns: the
    next exchange on the same communicator runs and moves the right bytes."""
    comm = D.Communicator(0, 1, D.Communicator.new_unique_id())
    buf = torch.arange(64, dtype=torch.float64, device=gpu)
    ref = buf.clone()
    kinds = np.array([D.EX_BCAST, D.EX_BCAST, D.EX_BCAST], np.int32)
    peers = np.zeros(3, np.int32)
    offs = np.array([0, 16, 32], np.int64)
    cnts = np.array([16, 16, 32], np.int64)
    ip, lp = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64)
    args = (comm.handle, kinds.ctypes.data_as(ip), peers.ctypes.data_as(ip), offs.ctypes.data_as(lp),
            cnts.ctypes.data_as(lp), 3, buf.data_ptr(), S.stream_handle())
    smfv._lib.lib.smfv_test_fail_exchange(2)  # the second op of the next group fails
    with pytest.raises(smfv.SmfvError, match="injected"):
        smfv._lib.call("smfv_comm_exchange_f64", *args)
    smfv._lib.call("smfv_comm_exchange_f64", *args)  # the group was closed: this one runs
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    # and a distributed plan on the same communicator still runs end to end
    A = smfv.gen_fem27(3000, 12, 12, 0.83, 5)
    X = np.random.default_rng(5).uniform(-1, 1, (A.numCols, 32))
    Yref = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
    Y = D.dist_spmm(comm, smfv.Variant.COLUMNWISE, smfv.DeviceCSR(A, gpu), torch.from_numpy(X).to(gpu), to_all=True)
    torch.cuda.synchronize()
    assert np.array_equal(bits(Y.cpu().numpy()), bits(Yref))
    comm.close()
