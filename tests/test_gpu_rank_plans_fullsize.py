"""(r4) Every rank plan of a p-GPU decomposition at FULL size, on one device:
p in {2, 3, 4, 5, 8} (r6: 3 and 5 split K = 32 into uneven column windows),
ROWWISE / COLUMNWISE / NONZERO, K = 32, on both cop20k_A stand-ins (the
27-point-stencil surrogate and the irregular k-NN one).

Each rank r runs its share through the product's rank plan
(smfv_dist_plan_create_rank: the partition of SC/...RowWise.cpp:26-29,
...ColumnWise.cpp:25-28, ...NonZeroElement.cpp:24-39 and the single-device
plan a rank of smfv_dist_plan_create builds -- tiled row blocks with a
non-zero first row, K/p column-window plans, nnz-range merge plans); the
shares are moved as the native exchange schedule says and assembled by the
device kernels, then compared with the oracle: ROWWISE / COLUMNWISE bit for
bit (the reference's RowWise / ColumnWise equal its serial result bitwise),
NONZERO within 1e-12 x sum|a||x| of the oracle's restated NonZeroElement at
that p (the reference's MPI_Reduce association is not restated).  The
fixtures of tests/golden pin the same plans to the reference's own bytes on
small patterns (test_gpu_dist_parity.py); these are the sizes the 8-GPU run
meets first.
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from test_gpu_dist_parity import assemble, bits, replay_exchange

import sparsematrixmultiplicationmpi_amd as smfv
from sparsematrixmultiplicationmpi_amd import dist as D

pytestmark = pytest.mark.gpu
NNZ_TOL = 1e-12
K = 32


@pytest.fixture(scope="module", params=["stencil", "irregular"])
def standin(request, gpu):
    A = smfv.cop20k_surrogate() if request.param == "stencil" else smfv.inputs.cop20k_irregular_surrogate()
    X = smfv.generateLargeFatVector(A.numCols, K)
    Yseq = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
    absY = oracle.spmm("sequential", A.rowPtr, A.colIndices, np.abs(A.values), np.abs(X))
    return request.param, A, X, Yseq, absY, smfv.DeviceCSR(A, gpu), torch.from_numpy(X).to(gpu)


# (r5) ROWWISE under the row partitions: blocks of equal work (opt-in,
# SMFV_DIST_BALANCED_ROWS), the reference's equal rows (the default,
# SC/...RowWise.cpp:26-29), and equal-work blocks cut into 3 chunks
# (SMFV_DIST_CHUNKS: one tiled plan per chunk).  COLUMNWISE / NONZERO ignore
# the row partition (their own reference decompositions)
PARTS = [(smfv.Variant.ROWWISE, "balanced", 1), (smfv.Variant.ROWWISE, "reference", 1),
         (smfv.Variant.ROWWISE, "balanced", 3), (smfv.Variant.COLUMNWISE, "balanced", 1),
         (smfv.Variant.NONZERO, "balanced", 1)]


@pytest.mark.parametrize("p", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("variant,partition,chunks", PARTS)
def test_rank_plans_full_size(gpu, standin, p, variant, partition, chunks):
    name, A, X, Yseq, absY, dA, dX = standin
    m = A.numRows
    root = p - 1
    dopts = D.dist_opts(partition, chunks)
    first, last, off, cnt = D.exchange_plan(variant, m, A.nnz, A.rowPtr, K, p, dopts)
    Y = torch.full((m, K), float("nan"), dtype=torch.float64, device=gpu)
    blocks = []
    for r in range(p):
        P = D.DistPlan(None, variant, dA, K, to_all=False, root=root, rank=(r, p), partition=partition,
                       chunks=chunks)
        pf, pl, _, _ = P.partition()  # the plan's own partition is the host function's
        assert np.array_equal(pf, first) and np.array_equal(pl, last)
        assert P.shape() == (p, r, chunks)
        P.run_local(dX, Y)
        blocks.append(P.exchange_buffer())
        st = P.stats()
        if variant == smfv.Variant.ROWWISE:
            # every row block of the stand-ins is big enough to tile; the
            # block's neighbours are its columns shifted by its first row
            assert st["tiled"] and st["row_begin"] == int(first[r]), (name, p, r, st)
        torch.cuda.synchronize()
    if variant != smfv.Variant.ROWWISE:
        xbuf = torch.full((max(int((off + cnt).max()), 1),), float("nan"), dtype=torch.float64, device=gpu)
        replay_exchange(variant, A, K, p, root, blocks, xbuf)
        assemble(variant, A, K, p, xbuf, Y, first, last)
    torch.cuda.synchronize()
    Yh = Y.cpu().numpy()
    if variant == smfv.Variant.NONZERO:
        Yz = oracle.spmm("nonzero", A.rowPtr, A.colIndices, A.values, X, p)
        err = float(np.max(np.abs(Yh - Yz) / np.maximum(absY, 1e-300)))
        assert err <= NNZ_TOL, (name, p, err)
        assert float(np.max(np.abs(Yh - Yseq) / np.maximum(absY, 1e-300))) <= NNZ_TOL
    else:
        assert np.array_equal(bits(Yh), bits(Yseq)), (name, p, variant)
