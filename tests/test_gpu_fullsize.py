"""BASELINE configs 4 and 5 checked at their FULL size (only
60k / 5k-row instances had been checked).  The full reference result is
too large for the host oracle in test time, so a row sample is checked:
the longest rows, every row open at a merge-path team boundary (carry rows,
from the library's own merge geometry), empty rows, the first / last rows
and random rows (sparsematrixmultiplicationmpi_amd/sampling.py), each
against the oracle's sequential sum of that row (SC/SparseMatrixFatVectorMultiply.cpp:17-27):
NONZERO within 1e-12 x sum|a||x| (the north star allows 1e-6 relative),
ROWWISE bit for bit."""
import numpy as np
import pytest
import torch

from oracle import oracle

import sparsematrixmultiplicationmpi_amd as smfv
from sparsematrixmultiplicationmpi_amd import sampling

pytestmark = pytest.mark.gpu


def check_sample(A, rows, dX, Ydev, exact: bool):
    """Oracle on the sampled rows (X rows gathered from the device)."""
    srp, scol, sval, ucols = sampling.sub_csr(A.rowPtr, A.colIndices, A.values, rows)
    Xs = dX[torch.from_numpy(ucols).to(dX.device)].cpu().numpy()
    Yref = oracle.spmm("sequential", srp, scol, sval, Xs)
    Ys = Ydev[torch.from_numpy(rows).to(Ydev.device)].cpu().numpy()
    if exact:
        assert np.array_equal(Ys.view(np.uint64), Yref.view(np.uint64))
    else:
        scale = oracle.spmm("sequential", srp, scol, np.abs(sval), np.abs(Xs))
        assert np.all(np.abs(Ys - Yref) <= 1e-12 * scale), float(np.max(np.abs(Ys - Yref) / np.maximum(scale, 1e-300)))
    return len(rows)


def test_config4_pow10m_nonzero_full_size(gpu):
    """Config 4: 10M x 10M power-law (alpha 2, cap 4096, mean 16), K = 32,
    NonZeroElement merge-path (k_merge_flat + k_carry_fixup) at full size,
    exactly the bench's input (bench.py --config pow10m_k32)."""
    m, K = 10_000_000, 32
    A = smfv.gen_random_rows(m, m, 16.0, 2.0, 4096, 42)
    dA = smfv.DeviceCSR(A, gpu)
    dX = torch.empty((m, K), dtype=torch.float64, device=gpu)
    smfv.fill_x_hash(dX, 43)
    Y = torch.full((m, K), np.nan, dtype=torch.float64, device=gpu)
    smfv.SpmmPlan(smfv.Variant.NONZERO, dA, K).run(dX, Y)
    torch.cuda.synchronize()
    rows = sampling.sample_rows(A.rowPtr, K)
    nb = len(sampling.merge_boundary_rows(A.rowPtr, K))
    assert nb > 10_000  # ~16k team boundaries at this size
    assert check_sample(A, rows, dX, Y, exact=False) > 5000
    assert not torch.isnan(Y).any()


@pytest.mark.parametrize("rank", [0, 7])
def test_config5_syn80m_rank_block_full_size(gpu, rank):
    """Config 5: 80M x 80M, 16 uniform-random columns per row, K = 32,
    row-partitioned over 8 ranks: rank `rank`'s 10M-row block generated
    alone (as each GPU does) against the full 80M-row X (20.5 GB, hash
    1..100), through the row-partitioned plan at one rank (its exchange is
    empty; the 8-rank schedule is replayed over gloo in test_dist_gloo.py)."""
    m = n = 80_000_000
    K, p = 32, 8
    from sparsematrixmultiplicationmpi_amd import dist as D
    first, last, _, _ = D.exchange_plan(smfv.Variant.ROWWISE, m, 0, None, K, p)
    r0, r1 = int(first[rank]), int(last[rank]) + 1
    A = smfv.gen_random_rows(m, n, 16.0, 0.0, 16, 42, r0, r1)
    dA = smfv.DeviceCSR(A, gpu)
    dX = torch.empty((n, K), dtype=torch.float64, device=gpu)
    smfv.fill_x_hash(dX, 43)
    Yb = torch.full((r1 - r0, K), np.nan, dtype=torch.float64, device=gpu)
    plan = smfv.SpmmPlan(smfv.Variant.ROWWISE, dA, K)
    assert not plan.stats()["tiled"]  # uniform random columns: no re-use to stage
    plan.run(dX, Yb)
    torch.cuda.synchronize()
    rows = sampling.sample_rows(A.rowPtr, K, n_random=4000)
    assert check_sample(A, rows, dX, Yb, exact=True) > 4000
    del dX
    torch.cuda.empty_cache()
