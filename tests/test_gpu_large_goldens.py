"""(r4) The product against the reference's own results at SURVEY 8(c)'s
sizes (tests/golden/make_golden_large.py): a 2,048-row random symmetric
pattern and a 20,000-row power-law pattern whose plan tiles in 8 XCD parts
and has direct rows, at K in {1, 3, 32, 128} and p in {1, 2, 3, 8}, with the
reference's X (rand()%100+1).

  one device   every variant's default plan (tiled where it pays, the K = 1
               chunk plan) -> the sha256 of the reference's sequential bytes;
               NONZERO on the merge path (untiled K, or tiles off): within
               1e-12 x sum|a||x| of the reference's NonZeroElement at p = 1
  p ranks      every rank plan (smfv_dist_plan_create_rank), the shares moved
               as the native exchange schedule says and assembled on the
               device -> the sha256 of the reference's RowWise / ColumnWise
               bytes at p; NonZeroElement within 1e-12 x sum|a||x| of the
               reference's own result at p (rebuilt exactly from the fixture)
"""
import numpy as np
import pytest
import torch

from conftest import golden_large_cases, golden_large_nnz, load_golden_large, sha_f64
from oracle import oracle
from test_gpu_dist_parity import assemble, replay_exchange

import sparsematrixmultiplicationmpi_amd as smfv
from sparsematrixmultiplicationmpi_amd import dist as D

pytestmark = pytest.mark.gpu
NNZ_TOL = 1e-12
CASES = [(name, K) for name, info in sorted(golden_large_cases().items()) for K in info["K"]]


@pytest.fixture(scope="module")
def problems(gpu):
    cache = {}

    def get(name, K):
        if (name, K) not in cache:
            g = load_golden_large(name)
            A = g["A"]
            X = smfv.generateLargeFatVector(A.numCols, K)  # the reference driver's X (pinned by test_oracle)
            Yseq = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
            assert sha_f64(Yseq) == str(g[f"sha_seq_k{K}"])  # the host copy IS the reference's bytes
            absY = oracle.spmm("sequential", A.rowPtr, A.colIndices, np.abs(A.values), X)
            cache.clear()
            cache[(name, K)] = (g, A, X, Yseq, absY, smfv.DeviceCSR(A, gpu), torch.from_numpy(X).to(gpu))
        return cache[(name, K)]
    return get


def rel(Y, R, absY):
    return float(np.max(np.abs(Y - R) / np.maximum(absY, 1e-300))) if Y.size else 0.0


@pytest.mark.parametrize("name,K", CASES)
def test_one_device_vs_reference(gpu, problems, name, K):
    g, A, X, Yseq, absY, dA, dX = problems(name, K)
    sha = str(g[f"sha_seq_k{K}"])
    for v in smfv.Variant:
        plan = smfv.SpmmPlan(v, dA, K)
        st = plan.stats()
        if name == "plaw20k" and K % 32 == 0:
            # the tiled plan in 8 XCD parts with direct rows (rows over 239 X rows)
            assert st["tiled"] and st["xcd_parts"] == 8 and st["direct_rows"] > 0, st
        Y = torch.full((A.numRows, K), np.nan, dtype=torch.float64, device=gpu)
        plan.run(dX, Y)
        torch.cuda.synchronize()
        if v == smfv.Variant.NONZERO and not st["tiled"]:
            # untiled NONZERO (K not a multiple of 32, no K = 1 chunk plan) is
            # the nnz-balanced merge path: reassociated, within tolerance
            assert rel(Y.cpu().numpy(), golden_large_nnz(g, K, 1, Yseq), absY) <= NNZ_TOL, (name, K)
        else:
            assert sha_f64(Y.cpu().numpy()) == sha, (name, K, v, st["tiled"])
    Y = torch.full((A.numRows, K), np.nan, dtype=torch.float64, device=gpu)
    smfv.SpmmPlan(smfv.Variant.NONZERO, dA, K, tiles="off").run(dX, Y)
    torch.cuda.synchronize()
    assert rel(Y.cpu().numpy(), golden_large_nnz(g, K, 1, Yseq), absY) <= NNZ_TOL


@pytest.mark.parametrize("name,K", CASES)
@pytest.mark.parametrize("variant", [smfv.Variant.ROWWISE, smfv.Variant.COLUMNWISE, smfv.Variant.NONZERO])
def test_rank_plans_vs_reference_large(gpu, problems, name, K, variant):
    g, A, X, Yseq, absY, dA, dX = problems(name, K)
    m = A.numRows
    for p in golden_large_cases()[name]["p"]:
        root = p - 1
        first, last, off, cnt = D.exchange_plan(variant, m, A.nnz, A.rowPtr, K, p)
        Y = torch.full((m, K), float("nan"), dtype=torch.float64, device=gpu)
        blocks = []
        for r in range(p):
            P = D.DistPlan(None, variant, dA, K, to_all=False, root=root, rank=(r, p))
            P.run_local(dX, Y)
            blocks.append(P.exchange_buffer())
            torch.cuda.synchronize()
        if variant != smfv.Variant.ROWWISE:
            xbuf = torch.full((max(int((off + cnt).max()), 1),), float("nan"), dtype=torch.float64, device=gpu)
            replay_exchange(variant, A, K, p, root, blocks, xbuf)
            assemble(variant, A, K, p, xbuf, Y, first, last)
        torch.cuda.synchronize()
        Yh = Y.cpu().numpy()
        if variant == smfv.Variant.NONZERO:
            assert rel(Yh, golden_large_nnz(g, K, p, Yseq), absY) <= NNZ_TOL, (name, K, p)
        else:
            key = f"sha_row_k{K}_p{p}" if variant == smfv.Variant.ROWWISE else f"sha_col_k{K}_p{p}"
            assert sha_f64(Yh) == str(g[key]), (name, K, p, variant)
