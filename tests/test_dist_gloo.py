"""Multi-process (world_size 2, 3 and (r6) 5, gloo, CPU) test of the distributed
exchange: each rank takes its part from the NATIVE plan (smfv_dist_plan --
the function the GPU path runs), computes it with the oracle, then replays
the NATIVE exchange schedule (smfv_dist_exchange_ops: the exact list of
all-gather / broadcast / send / recv operations smfv_dist_spmm_f64 and the
distributed plans issue to RCCL) with torch.distributed over gloo, assembles
Y as the device kernels do (panels_to_rowmajor, combine_row_blocks) and must
match the reference's sequential result -- on every rank for TO_ALL, on the
root for TO_ROOT (the reference's MPI_Gatherv / MPI_Reduce semantics,
SC/...RowWise.cpp:85-87, ...ColumnWise.cpp:82-84, ...NonZeroElement.cpp:88)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _local_part(variant, A, X, first, last, rank, p):
    from oracle import oracle
    rp, ci, va = A.rowPtr, A.colIndices, A.values
    if variant == 1:  # rows [first, last]
        sub = rp[first:last + 2] - rp[first]
        lo, hi = rp[first], rp[last + 1]
        return oracle.spmm("sequential", sub, ci[lo:hi], va[lo:hi], X).reshape(-1)
    if variant == 2:  # columns [first, last] -> [m x kc] panel
        return np.ascontiguousarray(oracle.spmm("sequential", rp, ci, va, X)[:, first:last + 1]).reshape(-1)
    # nnz range -> partial rows [first, last]
    s, e = oracle.partition_nnz(int(rp[-1]), p, rank)
    if e <= s:
        return np.zeros(0)
    sub = np.clip(rp[first:last + 2], s, e) - s
    return oracle.spmm("sequential", sub, ci[s:e], va[s:e], X).reshape(-1)


def run_ops(ops, xbuf: torch.Tensor, rank: int, p: int) -> None:
    """Replay a native exchange schedule over torch.distributed (gloo).  The
    ops of one schedule form one RCCL group (ncclGroupStart / End): a
    schedule of point-to-point ops (the chunked all-gatherv sends AND
    receives on every rank) is replayed as isend / irecv completed together,
    as the group completes them."""
    from sparsematrixmultiplicationmpi_amd.dist import EX_ALLGATHER, EX_BCAST, EX_RECV, EX_SEND
    if ops and all(k in (EX_SEND, EX_RECV) for k, _, _, _ in ops) and \
            any(k == EX_RECV for k, _, _, _ in ops) and any(k == EX_SEND for k, _, _, _ in ops):
        reqs, landing = [], []
        for kind, peer, off, cnt in ops:
            if kind == EX_SEND:
                reqs.append(dist.isend(xbuf[off:off + cnt].clone(), dst=peer))
            else:
                blk = torch.zeros(cnt, dtype=torch.float64)
                reqs.append(dist.irecv(blk, src=peer))
                landing.append((off, cnt, blk))
        for rq in reqs:
            rq.wait()
        for off, cnt, blk in landing:
            xbuf[off:off + cnt] = blk
        return
    for kind, peer, off, cnt in ops:
        if kind == EX_ALLGATHER:
            base = off - rank * cnt
            parts = [torch.zeros(cnt, dtype=torch.float64) for _ in range(p)]
            dist.all_gather(parts, xbuf[off:off + cnt].clone())
            for r in range(p):
                xbuf[base + r * cnt: base + (r + 1) * cnt] = parts[r]
        elif kind == EX_BCAST:
            blk = xbuf[off:off + cnt].clone()
            dist.broadcast(blk, src=peer)
            xbuf[off:off + cnt] = blk
        elif kind == EX_SEND:
            dist.send(xbuf[off:off + cnt].clone(), dst=peer)
        elif kind == EX_RECV:
            blk = torch.zeros(cnt, dtype=torch.float64)
            dist.recv(blk, src=peer)
            xbuf[off:off + cnt] = blk
        else:
            raise AssertionError(kind)


def _worker(rank, p, port, variant, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=p)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import sparsematrixmultiplicationmpi_amd as smfv
        from sparsematrixmultiplicationmpi_amd.dist import TO_ALL, exchange_ops, exchange_plan
        from oracle import oracle

        A = smfv.gen_random_rows(900, 700, 8, 2.0, 300, 31)
        K = 6
        X = np.random.default_rng(31).uniform(-1, 1, (A.numCols, K))
        m, nnz = A.numRows, A.nnz
        root = p - 1  # a root other than 0
        first, last, off, cnt = exchange_plan(variant, m, nnz, A.rowPtr, K, p)
        mine = _local_part(variant, A, X, first[rank], last[rank], rank, p)
        assert mine.size == cnt[rank]
        xbuf = torch.full((int((off + cnt).max()),), float("nan"), dtype=torch.float64)
        xbuf[off[rank]: off[rank] + cnt[rank]] = torch.from_numpy(mine)
        ops = exchange_ops(variant, mode, root, m, nnz, A.rowPtr, K, p, rank)
        run_ops(ops, xbuf, rank, p)
        if mode != TO_ALL and rank != root:
            q.put((rank, True, "not the root"))
            dist.destroy_process_group()
            return
        xb = xbuf.numpy()
        # assemble as the device code does
        if variant == 1:
            Y = xb.reshape(m, K)
        elif variant == 2:
            Y = np.zeros((m, K))
            for r in range(p):
                kc = last[r] - first[r] + 1
                if kc > 0:
                    Y[:, first[r]:last[r] + 1] = xb[off[r]: off[r] + m * kc].reshape(m, kc)
        else:
            Y = np.zeros((m, K))
            seen = np.zeros(m, bool)
            for r in range(p):
                nr = last[r] - first[r] + 1
                if nr <= 0:
                    continue
                blk = xb[off[r]: off[r] + nr * K].reshape(nr, K)
                rows = slice(first[r], last[r] + 1)
                Y[rows] = np.where(seen[rows, None], Y[rows] + blk, blk)
                seen[rows] = True
        Yref = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
        if variant == 3:
            err = float(np.max(np.abs(Y - Yref)))
            ok = err <= 1e-12
        else:
            ok = np.array_equal(Y.view(np.uint64), Yref.view(np.uint64))
            err = float(np.nanmax(np.abs(Y - Yref)))
        q.put((rank, ok, (err, ops)))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("p", [2, 3, 5])
@pytest.mark.parametrize("variant", [1, 2, 3])
def test_gloo_exchange(variant, p, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, p, port, variant, mode, q)) for r in range(p)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(p)]
    for pr in procs:
        pr.join(timeout=60)
    for rank, ok, err in res:
        assert ok, (variant, p, mode, rank, err)


def _rowpart_worker(rank, p, port, m, q):
    """Bench config 5's layout: rank r generates ONLY its RowWise rows
    (counter-based generator), computes them, and the native schedule
    (one all-gather of equal blocks, else broadcasts) assembles the full Y."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=p)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import sparsematrixmultiplicationmpi_amd as smfv
        from sparsematrixmultiplicationmpi_amd.dist import EX_ALLGATHER, TO_ALL, exchange_ops, exchange_plan
        from oracle import oracle

        K = 4
        first, last, off, cnt = exchange_plan(1, m, 0, None, K, p)
        A_loc = smfv.gen_random_rows(m, m, 16.0, 0.0, 16, 42, int(first[rank]), int(last[rank]) + 1)
        X = np.random.default_rng(7).uniform(-1, 1, (m, K))
        mine = oracle.spmm("sequential", A_loc.rowPtr, A_loc.colIndices, A_loc.values, X).reshape(-1)
        assert mine.size == cnt[rank] and off[rank] == first[rank] * K
        xbuf = torch.full((m * K,), float("nan"), dtype=torch.float64)
        xbuf[off[rank]: off[rank] + cnt[rank]] = torch.from_numpy(mine)
        ops = exchange_ops(1, TO_ALL, 0, m, 0, None, K, p, rank)
        run_ops(ops, xbuf, rank, p)
        Y = xbuf.numpy().reshape(m, K)
        A = smfv.gen_random_rows(m, m, 16.0, 0.0, 16, 42)
        Yref = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
        single = len(ops) == 1 and ops[0][0] == EX_ALLGATHER
        q.put((rank, bool(np.array_equal(Y.view(np.uint64), Yref.view(np.uint64))), single))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("p,m", [(2, 4000), (3, 4001)])
def test_gloo_rowpart(p, m):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rowpart_worker, args=(r, p, port, m, q)) for r in range(p)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(p)]
    for pr in procs:
        pr.join(timeout=60)
    for rank, ok, info in res:
        assert ok, (p, m, rank, info)
        assert info is (m % p == 0)  # equal blocks -> the single ncclAllGather op


def _golden_worker(rank, p, port, name, q):
    """The reference's own degenerate case at p = 8 (pat4x6_k3: K < p for
    ColumnWise, m < p for RowWise, nnz < p for NonZeroElement): every rank
    takes its part from the native plan, computes it with the oracle, and
    the native schedule, replayed over gloo, must give the reference's own
    results -- Y_seq bit for bit (RowWise / ColumnWise), the reference's
    NonZeroElement output at p (Y_nnz_p{p}) within 1e-12 x sum|a||x| --
    for every variant, on every rank (TO_ALL) or the root (TO_ROOT)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=p)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import sparsematrixmultiplicationmpi_amd as smfv
        from sparsematrixmultiplicationmpi_amd.dist import TO_ALL, exchange_ops, exchange_plan
        from conftest import load_golden
        from oracle import oracle

        g = load_golden(name)
        A = smfv.SparseMatrix(np.asarray(g["values"], np.float64), np.asarray(g["col_idx"], np.int32),
                              np.asarray(g["row_ptr"], np.int32), int(g["m"]), int(g["n"]))
        X = np.ascontiguousarray(g["X"], np.float64)
        K = X.shape[1]
        m, nnz = A.numRows, A.nnz
        absY = oracle.spmm("sequential", A.rowPtr, A.colIndices, np.abs(A.values), np.abs(X))
        results = []
        for variant in (1, 2, 3):
            first, last, off, cnt = exchange_plan(variant, m, nnz, A.rowPtr, K, p)
            for mode in (0, 1):
                root = p - 1
                mine = _local_part(variant, A, X, first[rank], last[rank], rank, p)
                assert mine.size == cnt[rank]
                xbuf = torch.full((max(int((off + cnt).max()), 1),), float("nan"), dtype=torch.float64)
                xbuf[off[rank]: off[rank] + cnt[rank]] = torch.from_numpy(mine)
                run_ops(exchange_ops(variant, mode, root, m, nnz, A.rowPtr, K, p, rank), xbuf, rank, p)
                if mode != TO_ALL and rank != root:
                    continue
                xb = xbuf.numpy()
                Y = np.zeros((m, K))
                if variant == 1:
                    Y = xb[:m * K].reshape(m, K)
                elif variant == 2:
                    for r in range(p):
                        kc = last[r] - first[r] + 1
                        if kc > 0:
                            Y[:, first[r]:last[r] + 1] = xb[off[r]: off[r] + m * kc].reshape(m, kc)
                else:
                    seen = np.zeros(m, bool)
                    for r in range(p):
                        nr = last[r] - first[r] + 1
                        if nr <= 0:
                            continue
                        blk = xb[off[r]: off[r] + nr * K].reshape(nr, K)
                        rows = slice(first[r], last[r] + 1)
                        Y[rows] = np.where(seen[rows, None], Y[rows] + blk, blk)
                        seen[rows] = True
                if variant == 3:
                    err = float(np.max(np.abs(Y - g[f"Y_nnz_p{p}"]) / np.maximum(absY, 1e-300)))
                    results.append((variant, mode, err <= 1e-12, err))
                else:
                    results.append((variant, mode, bool(np.array_equal(Y.view(np.uint64), g["Y_seq"].view(np.uint64))),
                                    None))
        q.put((rank, all(r[2] for r in results), results))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures
        q.put((rank, False, repr(e)))


def test_gloo_reference_degenerate_p8():
    """pat4x6_k3 at p = 8 over gloo: all three variants, both modes, root 7."""
    p = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_golden_worker, args=(r, p, port, "pat4x6_k3", q)) for r in range(p)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(p)]
    for pr in procs:
        pr.join(timeout=60)
    for rank, ok, info in res:
        assert ok, (rank, info)


def _chunked_worker(rank, p, port, partition, chunks, q):
    """(r5) The work-balanced ROWWISE partition and the chunked exchange
    (SMFV_DIST_CHUNKS): rank r's block [first, last] of the native balanced
    (or reference) partition, computed by the oracle, then the native
    per-chunk schedules run chunk after chunk -- point-to-point sends and
    receives of each chunk to every peer (TO_ALL) or the root (TO_ROOT) --
    must assemble the reference's sequential Y bit for bit."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=p)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import sparsematrixmultiplicationmpi_amd as smfv
        from sparsematrixmultiplicationmpi_amd.dist import TO_ALL, chunk_rows, dist_opts, exchange_ops, exchange_plan
        from oracle import oracle

        A = smfv.gen_random_rows(1500, 900, 8, 2.0, 300, 37)
        K = 5
        X = np.random.default_rng(37).uniform(-1, 1, (A.numCols, K))
        m, nnz = A.numRows, A.nnz
        dopts = dist_opts(partition, chunks)
        first, last, off, cnt = exchange_plan(1, m, nnz, A.rowPtr, K, p, dopts)
        # chunk boundaries tile the rank's block
        b = chunk_rows(1, dopts, m, nnz, A.rowPtr, K, p, rank)
        assert b[0] == first[rank] and b[-1] == last[rank] + 1 and len(b) == chunks + 1 and b == sorted(b)
        Yref = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
        out = []
        for mode in (0, 1):
            root = p - 1
            xbuf = torch.full((m * K,), float("nan"), dtype=torch.float64)
            mine = _local_part(1, A, X, first[rank], last[rank], rank, p)
            xbuf[off[rank]: off[rank] + cnt[rank]] = torch.from_numpy(mine)
            nops = 0
            for j in range(chunks):
                ops = exchange_ops(1, mode, root, m, nnz, A.rowPtr, K, p, rank, dopts, j)
                nops += len(ops)
                run_ops(ops, xbuf, rank, p)
            if mode != TO_ALL and rank != root:
                continue
            Y = xbuf.numpy().reshape(m, K)
            out.append((mode, bool(np.array_equal(Y.view(np.uint64), Yref.view(np.uint64))), nops))
        q.put((rank, all(o[1] for o in out), out))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures
        import traceback
        q.put((rank, False, traceback.format_exc()[-1500:]))


@pytest.mark.parametrize("p,partition,chunks", [(2, "balanced", 2), (3, "balanced", 3), (3, "reference", 2),
                                                (8, "balanced", 4), (2, "balanced", 1)])
def test_gloo_chunked_rowwise_exchange(p, partition, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunked_worker, args=(r, p, port, partition, chunks, q)) for r in range(p)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(p)]
    for pr in procs:
        pr.join(timeout=60)
    for rank, ok, info in res:
        assert ok, (p, partition, chunks, rank, info)
