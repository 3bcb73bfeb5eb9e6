// smfv_dist.cpp -- multi-GPU variants over RCCL (one process per GPU, xGMI).
//
// Each function mirrors one MPI decomposition of the reference
// (SC = /root/reference/Source Code) with the rank-local compute on the GPU
// and the single exchange step as RCCL point-to-point / collective calls:
//
//   ROWWISE    rows [r*q + min(r, m%p), ...)      SC/...RowWise.cpp:26-29
//              local block -> Y rows (in place)   :36-50
//              gather-to-root / all-gatherv       :85-87 (MPI_Gatherv)
//   COLUMNWISE K columns K/p, remainder last      SC/...ColumnWise.cpp:25-28
//              local [m x kc] panel               :34-48
//              gather panels + device transpose   :82-84, :109-126
//   NONZERO    nnz/p, remainder to lowest ranks   SC/...NonZeroElement.cpp:24-39
//              merge-path over the own nnz range, partial rows only
//              compact row blocks -> sum per row  :88 (MPI_Reduce SUM over m*K)
//
// The reference's NonZeroElement reduces a FULL m x K partial from every
// rank; here each rank ships only the rows its nnz range touches (the
// boundary rows are the only overlap), which is the same sum with p-fold
// less traffic.  Equal row blocks use ncclAllGather; unequal ones a grouped
// set of ncclBroadcast (all-gatherv) or ncclSend/ncclRecv to the root.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "smfv_internal.h"

struct smfv_comm_s {
    ncclComm_t nccl = nullptr;
    int rank = 0;
    int nranks = 1;
};

namespace {

#define SMFV_NCCL(call)                                                                     \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        if (r_ != ncclSuccess) {                                                            \
            ::smfv::set_error("%s failed: %s (%s:%d)", #call, ncclGetErrorString(r_),       \
                              __FILE__, __LINE__);                                          \
            return SMFV_ERR_COMM;                                                           \
        }                                                                                   \
    } while (0)

// the same inside ncclGroupStart / ncclGroupEnd: a failing call closes the
// group before returning, so the communicator's next collective starts clean
#define SMFV_NCCL_IN_GROUP(call)                                                            \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        if (r_ != ncclSuccess) {                                                            \
            (void)ncclGroupEnd();                                                           \
            ::smfv::set_error("%s failed: %s (%s:%d)", #call, ncclGetErrorString(r_),       \
                              __FILE__, __LINE__);                                          \
            return SMFV_ERR_COMM;                                                           \
        }                                                                                   \
    } while (0)

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// test hook (smfv_test_fail_exchange): the n-th exchange operation run by
// run_exchange fails as an RCCL error would, inside its open group -- the
// error path is exercised without a broken interconnect
long g_fail_exchange = 0;
bool injected_failure() { return g_fail_exchange > 0 && --g_fail_exchange == 0; }

}  // namespace

using smfv::set_error;

extern "C" {

SMFV_API int smfv_comm_unique_id(char out[SMFV_UNIQUE_ID_BYTES])
{
    SMFV_REQUIRE(out, "null output");
    static_assert(sizeof(ncclUniqueId) == SMFV_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId id;
    SMFV_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof id);
    return SMFV_OK;
}

SMFV_API int smfv_comm_init(smfv_comm_t *comm, int nranks, int rank,
                            const char id[SMFV_UNIQUE_ID_BYTES])
{
    SMFV_REQUIRE(comm && id && nranks > 0 && rank >= 0 && rank < nranks, "bad argument");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    auto *c = new smfv_comm_s;
    c->rank = rank;
    c->nranks = nranks;
    ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
        delete c;
        return SMFV_ERR_COMM;
    }
    *comm = c;
    return SMFV_OK;
}

SMFV_API int smfv_comm_destroy(smfv_comm_t comm)
{
    if (!comm) return SMFV_OK;
    ncclResult_t r = ncclCommDestroy(comm->nccl);
    delete comm;
    if (r != ncclSuccess) {
        set_error("ncclCommDestroy failed: %s", ncclGetErrorString(r));
        return SMFV_ERR_COMM;
    }
    return SMFV_OK;
}

SMFV_API int smfv_comm_rank(smfv_comm_t comm) { return comm ? comm->rank : -1; }
SMFV_API int smfv_comm_size(smfv_comm_t comm) { return comm ? comm->nranks : -1; }

SMFV_API int smfv_comm_count(smfv_comm_t comm, int *nranks)
{
    SMFV_REQUIRE(comm && nranks, "null argument");
    SMFV_NCCL(ncclCommCount(comm->nccl, nranks));
    return SMFV_OK;
}

SMFV_API int smfv_comm_bcast(smfv_comm_t comm, void *d_buf, size_t bytes, int root, void *stream)
{
    SMFV_REQUIRE(comm && (d_buf || bytes == 0) && root >= 0 && root < comm->nranks, "bad argument");
    if (comm->nranks == 1 || bytes == 0) return SMFV_OK;
    SMFV_NCCL(ncclBroadcast(d_buf, d_buf, bytes, ncclUint8, root, comm->nccl, smfv::as_stream(stream)));
    return SMFV_OK;
}

SMFV_API int smfv_dist_plan(int variant, int m, int64_t nnz, const int *h_row_ptr, int K, int p,
                            int *first, int *last, int64_t *offset, int64_t *count)
{
    SMFV_REQUIRE(m >= 0 && nnz >= 0 && K >= 0 && p > 0, "bad argument");
    SMFV_REQUIRE(first && last && offset && count, "null output array");
    switch (variant) {
    case SMFV_SEQUENTIAL:
    case SMFV_ROWWISE:
        for (int r = 0; r < p; ++r) {
            int s, e;
            smfv_partition_rows(m, p, r, &s, &e);
            first[r] = s;
            last[r] = e - 1;
            offset[r] = (int64_t)s * K;
            count[r] = (int64_t)(e - s) * K;
        }
        return SMFV_OK;
    case SMFV_COLUMNWISE:
        for (int r = 0; r < p; ++r) {
            int c0, c1;
            smfv_partition_cols(K, p, r, &c0, &c1);
            first[r] = c0;
            last[r] = c1 - 1;
            offset[r] = (int64_t)m * c0;
            count[r] = (int64_t)m * (c1 - c0);
        }
        return SMFV_OK;
    case SMFV_NONZERO: {
        SMFV_REQUIRE(h_row_ptr, "NONZERO needs the host row_ptr");
        SMFV_REQUIRE(h_row_ptr[m] == nnz, "row_ptr[m] != nnz");
        int64_t rows = 0;
        for (int r = 0; r < p; ++r) {
            int64_t s, e;
            smfv_partition_nnz(nnz, p, r, &s, &e);
            int rc = smfv_nnz_range_rows(m, h_row_ptr, s, e, &first[r], &last[r]);
            if (rc) return rc;
            const int64_t nr = std::max(0, last[r] - first[r] + 1);
            offset[r] = rows * K;
            count[r] = nr * K;
            rows += nr;
        }
        return SMFV_OK;
    }
    }
    set_error("unknown variant %d", variant);
    return SMFV_ERR_INVALID;
}

namespace {
// (r5) Cuts of rows [lo, hi) into c pieces of equal work, work(row i) =
// 12 B per non-zero + (8K + 4) B (its CSR and Y bytes): cut j is the first
// row i with W(i) >= W(lo) + (W(hi) - W(lo)) * j / c, W(i) = 12 rp[i] +
// (8K + 4) i.  Integer arithmetic only, so every rank computes the same
// cuts.  Without row_ptr: equal row counts.  cut[0] = lo, cut[c] = hi.
void work_cuts(const int *rp, int K, int lo, int hi, int c, int *cut)
{
    const int64_t per_row = 8 * (int64_t)K + 4;
    auto W = [&](int i) -> int64_t { return 12 * (int64_t)rp[i] + per_row * (int64_t)i; };
    cut[0] = lo;
    cut[c] = hi;
    for (int j = 1; j < c; ++j) {
        if (!rp) {
            cut[j] = lo + (int)((int64_t)(hi - lo) * j / c);
            continue;
        }
        const __int128 span = (__int128)(W(hi) - W(lo));
        const int64_t target = W(lo) + (int64_t)(span * j / c);
        int a = std::max(lo, cut[j - 1]), b = hi;  // first i in [a, b] with W(i) >= target
        while (a < b) {
            const int mid = a + (b - a) / 2;
            if (W(mid) >= target) b = mid; else a = mid + 1;
        }
        cut[j] = a;
    }
}
}  // namespace

SMFV_API int smfv_dist_plan_opts(int variant, int dopts, int m, int64_t nnz, const int *h_row_ptr, int K, int p,
                                 int *first, int *last, int64_t *offset, int64_t *count)
{
    const bool rows = variant == SMFV_ROWWISE || variant == SMFV_SEQUENTIAL;
    if (!rows || !(dopts & SMFV_DIST_BALANCED_ROWS) || !h_row_ptr)
        return smfv_dist_plan(variant, m, nnz, h_row_ptr, K, p, first, last, offset, count);
    SMFV_REQUIRE(m >= 0 && K >= 0 && p > 0, "bad argument");
    SMFV_REQUIRE(first && last && offset && count, "null output array");
    std::vector<int> cut((size_t)p + 1);
    work_cuts(h_row_ptr, K, 0, m, p, cut.data());
    for (int r = 0; r < p; ++r) {
        first[r] = cut[r];
        last[r] = cut[r + 1] - 1;
        offset[r] = (int64_t)cut[r] * K;
        count[r] = (int64_t)(cut[r + 1] - cut[r]) * K;
    }
    return SMFV_OK;
}

namespace {
struct Plan {
    std::vector<int> first, last;
    std::vector<int64_t> offset, count;
    int64_t total = 0;  // doubles in the exchange buffer
    int K = 0;
    int chunks = 1;         // (r5) ROWWISE: row chunks per rank, each exchanged on its own
    std::vector<int> cb;    // chunked: rank r's chunk j = rows [cb[r (chunks + 1) + j], cb[r (chunks + 1) + j + 1])
};
// (the plain host functions and the plan-less smfv_dist_spmm_f64 take the
// reference's partition; distributed plans pass their own options)
int make_plan(int variant, int m, int64_t nnz, const int *h_row_ptr, int K, int p, Plan &P, int dopts = 0)
{
    P.first.assign(p, 0);
    P.last.assign(p, -1);
    P.offset.assign(p, 0);
    P.count.assign(p, 0);
    P.K = K;
    int rc = smfv_dist_plan_opts(variant, dopts, m, nnz, h_row_ptr, K, p, P.first.data(), P.last.data(),
                                 P.offset.data(), P.count.data());
    if (rc) return rc;
    P.total = 0;
    for (int r = 0; r < p; ++r) P.total = std::max(P.total, P.offset[r] + P.count[r]);
    const int c = SMFV_DIST_CHUNKS_OF(dopts);
    P.chunks = 1;
    P.cb.clear();
    if (c > 1) {
        if (variant != SMFV_ROWWISE && variant != SMFV_SEQUENTIAL) {
            set_error("SMFV_DIST_CHUNKS applies to ROWWISE (variant %d)", variant);
            return SMFV_ERR_INVALID;
        }
        P.chunks = c;
        P.cb.assign((size_t)p * (c + 1), 0);
        for (int r = 0; r < p; ++r) work_cuts(h_row_ptr, K, P.first[r], P.last[r] + 1, c, &P.cb[(size_t)r * (c + 1)]);
    }
    return SMFV_OK;
}
}  // namespace

SMFV_API int smfv_dist_chunk_rows(int variant, int dopts, int m, int64_t nnz, const int *h_row_ptr, int K, int p,
                                  int rank, int *bounds, int *nchunks)
{
    SMFV_REQUIRE(bounds && nchunks && p > 0 && rank >= 0 && rank < p, "bad argument");
    Plan P;
    int rc = make_plan(variant, m, nnz, h_row_ptr, K, p, P, dopts);
    if (rc) return rc;
    *nchunks = P.chunks;
    if (P.chunks == 1) {
        bounds[0] = P.first[rank];
        bounds[1] = P.last[rank] + 1;
    } else {
        for (int j = 0; j <= P.chunks; ++j) bounds[j] = P.cb[(size_t)rank * (P.chunks + 1) + j];
    }
    return SMFV_OK;
}

SMFV_API int smfv_dist_workspace_bytes(smfv_comm_t comm, int variant, int m, int64_t nnz,
                                       const int *h_row_ptr, int K, size_t *bytes)
{
    SMFV_REQUIRE(comm && bytes && m >= 0 && nnz >= 0 && K >= 0, "bad argument");
    switch (variant) {
    case SMFV_SEQUENTIAL:
    case SMFV_ROWWISE:
        *bytes = 0;  // blocks are exchanged in place inside Y
        return SMFV_OK;
    case SMFV_COLUMNWISE:
        *bytes = align256((size_t)m * (size_t)K * sizeof(double));
        return SMFV_OK;
    case SMFV_NONZERO: {
        Plan P;
        int rc = make_plan(variant, m, nnz, h_row_ptr, K, comm->nranks, P);
        if (rc) return rc;
        const int r = comm->rank;
        int64_t s, e;
        smfv_partition_nnz(nnz, comm->nranks, r, &s, &e);
        const size_t merge =
            smfv::merge_workspace_bytes(std::max(0, P.last[r] - P.first[r] + 1), e - s, K);
        *bytes = align256((size_t)P.total * sizeof(double)) + merge;
        return SMFV_OK;
    }
    }
    set_error("unknown variant %d", variant);
    return SMFV_ERR_INVALID;
}

// The one exchange step of a distributed variant as data: gather-to-root
// (Gatherv / the Reduce's target) or all-gatherv of the ranks' blocks
// P.offset/P.count inside the exchange buffer; equal, back-to-back blocks
// go through one all-gather.
struct ExOp {
    int kind, peer;
    int64_t offset, count;
};

static std::vector<ExOp> exchange_schedule(const Plan &P, int p, int rank, bool may_be_equal, bool to_all,
                                           int root, int chunk = 0)
{
    std::vector<ExOp> ops;
    if (p <= 1) return ops;
    if (P.chunks > 1) {
        // (r5) chunk `chunk` of every rank's row block, point to point: every
        // rank sends its chunk to each peer (TO_ALL) or to the root, and
        // receives theirs -- one group; over xGMI's full mesh each link
        // carries one chunk per direction
        const int C1 = P.chunks + 1;
        auto blk = [&](int r, int64_t &off, int64_t &cnt) {
            const int s = P.cb[(size_t)r * C1 + chunk], e = P.cb[(size_t)r * C1 + chunk + 1];
            off = (int64_t)s * P.K;
            cnt = (int64_t)(e - s) * P.K;
        };
        int64_t off, cnt;
        blk(rank, off, cnt);
        if (to_all || rank != root) {
            if (cnt > 0)
                for (int r = 0; r < p; ++r)
                    if (r != rank && (to_all || r == root)) ops.push_back({SMFV_EX_SEND, r, off, cnt});
        }
        if (to_all || rank == root) {
            for (int r = 0; r < p; ++r) {
                if (r == rank) continue;
                blk(r, off, cnt);
                if (cnt > 0) ops.push_back({SMFV_EX_RECV, r, off, cnt});
            }
        }
        return ops;
    }
    bool equal = may_be_equal;
    for (int r = 1; r < p && equal; ++r)
        equal = P.count[r] == P.count[0] && P.offset[r] == P.offset[0] + r * P.count[0];
    if (to_all && equal && P.count[0] > 0) {
        ops.push_back({SMFV_EX_ALLGATHER, -1, P.offset[rank], P.count[0]});
        return ops;
    }
    for (int r = 0; r < p; ++r) {
        if (P.count[r] == 0) continue;
        if (to_all)
            ops.push_back({SMFV_EX_BCAST, r, P.offset[r], P.count[r]});
        else if (rank == root && r != root)
            ops.push_back({SMFV_EX_RECV, r, P.offset[r], P.count[r]});
        else if (rank == r && r != root)
            ops.push_back({SMFV_EX_SEND, root, P.offset[r], P.count[r]});
    }
    return ops;
}

// Runs a schedule with RCCL on `st` (one group; the all-gather alone).
// comm == NULL (a rank plan, smfv_dist_plan_create_rank) runs no exchange.
static int run_exchange(smfv_comm_t comm, const std::vector<ExOp> &ops, double *xbuf, hipStream_t st)
{
    if (ops.empty()) return SMFV_OK;
    if (!comm) {
        set_error("exchange needs a communicator (this plan was created for one rank alone)");
        return SMFV_ERR_COMM;
    }
    if (ops.size() == 1 && ops[0].kind == SMFV_EX_ALLGATHER) {
        const ExOp &o = ops[0];
        if (injected_failure()) {
            set_error("ncclAllGather failed: injected test failure (SMFV_TEST_FAIL_EXCHANGE)");
            return SMFV_ERR_COMM;
        }
        // block r lands at offset - rank * count + r * count
        SMFV_NCCL(ncclAllGather(xbuf + o.offset, xbuf + o.offset - (int64_t)comm->rank * o.count, (size_t)o.count,
                                ncclDouble, comm->nccl, st));
        return SMFV_OK;
    }
    SMFV_NCCL(ncclGroupStart());
    for (const ExOp &o : ops) {
        double *blk = xbuf + o.offset;
        const size_t cnt = (size_t)o.count;
        if (injected_failure()) {
            (void)ncclGroupEnd();
            set_error("exchange op %d failed: injected test failure (smfv_test_fail_exchange)", o.kind);
            return SMFV_ERR_COMM;
        }
        switch (o.kind) {
        case SMFV_EX_BCAST: SMFV_NCCL_IN_GROUP(ncclBroadcast(blk, blk, cnt, ncclDouble, o.peer, comm->nccl, st)); break;
        case SMFV_EX_RECV: SMFV_NCCL_IN_GROUP(ncclRecv(blk, cnt, ncclDouble, o.peer, comm->nccl, st)); break;
        case SMFV_EX_SEND: SMFV_NCCL_IN_GROUP(ncclSend(blk, cnt, ncclDouble, o.peer, comm->nccl, st)); break;
        default: (void)ncclGroupEnd(); set_error("bad exchange op %d", o.kind); return SMFV_ERR_INVALID;
        }
    }
    SMFV_NCCL(ncclGroupEnd());
    return SMFV_OK;
}

static int exchange_blocks(smfv_comm_t comm, const Plan &P, bool may_be_equal, bool to_all, int root,
                           double *xbuf, hipStream_t st)
{
    return run_exchange(comm, exchange_schedule(P, comm->nranks, comm->rank, may_be_equal, to_all, root), xbuf,
                        st);
}

SMFV_API int smfv_dist_exchange_ops(int variant, int mode, int root, int m, int64_t nnz, const int *h_row_ptr,
                                    int K, int p, int rank, int *kinds, int *peers, int64_t *offsets,
                                    int64_t *counts, int *nops)
{
    SMFV_REQUIRE(kinds && peers && offsets && counts && nops, "null output array");
    SMFV_REQUIRE(p > 0 && rank >= 0 && rank < p && root >= 0 && root < p, "bad rank / root");
    SMFV_REQUIRE(mode == SMFV_TO_ROOT || mode == SMFV_TO_ALL, "bad mode %d", mode);
    Plan P;
    int rc = make_plan(variant, m, nnz, h_row_ptr, K, p, P);
    if (rc) return rc;
    const auto ops = exchange_schedule(P, p, rank, variant != SMFV_NONZERO, mode == SMFV_TO_ALL, root);
    for (size_t i = 0; i < ops.size(); ++i) {
        kinds[i] = ops[i].kind;
        peers[i] = ops[i].peer;
        offsets[i] = ops[i].offset;
        counts[i] = ops[i].count;
    }
    *nops = (int)ops.size();
    return SMFV_OK;
}

SMFV_API int smfv_dist_exchange_ops_opts(int variant, int dopts, int mode, int root, int m, int64_t nnz,
                                         const int *h_row_ptr, int K, int p, int rank, int chunk, int *kinds,
                                         int *peers, int64_t *offsets, int64_t *counts, int *nops)
{
    SMFV_REQUIRE(kinds && peers && offsets && counts && nops, "null output array");
    SMFV_REQUIRE(p > 0 && rank >= 0 && rank < p && root >= 0 && root < p, "bad rank / root");
    SMFV_REQUIRE(mode == SMFV_TO_ROOT || mode == SMFV_TO_ALL, "bad mode %d", mode);
    Plan P;
    int rc = make_plan(variant, m, nnz, h_row_ptr, K, p, P, dopts);
    if (rc) return rc;
    SMFV_REQUIRE(chunk >= 0 && chunk < P.chunks, "chunk %d of %d", chunk, P.chunks);
    const auto ops = exchange_schedule(P, p, rank, variant != SMFV_NONZERO, mode == SMFV_TO_ALL, root, chunk);
    for (size_t i = 0; i < ops.size(); ++i) {
        kinds[i] = ops[i].kind;
        peers[i] = ops[i].peer;
        offsets[i] = ops[i].offset;
        counts[i] = ops[i].count;
    }
    *nops = (int)ops.size();
    return SMFV_OK;
}

SMFV_API int smfv_comm_exchange_f64(smfv_comm_t comm, const int *kinds, const int *peers, const int64_t *offsets,
                                    const int64_t *counts, int nops, double *d_buf, void *stream)
{
    SMFV_REQUIRE(comm && nops >= 0 && (nops == 0 || (kinds && peers && offsets && counts && d_buf)), "bad argument");
    std::vector<ExOp> ops((size_t)nops);
    for (int i = 0; i < nops; ++i) {
        SMFV_REQUIRE(kinds[i] >= SMFV_EX_ALLGATHER && kinds[i] <= SMFV_EX_RECV, "bad op kind %d", kinds[i]);
        SMFV_REQUIRE(offsets[i] >= 0 && counts[i] >= 0, "bad op range");
        SMFV_REQUIRE(kinds[i] == SMFV_EX_ALLGATHER || (peers[i] >= 0 && peers[i] < comm->nranks), "bad peer %d",
                     peers[i]);
        SMFV_REQUIRE(kinds[i] != SMFV_EX_ALLGATHER || (nops == 1 && offsets[i] >= (int64_t)comm->rank * counts[i]),
                     "an all-gather op runs alone and its blocks start at offset - rank * count >= 0");
        ops[(size_t)i] = {kinds[i], peers[i], offsets[i], counts[i]};
    }
    return run_exchange(comm, ops, d_buf, smfv::as_stream(stream));
}

SMFV_API void smfv_test_fail_exchange(int nth) { g_fail_exchange = nth > 0 ? nth : 0; }

SMFV_API int smfv_dist_spmm_f64(smfv_comm_t comm, int variant, int mode, int root, int m, int n,
                                int64_t nnz, const int *h_row_ptr, const int *d_row_ptr,
                                const int *d_col_idx, const double *d_values, const double *d_X,
                                int K, double *d_Y, void *d_workspace, size_t workspace_bytes,
                                void *stream)
{
    SMFV_REQUIRE(comm, "null communicator");
    SMFV_REQUIRE(mode == SMFV_TO_ROOT || mode == SMFV_TO_ALL, "bad mode %d", mode);
    SMFV_REQUIRE(m >= 0 && n >= 0 && nnz >= 0 && K >= 0, "negative size");
    const int p = comm->nranks, rank = comm->rank;
    SMFV_REQUIRE(root >= 0 && root < p, "bad root %d", root);
    hipStream_t st = smfv::as_stream(stream);
    size_t need = 0;
    int rc = smfv_dist_workspace_bytes(comm, variant, m, nnz, h_row_ptr, K, &need);
    if (rc) return rc;
    if (workspace_bytes < need || (need && !d_workspace)) {
        set_error("distributed workspace too small: %zu < %zu", workspace_bytes, need);
        return SMFV_ERR_WORKSPACE;
    }
    Plan P;
    rc = make_plan(variant, m, nnz, h_row_ptr, K, p, P);
    if (rc) return rc;
    const bool to_all = mode == SMFV_TO_ALL;

    // 1) rank-local compute into this rank's slot of the exchange buffer
    double *xbuf = nullptr;
    if (variant == SMFV_ROWWISE || variant == SMFV_SEQUENTIAL) {
        xbuf = d_Y;
        rc = smfv_spmm_rowblock_f64(P.first[rank], P.last[rank] + 1, n, d_row_ptr, d_col_idx,
                                    d_values, d_X, K, K, d_Y + P.offset[rank], K, stream);
    } else if (variant == SMFV_COLUMNWISE) {
        xbuf = static_cast<double *>(d_workspace);
        const int kc = P.last[rank] - P.first[rank] + 1;
        rc = smfv_spmm_colpanel_f64(m, n, P.first[rank], P.last[rank] + 1, d_row_ptr, d_col_idx,
                                    d_values, d_X, K, xbuf + P.offset[rank], std::max(1, kc),
                                    stream);
    } else if (variant == SMFV_NONZERO) {
        xbuf = static_cast<double *>(d_workspace);
        const size_t blocks_b = align256((size_t)P.total * sizeof(double));
        int64_t s, e;
        smfv_partition_nnz(nnz, p, rank, &s, &e);
        rc = smfv_spmm_nnzrange_f64(P.first[rank], P.last[rank], s, e, n, d_row_ptr, d_col_idx,
                                    d_values, d_X, K, K, xbuf + P.offset[rank], K,
                                    static_cast<char *>(d_workspace) + blocks_b,
                                    workspace_bytes - blocks_b, stream);
    } else {
        set_error("unknown variant %d", variant);
        return SMFV_ERR_INVALID;
    }
    if (rc) return rc;

    // 2) the one exchange step
    rc = exchange_blocks(comm, P, variant != SMFV_NONZERO, to_all, root, xbuf, st);
    if (rc) return rc;

    // 3) assemble Y where it is wanted
    if (!(to_all || rank == root)) return SMFV_OK;
    if (variant == SMFV_COLUMNWISE) return smfv_panels_to_rowmajor_f64(m, K, p, xbuf, d_Y, K, stream);
    if (variant == SMFV_NONZERO)
        return smfv_combine_row_blocks_f64(m, K, p, P.first.data(), P.last.data(), xbuf, d_Y, K,
                                           stream);
    return SMFV_OK;
}

SMFV_API int smfv_dist_rowpart_spmm_f64(smfv_comm_t comm, int mode, int root, int m, int n,
                                        const int *d_row_ptr_local, const int *d_col_idx_local,
                                        const double *d_values_local, const double *d_X, int K,
                                        double *d_Y, void *stream)
{
    SMFV_REQUIRE(comm, "null communicator");
    SMFV_REQUIRE(mode == SMFV_TO_ROOT || mode == SMFV_TO_ALL, "bad mode %d", mode);
    SMFV_REQUIRE(m >= 0 && n >= 0 && K >= 0, "negative size");
    const int p = comm->nranks, rank = comm->rank;
    SMFV_REQUIRE(root >= 0 && root < p, "bad root %d", root);
    hipStream_t st = smfv::as_stream(stream);
    Plan P;
    int rc = make_plan(SMFV_ROWWISE, m, 0, nullptr, K, p, P);
    if (rc) return rc;
    // 1) this rank's rows [first, last] from its local CSR, in place in Y
    const int mloc = P.last[rank] - P.first[rank] + 1;
    rc = smfv_spmm_rowblock_f64(0, mloc, n, d_row_ptr_local, d_col_idx_local, d_values_local, d_X, K, K,
                                d_Y + P.offset[rank], K, stream);
    if (rc) return rc;
    // 2) the one exchange step (all-gather of equal blocks / all-gatherv / gatherv)
    return exchange_blocks(comm, P, true, mode == SMFV_TO_ALL, root, d_Y, st);
}

// ---------------------------------------------------------------------------
// distributed plans
// ---------------------------------------------------------------------------
struct smfv_dist_plan_s {
    smfv_comm_t comm = nullptr;   // NULL: a rank plan (smfv_dist_plan_create_rank), no exchange
    int p = 1, rank = 0;          // this plan's rank of p
    int variant = 0, mode = 0, root = 0, m = 0, n = 0, K = 0;
    bool rowpart = false;
    Plan P;
    std::vector<ExOp> ops;
    smfv_plan_t local = nullptr;  // this rank's share as a single-device plan
    double *xbuf = nullptr;       // exchange buffer (COLUMNWISE panels / NONZERO row blocks)
    // (r5) chunked ROWWISE (SMFV_DIST_CHUNKS): one row-block plan and one
    // exchange per chunk; chunk j's exchange runs on xst after chunk j's
    // compute (event cev[j]) while chunk j + 1 computes; xdone joins back
    std::vector<smfv_plan_t> cplans;
    std::vector<std::vector<ExOp>> cops;
    hipStream_t xst = nullptr;
    std::vector<hipEvent_t> cev;
    hipEvent_t xdone = nullptr;
    ~smfv_dist_plan_s()
    {
        if (local) smfv_plan_destroy(local);
        for (smfv_plan_t c : cplans)
            if (c) smfv_plan_destroy(c);
        for (hipEvent_t e : cev) (void)hipEventDestroy(e);
        if (xdone) (void)hipEventDestroy(xdone);
        if (xst) (void)hipStreamDestroy(xst);
        if (xbuf) (void)hipFree(xbuf);
    }
    int chunk_begin(int j) const { return P.cb[(size_t)rank * (P.chunks + 1) + j]; }
};

static int dist_plan_finish(smfv_dist_plan_s *d, smfv_dist_plan_t *out)
{
    d->ops = exchange_schedule(d->P, d->p, d->rank, d->variant != SMFV_NONZERO, d->mode == SMFV_TO_ALL, d->root);
    if (d->P.chunks > 1) {
        d->cops.clear();
        for (int j = 0; j < d->P.chunks; ++j)
            d->cops.push_back(exchange_schedule(d->P, d->p, d->rank, true, d->mode == SMFV_TO_ALL, d->root, j));
        d->cev.assign((size_t)d->P.chunks, nullptr);
        hipError_t e = hipStreamCreateWithFlags(&d->xst, hipStreamNonBlocking);
        for (int j = 0; e == hipSuccess && j < d->P.chunks; ++j)
            e = hipEventCreateWithFlags(&d->cev[(size_t)j], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&d->xdone, hipEventDisableTiming);
        if (e != hipSuccess) {
            set_error("exchange stream / events: %s", hipGetErrorString(e));
            delete d;
            return SMFV_ERR_HIP;
        }
    }
    if (d->variant == SMFV_COLUMNWISE || d->variant == SMFV_NONZERO) {
        const size_t b = std::max<size_t>((size_t)d->P.total, 1) * sizeof(double);
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&d->xbuf), b);
        if (e != hipSuccess) {
            set_error("hipMalloc(exchange buffer): %s", hipGetErrorString(e));
            delete d;
            return SMFV_ERR_HIP;
        }
    }
    *out = d;
    return SMFV_OK;
}

// rank `rank` of `p` (comm may be NULL: a rank plan without exchange)
static int dist_plan_create(smfv_dist_plan_t *out, smfv_comm_t comm, int p, int rank, int variant, int mode,
                            int root, int m, int n, int64_t nnz, const int *h_row_ptr, const int *h_col_idx, int K,
                            int flags)
{
    SMFV_REQUIRE(out && h_row_ptr, "null plan / row_ptr");
    SMFV_REQUIRE(p > 0 && rank >= 0 && rank < p, "bad rank %d of %d", rank, p);
    SMFV_REQUIRE(mode == SMFV_TO_ROOT || mode == SMFV_TO_ALL, "bad mode %d", mode);
    SMFV_REQUIRE(root >= 0 && root < p, "bad root %d", root);
    SMFV_REQUIRE(m >= 0 && n >= 0 && nnz >= 0 && nnz <= 0x7fffffff && K >= 0 && h_row_ptr[m] == nnz, "bad sizes");
    SMFV_REQUIRE(variant >= SMFV_SEQUENTIAL && variant <= SMFV_NONZERO, "unknown variant %d", variant);
    auto *d = new smfv_dist_plan_s;
    d->comm = comm;
    d->p = p;
    d->rank = rank;
    d->variant = variant == SMFV_SEQUENTIAL ? SMFV_ROWWISE : variant;
    d->mode = mode;
    d->root = root;
    d->m = m;
    d->n = n;
    d->K = K;
    const int dopts = flags & SMFV_DIST_OPTS;
    flags &= ~SMFV_DIST_OPTS;
    int rc = make_plan(d->variant, m, nnz, h_row_ptr, K, p, d->P, dopts);
    if (!rc) {
        const int f = d->P.first[rank], l = d->P.last[rank];
        switch (d->variant) {
        case SMFV_ROWWISE:  // rows [f, l] (SC/...RowWise.cpp:26-50)
            if (d->P.chunks > 1) {  // (r5) one row-block plan per chunk (empty chunks: none)
                d->cplans.assign((size_t)d->P.chunks, nullptr);
                for (int j = 0; !rc && j < d->P.chunks; ++j)
                    if (d->chunk_begin(j + 1) > d->chunk_begin(j))
                        rc = smfv_plan_create_rows(&d->cplans[(size_t)j], SMFV_ROWWISE, d->chunk_begin(j),
                                                   d->chunk_begin(j + 1), n, h_row_ptr, h_col_idx, K, flags);
                break;
            }
            rc = smfv_plan_create_rows(&d->local, SMFV_ROWWISE, f, l + 1, n, h_row_ptr, h_col_idx, K, flags);
            break;
        case SMFV_COLUMNWISE:  // all rows, K columns [f, l] (SC/...ColumnWise.cpp:25-48)
            rc = smfv_plan_create(&d->local, SMFV_COLUMNWISE, m, n, nnz, h_row_ptr, h_col_idx, l - f + 1, flags);
            break;
        default: {  // nnz range [s, e) over rows [f, l] (SC/...NonZeroElement.cpp:24-67)
            int64_t s, e;
            smfv_partition_nnz(nnz, p, rank, &s, &e);
            // (r4) the pattern is passed: the range's whole rows take a row-block
            // plan, the cut rows the merge path (smfv::plan_create)
            rc = smfv::plan_create(&d->local, SMFV_NONZERO, f, std::max(0, l - f + 1), n, s, e, h_row_ptr, h_col_idx,
                                   K, flags, f);
        }
        }
    }
    if (rc) {
        delete d;
        return rc;
    }
    return dist_plan_finish(d, out);
}

SMFV_API int smfv_dist_plan_create(smfv_dist_plan_t *out, smfv_comm_t comm, int variant, int mode, int root, int m,
                                   int n, int64_t nnz, const int *h_row_ptr, const int *h_col_idx, int K, int flags)
{
    SMFV_REQUIRE(comm, "null communicator");
    return dist_plan_create(out, comm, comm->nranks, comm->rank, variant, mode, root, m, n, nnz, h_row_ptr, h_col_idx,
                            K, flags);
}

SMFV_API int smfv_dist_plan_create_rank(smfv_dist_plan_t *out, int p, int rank, int variant, int mode, int root,
                                        int m, int n, int64_t nnz, const int *h_row_ptr, const int *h_col_idx, int K,
                                        int flags)
{
    return dist_plan_create(out, nullptr, p, rank, variant, mode, root, m, n, nnz, h_row_ptr, h_col_idx, K, flags);
}

SMFV_API int smfv_dist_plan_create_rowpart(smfv_dist_plan_t *out, smfv_comm_t comm, int mode, int root, int m, int n,
                                           const int *h_row_ptr_local, const int *h_col_idx_local, int K, int flags)
{
    SMFV_REQUIRE(out && comm && h_row_ptr_local, "null plan / communicator / row_ptr");
    SMFV_REQUIRE(mode == SMFV_TO_ROOT || mode == SMFV_TO_ALL, "bad mode %d", mode);
    SMFV_REQUIRE(root >= 0 && root < comm->nranks, "bad root %d", root);
    SMFV_REQUIRE(m >= 0 && n >= 0 && K >= 0, "bad sizes");
    auto *d = new smfv_dist_plan_s;
    d->comm = comm;
    d->p = comm->nranks;
    d->rank = comm->rank;
    d->variant = SMFV_ROWWISE;
    d->rowpart = true;
    d->mode = mode;
    d->root = root;
    d->m = m;
    d->n = n;
    d->K = K;
    // (the rows are given: the reference partition, one block, SMFV_DIST_* ignored)
    flags &= ~SMFV_DIST_OPTS;
    int rc = make_plan(SMFV_ROWWISE, m, 0, nullptr, K, comm->nranks, d->P);
    const int first = d->P.first[comm->rank];
    const int mloc = d->P.last[comm->rank] - first + 1;
    // the local rows are global rows first.., so the pattern's column c is
    // local row c - first: the tile analysis' neighbours (col_base = first)
    if (!rc)
        rc = smfv::plan_create(&d->local, SMFV_ROWWISE, 0, mloc, n, 0, h_row_ptr_local[mloc], h_row_ptr_local,
                               h_col_idx_local, K, flags, first);
    if (rc) {
        delete d;
        return rc;
    }
    return dist_plan_finish(d, out);
}

SMFV_API int smfv_dist_plan_exchange_buffer(smfv_dist_plan_t d, double **d_buf, int64_t *doubles)
{
    SMFV_REQUIRE(d && d_buf && doubles, "null argument");
    *d_buf = d->xbuf;
    *doubles = d->xbuf ? d->P.total : 0;
    return SMFV_OK;
}

SMFV_API int smfv_dist_plan_partition(smfv_dist_plan_t d, int *first, int *last, int64_t *offset, int64_t *count)
{
    SMFV_REQUIRE(d && first && last && offset && count, "null argument");
    for (int r = 0; r < d->p; ++r) {
        first[r] = d->P.first[r];
        last[r] = d->P.last[r];
        offset[r] = d->P.offset[r];
        count[r] = d->P.count[r];
    }
    return SMFV_OK;
}

SMFV_API int smfv_dist_plan_shape(smfv_dist_plan_t d, int *p, int *rank, int *chunks)
{
    SMFV_REQUIRE(d && p && rank && chunks, "null argument");
    *p = d->p;
    *rank = d->rank;
    *chunks = d->P.chunks;
    return SMFV_OK;
}

SMFV_API int smfv_dist_plan_bind_values(smfv_dist_plan_t d, const double *d_values, void *stream)
{
    SMFV_REQUIRE(d, "null plan");
    if (d->P.chunks > 1) {
        for (smfv_plan_t c : d->cplans)
            if (c) {
                int rc = smfv_plan_bind_values(c, d_values, stream);
                if (rc) return rc;
            }
        return SMFV_OK;
    }
    return smfv_plan_bind_values(d->local, d_values, stream);
}

SMFV_API int smfv_dist_plan_execute_local(smfv_dist_plan_t d, const int *d_row_ptr, const int *d_col_idx,
                                          const double *d_values, const double *d_X, double *d_Y, void *stream)
{
    SMFV_REQUIRE(d, "null plan");
    SMFV_REQUIRE(d_Y || d->m == 0 || d->K == 0, "null Y");
    const int rank = d->rank, K = d->K;
    const int f = d->P.first[rank], l = d->P.last[rank];
    switch (d->variant) {
    case SMFV_ROWWISE:  // in place: this rank's rows of Y
        if (d->P.chunks > 1) {
            for (int j = 0; j < d->P.chunks; ++j)
                if (d->cplans[(size_t)j]) {
                    int rc = smfv_plan_execute(d->cplans[(size_t)j], d_row_ptr, d_col_idx, d_values, d_X, K,
                                               d_Y + (int64_t)d->chunk_begin(j) * K, K, stream);
                    if (rc) return rc;
                }
            return SMFV_OK;
        }
        return smfv_plan_execute(d->local, d_row_ptr, d_col_idx, d_values, d_X, K, d_Y + d->P.offset[rank], K,
                                 stream);
    case SMFV_COLUMNWISE: {  // [m x kc] panel from the X column window
        const int kc = l - f + 1;
        if (kc <= 0) return SMFV_OK;
        return smfv_plan_execute(d->local, d_row_ptr, d_col_idx, d_values, d_X + f, K, d->xbuf + d->P.offset[rank],
                                 kc, stream);
    }
    default:  // compact partial rows [f, l]
        if (l < f) return SMFV_OK;
        return smfv_plan_execute(d->local, d_row_ptr, d_col_idx, d_values, d_X, K, d->xbuf + d->P.offset[rank], K,
                                 stream);
    }
}

SMFV_API int smfv_dist_plan_exchange(smfv_dist_plan_t d, double *d_Y, void *stream)
{
    SMFV_REQUIRE(d, "null plan");
    hipStream_t st = smfv::as_stream(stream);
    double *buf = d->variant == SMFV_ROWWISE ? d_Y : d->xbuf;
    if (d->P.chunks > 1) {  // the chunks' exchanges back to back (the exchange alone)
        for (const auto &ops : d->cops) {
            int rc = run_exchange(d->comm, ops, buf, st);
            if (rc) return rc;
        }
        return SMFV_OK;
    }
    int rc = run_exchange(d->comm, d->ops, buf, st);
    if (rc) return rc;
    const int p = d->p;
    if (!(d->mode == SMFV_TO_ALL || d->rank == d->root)) return SMFV_OK;
    if (d->variant == SMFV_COLUMNWISE) return smfv_panels_to_rowmajor_f64(d->m, d->K, p, d->xbuf, d_Y, d->K, stream);
    if (d->variant == SMFV_NONZERO)
        return smfv_combine_row_blocks_f64(d->m, d->K, p, d->P.first.data(), d->P.last.data(), d->xbuf, d_Y, d->K,
                                           stream);
    return SMFV_OK;
}

#define SMFV_HIP_D(call)                                                                    \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess) {                                                             \
            set_error("%s: %s", #call, hipGetErrorString(e_));                              \
            return SMFV_ERR_HIP;                                                            \
        }                                                                                   \
    } while (0)

SMFV_API int smfv_dist_plan_execute(smfv_dist_plan_t d, const int *d_row_ptr, const int *d_col_idx,
                                    const double *d_values, const double *d_X, double *d_Y, void *stream)
{
    SMFV_REQUIRE(d, "null plan");
    if (d->P.chunks > 1) {
        // (r5) chunk j computes on `stream`; its exchange waits for it on the
        // plan's exchange stream and runs while chunk j + 1 computes; the
        // caller's stream waits for the last exchange.  (A capturing stream
        // forks to the exchange stream and joins back: graph-capturable.)
        // EXPERIMENTAL: its point-to-point RCCL groups have been replayed over
        // gloo and run at one rank, never between two GPUs.
        SMFV_REQUIRE(d_Y || d->m == 0 || d->K == 0, "null Y");
        hipStream_t st = smfv::as_stream(stream);
        const int K = d->K;
        // (r6) once anything was forked to the exchange stream,
        // every return joins it back: the caller's stream never runs ahead
        // of an exchange that may still write d_Y
        bool forked = false;
        auto join = [&](int rc) -> int {
            if (!forked) return rc;
            hipError_t e1 = hipEventRecord(d->xdone, d->xst);
            hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(st, d->xdone, 0) : e1;
            if (e2 != hipSuccess) {
                if (!rc) set_error("chunked execute join: %s", hipGetErrorString(e2));
                // the join itself failed: drain the exchange stream so nothing is left writing d_Y
                (void)hipStreamSynchronize(d->xst);
                return rc ? rc : SMFV_ERR_HIP;
            }
            return rc;
        };
        for (int j = 0; j < d->P.chunks; ++j) {
            if (d->cplans[(size_t)j]) {
                int rc = smfv_plan_execute(d->cplans[(size_t)j], d_row_ptr, d_col_idx, d_values, d_X, K,
                                           d_Y + (int64_t)d->chunk_begin(j) * K, K, stream);
                if (rc) return join(rc);
            }
            hipError_t e = hipEventRecord(d->cev[(size_t)j], st);
            if (e == hipSuccess) e = hipStreamWaitEvent(d->xst, d->cev[(size_t)j], 0);
            if (e != hipSuccess) {
                set_error("chunked execute fork (chunk %d): %s", j, hipGetErrorString(e));
                return join(SMFV_ERR_HIP);
            }
            forked = true;
            int rc = run_exchange(d->comm, d->cops[(size_t)j], d_Y, d->xst);
            if (rc) return join(rc);
        }
        return join(SMFV_OK);
    }
    int rc = smfv_dist_plan_execute_local(d, d_row_ptr, d_col_idx, d_values, d_X, d_Y, stream);
    return rc ? rc : smfv_dist_plan_exchange(d, d_Y, stream);
}

SMFV_API int smfv_dist_plan_stats(smfv_dist_plan_t d, double out[SMFV_PLAN_STATS])
{
    SMFV_REQUIRE(d, "null plan");
    if (d->P.chunks > 1) {
        // the first chunk's stats; counts summed over the chunks (tiles, staged
        // rows, device bytes, direct rows, analysis time, snapshot entries),
        // re-use weighted by staged rows, tiled only if every chunk is
        for (int i = 0; i < SMFV_PLAN_STATS; ++i) out[i] = 0.0;
        bool first = true;
        double reuse_w = 0.0;
        for (smfv_plan_t c : d->cplans) {
            if (!c) continue;
            double o[SMFV_PLAN_STATS];
            int rc = smfv_plan_stats(c, o);
            if (rc) return rc;
            if (first) {
                for (int i = 0; i < SMFV_PLAN_STATS; ++i) out[i] = o[i];
                for (int i : {1, 2, 4, 5, 8, 9, 17}) out[i] = 0.0;
                first = false;
            }
            out[0] = out[0] && o[0];
            for (int i : {1, 2, 4, 5, 8, 9, 17}) out[i] += o[i];
            reuse_w += o[3] * o[2];
        }
        out[3] = out[2] > 0 ? reuse_w / out[2] : 0.0;
        out[6] = d->P.first[d->rank];
        return SMFV_OK;
    }
    return smfv_plan_stats(d->local, out);
}

SMFV_API int smfv_dist_plan_destroy(smfv_dist_plan_t d)
{
    delete d;
    return SMFV_OK;
}

}  // extern "C"
