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

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

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
struct Plan {
    std::vector<int> first, last;
    std::vector<int64_t> offset, count;
    int64_t total = 0;  // doubles in the exchange buffer
};
int make_plan(int variant, int m, int64_t nnz, const int *h_row_ptr, int K, int p, Plan &P)
{
    P.first.assign(p, 0);
    P.last.assign(p, -1);
    P.offset.assign(p, 0);
    P.count.assign(p, 0);
    int rc = smfv_dist_plan(variant, m, nnz, h_row_ptr, K, p, P.first.data(), P.last.data(),
                            P.offset.data(), P.count.data());
    if (rc) return rc;
    P.total = 0;
    for (int r = 0; r < p; ++r) P.total = std::max(P.total, P.offset[r] + P.count[r]);
    return SMFV_OK;
}
}  // namespace

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

// The one exchange step of a distributed variant: gather-to-root (Gatherv /
// Reduce target) or all-gatherv of the ranks' blocks P.offset/P.count inside
// xbuf; equal, back-to-back blocks go through one ncclAllGather.
static int exchange_blocks(smfv_comm_t comm, const Plan &P, bool may_be_equal, bool to_all, int root,
                           double *xbuf, hipStream_t st)
{
    const int p = comm->nranks, rank = comm->rank;
    if (p > 1) {
        bool equal = may_be_equal;
        for (int r = 1; r < p && equal; ++r)
            equal = P.count[r] == P.count[0] && P.offset[r] == P.offset[0] + r * P.count[0];
        if (to_all && equal && P.count[0] > 0) {
            SMFV_NCCL(ncclAllGather(xbuf + P.offset[rank], xbuf, (size_t)P.count[0], ncclDouble,
                                    comm->nccl, st));
        } else {
            SMFV_NCCL(ncclGroupStart());
            for (int r = 0; r < p; ++r) {
                if (P.count[r] == 0) continue;
                double *blk = xbuf + P.offset[r];
                const size_t cnt = (size_t)P.count[r];
                if (to_all) {
                    SMFV_NCCL(ncclBroadcast(blk, blk, cnt, ncclDouble, r, comm->nccl, st));
                } else if (rank == root && r != root) {
                    SMFV_NCCL(ncclRecv(blk, cnt, ncclDouble, r, comm->nccl, st));
                } else if (rank == r && r != root) {
                    SMFV_NCCL(ncclSend(blk, cnt, ncclDouble, root, comm->nccl, st));
                }
            }
            SMFV_NCCL(ncclGroupEnd());
        }
    }

    return SMFV_OK;
}

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

}  // extern "C"
