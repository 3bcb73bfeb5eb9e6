// dropin.cpp -- the reference's C++ call surface over the libsmfv C ABI
// (libsmfv_mpi.so).  Callers written against SC/SparseMatrixFatVectorMultiply*.h
// and SC/utils.h link this instead of the reference's .cpp files.
//
//   sparseMatrixFatVectorMultiply*   SC/SparseMatrixFatVectorMultiply*.cpp
//   areMatricesEqual                 SC/utils.cpp:38-63
//   readMatrixMarketFile             SC/utils.cpp:70-185   (-> smfv_mtx_read)
//   generateLargeFatVector           SC/utils.cpp:193-209  (rand() % 100 + 1)
//   serialize / deserialize          SC/utils.cpp:216-253
//
// Device placement: rank r of MPI_COMM_WORLD uses GPU (local rank % devices).
// The RCCL communicator is created on first collective use (rank 0 makes the
// unique id, MPI_Bcast hands it out: MPI is only the bootstrap, every data
// movement of the SpMM itself is RCCL over xGMI).
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "SparseMatrixFatVectorMultiply.h"
#include "SparseMatrixFatVectorMultiplyColumnWise.h"
#include "SparseMatrixFatVectorMultiplyNonZeroElement.h"
#include "SparseMatrixFatVectorMultiplyRowWise.h"
#include "smfv.h"
#include "smfv_host.h"
#include "utils.h"

#define DROPIN_API __attribute__((visibility("default")))

namespace {

struct Context {
    bool init = false;
    bool mpi = false;
    int rank = 0, size = 1;
    smfv_comm_t comm = nullptr;
    hipStream_t stream = nullptr;
};

Context g_ctx;

[[noreturn]] void fail(const std::string &what)
{
    int mpi_on = 0, fin = 0;
    MPI_Initialized(&mpi_on);
    MPI_Finalized(&fin);
    if (mpi_on && !fin) {
        std::fprintf(stderr, "smfv: %s\n", what.c_str());
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    throw std::runtime_error("smfv: " + what);
}

void check(int rc, const char *where)
{
    if (rc != SMFV_OK) fail(std::string(where) + ": " + smfv_last_error());
}

void hip_check(hipError_t e, const char *where)
{
    if (e != hipSuccess) fail(std::string(where) + ": " + hipGetErrorString(e));
}

Context &ctx()
{
    if (g_ctx.init) return g_ctx;
    int on = 0;
    MPI_Initialized(&on);
    g_ctx.mpi = on != 0;
    int local = 0;
    if (g_ctx.mpi) {
        MPI_Comm_rank(MPI_COMM_WORLD, &g_ctx.rank);
        MPI_Comm_size(MPI_COMM_WORLD, &g_ctx.size);
        MPI_Comm node;
        MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, g_ctx.rank, MPI_INFO_NULL, &node);
        MPI_Comm_rank(node, &local);
        MPI_Comm_free(&node);
    }
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev <= 0) fail("no HIP device");
    hip_check(hipSetDevice(local % ndev), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking), "hipStreamCreate");
    g_ctx.init = true;
    return g_ctx;
}

smfv_comm_t comm_world()
{
    Context &c = ctx();
    if (c.comm || c.size == 1) return c.comm;
    char id[SMFV_UNIQUE_ID_BYTES] = {0};
    if (c.rank == 0) check(smfv_comm_unique_id(id), "smfv_comm_unique_id");
    MPI_Bcast(id, SMFV_UNIQUE_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
    check(smfv_comm_init(&c.comm, c.size, c.rank, id), "smfv_comm_init");
    return c.comm;
}

// Buffers reused across calls (grow-only): the device copies of A, X, Y and
// the workspace, and pinned host staging for X (in) and Y (out), so a call
// pays no hipMalloc and its X / Y transfers run at pinned-copy speed
// (the FatVector <-> flat conversion and the rank-0
// rebuild are a large share of the reference's RowWise time).
struct Cached {
    void *p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    void *get(size_t bytes)
    {
        if (bytes <= cap) return p;
        release();
        const size_t b = std::max<size_t>(bytes, 256);
        if (pinned)
            hip_check(hipHostMalloc(&p, b, hipHostMallocDefault), "hipHostMalloc");
        else
            hip_check(hipMalloc(&p, b), "hipMalloc");
        cap = b;
        return p;
    }
    void release()
    {
        if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        cap = 0;
    }
};

struct Buffers {
    Cached rp, ci, va, X, Y, ws, hX{nullptr, 0, true}, hY{nullptr, 0, true};
};

Buffers &bufs()
{
    static Buffers *b = new Buffers;  // process lifetime (freed with the context at exit)
    return *b;
}

// host rows [0, rows) copied in parallel (plain threads: the copies are
// memory-bound and the FatVector side is m separate allocations)
template <class F> void par_rows(int rows, F f)
{
    const int nt = rows < 4096 ? 1 : (int)std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency()));
    if (nt == 1) {
        f(0, rows);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(f, (int)((int64_t)rows * t / nt), (int)((int64_t)rows * (t + 1) / nt));
    for (auto &x : th) x.join();
}

// A and X resident on the device for one call
struct Problem {
    int m, n, K;
    int64_t nnz;
    int *rp, *ci;
    double *va, *X, *Y;
    Problem(const SparseMatrix &A, const FatVector &fat, int K_, hipStream_t st)
        : m(A.numRows), n(A.numCols), K(K_), nnz((int64_t)A.values.size())
    {
        if ((int)A.rowPtr.size() != m + 1 || (int64_t)A.colIndices.size() != nnz ||
            (m >= 0 && A.rowPtr.size() && A.rowPtr[m] != nnz))
            fail("malformed SparseMatrix (rowPtr / colIndices / values sizes)");
        if ((int)fat.size() != n) fail("fatVector has " + std::to_string(fat.size()) + " rows, matrix has " + std::to_string(n) + " columns");
        for (const auto &r : fat)
            if ((int)r.size() != K) fail("fatVector rows must have vecCols entries");
        Buffers &B = bufs();
        rp = static_cast<int *>(B.rp.get(A.rowPtr.size() * sizeof(int)));
        ci = static_cast<int *>(B.ci.get(A.colIndices.size() * sizeof(int)));
        va = static_cast<double *>(B.va.get(A.values.size() * sizeof(double)));
        X = static_cast<double *>(B.X.get((size_t)n * K * sizeof(double)));
        Y = static_cast<double *>(B.Y.get((size_t)m * K * sizeof(double)));
        // serialize (SC/utils.cpp:216-228) straight into pinned staging
        double *hx = static_cast<double *>(B.hX.get((size_t)n * K * sizeof(double)));
        par_rows(n, [&](int a, int b) {
            for (int i = a; i < b; ++i) std::copy(fat[i].begin(), fat[i].end(), hx + (size_t)i * K);
        });
        auto up = [&](void *d, const void *h, size_t bytes) {
            if (bytes) hip_check(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
        };
        up(rp, A.rowPtr.data(), A.rowPtr.size() * sizeof(int));
        up(ci, A.colIndices.data(), A.colIndices.size() * sizeof(int));
        up(va, A.values.data(), A.values.size() * sizeof(double));
        up(X, hx, (size_t)n * K * sizeof(double));
    }
    void *workspace(size_t bytes) { return bytes ? bufs().ws.get(bytes) : nullptr; }
    FatVector download(hipStream_t st)
    {
        double *hy = static_cast<double *>(bufs().hY.get((size_t)m * K * sizeof(double)));
        if ((size_t)m * K)
            hip_check(hipMemcpyAsync(hy, Y, (size_t)m * K * sizeof(double), hipMemcpyDeviceToHost, st),
                      "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
        // deserialize (SC/utils.cpp:238-253): the m row vectors built in parallel
        FatVector out((size_t)m);
        par_rows(m, [&](int a, int b) {
            for (int i = a; i < b; ++i) out[i].assign(hy + (size_t)i * K, hy + (size_t)(i + 1) * K);
        });
        return out;
    }
};

FatVector local_run(int variant, const SparseMatrix &A, const FatVector &fat, int K)
{
    Context &c = ctx();
    Problem P(A, fat, K, c.stream);
    size_t wsb = 0;
    check(smfv_spmm_workspace_bytes(variant, P.m, P.nnz, K, &wsb), "smfv_spmm_workspace_bytes");
    check(smfv_spmm_csr_f64(variant, P.m, P.n, P.nnz, P.rp, P.ci, P.va, P.X, K, K, P.Y, K, P.workspace(wsb), wsb,
                            c.stream),
          "smfv_spmm_csr_f64");
    return P.download(c.stream);
}

FatVector collective_run(int variant, const SparseMatrix &A, const FatVector &fat, int K)
{
    Context &c = ctx();
    if (c.size == 1) return local_run(variant, A, fat, K);
    smfv_comm_t comm = comm_world();
    Problem P(A, fat, K, c.stream);
    size_t wsb = 0;
    check(smfv_dist_workspace_bytes(comm, variant, P.m, P.nnz, A.rowPtr.data(), K, &wsb),
          "smfv_dist_workspace_bytes");
    check(smfv_dist_spmm_f64(comm, variant, SMFV_TO_ROOT, 0, P.m, P.n, P.nnz, A.rowPtr.data(), P.rp, P.ci,
                             P.va, P.X, K, P.Y, P.workspace(wsb), wsb, c.stream),
          "smfv_dist_spmm_f64");
    if (c.rank != 0) {
        hip_check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
        return FatVector{};
    }
    return P.download(c.stream);
}

}  // namespace

DROPIN_API FatVector sparseMatrixFatVectorMultiply(const SparseMatrix &sparseMatrix,
                                                   const FatVector &fatVector, int vecCols)
{
    return local_run(SMFV_SEQUENTIAL, sparseMatrix, fatVector, vecCols);
}

DROPIN_API FatVector sparseMatrixFatVectorMultiplyRowWise(const SparseMatrix &sparseMatrix,
                                                          const FatVector &fatVector, int vecCols)
{
    return collective_run(SMFV_ROWWISE, sparseMatrix, fatVector, vecCols);
}

DROPIN_API FatVector sparseMatrixFatVectorMultiplyColumnWise(const SparseMatrix &sparseMatrix,
                                                             const FatVector &fatVector, int vecCols)
{
    return collective_run(SMFV_COLUMNWISE, sparseMatrix, fatVector, vecCols);
}

DROPIN_API FatVector sparseMatrixFatVectorMultiplyNonZeroElement(const SparseMatrix &sparseMatrix,
                                                                 const FatVector &fatVector, int vecCols)
{
    return collective_run(SMFV_NONZERO, sparseMatrix, fatVector, vecCols);
}

DROPIN_API bool areMatricesEqual(const FatVector &mat1, const FatVector &mat2, double tolerance)
{
    if (mat1.size() != mat2.size()) return false;
    for (size_t i = 0; i < mat1.size(); ++i) {
        if (mat1[i].size() != mat2[i].size()) return false;
        for (size_t j = 0; j < mat1[i].size(); ++j)
            if (std::fabs(mat1[i][j] - mat2[i][j]) > tolerance) return false;
    }
    return true;
}

DROPIN_API SparseMatrix readMatrixMarketFile(const std::string &filename)
{
    int m = 0, n = 0;
    int64_t nnz = 0;
    int *rp = nullptr, *ci = nullptr;
    double *va = nullptr;
    if (smfv_mtx_read(filename.c_str(), &m, &n, &nnz, &rp, &ci, &va) != SMFV_OK)
        throw std::runtime_error(smfv_last_error());
    SparseMatrix A;
    A.numRows = m;
    A.numCols = n;
    A.rowPtr.assign(rp, rp + m + 1);
    A.colIndices.assign(ci, ci + nnz);
    A.values.assign(va, va + nnz);
    smfv_free(rp);
    smfv_free(ci);
    smfv_free(va);
    return A;
}

DROPIN_API FatVector generateLargeFatVector(int n, int k)
{
    // the process-global rand() stream, exactly as SC/utils.cpp:203
    FatVector v((size_t)n, std::vector<double>((size_t)k));
    for (auto &row : v)
        for (auto &x : row) x = rand() % 100 + 1;
    return v;
}

DROPIN_API std::vector<double> serialize(const FatVector &denseVec)
{
    size_t total = 0;
    for (const auto &r : denseVec) total += r.size();
    std::vector<double> flat;
    flat.reserve(total);
    for (const auto &r : denseVec) flat.insert(flat.end(), r.begin(), r.end());
    return flat;
}

DROPIN_API FatVector deserialize(const std::vector<double> &flat, int rows, int cols)
{
    FatVector out((size_t)rows, std::vector<double>((size_t)cols));
    for (int i = 0; i < rows; ++i)
        std::copy(flat.begin() + (size_t)i * cols, flat.begin() + (size_t)(i + 1) * cols, out[i].begin());
    return out;
}
