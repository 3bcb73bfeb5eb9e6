// dropin_multirank.cpp -- the C++ drop-in (libsmfv_mpi.so) called repeatedly
// by several MPI ranks (the tiled distributed plan is built on
// every rank at a pattern's SECOND call, SC/...RowWise.cpp:12-126 et al.).
//
//   mpiexec -n p smfv_dropin_multirank <a.smfvcsr> <x.smfvdns> <y_seq.smfvdns> [calls]
//
// Each of the three MPI variants is called `calls` times (default 4: call 1
// runs the untiled plan, call 2 builds and runs the tiled one on every rank,
// later calls hit the cache).  Rank 0's result must equal the reference's
// sequential Y bit for bit (RowWise, ColumnWise) or within 1e-12 x
// sum|a||x| (NonZeroElement) at EVERY call; the other ranks must get
// FatVector{} (SC/...RowWise.cpp:125).  Rank 0 prints the per-call times
// and "DROPIN MULTIRANK OK", exits 0; any failure exits 1.
#include <mpi.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <string>
#include <vector>

#include "SparseMatrixFatVectorMultiplyColumnWise.h"
#include "SparseMatrixFatVectorMultiplyNonZeroElement.h"
#include "SparseMatrixFatVectorMultiplyRowWise.h"
#include "smfv.h"
#include "smfv_host.h"

static FatVector read_dense(const char *path)
{
    std::ifstream f(path, std::ios::binary);
    char magic[8];
    int64_t rc[2];
    if (!f.read(magic, 8) || std::memcmp(magic, "SMFVDNS1", 8) || !f.read(reinterpret_cast<char *>(rc), 16)) {
        std::fprintf(stderr, "bad dense file %s\n", path);
        std::exit(2);
    }
    FatVector out((size_t)rc[0], std::vector<double>((size_t)rc[1]));
    for (auto &r : out) f.read(reinterpret_cast<char *>(r.data()), (std::streamsize)(r.size() * 8));
    return out;
}

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    int rank = 0, world = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &world);
    if (argc < 4) {
        if (rank == 0) std::fprintf(stderr, "usage: %s <a.smfvcsr> <x.smfvdns> <y_seq.smfvdns> [calls]\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    const int calls = argc > 4 ? std::atoi(argv[4]) : 4;
    int m, n, *rp, *ci;
    int64_t nnz;
    double *va;
    if (smfv_csr_read_bin(argv[1], &m, &n, &nnz, &rp, &ci, &va) != SMFV_OK) {
        std::fprintf(stderr, "%s\n", smfv_last_error());
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    SparseMatrix A;
    A.numRows = m;
    A.numCols = n;
    A.rowPtr.assign(rp, rp + m + 1);
    A.colIndices.assign(ci, ci + nnz);
    A.values.assign(va, va + nnz);
    smfv_free(rp);
    smfv_free(ci);
    smfv_free(va);
    const FatVector X = read_dense(argv[2]);
    const FatVector Yseq = read_dense(argv[3]);
    const int K = X.empty() ? 0 : (int)X[0].size();
    std::vector<double> scale((size_t)m * K, 0.0);
    for (int i = 0; i < m; ++i)
        for (int j = A.rowPtr[i]; j < A.rowPtr[i + 1]; ++j)
            for (int k = 0; k < K; ++k) scale[(size_t)i * K + k] += std::fabs(A.values[j]) * std::fabs(X[A.colIndices[j]][k]);
    auto exact = [&](const FatVector &Y) {
        if (Y.size() != Yseq.size()) return false;
        for (size_t i = 0; i < Y.size(); ++i)
            if (Y[i].size() != Yseq[i].size() || std::memcmp(Y[i].data(), Yseq[i].data(), Y[i].size() * 8)) return false;
        return true;
    };
    auto close = [&](const FatVector &Y) {
        if (Y.size() != Yseq.size()) return false;
        for (int i = 0; i < m; ++i)
            for (int k = 0; k < K; ++k)
                if (!(std::fabs(Y[i][k] - Yseq[i][k]) <= 1e-12 * scale[(size_t)i * K + k])) return false;
        return true;
    };
    struct Variant {
        const char *name;
        std::function<FatVector()> call;
        std::function<bool(const FatVector &)> ok;
    };
    const Variant vars[] = {
        {"RowWise", [&] { return sparseMatrixFatVectorMultiplyRowWise(A, X, K); }, exact},
        {"ColumnWise", [&] { return sparseMatrixFatVectorMultiplyColumnWise(A, X, K); }, exact},
        {"NonZeroElement", [&] { return sparseMatrixFatVectorMultiplyNonZeroElement(A, X, K); }, close},
    };
    int failures = 0;
    for (const Variant &v : vars)
        for (int c = 1; c <= calls; ++c) {
            MPI_Barrier(MPI_COMM_WORLD);
            const auto t0 = std::chrono::steady_clock::now();
            const FatVector Y = v.call();
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            const int bad = rank == 0 ? !v.ok(Y) : !Y.empty();
            int any = 0;
            MPI_Allreduce(&bad, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
            if (bad) std::printf("FAIL rank %d %s call %d\n", rank, v.name, c);
            failures += any;
            if (rank == 0) std::printf("%s call %d: %.3f ms%s\n", v.name, c, ms, any ? " FAILED" : "");
        }
    if (rank == 0) std::printf(failures ? "DROPIN MULTIRANK FAILED (%d) world %d\n" : "DROPIN MULTIRANK OK%.0d world %d\n", failures, world);
    MPI_Finalize();
    return failures ? 1 : 0;
}
