// dropin_golden.cpp -- pins the C++ drop-in (libsmfv_mpi.so) to the golden
// fixtures made by the reference itself (tests/golden/make_golden.py).
//
//   mpiexec -n 1 smfv_dropin_golden <a.smfvcsr> <x.smfvdns> <y_seq.smfvdns>
//
// Calls the reference's four signatures (SC/SparseMatrixFatVectorMultiply*.h)
// on the golden A and X and compares with the reference's sequential Y:
// bit for bit for the sequential / RowWise / ColumnWise variants, within
// 1e-12 x sum|a||x| for NonZeroElement (and the reference's own check,
// areMatricesEqual 1e-6, SC/utils.cpp:55).  Then the same calls with the
// inputs made device-resident by smfvDistributeInputs, the device-side
// result check (smfvCompareWithReference), and a repeated call (plan cache).
// Prints "DROPIN GOLDEN OK" and exits 0, or names the failure and exits 1.
#include <mpi.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <thread>
#include <utility>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "SparseMatrixFatVectorMultiply.h"
#include "SparseMatrixFatVectorMultiplyColumnWise.h"
#include "SparseMatrixFatVectorMultiplyNonZeroElement.h"
#include "SparseMatrixFatVectorMultiplyRowWise.h"
#include "smfv.h"
#include "smfv_dropin.h"
#include "smfv_host.h"
#include "utils.h"

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

static int failures = 0;

static void expect(bool ok, const std::string &what)
{
    if (!ok) {
        std::printf("FAIL %s\n", what.c_str());
        ++failures;
    }
}

// the reference's loop (SC/SparseMatrixFatVectorMultiply.cpp:17-27): per
// row, non-zeros in CSR order, y += a * x with a separate multiply and add
// (this file is built with -ffp-contract=off)
static FatVector host_spmm(const SparseMatrix &A, const FatVector &X, int K)
{
    FatVector Y((size_t)A.numRows, std::vector<double>((size_t)K, 0.0));
    for (int i = 0; i < A.numRows; ++i)
        for (int j = A.rowPtr[i]; j < A.rowPtr[i + 1]; ++j)
            for (int k = 0; k < K; ++k) Y[i][k] += A.values[j] * X[A.colIndices[j]][k];
    return Y;
}

static bool same_bits(const FatVector &a, const FatVector &b)
{
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i].size() != b[i].size() || std::memcmp(a[i].data(), b[i].data(), a[i].size() * 8)) return false;
    return true;
}

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s <a.smfvcsr> <x.smfvdns> <y_seq.smfvdns>\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
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
    FatVector X = read_dense(argv[2]);
    const FatVector Yseq = read_dense(argv[3]);
    const int K = X.empty() ? 0 : (int)X[0].size();
    // |A||X|: the scale a reassociated (NonZeroElement) sum is compared against
    std::vector<double> scale((size_t)m * K, 0.0);
    for (int i = 0; i < m; ++i)
        for (int j = A.rowPtr[i]; j < A.rowPtr[i + 1]; ++j)
            for (int k = 0; k < K; ++k) scale[(size_t)i * K + k] += std::fabs(A.values[j]) * std::fabs(X[A.colIndices[j]][k]);
    auto nz_ok = [&](const FatVector &Y) {
        if (Y.size() != Yseq.size()) return false;
        for (int i = 0; i < m; ++i)
            for (int k = 0; k < K; ++k)
                if (!(std::fabs(Y[i][k] - Yseq[i][k]) <= 1e-12 * scale[(size_t)i * K + k])) return false;
        return areMatricesEqual(Y, Yseq, 1e-6);
    };

    for (int pass = 0; pass < 2; ++pass) {  // pass 1: plans come from the cache
        const std::string tag = pass ? " (cached plan)" : "";
        expect(same_bits(sparseMatrixFatVectorMultiply(A, X, K), Yseq), "sequential" + tag);
        expect(same_bits(sparseMatrixFatVectorMultiplyRowWise(A, X, K), Yseq), "RowWise" + tag);
        expect(same_bits(sparseMatrixFatVectorMultiplyColumnWise(A, X, K), Yseq), "ColumnWise" + tag);
        expect(nz_ok(sparseMatrixFatVectorMultiplyNonZeroElement(A, X, K)), "NonZeroElement" + tag);
    }
    // device-resident inputs + device-side check against the kept serial result
    FatVector serial = sparseMatrixFatVectorMultiply(A, X, K);
    smfvKeepResultAsReference();
    smfvDistributeInputs(A, X, K);
    expect(same_bits(sparseMatrixFatVectorMultiplyRowWise(A, X, K), Yseq), "RowWise (resident inputs)");
    double d = -1.0;
    expect(smfvCompareWithReference(0.0, &d) && d == 0.0, "device compare RowWise");
    expect(same_bits(sparseMatrixFatVectorMultiplyColumnWise(A, X, K), Yseq), "ColumnWise (resident inputs)");
    expect(nz_ok(sparseMatrixFatVectorMultiplyNonZeroElement(A, X, K)), "NonZeroElement (resident inputs)");
    expect(smfvCompareWithReference(1e-6, &d), "device compare NonZeroElement");
    smfvReleaseInputs();
    // a changed value after release: a fresh upload sees it
    if (m > 0 && !A.values.empty() && K > 0) {
        A.values[0] += 1.0;
        FatVector Y2 = sparseMatrixFatVectorMultiplyRowWise(A, X, K);
        int r0 = 0;
        while (A.rowPtr[r0 + 1] == 0) ++r0;  // the row holding value 0
        expect(Y2[r0][0] != Yseq[r0][0] || X[A.colIndices[0]][0] == 0.0, "value change seen after release");
        double dd = -1.0;
        const bool same = smfvCompareWithReference(0.0, &dd);
        if (same) std::printf("note: r0=%d y2=%.17g yseq=%.17g x=%.17g d=%.17g\n", r0, Y2[r0][0], Yseq[r0][0],
                              X[A.colIndices[0]][0], dd);
        expect(!same || X[A.colIndices[0]][0] == 0.0, "device compare sees the change");
    }
    // (r3) resident inputs changed IN PLACE (same objects, same addresses)
    // after smfvDistributeInputs: the call sees the new values and X
    if (m > 0 && !A.values.empty() && K > 0) {
        FatVector X2 = X;
        smfvDistributeInputs(A, X2, K);
        expect(same_bits(sparseMatrixFatVectorMultiplyRowWise(A, X2, K), host_spmm(A, X2, K)), "resident (unchanged)");
        A.values[A.values.size() / 2] = -3.25;
        X2[A.colIndices[0]][K - 1] += 7.0;
        expect(same_bits(sparseMatrixFatVectorMultiplyRowWise(A, X2, K), host_spmm(A, X2, K)),
               "resident inputs edited in place are re-uploaded");
        expect(same_bits(sparseMatrixFatVectorMultiply(A, X2, K), host_spmm(A, X2, K)), "resident, sequential");
        smfvReleaseInputs();
    }
    // (r3) another pattern with the same sizes: a plan-cache key match (forced
    // by SMFV_TEST_PLAN_KEY_BITS=0 in the test) must not run the first
    // pattern's plan
    if (m > 1 && n > 1 && nnz > 0 && K > 0) {
        SparseMatrix B = A;
        for (int i = 0; i < m; ++i) {  // every column shifted by one, rows re-sorted by (col, value)
            std::vector<std::pair<int, double>> row;
            for (int j = A.rowPtr[i]; j < A.rowPtr[i + 1]; ++j) row.push_back({(A.colIndices[j] + 1) % n, A.values[j]});
            std::sort(row.begin(), row.end());
            for (int j = A.rowPtr[i], q = 0; j < A.rowPtr[i + 1]; ++j, ++q) {
                B.colIndices[j] = row[q].first;
                B.values[j] = row[q].second;
            }
        }
        for (int pass = 0; pass < 3; ++pass) {  // the third pass may run a background-built tiled plan
            expect(same_bits(sparseMatrixFatVectorMultiplyRowWise(B, X, K), host_spmm(B, X, K)),
                   "second pattern, same sizes (RowWise)");
            expect(same_bits(sparseMatrixFatVectorMultiplyRowWise(A, X, K), host_spmm(A, X, K)),
                   "first pattern again (RowWise)");
            if (pass == 1) std::this_thread::sleep_for(std::chrono::milliseconds(500));
        }
    }
    std::printf(failures ? "DROPIN GOLDEN FAILED (%d)\n" : "DROPIN GOLDEN OK%.0d\n", failures);
    MPI_Finalize();
    return failures ? 1 : 0;
}
