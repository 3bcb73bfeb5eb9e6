// ref_driver.cpp -- drives the REFERENCE's own four SpMM functions, compiled
// unmodified from /root/reference/Source Code (see oracle/Makefile, target
// `ref`).  TEST INFRASTRUCTURE ONLY: used to produce the golden fixtures in
// tests/golden/ and, on the GPU box, as the reference CPU/MPI baseline that
// bench.py times beside the GPU (cpu_baseline.kind = "reference").
//
// This is NOT the reference's main.cpp (that one needs PETSc, absent here);
// it follows main.cpp's sequence: rank 0 loads A and X (SC/main.cpp:53-69),
// times the serial kernel (:74-81), broadcasts A and X (:106-143), and times
// each MPI variant with a barrier + MPI_Wtime around the call (:161-163,
// :204-206, :247-249).  Input is the SMFV binary CSR container written by
// the tests (magic "SMFVCSR1"); X is either read from an SMFV dense file or
// generated exactly as SC/utils.cpp:193-209 does (rand()%100+1, no srand).
//
// usage: ref_driver <csr.bin> <K> [--x dense.bin] [--out prefix]
//                   [--reps R] [--variants SRCZ]
#include <mpi.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>
#include <algorithm>

#include "SparseMatrixFatVectorMultiply.h"
#include "SparseMatrixFatVectorMultiplyRowWise.h"
#include "SparseMatrixFatVectorMultiplyColumnWise.h"
#include "SparseMatrixFatVectorMultiplyNonZeroElement.h"

static bool read_csr(const char *path, SparseMatrix &A)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    char magic[8];
    int32_t m, n;
    int64_t nnz;
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "SMFVCSR1", 8) == 0 &&
              std::fread(&m, 4, 1, f) == 1 && std::fread(&n, 4, 1, f) == 1 &&
              std::fread(&nnz, 8, 1, f) == 1;
    if (ok) {
        A.numRows = m;
        A.numCols = n;
        A.rowPtr.resize((size_t)m + 1);
        A.colIndices.resize((size_t)nnz);
        A.values.resize((size_t)nnz);
        ok = std::fread(A.rowPtr.data(), 4, (size_t)m + 1, f) == (size_t)m + 1 &&
             std::fread(A.colIndices.data(), 4, (size_t)nnz, f) == (size_t)nnz &&
             std::fread(A.values.data(), 8, (size_t)nnz, f) == (size_t)nnz;
    }
    std::fclose(f);
    return ok;
}

static bool read_dense(const char *path, std::vector<double> &flat, int64_t &rows, int64_t &cols)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    char magic[8];
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "SMFVDNS1", 8) == 0 &&
              std::fread(&rows, 8, 1, f) == 1 && std::fread(&cols, 8, 1, f) == 1;
    if (ok) {
        flat.resize((size_t)(rows * cols));
        ok = std::fread(flat.data(), 8, flat.size(), f) == flat.size();
    }
    std::fclose(f);
    return ok;
}

static void write_dense(const std::string &path, const FatVector &Y, int K)
{
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return;
    int64_t rows = (int64_t)Y.size(), cols = K;
    std::fwrite("SMFVDNS1", 1, 8, f);
    std::fwrite(&rows, 8, 1, f);
    std::fwrite(&cols, 8, 1, f);
    for (const auto &r : Y) std::fwrite(r.data(), 8, r.size(), f);
    std::fclose(f);
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    int rank, size;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    if (argc < 3) {
        if (rank == 0) std::fprintf(stderr, "usage: %s <csr.bin> <K> [--x dense.bin] [--out prefix] [--reps R] [--variants SRCZ]\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    const char *csrPath = argv[1];
    int k = std::atoi(argv[2]);
    const char *xPath = nullptr;
    std::string out;
    int reps = 1;
    std::string variants = "SRCZ";
    for (int i = 3; i + 1 < argc; i += 2) {
        if (!std::strcmp(argv[i], "--x")) xPath = argv[i + 1];
        else if (!std::strcmp(argv[i], "--out")) out = argv[i + 1];
        else if (!std::strcmp(argv[i], "--reps")) reps = std::atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--variants")) variants = argv[i + 1];
    }

    SparseMatrix M;
    FatVector v;
    std::vector<double> flat;
    int dataSize = 0;
    if (rank == 0) {
        if (!read_csr(csrPath, M)) {
            std::fprintf(stderr, "cannot read %s\n", csrPath);
            MPI_Abort(MPI_COMM_WORLD, 2);
        }
        std::printf("World size: %d\nSparse matrix: %s\nMatrix size: %dx%d\nVector size: %dx%d\n",
                    size, csrPath, M.numRows, M.numCols, M.numCols, k);
        if (xPath) {
            int64_t r, c;
            if (!read_dense(xPath, flat, r, c) || r != M.numCols || c != k) {
                std::fprintf(stderr, "bad X file %s\n", xPath);
                MPI_Abort(MPI_COMM_WORLD, 3);
            }
        } else {
            flat.resize((size_t)M.numCols * (size_t)k);
            for (auto &x : flat) x = rand() % 100 + 1;  // SC/utils.cpp:203, no srand
        }
        v.assign((size_t)M.numCols, std::vector<double>((size_t)k));
        for (int i = 0; i < M.numCols; ++i)
            for (int j = 0; j < k; ++j) v[i][j] = flat[(size_t)i * k + j];
        dataSize = (int)flat.size();
    }

    FatVector ySeq;
    if (rank == 0 && variants.find('S') != std::string::npos) {
        std::vector<double> ts;
        for (int r = 0; r < reps; ++r) {
            double t0 = MPI_Wtime();
            ySeq = sparseMatrixFatVectorMultiply(M, v, k);
            ts.push_back(MPI_Wtime() - t0);
        }
        std::printf("Serial Algo Execution time: %.9g\n", median(ts));
        if (!out.empty()) write_dense(out + ".seq.bin", ySeq, k);
    }

    // broadcast A and X to every rank (SC/main.cpp:106-143)
    MPI_Barrier(MPI_COMM_WORLD);
    int nv = (int)M.values.size(), nc = (int)M.colIndices.size(), nr = (int)M.rowPtr.size();
    MPI_Bcast(&M.numRows, 1, MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(&M.numCols, 1, MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(&nv, 1, MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(&nc, 1, MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(&nr, 1, MPI_INT, 0, MPI_COMM_WORLD);
    if (rank != 0) {
        M.values.resize(nv);
        M.colIndices.resize(nc);
        M.rowPtr.resize(nr);
    }
    MPI_Bcast(M.values.data(), nv, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    MPI_Bcast(M.colIndices.data(), nc, MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(M.rowPtr.data(), nr, MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(&dataSize, 1, MPI_INT, 0, MPI_COMM_WORLD);
    if (rank != 0) flat.resize(dataSize);
    MPI_Bcast(flat.data(), dataSize, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    if (rank != 0) {
        v.assign((size_t)M.numCols, std::vector<double>((size_t)k));
        for (int i = 0; i < M.numCols; ++i)
            for (int j = 0; j < k; ++j) v[i][j] = flat[(size_t)i * k + j];
    }
    MPI_Barrier(MPI_COMM_WORLD);

    struct V { char tag; const char *name; const char *suffix; FatVector (*fn)(const SparseMatrix &, const FatVector &, int); };
    const V vs[] = {
        {'R', "Row-wise", "row", sparseMatrixFatVectorMultiplyRowWise},
        {'C', "Column-wise", "col", sparseMatrixFatVectorMultiplyColumnWise},
        {'Z', "Non-zero Elements", "nnz", sparseMatrixFatVectorMultiplyNonZeroElement},
    };
    for (const V &x : vs) {
        if (variants.find(x.tag) == std::string::npos) continue;
        std::vector<double> ts;
        FatVector y;
        for (int r = 0; r < reps; ++r) {
            MPI_Barrier(MPI_COMM_WORLD);
            double t0 = MPI_Wtime();
            y = x.fn(M, v, k);
            ts.push_back(MPI_Wtime() - t0);
        }
        if (rank == 0) {
            std::printf("%s Execution time: %.9g\n", x.name, median(ts));
            if (!ySeq.empty()) {
                double mx = 0;
                bool same = y.size() == ySeq.size();
                for (size_t i = 0; same && i < y.size(); ++i)
                    for (size_t j = 0; j < y[i].size(); ++j) mx = std::max(mx, std::abs(y[i][j] - ySeq[i][j]));
                std::printf("%s: Results are %s!\n", x.name, (same && mx <= 1e-6) ? "the same" : "different");
            }
            if (!out.empty()) write_dense(out + "." + x.suffix + ".bin", y, k);
        }
    }
    MPI_Finalize();
    return 0;
}
