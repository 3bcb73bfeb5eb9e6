// main.cpp -- smfv_main, the drop-in for the reference CLI (SC/main.cpp):
//
//   mpirun -np P ./smfv_main <k> <matrix.mtx>
//
// Same arguments (SC/main.cpp:23-34), same sequence (rank-0 read + fat
// vector :53-69, serial run :74-81, broadcast of A and X :106-143, the three
// MPI variants timed with MPI_Wtime :161-163 / :204-206 / :247-249) and the
// same stdout lines the reference's CSV scrapers parse
// (SC/scripts/get_csv_all.sh:18-48).  Every SpMM runs on the rank's MI355X
// through libsmfv; the timed region of each call is the API end-to-end time
// (host FatVector -> device -> kernel -> RCCL gather -> host FatVector).  The
// PETSc comparison block (SC/main.cpp:282-402) is not part of this engine.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "SparseMatrixFatVectorMultiply.h"
#include "SparseMatrixFatVectorMultiplyColumnWise.h"
#include "SparseMatrixFatVectorMultiplyNonZeroElement.h"
#include "SparseMatrixFatVectorMultiplyRowWise.h"
#include "utils.h"

namespace {

void bcast_inputs(SparseMatrix &M, FatVector &v, int k, int rank)
{
    int dims[5] = {M.numRows, M.numCols, (int)M.values.size(), (int)M.colIndices.size(),
                   (int)M.rowPtr.size()};
    MPI_Bcast(dims, 5, MPI_INT, 0, MPI_COMM_WORLD);
    M.numRows = dims[0];
    M.numCols = dims[1];
    if (rank != 0) {
        M.values.resize(dims[2]);
        M.colIndices.resize(dims[3]);
        M.rowPtr.resize(dims[4]);
    }
    MPI_Bcast(M.values.data(), dims[2], MPI_DOUBLE, 0, MPI_COMM_WORLD);
    MPI_Bcast(M.colIndices.data(), dims[3], MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(M.rowPtr.data(), dims[4], MPI_INT, 0, MPI_COMM_WORLD);
    std::vector<double> flat;
    if (rank == 0) flat = serialize(v);
    flat.resize((size_t)M.numCols * k);
    MPI_Bcast(flat.data(), (int)flat.size(), MPI_DOUBLE, 0, MPI_COMM_WORLD);
    if (rank != 0) v = deserialize(flat, M.numCols, k);
}

void run_variant(const char *name, FatVector (*fn)(const SparseMatrix &, const FatVector &, int),
                 const SparseMatrix &M, const FatVector &v, int k, const FatVector &serial, int rank)
{
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    FatVector y = fn(M, v, k);
    const double t1 = MPI_Wtime();
    if (rank == 0) {
        std::cout << name << " Execution time: " << (t1 - t0) << std::endl;
        std::cout << name << ": Results are "
                  << (areMatricesEqual(serial, y, 1e-6) ? "the same!" : "different!") << std::endl;
    }
}

}  // namespace

int main(int argc, char *argv[])
{
    MPI_Init(&argc, &argv);
    int rank = 0, size = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    if (argc != 3) {
        if (rank == 0) std::cerr << "Usage: " << argv[0] << " <number of columns> <matrix file path>" << std::endl;
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    const int k = std::atoi(argv[1]);
    const std::string filename = argv[2];

    SparseMatrix M;
    FatVector v, serial;
    if (rank == 0) {
        std::cout << "World size: " << size << std::endl;
        std::cout << "Sparse matrix: " << filename << std::endl;
        try {
            M = readMatrixMarketFile(filename);
        } catch (const std::exception &e) {
            std::cerr << e.what() << std::endl;
            MPI_Abort(MPI_COMM_WORLD, 1);
        }
        std::cout << "Matrix size: " << M.numRows << "x" << M.numCols << std::endl;
        v = generateLargeFatVector(M.numCols, k);
        std::cout << "Vector size: " << M.numCols << "x" << k << std::endl;
        const double t0 = MPI_Wtime();
        serial = sparseMatrixFatVectorMultiply(M, v, k);
        const double t1 = MPI_Wtime();
        std::cout << "Serial Algo Execution time: " << (t1 - t0) << std::endl;
    }
    MPI_Barrier(MPI_COMM_WORLD);
    bcast_inputs(M, v, k, rank);
    MPI_Barrier(MPI_COMM_WORLD);

    run_variant("Row-wise", sparseMatrixFatVectorMultiplyRowWise, M, v, k, serial, rank);
    run_variant("Column-wise", sparseMatrixFatVectorMultiplyColumnWise, M, v, k, serial, rank);
    run_variant("Non-zero Elements", sparseMatrixFatVectorMultiplyNonZeroElement, M, v, k, serial, rank);

    MPI_Barrier(MPI_COMM_WORLD);
    MPI_Finalize();
    return 0;
}
