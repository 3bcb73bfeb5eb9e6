// MatrixDefinitions.h -- drop-in for SC/MatrixDefinitions.h:14-22 of the
// reference (AlexisBalayre/SparseMatrixMultiplicationMPI).
//
// Same type names and members, plus the two int dimensions every reference
// source reads (SC/main.cpp:111-112 broadcasts them as MPI_INT) and the
// shipped header forgot.  0-based CSR, int32 indices, fp64 values.
#ifndef MATRIXDEFINITIONS_H
#define MATRIXDEFINITIONS_H

#include <vector>

struct SparseMatrix
{
    std::vector<double> values;   // nnz non-zero values, row by row
    std::vector<int> colIndices;  // nnz column indices (sorted inside a row)
    std::vector<int> rowPtr;      // numRows + 1 offsets into values/colIndices
    int numRows = 0;
    int numCols = 0;
};

// dense numCols x K "fat vector", one std::vector per row
typedef std::vector<std::vector<double>> FatVector;

#endif
