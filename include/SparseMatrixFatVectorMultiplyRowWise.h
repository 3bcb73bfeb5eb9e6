// SparseMatrixFatVectorMultiplyRowWise.h -- drop-in for SC/SparseMatrixFatVectorMultiplyRowWise.h:15-17.
//
// Y = sparseMatrix * fatVector on MI355X through libsmfv (include/smfv.h):
// row blocks per rank + gather to rank 0 (SMFV_ROWWISE).
// Collective over MPI_COMM_WORLD when MPI is initialised (one GPU per rank,
// RCCL over xGMI for the exchange); every rank passes the full matrix and
// fat vector.  Rank 0 receives the numRows x vecCols result, the other ranks
// an empty FatVector -- the reference's contract.  Without MPI it runs on
// the local GPU.  Failures abort the MPI job (or throw std::runtime_error
// when MPI is not initialised).
#ifndef SPARSEMATRIXFATVECTORMULTIPLYROWWISE_H
#define SPARSEMATRIXFATVECTORMULTIPLYROWWISE_H

#include "MatrixDefinitions.h"

FatVector sparseMatrixFatVectorMultiplyRowWise(const SparseMatrix &sparseMatrix,
                                            const FatVector &fatVector, int vecCols);

#endif
