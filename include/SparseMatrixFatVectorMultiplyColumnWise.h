// SparseMatrixFatVectorMultiplyColumnWise.h -- drop-in for SC/SparseMatrixFatVectorMultiplyColumnWise.h:15.
//
// Y = sparseMatrix * fatVector on MI355X through libsmfv (include/smfv.h):
// K-column panels per rank + gather + transpose (SMFV_COLUMNWISE).
// Collective over MPI_COMM_WORLD when MPI is initialised (one GPU per rank,
// RCCL over xGMI for the exchange); every rank passes the full matrix and
// fat vector.  Rank 0 receives the numRows x vecCols result, the other ranks
// an empty FatVector -- the reference's contract.  Without MPI it runs on
// the local GPU.  Failures abort the MPI job (or throw std::runtime_error
// when MPI is not initialised).
#ifndef SPARSEMATRIXFATVECTORMULTIPLYCOLUMNWISE_H
#define SPARSEMATRIXFATVECTORMULTIPLYCOLUMNWISE_H

#include "MatrixDefinitions.h"

FatVector sparseMatrixFatVectorMultiplyColumnWise(const SparseMatrix &sparseMatrix,
                                            const FatVector &fatVector, int vecCols);

#endif
