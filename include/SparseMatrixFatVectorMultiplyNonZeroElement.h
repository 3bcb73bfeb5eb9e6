// SparseMatrixFatVectorMultiplyNonZeroElement.h -- drop-in for SC/SparseMatrixFatVectorMultiplyNonZeroElement.h:15.
//
// Y = sparseMatrix * fatVector on MI355X through libsmfv (include/smfv.h):
// nnz ranges per rank (merge-path) + row-block sum (SMFV_NONZERO).
// Collective over MPI_COMM_WORLD when MPI is initialised (one GPU per rank,
// RCCL over xGMI for the exchange); every rank passes the full matrix and
// fat vector.  Rank 0 receives the numRows x vecCols result, the other ranks
// an empty FatVector -- the reference's contract.  Without MPI it runs on
// the local GPU.  Failures abort the MPI job (or throw std::runtime_error
// when MPI is not initialised).
#ifndef SPARSEMATRIXFATVECTORMULTIPLYNONZEROELEMENT_H
#define SPARSEMATRIXFATVECTORMULTIPLYNONZEROELEMENT_H

#include "MatrixDefinitions.h"

FatVector sparseMatrixFatVectorMultiplyNonZeroElement(const SparseMatrix &sparseMatrix,
                                            const FatVector &fatVector, int vecCols);

#endif
