// SparseMatrixFatVectorMultiply.h -- drop-in for SC/SparseMatrixFatVectorMultiply.h:14-15.
//
// Y = sparseMatrix * fatVector on MI355X through libsmfv (include/smfv.h):
// sequential order (SMFV_SEQUENTIAL); local GPU, not collective.
#ifndef SPARSEMATRIXFATVECTORMULTIPLY_H
#define SPARSEMATRIXFATVECTORMULTIPLY_H

#include "MatrixDefinitions.h"

FatVector sparseMatrixFatVectorMultiply(const SparseMatrix &sparseMatrix,
                                            const FatVector &fatVector, int vecCols);

#endif
