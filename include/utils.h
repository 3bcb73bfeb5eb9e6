// utils.h -- drop-in for the hot-path helpers of SC/utils.h (reference).
//
// The PETSc conversion (SC/utils.h:24) is out of scope: PETSc is not part of
// this engine; the vendor-library comparison uses rocSPARSE.
#ifndef UTILS_H
#define UTILS_H

#include <string>
#include <vector>

#include "MatrixDefinitions.h"

// |a - b| <= tolerance element-wise, same shapes      (SC/utils.cpp:38-63)
bool areMatricesEqual(const FatVector &mat1, const FatVector &mat2, double tolerance);
// Matrix Market -> CSR; throws std::runtime_error       (SC/utils.cpp:70-185)
SparseMatrix readMatrixMarketFile(const std::string &filename);
// n x k, rand() % 100 + 1                                (SC/utils.cpp:193-209)
FatVector generateLargeFatVector(int n, int k);
// FatVector <-> row-major flat array                    (SC/utils.cpp:216-253)
std::vector<double> serialize(const FatVector &denseVec);
FatVector deserialize(const std::vector<double> &flat, int rows, int cols);

#endif
