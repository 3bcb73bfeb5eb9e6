// relink_caller.cpp -- a caller written against the REFERENCE's own headers
// (compiled with -I"<reference>/Source Code", so its quoted includes resolve
// there first, as SC/main.cpp's do) and re-linked to libsmfv_mpi.so, the
// INTEGRATION.md section 1 recipe.  The drop-in struct reaches it through
// `-include <repo>/include/MatrixDefinitions.h`: that header defines the
// reference header's own guard (MATRIXDEFINITIONS_H), so the reference's
// SparseMatrix (no numRows / numCols, SC/MatrixDefinitions.h:14-19) is never
// seen.  Compiled and linked by tests/test_host.py::test_relink_recipe (no
// GPU: it is not run).
#include "SparseMatrixFatVectorMultiply.h"
#include "SparseMatrixFatVectorMultiplyColumnWise.h"
#include "SparseMatrixFatVectorMultiplyNonZeroElement.h"
#include "SparseMatrixFatVectorMultiplyRowWise.h"

int main()
{
    SparseMatrix A;
    A.numRows = 1;  // the members SC/main.cpp:111-112 broadcast
    A.numCols = 1;
    A.rowPtr = {0, 1};
    A.colIndices = {0};
    A.values = {2.0};
    FatVector X(1, std::vector<double>(1, 3.0));
    FatVector (*fns[])(const SparseMatrix &, const FatVector &, int) = {
        sparseMatrixFatVectorMultiply, sparseMatrixFatVectorMultiplyRowWise,
        sparseMatrixFatVectorMultiplyColumnWise, sparseMatrixFatVectorMultiplyNonZeroElement};
    return fns[0] == nullptr ? 1 : 0;
}
