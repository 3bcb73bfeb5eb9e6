// smfv_dropin.h -- extensions of the reference's C++ call surface in
// libsmfv_mpi.so (not part of the reference's headers, which stay verbatim
// in SparseMatrixFatVectorMultiply*.h / utils.h / MatrixDefinitions.h).
//
// They let a caller written against the reference keep A and X resident on
// the GPUs between calls and check results on the device:
//
//   smfvDistributeInputs   replaces the 9 host MPI_Bcast of A and the fat
//                          vector (SC/main.cpp:106-143) with one H2D on rank
//                          0 and ncclBroadcast of the device copies over
//                          xGMI; every rank ends with A and X on its GPU and
//                          (as after the reference's broadcast) on the host
//   smfvKeepResultAsReference / smfvCompareWithReference
//                          the reference's areMatricesEqual check
//                          (SC/utils.cpp:38-63, called at SC/main.cpp:184,
//                          227, 270) on the device: the last call's result is
//                          compared where it already is, no D2H, no FatVector
#ifndef SMFV_DROPIN_H
#define SMFV_DROPIN_H

#include "MatrixDefinitions.h"

// Collective over MPI_COMM_WORLD.  Rank 0's A and fatVector (n x k) are
// uploaded once and broadcast device-to-device; the other ranks' A and
// fatVector are overwritten with rank 0's.  Until smfvReleaseInputs(), calls
// of the four functions with these SAME objects (same addresses, same
// sizes) use the resident device copies instead of uploading A and X again:
// the caller must not modify them in between.  Returns the wall time of the
// distribution (seconds, rank-local).
double smfvDistributeInputs(SparseMatrix &A, FatVector &fatVector, int k);
void smfvReleaseInputs();

// Rank 0: keep the device result of the last call (e.g. the serial one) as
// the reference.  smfvCompareWithReference: areMatricesEqual(reference,
// last result, tolerance) evaluated on the device (max |a - b|, NaN counts as
// a difference); *max_abs_diff receives the maximum (may be NULL).  Both
// apply to rank 0's last result; on other ranks they return false / do
// nothing.
void smfvKeepResultAsReference();
bool smfvCompareWithReference(double tolerance, double *max_abs_diff);

#endif
