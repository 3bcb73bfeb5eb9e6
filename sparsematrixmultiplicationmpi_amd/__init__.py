"""MI355X-native CSR x fat-vector SpMM engine (drop-in for the hot path of
AlexisBalayre/SparseMatrixMultiplicationMPI).

    Y[m x K] = A_csr[m x n] * X[n x K]   (fp64)

The product is libsmfv.so (HIP kernels for gfx950 + C ABI in include/smfv.h)
and libsmfv_mpi.so / smfv_main (the reference's C++ call surface and CLI).
This package is the Python host binding used by the tests and bench.py.
"""
from ._lib import LIB_PATH, SmfvError, lib  # noqa: F401  (raises if the library is missing)
from .inputs import (  # noqa: F401
    COP20K_M,
    COP20K_NNZ,
    SparseMatrix,
    areMatricesEqual,
    cop20k_surrogate,
    deserialize,
    gen_fem27,
    gen_random_rows,
    generateLargeFatVector,
    readMatrixMarketFile,
    serialize,
    writeMatrixMarketFile,
)
from .engine import (  # noqa: F401
    DeviceCSR,
    SpmmPlan,
    VendorSpmm,
    Variant,
    compare,
    fill_x_hash,
    sparseMatrixFatVectorMultiply,
    sparseMatrixFatVectorMultiplyColumnWise,
    sparseMatrixFatVectorMultiplyNonZeroElement,
    sparseMatrixFatVectorMultiplyRowWise,
    spmm,
)

__version__ = "0.1.0"
