// smfv_vendor.cpp -- the vendor-library comparator: Y = A * X with rocSPARSE's
// generic SpMM (CSR, int32 indices, f64, row-major dense operands).
//
// This is the analogue of the reference's PETSc block (SC/main.cpp:289-402:
// MatMatMult on the same A and fat vector, timed and checked against the
// serial result).  It is NOT on the product path: smfv_main prints it as the
// "rocSPARSE" line and bench.py times it beside the engine's own kernel.
#include <rocsparse/rocsparse.h>

#include <cstdint>

#include "smfv_internal.h"

using smfv::set_error;

struct smfv_vendor_s {
    rocsparse_handle handle = nullptr;
    rocsparse_spmat_descr A = nullptr;
    rocsparse_dnmat_descr X = nullptr, Y = nullptr;
    rocsparse_spmm_alg alg = rocsparse_spmm_alg_default;
    void *buffer = nullptr;
    size_t buffer_bytes = 0;
    ~smfv_vendor_s()
    {
        if (A) rocsparse_destroy_spmat_descr(A);
        if (X) rocsparse_destroy_dnmat_descr(X);
        if (Y) rocsparse_destroy_dnmat_descr(Y);
        if (handle) rocsparse_destroy_handle(handle);
        if (buffer) (void)hipFree(buffer);
    }
};

#define SMFV_SPARSE(call)                                                          \
    do {                                                                           \
        rocsparse_status s_ = (call);                                              \
        if (s_ != rocsparse_status_success) {                                      \
            set_error("%s failed: rocsparse status %d", #call, (int)s_);           \
            delete h;                                                              \
            return SMFV_ERR_HIP;                                                   \
        }                                                                          \
    } while (0)

extern "C" {

SMFV_API int smfv_vendor_spmm_create(smfv_vendor_t *out, int alg, int m, int n, int64_t nnz,
                                     const int *d_row_ptr, const int *d_col_idx, const double *d_values,
                                     const double *d_X, int64_t ldx, int K, double *d_Y, int64_t ldy,
                                     void *stream)
{
    SMFV_REQUIRE(out, "null handle pointer");
    SMFV_REQUIRE(m > 0 && n > 0 && nnz >= 0 && K > 0, "bad sizes (m=%d n=%d nnz=%lld K=%d)", m, n,
                 (long long)nnz, K);
    SMFV_REQUIRE(ldx >= K && ldy >= K, "leading dimension smaller than K");
    SMFV_REQUIRE(d_row_ptr && d_X && d_Y && (nnz == 0 || (d_col_idx && d_values)), "null pointer");
    SMFV_REQUIRE(alg >= 0 && alg <= 2, "alg: 0 default, 1 csr row split, 2 csr merge path");
    auto *h = new smfv_vendor_s;
    h->alg = alg == 1 ? rocsparse_spmm_alg_csr_row_split
           : alg == 2 ? rocsparse_spmm_alg_csr_merge_path : rocsparse_spmm_alg_default;
    SMFV_SPARSE(rocsparse_create_handle(&h->handle));
    SMFV_SPARSE(rocsparse_set_stream(h->handle, smfv::as_stream(stream)));
    SMFV_SPARSE(rocsparse_create_csr_descr(&h->A, m, n, nnz, const_cast<int *>(d_row_ptr),
                                           const_cast<int *>(d_col_idx), const_cast<double *>(d_values),
                                           rocsparse_indextype_i32, rocsparse_indextype_i32,
                                           rocsparse_index_base_zero, rocsparse_datatype_f64_r));
    SMFV_SPARSE(rocsparse_create_dnmat_descr(&h->X, n, K, ldx, const_cast<double *>(d_X),
                                             rocsparse_datatype_f64_r, rocsparse_order_row));
    SMFV_SPARSE(rocsparse_create_dnmat_descr(&h->Y, m, K, ldy, d_Y, rocsparse_datatype_f64_r,
                                             rocsparse_order_row));
    const double one = 1.0, zero = 0.0;
    SMFV_SPARSE(rocsparse_spmm(h->handle, rocsparse_operation_none, rocsparse_operation_none, &one, h->A, h->X,
                               &zero, h->Y, rocsparse_datatype_f64_r, h->alg, rocsparse_spmm_stage_buffer_size,
                               &h->buffer_bytes, nullptr));
    if (h->buffer_bytes) {
        hipError_t e = hipMalloc(&h->buffer, h->buffer_bytes);
        if (e != hipSuccess) {
            set_error("hipMalloc(rocsparse buffer %zu): %s", h->buffer_bytes, hipGetErrorString(e));
            delete h;
            return SMFV_ERR_HIP;
        }
    }
    SMFV_SPARSE(rocsparse_spmm(h->handle, rocsparse_operation_none, rocsparse_operation_none, &one, h->A, h->X,
                               &zero, h->Y, rocsparse_datatype_f64_r, h->alg, rocsparse_spmm_stage_preprocess,
                               &h->buffer_bytes, h->buffer));
    *out = h;
    return SMFV_OK;
}

SMFV_API int smfv_vendor_spmm_execute(smfv_vendor_t h)
{
    SMFV_REQUIRE(h, "null handle");
    const double one = 1.0, zero = 0.0;
    const rocsparse_status s =
        rocsparse_spmm(h->handle, rocsparse_operation_none, rocsparse_operation_none, &one, h->A, h->X, &zero,
                       h->Y, rocsparse_datatype_f64_r, h->alg, rocsparse_spmm_stage_compute, &h->buffer_bytes,
                       h->buffer);
    if (s != rocsparse_status_success) {
        set_error("rocsparse_spmm(compute) failed: status %d", (int)s);
        return SMFV_ERR_HIP;
    }
    return SMFV_OK;
}

SMFV_API int smfv_vendor_spmm_destroy(smfv_vendor_t h)
{
    delete h;
    return SMFV_OK;
}

}  // extern "C"
