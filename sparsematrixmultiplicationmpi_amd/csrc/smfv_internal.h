// smfv_internal.h -- shared helpers of libsmfv (error state, checks).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "smfv.h"

namespace smfv {

void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#define SMFV_REQUIRE(cond, ...)                   \
    do {                                          \
        if (!(cond)) {                            \
            ::smfv::set_error(__VA_ARGS__);       \
            return SMFV_ERR_INVALID;              \
        }                                         \
    } while (0)

#define SMFV_HIP(call)                                                               \
    do {                                                                             \
        hipError_t e_ = (call);                                                      \
        if (e_ != hipSuccess) {                                                      \
            ::smfv::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                              __FILE__, __LINE__);                                   \
            return SMFV_ERR_HIP;                                                     \
        }                                                                            \
    } while (0)

// launch-error check after a <<<>>> launch
#define SMFV_LAUNCHED() SMFV_HIP(hipGetLastError())

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// merge-path geometry shared by the kernels and the workspace query
struct MergeGeom {
    int64_t items;   // rows + nnz
    int64_t ipt;     // merge-path items per team
    int64_t nteams;
};
MergeGeom merge_geom(int nrows, int64_t nnz, int K);
size_t merge_workspace_bytes(int nrows, int64_t nnz, int K);

// smfv_plan_create / smfv_plan_create_rows with an explicit non-zero range
// (NONZERO rank-local plans: rows [row_begin, row_begin + m) restricted to
// the non-zeros [nnz_base, nnz_end)); h_rp / h_ci: the whole matrix or NULL.
// col_base: the global row of the block's first row, for a square pattern's
// neighbour lookup in the tile analysis (column c = block row c - col_base);
// -1 = row_begin (the block is a slice of the whole matrix), a local CSR of
// a row partition passes its first global row.
int plan_create(smfv_plan_t *out, int variant, int row_begin, int m, int n, int64_t nnz_base, int64_t nnz_end,
                const int *h_rp, const int *h_ci, int K, int flags, int col_base = -1);

}  // namespace smfv
