/*
 * smfv_host.h -- host-side inputs of the SpMM engine (no device needed).
 *
 *   reference function (replaced)                   entry point here
 *   ---------------------------------------------   -----------------------------
 *   SC/utils.cpp:70-185  readMatrixMarketFile       smfv_mtx_read
 *   SC/utils.cpp:193-209 generateLargeFatVector     smfv_fatvector_rand
 *   SC/utils.cpp:216-253 serialize / deserialize    (the flat row-major layout of
 *                                                    every X / Y buffer in smfv.h)
 *
 * plus synthetic CSR generators for the bench configurations that have no
 * input file in this environment (BASELINE.json configs 2-5; cop20k_A.mtx
 * is not available offline, so a labelled surrogate with its m and nnz is
 * generated instead) and a small binary CSR/dense container ("SMFV") used
 * by the tests and the reference driver.
 *
 * Arrays returned through `**out` pointers are malloc'd by the library and
 * released with smfv_free().  Return codes as in smfv.h.
 */
#ifndef SMFV_HOST_H
#define SMFV_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef SMFV_API
#define SMFV_API __attribute__((visibility("default")))
#endif

SMFV_API void smfv_free(void *p);

/* Matrix Market reader with the reference's semantics (SC/utils.cpp:70-185):
 * '%' lines are comments and set the symmetric / pattern flags by substring;
 * pattern entries are 1.0; symmetric off-diagonal entries are mirrored
 * without negation; each row is sorted by (column, value); duplicates are
 * kept.  Malformed input is an error here (the reference has undefined
 * behaviour on a blank size line). */
SMFV_API int smfv_mtx_read(const char *path, int *m, int *n, int64_t *nnz, int **row_ptr,
                           int **col_idx, double **values);
/* Writes a general (or, with symmetric=1, the lower triangle of a
 * symmetric) real coordinate Matrix Market file. */
SMFV_API int smfv_mtx_write(const char *path, int m, int n, const int *row_ptr, const int *col_idx,
                            const double *values, int symmetric);

/* X[i][j] = rand() % 100 + 1, row-major, from glibc's rand() stream with
 * its default seed 1 (SC/utils.cpp:203 never calls srand) -- restated
 * (TYPE_3 additive feedback generator) so the result does not depend on
 * other rand() calls in the process. */
SMFV_API void smfv_fatvector_rand(int64_t n, int K, double *X);

/* SMFV binary containers (little-endian):
 *   CSR   "SMFVCSR1" int32 m, int32 n, int64 nnz, int32 row_ptr[m+1],
 *         int32 col_idx[nnz], f64 values[nnz]
 *   dense "SMFVDNS1" int64 rows, int64 cols, f64 data[rows*cols]        */
SMFV_API int smfv_csr_write_bin(const char *path, int m, int n, const int *row_ptr,
                                const int *col_idx, const double *values);
SMFV_API int smfv_csr_read_bin(const char *path, int *m, int *n, int64_t *nnz, int **row_ptr,
                               int **col_idx, double **values);
SMFV_API int smfv_dense_write_bin(const char *path, int64_t rows, int64_t cols, const double *data);

/* Symmetric 3-D 27-point-stencil surrogate ("fem27"): grid nx*ny*(...) in
 * natural order truncated to m points; every stencil pair is kept with
 * probability keep (hash of the pair, so A is exactly symmetric), diagonal
 * always; values in [-1, 1) (diagonal in [1, 2)).  Used as the labelled
 * stand-in for SuiteSparse cop20k_A (m = 121192, nnz ~ 2.62M). */
SMFV_API int smfv_gen_fem27(int m, int nx, int ny, double keep, uint64_t seed, int64_t *nnz,
                            int **row_ptr, int **col_idx, double **values);

/* Irregular FEM-like surrogate (a second stand-in for cop20k_A with the
 * same m and nnz but no stencil regularity): m points in the unit cube, 70 %
 * uniform and 30 % in Gaussian clusters, each joined to its k_i nearest
 * points (k_i in [3, 48], log-graded along the cube's diagonal, times a
 * scale bisected so that nnz is
 * as close to target_nnz as the scale allows), symmetrised, diagonal
 * added, rows numbered in Morton order of the points.  Row degrees spread
 * ~5..80; values symmetric as smfv_gen_fem27. */
SMFV_API int smfv_gen_knn3d(int m, int64_t target_nnz, uint64_t seed, int64_t *nnz, int **row_ptr, int **col_idx,
                            double **values);

/* Rows [row_begin, row_end) of an m x n matrix with row lengths drawn from
 * a truncated power law (P(L >= x) ~ x^(1-alpha), cap `cap`) scaled to the
 * requested mean, columns uniform and distinct per row, sorted; values in
 * [-1, 1).  alpha <= 0 -> every row has exactly round(mean) entries
 * (BASELINE config 5's "~16 nnz/row uniform").  Row lengths and entries
 * depend only on (seed, global row), so any row block can be generated
 * alone.  row_ptr of the block starts at 0. */
SMFV_API int smfv_gen_random_rows(int64_t m, int64_t n, int64_t row_begin, int64_t row_end,
                                  double mean, double alpha, int cap, uint64_t seed,
                                  int64_t *nnz, int **row_ptr, int **col_idx, double **values);

#ifdef __cplusplus
}
#endif

#endif /* SMFV_HOST_H */
