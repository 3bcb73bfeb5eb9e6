/*
 * smfv_oracle.c -- CPU parity ORACLE for the CSR x fat-vector SpMM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the reported CPU baseline), never as the thing measured or shipped.
 * The product path (libsmfv.so) never links or calls it.
 *
 * This is a plain-C restatement of the reference algorithms
 * (AlexisBalayre/SparseMatrixMultiplicationMPI, "Source Code/" = SC/):
 *
 *   oracle_spmm_sequential  <- SC/SparseMatrixFatVectorMultiply.cpp:11-31
 *   oracle_spmm_rowwise     <- SC/SparseMatrixFatVectorMultiplyRowWise.cpp:12-126
 *   oracle_spmm_columnwise  <- SC/SparseMatrixFatVectorMultiplyColumnWise.cpp:13-131
 *   oracle_spmm_nonzero     <- SC/SparseMatrixFatVectorMultiplyNonZeroElement.cpp:12-120
 *   oracle_mtx_read         <- SC/utils.cpp:70-185 (readMatrixMarketFile)
 *   oracle_fatvector_rand   <- SC/utils.cpp:193-209 (generateLargeFatVector)
 *   oracle_max_abs_diff     <- SC/utils.cpp:38-63 (areMatricesEqual)
 *
 * The MPI variants are restated for p simulated ranks inside one process:
 * the same partition formulas, the same local loop order, and the
 * collective's data movement (Gatherv = concatenation by displacement,
 * Reduce(SUM) = binomial-tree sum).  All arithmetic is fp64 with separate
 * multiply and add (built with -ffp-contract=off), which is what the
 * reference gets from g++ on x86-64 without -mfma.
 *
 * Parity pinning: the sequential / row-wise / column-wise restatements are
 * checked bit-for-bit against the reference's own four kernel sources
 * compiled unmodified from /root/reference (oracle/Makefile target `ref`,
 * output oracle/_ref/) via the golden fixtures in tests/golden/.  The
 * Matrix Market reader cannot be built from the reference (utils.cpp needs
 * PETSc, absent from the image); it is pinned by known-answer tests only.
 *
 * Indices: int32 rowPtr / colIdx exactly as SC/MatrixDefinitions.h:14-19;
 * dense offsets are int64 here (the reference uses int and overflows at
 * m*K >= 2^31 -- SURVEY.md section 7 item 5).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define ORACLE_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* Sequential: SC/SparseMatrixFatVectorMultiply.cpp:15-27                    */
/* result(m x K) zero-initialised (:15); row -> nnz -> k (:17-27)            */
/* ------------------------------------------------------------------------ */
ORACLE_API int oracle_spmm_sequential(int m, const int *rowPtr, const int *colIdx,
                                      const double *vals, const double *X, int K,
                                      double *Y)
{
    if (m < 0 || K < 0) return -1;
    memset(Y, 0, sizeof(double) * (size_t)m * (size_t)K);
    for (int i = 0; i < m; ++i) {
        double *yi = Y + (int64_t)i * K;
        for (int j = rowPtr[i]; j < rowPtr[i + 1]; ++j) {
            const double v = vals[j];
            const double *xc = X + (int64_t)colIdx[j] * K;
            for (int k = 0; k < K; ++k) {
                double prod = v * xc[k];
                yi[k] = yi[k] + prod;
            }
        }
    }
    return 0;
}

/* RowWise partition: SC/...RowWise.cpp:26-29 (remainder to the lowest ranks) */
ORACLE_API void oracle_partition_rows(int m, int p, int r, int *start, int *end)
{
    int q = m / p, extra = m % p;
    int s = r * q + (r < extra ? r : extra);
    *start = s;
    *end = s + q + (r < extra ? 1 : 0);
}

/* ColumnWise partition: SC/...ColumnWise.cpp:25-28 (remainder to the LAST rank) */
ORACLE_API void oracle_partition_cols(int K, int p, int r, int *start, int *end)
{
    int q = K / p, extra = K % p;
    int s = r * q;
    *start = s;
    *end = (r != p - 1) ? s + q : s + q + extra;
}

/* NonZeroElement partition: SC/...NonZeroElement.cpp:24-39 */
ORACLE_API void oracle_partition_nnz(int64_t nnz, int p, int r, int64_t *start, int64_t *end)
{
    int64_t q = nnz / p, extra = nnz % p;
    if (r < extra) {
        *start = (int64_t)r * (q + 1);
        *end = *start + q + 1;
    } else {
        *start = (int64_t)r * q + extra;
        *end = *start + q;
    }
}

/* ------------------------------------------------------------------------ */
/* RowWise: SC/SparseMatrixFatVectorMultiplyRowWise.cpp                      */
/* local flat (end-start) x K block (:32-50), Gatherv into rank order by      */
/* displacement (:63-87), rank-0 rebuild row-major (:111-121).               */
/* ------------------------------------------------------------------------ */
ORACLE_API int oracle_spmm_rowwise(int p, int m, const int *rowPtr, const int *colIdx,
                                   const double *vals, const double *X, int K, double *Y)
{
    if (p <= 0 || m < 0 || K < 0) return -1;
    int64_t displ = 0;
    for (int r = 0; r < p; ++r) {
        int s, e;
        oracle_partition_rows(m, p, r, &s, &e);
        int64_t localSize = (int64_t)(e - s) * K;
        double *local = (double *)calloc((size_t)(localSize > 0 ? localSize : 1), sizeof(double));
        if (!local) return -2;
        for (int i = s; i < e; ++i) {
            for (int j = rowPtr[i]; j < rowPtr[i + 1]; ++j) {
                int c = colIdx[j];
                for (int k = 0; k < K; ++k) {
                    int64_t li = (int64_t)(i - s) * K + k;
                    double prod = vals[j] * X[(int64_t)c * K + k];
                    local[li] = local[li] + prod;
                }
            }
        }
        /* MPI_Gatherv: rank r's block lands at displacement sum(recvCounts[<r]) */
        memcpy(Y + displ, local, sizeof(double) * (size_t)localSize);
        displ += localSize;
        free(local);
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* ColumnWise: SC/SparseMatrixFatVectorMultiplyColumnWise.cpp                 */
/* per owned column: per row dot product with a scalar sum (:34-48), local   */
/* panel [m x kc] row-major (:46), Gatherv rank-major (:82-84), rebuild      */
/* interleaving panels back into row-major (:109-126).                       */
/* ------------------------------------------------------------------------ */
ORACLE_API int oracle_spmm_columnwise(int p, int m, const int *rowPtr, const int *colIdx,
                                      const double *vals, const double *X, int K, double *Y)
{
    if (p <= 0 || m < 0 || K < 0) return -1;
    /* gathered buffer, rank-major panels */
    double *gathered = (double *)malloc(sizeof(double) * ((size_t)m * (size_t)K + 1));
    if (!gathered) return -2;
    int64_t displ = 0;
    for (int r = 0; r < p; ++r) {
        int c0, c1;
        oracle_partition_cols(K, p, r, &c0, &c1);
        int kc = c1 - c0;
        double *panel = gathered + displ;
        for (int col = c0; col < c1; ++col) {
            for (int i = 0; i < m; ++i) {
                double sum = 0.0;
                for (int j = rowPtr[i]; j < rowPtr[i + 1]; ++j) {
                    double prod = vals[j] * X[(int64_t)colIdx[j] * K + col];
                    sum = sum + prod;
                }
                panel[(int64_t)i * kc + (col - c0)] = sum;
            }
        }
        displ += (int64_t)m * kc;
    }
    /* rank-0 rebuild (:112-125) */
    int64_t idx = 0;
    for (int r = 0; r < p; ++r) {
        int c0, c1;
        oracle_partition_cols(K, p, r, &c0, &c1);
        for (int row = 0; row < m; ++row)
            for (int col = 0; col < c1 - c0; ++col)
                Y[(int64_t)row * K + c0 + col] = gathered[idx++];
    }
    free(gathered);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* NonZeroElement: SC/SparseMatrixFatVectorMultiplyNonZeroElement.cpp        */
/* nnz range per rank (:24-39), nnz->row map (:42-51), full m x K partial    */
/* per rank (:54-67), MPI_Reduce(SUM) to rank 0 (:88), rebuild (:112-115).   */
/* The reduce is restated as a binomial tree over ranks (MPICH's short-       */
/* message algorithm); MPICH may pick another association for large          */
/* messages, so this variant is compared with a tolerance, never bitwise,   */
/* for p > 2.                                                                */
/* ------------------------------------------------------------------------ */
ORACLE_API int oracle_spmm_nonzero(int p, int m, const int *rowPtr, const int *colIdx,
                                   const double *vals, const double *X, int K, double *Y)
{
    if (p <= 0 || m < 0 || K < 0) return -1;
    int64_t nnz = rowPtr[m];
    int64_t mk = (int64_t)m * K;
    int *rowOf = (int *)malloc(sizeof(int) * (size_t)(nnz > 0 ? nnz : 1));
    double *part = (double *)calloc((size_t)p * (size_t)(mk > 0 ? mk : 1), sizeof(double));
    if (!rowOf || !part) { free(rowOf); free(part); return -2; }
    for (int row = 0, idx = 0; row < m; ++row)
        for (; idx < rowPtr[row + 1]; ++idx) rowOf[idx] = row;
    for (int r = 0; r < p; ++r) {
        int64_t s, e;
        oracle_partition_nnz(nnz, p, r, &s, &e);
        double *local = part + (int64_t)r * mk;
        for (int64_t idx = s; idx < e; ++idx) {
            int row = rowOf[idx];
            int col = colIdx[idx];
            double v = vals[idx];
            for (int k = 0; k < K; ++k) {
                double prod = v * X[(int64_t)col * K + k];
                local[(int64_t)row * K + k] = local[(int64_t)row * K + k] + prod;
            }
        }
    }
    /* binomial-tree reduce to rank 0 */
    for (int mask = 1; mask < p; mask <<= 1)
        for (int r = 0; r < p; r += 2 * mask)
            if (r + mask < p) {
                double *a = part + (int64_t)r * mk, *b = part + (int64_t)(r + mask) * mk;
                for (int64_t t = 0; t < mk; ++t) a[t] = a[t] + b[t];
            }
    memcpy(Y, part, sizeof(double) * (size_t)mk);
    free(rowOf);
    free(part);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* areMatricesEqual: SC/utils.cpp:38-63 -- absolute |a-b| > tol fails.       */
/* Returns the max absolute difference (the caller applies the tolerance).  */
/* ------------------------------------------------------------------------ */
ORACLE_API double oracle_max_abs_diff(const double *a, const double *b, int64_t count)
{
    double mx = 0.0;
    for (int64_t i = 0; i < count; ++i) {
        double d = fabs(a[i] - b[i]);
        if (d > mx || d != d) mx = (d != d) ? INFINITY : d;
    }
    return mx;
}

/* ------------------------------------------------------------------------ */
/* generateLargeFatVector: SC/utils.cpp:193-209.  X[i][j] = rand()%100 + 1,  */
/* row-major, glibc rand() never seeded (= srand(1) stream).                 */
/* ------------------------------------------------------------------------ */
ORACLE_API void oracle_fatvector_rand(int n, int K, double *X)
{
    srand(1);
    for (int64_t i = 0; i < (int64_t)n * K; ++i) X[i] = (double)(rand() % 100 + 1);
}

/* ------------------------------------------------------------------------ */
/* readMatrixMarketFile: SC/utils.cpp:70-185.                                */
/*  - leading lines whose first char is '%' are comments; any of them        */
/*    containing "symmetric" / "pattern" sets the flag (:84-105)             */
/*  - first non-comment line: rows cols nnz (:109)                           */
/*  - nnz entries "r c [v]" read as whitespace-separated tokens (:124-141);  */
/*    pattern -> 1.0 (:130); 1-based -> 0-based (:143-144)                   */
/*  - symmetric: off-diagonal entries mirrored, value NOT negated (:149-152) */
/*  - each row sorted by (col, value) (:156-159); duplicates kept           */
/*  - CSR built row by row (:162-181)                                        */
/* Returns 0 on success, <0 on error (the reference throws runtime_error).  */
/* ------------------------------------------------------------------------ */
typedef struct { int col; double val; } oracle_entry;

static int entry_cmp(const void *a, const void *b)
{
    const oracle_entry *x = (const oracle_entry *)a, *y = (const oracle_entry *)b;
    if (x->col != y->col) return x->col < y->col ? -1 : 1;
    if (x->val < y->val) return -1;
    if (x->val > y->val) return 1;
    return 0;
}

ORACLE_API int oracle_mtx_read(const char *path, int *out_m, int *out_n, int64_t *out_nnz,
                               int **out_rowPtr, int **out_colIdx, double **out_vals)
{
    FILE *f = fopen(path, "r");
    if (!f) return -1; /* "Unable to open file" (:75-78) */
    char *line = NULL;
    size_t cap = 0;
    ssize_t len;
    int isSym = 0, isPat = 0, have = 0;
    while ((len = getline(&line, &cap, f)) >= 0) {
        if (line[0] == '%') {
            if (strstr(line, "symmetric")) isSym = 1;
            if (strstr(line, "pattern")) isPat = 1;
        } else {
            have = 1;
            break;
        }
    }
    int m, n;
    long long nz;
    if (!have || sscanf(line, "%d %d %lld", &m, &n, &nz) != 3 || m < 0 || n < 0 || nz < 0) {
        free(line);
        fclose(f);
        return -2; /* "Failed to read matrix dimensions" (:112-115) */
    }
    free(line);
    int64_t total = isSym ? 2 * nz : nz;
    int *rows = (int *)malloc(sizeof(int) * (size_t)(total > 0 ? total : 1));
    oracle_entry *ent = (oracle_entry *)malloc(sizeof(oracle_entry) * (size_t)(total > 0 ? total : 1));
    int *cnt = (int *)calloc((size_t)m + 1, sizeof(int));
    if (!rows || !ent || !cnt) { fclose(f); free(rows); free(ent); free(cnt); return -3; }
    int64_t t = 0;
    for (long long i = 0; i < nz; ++i) {
        int r, c;
        double v = 1.0;
        if (fscanf(f, "%d %d", &r, &c) != 2) goto bad;
        if (!isPat && fscanf(f, "%lf", &v) != 1) goto bad;
        r--; c--;
        if (r < 0 || r >= m || c < 0) goto bad; /* reference: UB; here an error */
        rows[t] = r; ent[t].col = c; ent[t].val = v; t++;
        if (isSym && r != c) {
            if (c >= m) goto bad;
            rows[t] = c; ent[t].col = r; ent[t].val = v; t++;
        }
    }
    fclose(f);
    /* counting sort by row keeps insertion order inside a row, then sort */
    for (int64_t i = 0; i < t; ++i) cnt[rows[i] + 1]++;
    for (int i = 0; i < m; ++i) cnt[i + 1] += cnt[i];
    int *rowPtr = (int *)malloc(sizeof(int) * ((size_t)m + 1));
    int *colIdx = (int *)malloc(sizeof(int) * (size_t)(t > 0 ? t : 1));
    double *vals = (double *)malloc(sizeof(double) * (size_t)(t > 0 ? t : 1));
    oracle_entry *sorted = (oracle_entry *)malloc(sizeof(oracle_entry) * (size_t)(t > 0 ? t : 1));
    int *fill = (int *)malloc(sizeof(int) * ((size_t)m + 1));
    if (!rowPtr || !colIdx || !vals || !sorted || !fill) {
        free(rowPtr); free(colIdx); free(vals); free(sorted); free(fill);
        free(rows); free(ent); free(cnt);
        return -3;
    }
    memcpy(rowPtr, cnt, sizeof(int) * ((size_t)m + 1));
    memcpy(fill, cnt, sizeof(int) * ((size_t)m + 1));
    for (int64_t i = 0; i < t; ++i) sorted[fill[rows[i]]++] = ent[i];
    for (int i = 0; i < m; ++i)
        qsort(sorted + rowPtr[i], (size_t)(rowPtr[i + 1] - rowPtr[i]), sizeof(oracle_entry), entry_cmp);
    for (int64_t i = 0; i < t; ++i) { colIdx[i] = sorted[i].col; vals[i] = sorted[i].val; }
    free(sorted); free(fill); free(rows); free(ent); free(cnt);
    *out_m = m; *out_n = n; *out_nnz = t;
    *out_rowPtr = rowPtr; *out_colIdx = colIdx; *out_vals = vals;
    return 0;
bad:
    fclose(f);
    free(rows); free(ent); free(cnt);
    return -4; /* "Failed to read data from file" (:138-141) */
}

ORACLE_API void oracle_free(void *p) { free(p); }
