/*
 * smfv.h -- C ABI of the MI355X-native CSR x fat-vector SpMM engine.
 *
 *   Y[m x K] = A_csr[m x n] * X[n x K]        (fp64, int32 CSR indices)
 *
 * This is the drop-in boundary for the reference's hot path
 * (AlexisBalayre/SparseMatrixMultiplicationMPI, "Source Code/" = SC/):
 *
 *   reference interface (replaced)                              entry point here
 *   ---------------------------------------------------------  ---------------------------
 *   SC/SparseMatrixFatVectorMultiply.h:14-15  (sequential)      smfv_spmm_csr_f64(SMFV_SEQUENTIAL)
 *   SC/SparseMatrixFatVectorMultiplyRowWise.h:15-17             smfv_spmm_csr_f64(SMFV_ROWWISE),
 *                                                               smfv_dist_spmm_f64(SMFV_ROWWISE)
 *   SC/SparseMatrixFatVectorMultiplyColumnWise.h:15             smfv_spmm_csr_f64(SMFV_COLUMNWISE),
 *                                                               smfv_dist_spmm_f64(SMFV_COLUMNWISE)
 *   SC/SparseMatrixFatVectorMultiplyNonZeroElement.h:15         smfv_spmm_csr_f64(SMFV_NONZERO),
 *                                                               smfv_dist_spmm_f64(SMFV_NONZERO)
 *   SC/MatrixDefinitions.h:14-22 (SparseMatrix, FatVector)      plain pointers + sizes below
 *   partition formulas SC/...RowWise.cpp:26-29,                 smfv_partition_{rows,cols,nnz}
 *     ...ColumnWise.cpp:25-28, ...NonZeroElement.cpp:24-39
 *   SC/utils.cpp:38-63 (areMatricesEqual)                       smfv_compare_f64 (device-side)
 *
 * The C++ signatures of the reference (FatVector by value, MPI collective)
 * are kept verbatim in include/SparseMatrixFatVectorMultiply*.h; they are
 * thin host wrappers over this ABI (libsmfv_mpi.so).
 *
 * Conventions (all functions):
 *   - every pointer named d_* is a DEVICE pointer on the current HIP device;
 *   - CSR is 0-based: row_ptr[m+1], col_idx[nnz], values[nnz], with
 *     row_ptr[0] == 0 and row_ptr[m] == nnz (as built by SC/utils.cpp:162-181);
 *   - X and Y are row-major with leading dimensions ldx >= K, ldy >= K
 *     (the SC/utils.cpp:216-228 `serialize` layout when ld == K);
 *   - `stream` is a hipStream_t (NULL = default stream); every call is
 *     asynchronous on it and captures into a hipGraph (no allocation, no
 *     synchronisation inside);
 *   - results of SEQUENTIAL, ROWWISE and COLUMNWISE are bit-identical to the
 *     reference's sequential kernel (per-row nnz-ascending sums, separate
 *     multiply and add); NONZERO (merge-path) sums a row split across
 *     partitions in a different association, like the reference's own
 *     MPI_Reduce(SUM) -- deterministic, within 1e-12 relative in practice;
 *   - return value: SMFV_OK (0) or a negative smfv_status; the message of
 *     the last failure on the calling thread is smfv_last_error().  No C++
 *     exception crosses this boundary.
 */
#ifndef SMFV_H
#define SMFV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMFV_API __attribute__((visibility("default")))

typedef enum smfv_variant {
    SMFV_SEQUENTIAL = 0, /* SC/SparseMatrixFatVectorMultiply.cpp:11-31            */
    SMFV_ROWWISE = 1,    /* SC/SparseMatrixFatVectorMultiplyRowWise.cpp:12-126    */
    SMFV_COLUMNWISE = 2, /* SC/SparseMatrixFatVectorMultiplyColumnWise.cpp:13-131 */
    SMFV_NONZERO = 3     /* SC/SparseMatrixFatVectorMultiplyNonZeroElement.cpp:12-120 */
} smfv_variant;

typedef enum smfv_status {
    SMFV_OK = 0,
    SMFV_ERR_INVALID = -1,   /* bad sizes / null pointers / unknown variant */
    SMFV_ERR_WORKSPACE = -2, /* workspace missing or too small            */
    SMFV_ERR_HIP = -3,       /* a HIP runtime call failed                 */
    SMFV_ERR_COMM = -4,      /* an RCCL call failed                       */
    SMFV_ERR_HOST = -5       /* host-side failure (I/O, allocation)       */
} smfv_status;

/* ---- library ------------------------------------------------------------ */
SMFV_API const char *smfv_last_error(void);
SMFV_API const char *smfv_version(void);
/* Creates the HIP context on the current device, loads the library's code
 * object (one empty kernel launch on `stream`) and starts the runtime's
 * host<->device copy path (one 1 MiB copy each way: the process's first
 * copy of that size costs 10-30 ms once), synchronised: the one-time device
 * start-up a CPU caller never pays, done before a timed call so that call's
 * time is the SpMM's. */
SMFV_API int smfv_device_init(void *stream);

/* ---- partitions (pure host functions, no device needed) ----------------- */
/* RowWise: q = m/p, rows [r*q + min(r, m%p), +q + (r < m%p))  (RowWise.cpp:26-29) */
SMFV_API void smfv_partition_rows(int m, int p, int r, int *start, int *end);
/* ColumnWise: K/p columns, remainder to the LAST rank        (ColumnWise.cpp:25-28) */
SMFV_API void smfv_partition_cols(int K, int p, int r, int *start, int *end);
/* NonZeroElement: nnz/p, remainder to the lowest ranks        (NonZeroElement.cpp:24-39) */
SMFV_API void smfv_partition_nnz(int64_t nnz, int p, int r, int64_t *start, int64_t *end);

/* ---- single-device SpMM ------------------------------------------------- */
/* Merge-path geometry of SMFV_NONZERO over nrows rows / nnz non-zeros
 * (host): out[0] merge items (rows + non-zeros), [1] items per team, [2]
 * teams.  Team t walks diagonals [t * out[1], (t + 1) * out[1]); a row open at
 * a team boundary is finished by the carry fix-up (tests sample those rows). */
SMFV_API int smfv_merge_geometry(int nrows, int64_t nnz, int K, int64_t out[3]);

/* Device workspace (bytes) smfv_spmm_csr_f64 needs for `variant`; 0 for all
 * but SMFV_NONZERO (merge-path carry slots). */
SMFV_API int smfv_spmm_workspace_bytes(int variant, int m, int64_t nnz, int K, size_t *bytes);

/* Y = A * X on the current device.  `workspace` may be NULL when the
 * workspace size is 0. */
SMFV_API int smfv_spmm_csr_f64(int variant, int m, int n, int64_t nnz,
                               const int *d_row_ptr, const int *d_col_idx, const double *d_values,
                               const double *d_X, int64_t ldx, int K,
                               double *d_Y, int64_t ldy,
                               void *d_workspace, size_t workspace_bytes, void *stream);

/* ---- plans: analysed once per (matrix pattern, K), executed many times --
 * The plan owns all device workspace (merge-path carries for NONZERO) and,
 * with K a multiple of 32 (or K = 4, 8, 16: one narrow column window, e.g. a
 * ColumnWise rank's K/p panel; the kernel stages and stores only the window's
 * columns, X and Y 16-byte aligned with even strides), a clustered
 * row-tile analysis of the pattern (h_col_idx needed): tiles of <= 64 rows
 * grown by adjacency whose distinct X rows (<= 239) fit a 60 KiB LDS image,
 * with a tile-ordered copy of the values and 16-bit X-row offsets.  The tiled
 * kernel (one warp-specialised block per CU, double-buffered LDS-DMA staging)
 * stages each tile's X rows once and reads them from LDS -- same per-row
 * order and arithmetic, bit-identical result; rows over a cap alone are
 * gathered straight from X by a second launch.  Tiling is used when the
 * re-use (non-zeros per staged X row) is >= 3 -- estimated first on 128 tiles
 * grown in the full pattern, so the decision does not depend on the row
 * numbering -- or when SMFV_PLAN_FORCE_TILES is set.  A NONZERO plan over
 * whole rows takes the same tiled kernel under the same rule (bit-identical
 * to the reference's NonZeroElement with one rank, which sums every row in
 * CSR order); otherwise, and with SMFV_PLAN_NO_TILES, it runs the merge path.
 * With K == 1 (SpMV) a plan over whole rows takes the chunk layout of
 * k_spmv_chunks wherever the pattern fits it (smfv_spmv_chunks_analyse):
 * consecutive rows packed into 1,024-entry chunks at fixed addresses, the
 * values snapshot and 16-bit column offsets (10 B per entry against CSR's
 * 12; 32-bit columns where a row spans more than 65,535 columns); it is a
 * tiled plan for the values contract below.
 *
 * Values contract of a TILED plan: smfv_plan_bind_values gathers a snapshot
 * of A's device values (tile order, and the directly-gathered rows) and the
 * plan computes with that snapshot until the next bind.  After the values
 * change -- at the same address or not -- the caller must bind again;
 * execute refuses a d_values pointer other than the bound one.  Untiled plans
 * read the live values.  The pattern (row_ptr / col_idx) must not change over
 * a plan's life.
 *
 * Streams: create allocates device memory and synchronises; bind and execute
 * are asynchronous and graph-capturable.  An execute on a stream other than
 * the bind's waits for the bind's gather (hipStreamWaitEvent; while capturing
 * it requires the gather to have completed).  A plan is not thread-safe. */
typedef struct smfv_plan_s *smfv_plan_t;
#define SMFV_PLAN_NO_TILES 1
#define SMFV_PLAN_FORCE_TILES 2
/* Opt-in: the tiled kernel sums each term with one fused multiply-add
 * instead of the reference's separate multiply and add.  Same per-row order;
 * results differ from the reference by rounding only (well inside the 1e-6
 * relative tolerance) and are no longer bit-identical. */
#define SMFV_PLAN_FMA 4
/* Tiles are seeded at the oldest unassigned neighbour of the tiles built so
 * far (a wavefront through the pattern's graph: neighbouring tiles run
 * together on one XCD and share X rows in its L2, whatever the row
 * numbering).  This flag seeds them in row order instead (A/B). */
#define SMFV_PLAN_NATURAL_SEEDS 8
/* Opt-in (BASELINE config 3's "MFMA K-panel", kept as a measured
 * alternative): the tiles run as dense 16 x 4 blocks of A on
 * v_mfma_f64_16x16x4f64 (k_rows_mfma).  Sums are reassociated by the MFMA:
 * within tolerance, not bit-identical. */
#define SMFV_PLAN_MFMA 16
/* Opt-in (measured slower, kept for A/B): the tiled plan cuts the first
 * tile of each of the kernel's blocks in two and runs the halves first and
 * last, halving the unoverlapped staging of a block's first tile and the
 * unoverlapped compute of its last -- at the cost of one more unit per block
 * (26.5 -> 27.2 us on the cop20k surrogate, K = 32). */
#define SMFV_PLAN_SPLIT_ENDS 32
/* Each XCD has its own L2, so the tiled plan splits the rows into 8 parts
 * of equal non-zero count -- row ranges, or shares of the rows' breadth-first
 * order, whichever reads fewer X rows summed over the parts -- tiles each
 * part as its own wavefront and runs part x on XCD x.  This flag keeps one
 * wavefront over the whole pattern cut into 8 consecutive shares (A/B). */
#define SMFV_PLAN_ONE_WAVEFRONT 64
/* Untiled, and the simplest row kernel for any K (one double per lane,
 * k_rows): an independent computation of the same per-row sums, used by the
 * C++ drop-in for the sequential function -- the result the parallel
 * variants are checked against (SC/main.cpp:184) -- so that check does not
 * compare a kernel with itself.  Ignored for SMFV_NONZERO. */
#define SMFV_PLAN_SIMPLE_ROWS 128
/* RETIRED (ignored): column-streamed tiles (k_rows_cs), measured 3.4x slower
 * than k_rows_ws (profiles/r03/ab_s2/); the r2-r4 lab build that kept it was
 * removed in r5.  The value stays reserved. */
#define SMFV_PLAN_CS 256
/* The tiled kernel k_rows_ws (~60-row tiles whose whole X union sits in
 * LDS), asked for explicitly (with a geometry flag below: A/B). */
#define SMFV_PLAN_WS 512
/* (r4) The geometry of k_rows_ws (A/B; without either flag the library's
 * default): GEOM1 one 1024-lane block per CU (8 compute + 8 loader waves,
 * tiles of <= 64 rows and <= 239 staged X rows, 158 KiB of LDS); GEOM2 two
 * independent 512-lane blocks per CU (4 + 4 waves, tiles of <= 32 rows and
 * <= 125 X rows, 80 KiB of LDS each), so one block's per-tile hand-off hides
 * behind the other's work.  Same per-row order: bit-identical either way.
 * Without a flag a plan takes GEOM1, except a SMALL plan (fewer than 1.5
 * GEOM1 tiles per CU, e.g. a rank's row block at p = 8), which takes GEOM2
 * when its 32-row tiles keep the re-use and add no direct rows: there one
 * unit per block is all fill and drain, and half-size units halve it
 * (7.9 -> 7.1 us on a cop20k rank block).  On whole cop20k GEOM2 is slower
 * (2.6x the units: profiles/r04/ab_geom). */
#define SMFV_PLAN_WS_GEOM1 1024
#define SMFV_PLAN_WS_GEOM2 2048
/* (r4) GEOM3: one 768-lane block per CU, 8 compute + 4 loader waves (16 X
 * pieces each), 64-row tiles: 3 waves per SIMD, so the compute waves may hold
 * up to 168 VGPRs (deeper LDS read-ahead). */
#define SMFV_PLAN_WS_GEOM3 4096
/* (r5) Live values: the tiled kernel's loaders DMA each row's value pairs
 * straight from the caller's CSR values (no snapshot, no bind pass: a bind is
 * a no-op and every execute reads the values it is given, like an untiled
 * plan).  Bit-identical to the snapshot path.  Tiled k_rows_ws plans only
 * (K = 1 chunk plans and SMFV_PLAN_MFMA keep their snapshot). */
#define SMFV_PLAN_LIVE_VALUES 8192
/* (r5) Row pairs: a k_rows_ws tile may hold up to twice its teams in rows,
 * the shortest rows riding as second rows of the teams of the next shortest
 * (a team sums its first row, stores it, then sums its second; no pair runs
 * more than one batch of 8 past the tile's longest row), with a larger entry
 * cap (2,048 against 1,792), so the tiles of short-row patterns stop at the
 * X-row cap instead of the row count.  Same per-row order: bit-identical.
 * Without either flag a plan builds both and keeps the one whose busiest
 * block runs fewer tiles (ties: one row per team): the irregular cop20k
 * stand-in pairs (10 -> 8 rounds, 27.6 -> 25.7 us), the stencil one does not
 * (8 rounds either way, and bigger tiles make longer units).  SINGLE_ROWS
 * forces one row per team, ROW_PAIRS forces pairs (A/B, tests). */
#define SMFV_PLAN_SINGLE_ROWS 16384
#define SMFV_PLAN_ROW_PAIRS 32768
SMFV_API int smfv_plan_create(smfv_plan_t *plan, int variant, int m, int n, int64_t nnz,
                              const int *h_row_ptr, const int *h_col_idx, int K, int flags);
/* Plan of the row block [row_begin, row_end) of a CSR matrix (h_row_ptr /
 * h_col_idx: host arrays of the WHOLE matrix; the analysis runs on the
 * block's own rows): what one rank of SC/...RowWise.cpp:36-50 computes.
 * Execute takes the whole matrix's device arrays and writes the block's rows
 * to d_Y (row i of the block at d_Y + i * ldy), as smfv_spmm_rowblock_f64. */
SMFV_API int smfv_plan_create_rows(smfv_plan_t *plan, int variant, int row_begin, int row_end, int n,
                                   const int *h_row_ptr, const int *h_col_idx, int K, int flags);
/* Host threads a plan analysis started on the CALLING thread may use (the
 * tile analysis runs its 8 XCD parts in parallel): 0 = the default (up to 8);
 * a library building plans in the background lowers it so the caller's own
 * work keeps its cores. */
SMFV_API void smfv_set_analysis_threads(int threads);
SMFV_API int smfv_plan_bind_values(smfv_plan_t plan, const double *d_values, void *stream);
/* Host-only diagnostic: run the clustered tile analysis and build the tiled
 * kernel's plan, verify the invariants the kernel relies on (every row in
 * exactly one tile or the direct list, caps, CSR order inside rows, union
 * positions, pads on the zero row -- by replaying the kernel's reads) and
 * report out[0] tiles, [1] staged X rows, [2] re-use, [3] direct rows,
 * [4] tile entries (incl. pads), [5] non-zeros in tiles.  No device needed. */
SMFV_API int smfv_plan_analyse(int m, int n, const int *h_row_ptr, const int *h_col_idx,
                               double out[6]);
/* The same for the row block [row_begin, row_end) with the caps a plan of
 * these flags uses (smfv_plan_create_rows; (r5) SMFV_PLAN_LIVE_VALUES builds
 * and verifies the live-values layout): out[0..5] as above, [6] XCD
 * parts (8 or 1), [7] X footprint of the 8 parts (-1: not computed),
 * [8] X footprint of the plan's 8 XCD tile ranges (distinct X rows each
 * reads, summed, over the block's distinct X rows).  No device needed. */
/* (r5) The narrow-team plan of a kw = 4 / 8 column window (k_rows_wsn) for
 * the row block [row_begin, row_end), built and verified on the host (the
 * kernel's reads replayed): out[0] tiles, [1] staged X rows, [2] re-use,
 * [3] direct rows, [4] rows of the fullest tile, [5] padded entries; (r6)
 * the modelled LDS cycles of the kernel's X reads (ds_read_b128 lane groups,
 * one cycle each when conflict-free, plus one per extra distinct address on a
 * bank): [6] lane groups (the conflict-free count), [7] cycles with the
 * plan's bank-coloured image slots, [8] cycles with first-use slots.  No
 * device needed.  (SC/...ColumnWise.cpp:34-48 on a rank's K/p panel.) */
SMFV_API int smfv_wsn_plan_analyse(int row_begin, int row_end, int n, const int *h_row_ptr,
                                   const int *h_col_idx, int kw, double out[9]);
SMFV_API int smfv_plan_analyse_rows(int row_begin, int row_end, int n, const int *h_row_ptr,
                                    const int *h_col_idx, int flags, double out[9]);
/* The K = 1 chunk layout (k_spmv_chunks) of the row block [row_begin,
 * row_end) with `cap` entry slots per chunk (512, 1024 or 2048; 0: the plans'
 * default), built and verified as smfv_plan_create builds it for K = 1:
 * out[0] 1 if the pattern fits the layout (else 0: a row longer than a
 * chunk), [1] chunks, [2] non-zeros placed, [3] most rows in a chunk, [4]
 * mean fill of a chunk's slots, [5] 1 for the wide layout (32-bit columns:
 * some row spans more than 65,535 columns), 0 for 16-bit offsets.  No device
 * needed.  (SC/SparseMatrixFatVectorMultiply.cpp:17-27 at vecCols = 1.) */
SMFV_API int smfv_spmv_chunks_analyse(int row_begin, int row_end, int n, const int *h_row_ptr,
                                      const int *h_col_idx, int cap, double out[6]);
SMFV_API int smfv_plan_execute(smfv_plan_t plan, const int *d_row_ptr, const int *d_col_idx,
                               const double *d_values, const double *d_X, int64_t ldx,
                               double *d_Y, int64_t ldy, void *stream);
/* out[0] tiled (0/1), [1] tiles, [2] staged X rows per panel, [3] re-use
 * (tiled non-zeros / staged rows), [4] plan device bytes, [5] direct rows,
 * [6] first row of the block, [7] re-use estimated on the sample tiles (-1:
 * not sampled), [8] host analysis + upload time (ms), [9] values gathered
 * by each bind (snapshot entries, pads included), [10] 1 if the tiles run on
 * the MFMA kernel (SMFV_PLAN_MFMA), [11] XCD parts (8: one part of the
 * rows per XCD, 1: one wavefront), [12] X rows the 8 parts read, summed,
 * over the pattern's X rows (-1: not computed), [13] the kernel a tiled
 * plan runs: 0 none (untiled), 1 k_rows_ws, 2 k_rows_mfma, 3 k_spmv_chunks,
 * (r5) 5 k_rows_wsn (narrow-team tiles of a K = 4 / 8 window),
 * (4 was the retired k_rows_cs); [14] (r5) 1 if the tiled plan reads live
 * values (SMFV_PLAN_LIVE_VALUES), else 0; [15] (r4) the k_rows_ws
 * geometry (1: one 1024-lane block per CU, 2: two 512-lane blocks, 3: one
 * 768-lane block; 0 other); [16] (r4) 1 if a bind writes the snapshot's real
 * entries from bind items of up to 4 consecutive non-zeros (pads written once
 * at create: k_bind_items), 0 if it gathers every entry by index; [17] (r5)
 * rows summed as a team's second row (SMFV_PLAN_SINGLE_ROWS) */
#define SMFV_PLAN_STATS 18
SMFV_API int smfv_plan_stats(smfv_plan_t plan, double out[SMFV_PLAN_STATS]);
SMFV_API int smfv_plan_destroy(smfv_plan_t plan);

/* HBM streaming probe for the bench (not the SpMM path): d_dst = d_src,
 * `bytes` (multiple of 16, 16-B aligned pointers) by a 16-byte-per-lane
 * non-temporal copy kernel.  Read + write bytes / time = the measured
 * streaming ceiling quoted beside the 8 TB/s spec. */
SMFV_API int smfv_stream_copy(void *d_dst, const void *d_src, size_t bytes, void *stream);
/* (r6) Floor probe of the SpMM's 2:1 read:write mix (bench only).
 * unit_kib <= 0: a plain non-temporal stream, each 16 B written is the sum of
 * 32 B read (rbytes == 2 * wbytes).  unit_kib in 1..64: the same kind of
 * bytes through k_rows_ws's pipeline shape -- one 1024-lane block per CU,
 * loader waves staging units of unit_kib KiB of d_src into LDS by
 * non-temporal LDS-DMA (double-buffered), writer waves storing each unit's
 * share of wbytes from LDS; rbytes < 2 GiB, rbytes >= wbytes.  d_dst gets
 * no meaningful values. */
SMFV_API int smfv_stream_mix(void *d_dst, size_t wbytes, const void *d_src, size_t rbytes, int unit_kib,
                             void *stream);

/* Rank-local building blocks of the distributed variants (also usable on
 * their own).  Row block [row_begin, row_end) of Y (row-major, ldy):
 * what one rank of SC/...RowWise.cpp:36-50 computes.  n = rows of X (all
 * rank-local functions take it: it bounds every X access). */
SMFV_API int smfv_spmm_rowblock_f64(int row_begin, int row_end, int n, const int *d_row_ptr,
                                    const int *d_col_idx, const double *d_values,
                                    const double *d_X, int64_t ldx, int K,
                                    double *d_Yblock, int64_t ldy, void *stream);

/* Column panel [col_begin, col_end) of Y for all m rows, written as a
 * [m x (col_end-col_begin)] panel with leading dimension ldp: what one rank
 * of SC/...ColumnWise.cpp:34-48 computes. */
SMFV_API int smfv_spmm_colpanel_f64(int m, int n, int col_begin, int col_end, const int *d_row_ptr,
                                    const int *d_col_idx, const double *d_values,
                                    const double *d_X, int64_t ldx,
                                    double *d_panel, int64_t ldp, void *stream);

/* nnz range [nnz_begin, nnz_end) (SC/...NonZeroElement.cpp:56-67): partial
 * rows [row_first, row_last] written compactly to d_Ypart (row_last -
 * row_first + 1 rows, ldy).  row_first/row_last are returned by
 * smfv_nnz_range_rows (host, reads the host copy of row_ptr). */
SMFV_API int smfv_nnz_range_rows(int m, const int *h_row_ptr, int64_t nnz_begin, int64_t nnz_end,
                                 int *row_first, int *row_last);
SMFV_API int smfv_spmm_nnzrange_workspace_bytes(int nrows, int64_t nnz_count, int K, size_t *bytes);
SMFV_API int smfv_spmm_nnzrange_f64(int row_first, int row_last, int64_t nnz_begin, int64_t nnz_end,
                                    int n, const int *d_row_ptr, const int *d_col_idx,
                                    const double *d_values, const double *d_X, int64_t ldx, int K,
                                    double *d_Ypart, int64_t ldy,
                                    void *d_workspace, size_t workspace_bytes, void *stream);

/* Rebuild row-major Y from rank-major column panels (the rank-0 loop of
 * SC/...ColumnWise.cpp:109-126, on device): panels of p ranks laid out back
 * to back, rank r's panel is [m x kc_r] at offset sum_{q<r} m*kc_q. */
SMFV_API int smfv_panels_to_rowmajor_f64(int m, int K, int p, const double *d_panels,
                                         double *d_Y, int64_t ldy, void *stream);

/* Sum compact partial row blocks (one per rank, rank order) into Y, zeroing
 * rows no rank covers: the MPI_Reduce(SUM) of SC/...NonZeroElement.cpp:88
 * restricted to the rows each rank touched.  h_row_first/h_row_last are
 * host arrays of p entries; block r sits at d_blocks + offset_r where
 * offset_r = K * sum_{q<r} (row_last_q - row_first_q + 1) (empty ranks have
 * row_last = row_first - 1). */
SMFV_API int smfv_combine_row_blocks_f64(int m, int K, int p, const int *h_row_first,
                                         const int *h_row_last, const double *d_blocks,
                                         double *d_Y, int64_t ldy, void *stream);

/* Device-side areMatricesEqual (SC/utils.cpp:38-63): writes max |a-b| and
 * max |a-b|/max(|b|, tiny) over the m x K matrices into h_out[0..1]
 * (host memory; synchronises the stream). */
SMFV_API int smfv_compare_f64(int m, int K, const double *d_A, int64_t lda, const double *d_B,
                              int64_t ldb, double *h_out, void *stream);

/* ---- synthetic inputs generated on device (bench configs 4-5) ----------- */
/* X[i][k] = 1 + (splitmix64(seed ^ (i*K + k)) % 100): integers 1..100 like
 * SC/utils.cpp:203, but counter-based so any shard can be generated alone. */
SMFV_API int smfv_fill_x_hash_f64(int64_t n, int K, uint64_t seed, double *d_X, int64_t ldx,
                                  void *stream);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) -------------------- */
typedef struct smfv_comm_s *smfv_comm_t;
#define SMFV_UNIQUE_ID_BYTES 128
SMFV_API int smfv_comm_unique_id(char out[SMFV_UNIQUE_ID_BYTES]);
SMFV_API int smfv_comm_init(smfv_comm_t *comm, int nranks, int rank,
                            const char id[SMFV_UNIQUE_ID_BYTES]);
SMFV_API int smfv_comm_destroy(smfv_comm_t comm);
SMFV_API int smfv_comm_rank(smfv_comm_t comm);
SMFV_API int smfv_comm_size(smfv_comm_t comm);
/* The number of ranks the RCCL communicator itself reports (ncclCommCount),
 * i.e. how many processes actually joined it -- not the size the caller
 * asked for.  (the reference's MPI_Comm_size(MPI_COMM_WORLD), SC/main.cpp:16) */
SMFV_API int smfv_comm_count(smfv_comm_t comm, int *nranks);
/* In-place broadcast of `bytes` device bytes from root's d_buf to every
 * rank's d_buf (ncclBroadcast over xGMI): the device-resident form of the
 * reference's input distribution (SC/main.cpp:106-143, 9x MPI_Bcast).
 * Collective, asynchronous on `stream`. */
SMFV_API int smfv_comm_bcast(smfv_comm_t comm, void *d_buf, size_t bytes, int root, void *stream);

/* Collective over `comm` (every rank calls it with the full A and X
 * resident on its device, as after SC/main.cpp:106-143):
 *   SMFV_ROWWISE    rank-local row block + gather (RowWise.cpp:85-87)
 *   SMFV_COLUMNWISE rank-local K panel + gather + device transpose (:82-84, :109-126)
 *   SMFV_NONZERO    rank-local nnz range + row-block reduce (NonZeroElement.cpp:88)
 * mode SMFV_TO_ROOT: the full Y lands on rank `root` only (reference
 * semantics, other ranks' d_Y untouched); SMFV_TO_ALL: every rank gets Y
 * (all-gather).  h_row_ptr is the host copy of row_ptr (NONZERO needs it to
 * find each rank's boundary rows).  Workspace: smfv_dist_workspace_bytes. */
/* Exchange plan of a distributed variant for p ranks (pure host; the same
 * function drives smfv_dist_spmm_f64).  For rank r:
 *   ROWWISE     first/last = its rows [first, last]            (RowWise.cpp:26-29)
 *   COLUMNWISE  first/last = its K columns [first, last]       (ColumnWise.cpp:25-28)
 *   NONZERO     first/last = the rows its nnz range touches    (NonZeroElement.cpp:24-39)
 * and offset/count (in doubles) = where its block sits in the exchange
 * buffer: Y itself for ROWWISE (offset = first*K), the rank-major panel
 * buffer for COLUMNWISE (offset = m*first), the compact row-block buffer for
 * NONZERO.  Empty ranks have last = first - 1 and count = 0.  Arrays hold p
 * entries; h_row_ptr is needed for NONZERO only. */
SMFV_API int smfv_dist_plan(int variant, int m, int64_t nnz, const int *h_row_ptr, int K, int p,
                            int *first, int *last, int64_t *offset, int64_t *count);

/* (r5) Distribution options: the high byte of a distributed plan's flags
 * (the low bits stay smfv_plan_create's SMFV_PLAN_* flags for the rank's
 * share), and the `dopts` of the *_opts host functions below.  0 = the
 * reference's decomposition.
 *   SMFV_DIST_BALANCED_ROWS  ROWWISE row blocks of equal WORK, 12 B per
 *        non-zero + 8K + 4 B per row (the block's CSR and Y bytes), instead
 *        of the reference's equal row counts (SC/...RowWise.cpp:26-29).  The
 *        result is bit-identical either way: each row is summed in CSR order
 *        by the one rank that owns it, and the Gatherv / all-gatherv exchange
 *        takes any block sizes.  Opt-in: measured on the irregular cop20k_A
 *        stand-in at p = 8 it cuts the slowest rank's kernel 12.1 -> 11.5 us
 *        but makes the Y blocks unequal (the largest 3.9 -> 5.6 MB), so the
 *        exchange, which dominates the step, loses the single ncclAllGather
 *        and moves more bytes per link.
 *   SMFV_DIST_CHUNKS(c)  ROWWISE, c = 2..7: the rank's block is cut into c
 *        row chunks of equal work, each a row-block plan of its own; chunk
 *        j's exchange is issued on the plan's exchange stream as soon as
 *        chunk j is computed, while chunk j + 1 computes (the exchange of
 *        one problem overlapped with its own compute).  A chunk's exchange
 *        is point to point: ncclSend of the chunk to every peer and ncclRecv
 *        of theirs (TO_ALL, an all-gatherv over the full xGMI mesh) or to the
 *        root (TO_ROOT, the Gatherv).  0 / 1: one block, one exchange.
 *        EXPERIMENTAL: the schedule is pinned over gloo (2 / 3 / 8 ranks) and
 *        at one rank on the GPU; its RCCL point-to-point groups have not yet
 *        moved data between two GPUs, so bench.py defaults to --chunks 1.
 * Row-partitioned plans (A not replicated) always use the reference rows. */
#define SMFV_DIST_BALANCED_ROWS (1 << 24)
#define SMFV_DIST_CHUNKS(c) (((c) & 7) << 25)
#define SMFV_DIST_CHUNKS_OF(f) (((f) >> 25) & 7)
#define SMFV_DIST_OPTS ((int)0xFF000000u) /* (r6) no signed shift into the sign bit */
/* smfv_dist_plan under distribution options (h_row_ptr needed for
 * work-balanced ROWWISE blocks; NULL falls back to the reference rows).
 * smfv_dist_plan(...) = smfv_dist_plan_opts(..., 0). */
SMFV_API int smfv_dist_plan_opts(int variant, int dopts, int m, int64_t nnz, const int *h_row_ptr, int K, int p,
                                 int *first, int *last, int64_t *offset, int64_t *count);
/* ROWWISE under SMFV_DIST_CHUNKS(c): rank `rank`'s chunk boundaries,
 * chunk j = rows [bounds[j], bounds[j + 1]); bounds holds >= 8 entries,
 * *nchunks receives c (1 when unchunked: bounds = [first, last + 1]). */
SMFV_API int smfv_dist_chunk_rows(int variant, int dopts, int m, int64_t nnz, const int *h_row_ptr, int K, int p,
                                  int rank, int *bounds, int *nchunks);

typedef enum smfv_dist_mode { SMFV_TO_ROOT = 0, SMFV_TO_ALL = 1 } smfv_dist_mode;
SMFV_API int smfv_dist_workspace_bytes(smfv_comm_t comm, int variant, int m, int64_t nnz,
                                       const int *h_row_ptr, int K, size_t *bytes);
SMFV_API int smfv_dist_spmm_f64(smfv_comm_t comm, int variant, int mode, int root, int m, int n,
                                int64_t nnz, const int *h_row_ptr, const int *d_row_ptr,
                                const int *d_col_idx, const double *d_values, const double *d_X,
                                int K, double *d_Y, void *d_workspace, size_t workspace_bytes,
                                void *stream);

/* Row-partitioned ROWWISE (bench config 5: the matrix does not fit, or is
 * not wanted, on every rank).  Unlike smfv_dist_spmm_f64, A is NOT
 * replicated: rank r passes only its rows [first, last] of the RowWise
 * partition (SC/...RowWise.cpp:26-29; smfv_dist_plan) as a local CSR
 * (row_ptr 0-based, column ids global), X (n x K, row-major) replicated.
 * Rank r computes its block in place at d_Y + first*K (d_Y is m x K on
 * every rank), then the RowWise exchange: SMFV_TO_ALL all-gathers (one
 * ncclAllGather when the blocks are equal, else all-gatherv),
 * SMFV_TO_ROOT gathers to root (SC/...RowWise.cpp:85-87).  Collective. */
SMFV_API int smfv_dist_rowpart_spmm_f64(smfv_comm_t comm, int mode, int root, int m, int n,
                                        const int *d_row_ptr_local, const int *d_col_idx_local,
                                        const double *d_values_local, const double *d_X, int K,
                                        double *d_Y, void *stream);

/* The exchange step as a list of operations (pure host; the schedule
 * smfv_dist_spmm_f64 and the distributed plans execute with RCCL, exposed so
 * it can be replayed over another transport in tests).  For rank `rank` of
 * p: op i is kinds[i] (SMFV_EX_*) with peer, offset and count (doubles,
 * into the exchange buffer of smfv_dist_plan); ops run in order, inside
 * one group.  Arrays hold >= 2p entries; *nops receives the count. */
#define SMFV_EX_ALLGATHER 1 /* ncclAllGather(buf + offset, buf + offset - rank * count, count): equal
                              back-to-back blocks, rank r's at offset - (rank - r) * count */
#define SMFV_EX_BCAST 2     /* ncclBroadcast(buf + offset, count, root = peer): one block of an all-gatherv */
#define SMFV_EX_SEND 3      /* ncclSend(buf + offset, count, to peer): own block to the root */
#define SMFV_EX_RECV 4      /* ncclRecv(buf + offset, count, from peer): a rank's block at the root */
SMFV_API int smfv_dist_exchange_ops(int variant, int mode, int root, int m, int64_t nnz,
                                    const int *h_row_ptr, int K, int p, int rank, int *kinds, int *peers,
                                    int64_t *offsets, int64_t *counts, int *nops);
/* (r5) The same under distribution options: the ops of chunk `chunk` (0 when
 * unchunked); a chunked plan runs chunk j's ops after chunk j's compute. */
SMFV_API int smfv_dist_exchange_ops_opts(int variant, int dopts, int mode, int root, int m, int64_t nnz,
                                         const int *h_row_ptr, int K, int p, int rank, int chunk, int *kinds,
                                         int *peers, int64_t *offsets, int64_t *counts, int *nops);
/* Runs an exchange schedule (ops as smfv_dist_exchange_ops returns them, or
 * any list of the same form) on `comm` over the device buffer d_buf:
 * ncclAllGather alone, else one ncclGroupStart / ncclGroupEnd around the
 * broadcasts / sends / receives.  A failing RCCL call closes the group
 * before the error returns, so the communicator's next call starts clean.
 * Collective; asynchronous on `stream`. */
SMFV_API int smfv_comm_exchange_f64(smfv_comm_t comm, const int *kinds, const int *peers, const int64_t *offsets,
                                    const int64_t *counts, int nops, double *d_buf, void *stream);
/* Test hook: the nth exchange operation run from now on (any communicator,
 * any plan) fails as an RCCL error would, inside its open group; 0 = off. */
SMFV_API void smfv_test_fail_exchange(int nth);

/* ---- distributed plans: the rank-local part analysed once --------------
 * A distributed plan holds this rank's share of a variant (RowWise row
 * block, ColumnWise K-column window, NonZeroElement nnz range) as a
 * single-device plan -- so the rank-local compute runs the tiled kernel
 * where it pays, as smfv_plan_* does -- plus the exchange buffers and the
 * exchange schedule.  h_col_idx may be NULL (no tiling).  Values contract as
 * for smfv_plan_t (bind after a change).  execute = execute_local +
 * exchange on the same stream; the two halves are exposed separately for
 * timing.  mode / root as smfv_dist_spmm_f64; d_Y is m x K, row-major.
 * Collective: every rank creates and executes its plan. */
typedef struct smfv_dist_plan_s *smfv_dist_plan_t;
SMFV_API int smfv_dist_plan_create(smfv_dist_plan_t *plan, smfv_comm_t comm, int variant, int mode, int root,
                                   int m, int n, int64_t nnz, const int *h_row_ptr, const int *h_col_idx, int K,
                                   int flags);
/* Row-partitioned ROWWISE (A not replicated, as smfv_dist_rowpart_spmm_f64):
 * the rank's local CSR rows of the RowWise partition of an m-row matrix. */
SMFV_API int smfv_dist_plan_create_rowpart(smfv_dist_plan_t *plan, smfv_comm_t comm, int mode, int root, int m,
                                           int n, const int *h_row_ptr_local, const int *h_col_idx_local, int K,
                                           int flags);
/* The plan of rank `rank` of `p` with no communicator: the rank-local share
 * exactly as a rank of smfv_dist_plan_create computes it (same partition,
 * same single-device plan), execute_local only -- exchange and execute
 * return SMFV_ERR_COMM when the schedule has operations.  Lets one device
 * run every rank of a p-rank decomposition (tests, replays). */
SMFV_API int smfv_dist_plan_create_rank(smfv_dist_plan_t *plan, int p, int rank, int variant, int mode, int root,
                                        int m, int n, int64_t nnz, const int *h_row_ptr, const int *h_col_idx, int K,
                                        int flags);
/* The plan's exchange buffer (device; COLUMNWISE rank-major panels, NONZERO
 * compact row blocks, at smfv_dist_plan's offset / count) and its size in
 * doubles; NULL / 0 for ROWWISE, whose exchange runs in Y. */
SMFV_API int smfv_dist_plan_exchange_buffer(smfv_dist_plan_t plan, double **d_buf, int64_t *doubles);
/* (r5) The partition the plan was created with (p entries each, as
 * smfv_dist_plan_opts returns them) and its p, rank and chunks per rank. */
SMFV_API int smfv_dist_plan_partition(smfv_dist_plan_t plan, int *first, int *last, int64_t *offset,
                                      int64_t *count);
SMFV_API int smfv_dist_plan_shape(smfv_dist_plan_t plan, int *p, int *rank, int *chunks);
SMFV_API int smfv_dist_plan_bind_values(smfv_dist_plan_t plan, const double *d_values, void *stream);
SMFV_API int smfv_dist_plan_execute(smfv_dist_plan_t plan, const int *d_row_ptr, const int *d_col_idx,
                                    const double *d_values, const double *d_X, double *d_Y, void *stream);
SMFV_API int smfv_dist_plan_execute_local(smfv_dist_plan_t plan, const int *d_row_ptr, const int *d_col_idx,
                                          const double *d_values, const double *d_X, double *d_Y, void *stream);
SMFV_API int smfv_dist_plan_exchange(smfv_dist_plan_t plan, double *d_Y, void *stream);
/* the rank-local plan's smfv_plan_stats */
SMFV_API int smfv_dist_plan_stats(smfv_dist_plan_t plan, double out[SMFV_PLAN_STATS]);
SMFV_API int smfv_dist_plan_destroy(smfv_dist_plan_t plan);

/* ---- vendor-library comparator (not on the product path) ---------------
 * Y = A * X by rocSPARSE's generic SpMM (CSR int32 / f64, row-major X and
 * Y), the analogue of the reference's PETSc MatMatMult comparison block
 * (SC/main.cpp:289-402).  create binds the operands, sizes and allocates the
 * rocSPARSE buffer and runs its preprocess stage; execute runs the compute
 * stage on the stream given at creation.  alg: 0 rocSPARSE default, 1 CSR
 * row split, 2 CSR merge path.  rocSPARSE's summation order is its own: its
 * result matches the reference within tolerance, not bit for bit. */
typedef struct smfv_vendor_s *smfv_vendor_t;
SMFV_API int smfv_vendor_spmm_create(smfv_vendor_t *handle, int alg, int m, int n, int64_t nnz,
                                     const int *d_row_ptr, const int *d_col_idx, const double *d_values,
                                     const double *d_X, int64_t ldx, int K, double *d_Y, int64_t ldy,
                                     void *stream);
SMFV_API int smfv_vendor_spmm_execute(smfv_vendor_t handle);
SMFV_API int smfv_vendor_spmm_destroy(smfv_vendor_t handle);

#ifdef __cplusplus
}
#endif

#endif /* SMFV_H */
