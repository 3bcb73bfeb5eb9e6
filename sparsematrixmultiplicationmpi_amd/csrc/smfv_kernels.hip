// smfv_kernels.hip -- CDNA4 (gfx950) kernels of the CSR x fat-vector SpMM
// hot path and the single-device C ABI (include/smfv.h).
//
// Reference loops replaced (SC = /root/reference/Source Code):
//   k_rows_ws (tiled plan, K % 32 == 0), k_rows_mh / k_rows (no plan),
//   k_rows_list (a plan's direct rows)
//            <- SC/SparseMatrixFatVectorMultiply.cpp:17-27 (sequential) and
//               SC/SparseMatrixFatVectorMultiplyRowWise.cpp:36-50 (row block)
//   the same with a column window (colpanel)
//            <- SC/SparseMatrixFatVectorMultiplyColumnWise.cpp:34-48
//   k_merge_flat / k_merge + k_carry_fixup
//            <- SC/SparseMatrixFatVectorMultiplyNonZeroElement.cpp:24-67 (nnz
//               partition) + :88 (sum of partial rows)
//   k_panels_to_rowmajor <- SC/...ColumnWise.cpp:109-126 (rank-0 rebuild)
//   k_combine_blocks     <- SC/...NonZeroElement.cpp:88 (MPI_Reduce SUM)
//   k_compare            <- SC/utils.cpp:38-63 (areMatricesEqual)
//   k_copy16             bench probe: measured HBM streaming rate
//
// Layout: X[n x K] and Y[m x K] row-major (SC/utils.cpp:216-228 serialize),
// CSR int32/f64 as SC/MatrixDefinitions.h:14-19.
//
// Thread mapping ("row team"): a team of TEAM lanes owns one CSR row; lane t
// of the team owns VEC consecutive doubles of the output row (VEC = 2 ->
// 16-byte loads/stores; a K = 32 row of X is one 256-byte, 2-cache-line
// read by a 16-lane team).  The team reads TEAM (col, val) pairs with one
// coalesced load and broadcasts them inside the team with ds_bpermute, so
// each non-zero costs one 16-B/lane X gather.  Non-zeros of a row are
// accumulated strictly in CSR order with a separate multiply and add (fp
// contraction is off for this file), which makes SEQUENTIAL / ROWWISE /
// COLUMNWISE bit-identical to the reference's x86-64 loop.
//
// Workgroups are remapped XCD-major (bijective): blocks dealt round-robin to
// the 8 XCDs receive contiguous row ranges, so the X rows a band of the
// matrix touches stay in one XCD's L2.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "smfv_internal.h"
#include "smfv_plan.h"

#pragma clang fp contract(off)

namespace smfv {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int xcd_remap(int b, int nwg)
{
    // blocks b, b+8, ... share an XCD; give each such group a contiguous
    // range of logical block ids (bijective for any nwg; guide T1).
    const int x = b & 7, q = nwg >> 3, r = nwg & 7;
    const int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + (b >> 3);
}

template <int VEC> struct VecT;
template <> struct VecT<1> {
    using T = double;
    __device__ static T load(const double *p) { return *p; }
    __device__ static void store(double *p, T v) { *p = v; }
    __device__ static T zero() { return 0.0; }
    __device__ static T madd(T acc, double v, T x)
    {
        double p = v * x;
        return acc + p;
    }
};
template <> struct VecT<2> {
    using T = double2;
    __device__ static T load(const double *p) { return *reinterpret_cast<const double2 *>(p); }
    __device__ static void store(double *p, T v) { *reinterpret_cast<double2 *>(p) = v; }
    __device__ static T zero() { return make_double2(0.0, 0.0); }
    __device__ static T madd(T acc, double v, T x)
    {
        double px = v * x.x, py = v * x.y;
        return make_double2(acc.x + px, acc.y + py);
    }
};

// Accumulate nnz [js, je) of one row into acc (team-uniform control flow).
// X is indexed at column offset c (this lane's VEC columns); cok = lane owns
// a valid column.  Strict CSR order, separate multiply/add.
template <int TEAM, int VEC>
__device__ __forceinline__ typename VecT<VEC>::T
row_segment(int js, int je, const int *__restrict__ ci, const double *__restrict__ va,
            const double *__restrict__ X, int64_t ldx, int c, bool cok,
            typename VecT<VEC>::T acc)
{
    using V = VecT<VEC>;
    if constexpr (TEAM == 1) {
        int j = js;
        for (; j + 4 <= je; j += 4) {
            int c0 = ci[j], c1 = ci[j + 1], c2 = ci[j + 2], c3 = ci[j + 3];
            double v0 = va[j], v1 = va[j + 1], v2 = va[j + 2], v3 = va[j + 3];
            typename V::T x0 = V::zero(), x1 = V::zero(), x2 = V::zero(), x3 = V::zero();
            if (cok) {
                x0 = V::load(X + (int64_t)c0 * ldx + c);
                x1 = V::load(X + (int64_t)c1 * ldx + c);
                x2 = V::load(X + (int64_t)c2 * ldx + c);
                x3 = V::load(X + (int64_t)c3 * ldx + c);
            }
            acc = V::madd(acc, v0, x0);
            acc = V::madd(acc, v1, x1);
            acc = V::madd(acc, v2, x2);
            acc = V::madd(acc, v3, x3);
        }
        for (; j < je; ++j) {
            const int cc = ci[j];
            const double vv = va[j];
            typename V::T x = V::zero();
            if (cok) x = V::load(X + (int64_t)cc * ldx + c);
            acc = V::madd(acc, vv, x);
        }
        return acc;
    } else {
        constexpr int U = TEAM < 8 ? TEAM : 8;
        const int lane = threadIdx.x & 63;
        const int tl = lane & (TEAM - 1);
        const int tbase = lane & ~(TEAM - 1);
        for (int j0 = js; j0 < je; j0 += TEAM) {
            const int n = min(TEAM, je - j0);
            int myc = 0;
            double myv = 0.0;
            if (tl < n) {
                myc = ci[j0 + tl];
                myv = va[j0 + tl];
            }
            for (int t0 = 0; t0 < n; t0 += U) {
                int cc[U];
                double vv[U];
                typename V::T x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int src = tbase + min(t0 + u, TEAM - 1);
                    cc[u] = __shfl(myc, src);
                    vv[u] = __shfl(myv, src);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    x[u] = V::zero();
                    if (cok && t0 + u < n) x[u] = V::load(X + (int64_t)cc[u] * ldx + c);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (t0 + u < n) acc = V::madd(acc, vv[u], x[u]);
            }
        }
        return acc;
    }
}

// ---------------------------------------------------------------------------
// k_rows: rows [row_begin, row_begin + nrows) of Y (written at Y + lrow*ldy),
// columns [0, K) of the (possibly offset) X.
// ---------------------------------------------------------------------------
template <int TEAM, int VEC>
__global__ __launch_bounds__(256) void k_rows(int row_begin, int nrows, const int *__restrict__ rp,
                                              const int *__restrict__ ci,
                                              const double *__restrict__ va,
                                              const double *__restrict__ X, int64_t ldx, int K,
                                              double *__restrict__ Y, int64_t ldy)
{
    using V = VecT<VEC>;
    constexpr int RPB = 256 / TEAM;  // rows per block
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int lrow = blk * RPB + (int)(threadIdx.x / TEAM);
    if (lrow >= nrows) return;  // whole team leaves together
    const int tl = threadIdx.x & (TEAM - 1);
    const int row = row_begin + lrow;
    const int js = rp[row], je = rp[row + 1];
    double *yrow = Y + (int64_t)lrow * ldy;
    const int npass = (K + TEAM * VEC - 1) / (TEAM * VEC);
    for (int p = 0; p < npass; ++p) {
        const int c = p * TEAM * VEC + tl * VEC;
        const bool cok = c < K;
        typename V::T acc = row_segment<TEAM, VEC>(js, je, ci, va, X, ldx, c, cok, V::zero());
        if (cok) V::store(yrow + c, acc);
    }
}

// ---------------------------------------------------------------------------
// k_spmv_stream: K = 1 (SpMV, BASELINE config 1 on the GPU).  One lane per
// row, RPB consecutive rows per NT-lane block.  The block's non-zeros are streamed in
// chunks of CH: every lane loads CH / NT (col, val) pairs with coalesced
// loads, gathers X (n doubles, L2-resident for cop20k) and writes the
// products a_j * x_j to LDS; then each lane adds its row's products of the
// chunk in CSR order, carrying the partial sum across chunks.  The product
// is rounded before the add exactly as in the reference's y += a * x
// (SC/SparseMatrixFatVectorMultiply.cpp:22-24), so the result is
// bit-identical.
// ---------------------------------------------------------------------------
template <int NT, int RPB, int CH>
__global__ __launch_bounds__(NT) void k_spmv_stream(int row_begin, int nrows, const int *__restrict__ rp,
                                                    const int *__restrict__ ci,
                                                    const double *__restrict__ va,
                                                    const double *__restrict__ X, int64_t ldx,
                                                    double *__restrict__ Y, int64_t ldy)
{
    static_assert(CH % NT == 0 && RPB <= NT, "whole products per lane, one lane per row");
    constexpr int PER = CH / NT;
    __shared__ double prod[CH];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int lr0 = blk * RPB;
    const int nr = min(RPB, nrows - lr0);
    if (nr <= 0) return;  // block-uniform
    const int r0 = row_begin + lr0, t = threadIdx.x;
    const int e0 = rp[r0], e1 = rp[r0 + nr];
    int js = 0, je = 0;
    if (t < nr) js = rp[r0 + t], je = rp[r0 + t + 1];
    double acc = 0.0;
    for (int64_t c0 = e0; c0 < e1; c0 += CH) {  // (int64: c0 + CH may pass INT_MAX)
        const int cn = (int)min((int64_t)CH, (int64_t)e1 - c0);
        int c[PER];
        double v[PER], x[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = t + i * NT;
            c[i] = e < cn ? __builtin_nontemporal_load(ci + c0 + e) : 0;
            v[i] = e < cn ? __builtin_nontemporal_load(va + c0 + e) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) x[i] = t + i * NT < cn ? X[(int64_t)c[i] * ldx] : 0.0;
#pragma unroll
        for (int i = 0; i < PER; ++i) prod[t + i * NT] = v[i] * x[i];
        __syncthreads();
        int j = (int)(max((int64_t)js, c0) - c0);
        const int b = (int)(min((int64_t)je, c0 + cn) - c0);
        for (; j + 4 <= b; j += 4) {
            const double p0 = prod[j], p1 = prod[j + 1], p2 = prod[j + 2], p3 = prod[j + 3];
            acc = acc + p0;
            acc = acc + p1;
            acc = acc + p2;
            acc = acc + p3;
        }
        for (; j < b; ++j) acc = acc + prod[j];
        __syncthreads();
    }
    if (t < nr) Y[(int64_t)(lr0 + t) * ldy] = acc;
}

// ---------------------------------------------------------------------------
// k_spmv_chunks: K = 1 on a chunk plan (build_spmv_chunks).  Block c owns the
// rows of chunk c; its CH entry slots start at c * CH, so every lane issues
// its value (16-B pairs) and column-offset loads (two u16 per dword) at
// launch, beside the scalar header load, with no row_ptr round trip in
// front of them.  Lane t holds entries 2 (k NT + t) + {0, 1}: each load
// instruction of the wave reads one contiguous run.  The products a_j * x_j
// go to LDS; lane t < rows then adds its row's products in CSR order (the
// row starts come from the plan), exactly the reference's y += a * x.
// ---------------------------------------------------------------------------
typedef double chunk_d2 __attribute__((ext_vector_type(2)));
constexpr int K1_NT = 256;  // lanes per chunk block = row cap of a chunk

// entry slots per chunk (1,024; 512 and 2,048 measured slower: DESIGN.md 4.1)
static int spmv_chunk_cap()
{
    return 1024;
}


template <int NT, int CH, bool WIDE>
__global__ __launch_bounds__(NT) void k_spmv_chunks(const int4 *__restrict__ hdr, const uint16_t *__restrict__ rs,
                                                    const uint16_t *__restrict__ off, const int *__restrict__ col,
                                                    const double *__restrict__ vals,
                                                    const double *__restrict__ X, int64_t ldx,
                                                    double *__restrict__ Y, int64_t ldy)
{
    static_assert(CH % (2 * NT) == 0, "whole entry pairs per lane");
    constexpr int V2 = CH / (2 * NT);
    __shared__ chunk_d2 prod[CH / 2];
    const int c = xcd_remap(blockIdx.x, gridDim.x);
    const int t = threadIdx.x;
    const int4 h = hdr[c];  // first row, rows, base column, entries (scalar load, in flight with the stream)
    const chunk_d2 *v2 = reinterpret_cast<const chunk_d2 *>(vals + (int64_t)c * CH);
    const uint32_t *o2 = reinterpret_cast<const uint32_t *>(off + (int64_t)c * CH);
    const uint64_t *c2 = reinterpret_cast<const uint64_t *>(col + (int64_t)c * CH);
    chunk_d2 v[V2];
    uint32_t o[V2];
    uint64_t cc[V2];
#pragma unroll
    for (int k = 0; k < V2; ++k) {
        v[k] = __builtin_nontemporal_load(v2 + k * NT + t);
        if constexpr (WIDE) {
            cc[k] = __builtin_nontemporal_load(c2 + k * NT + t);  // two 32-bit columns
        } else {
            o[k] = __builtin_nontemporal_load(o2 + k * NT + t);
        }
    }
    const uint16_t *rsc = rs + (int64_t)c * (NT + 1);
    const int a = rsc[t], b = rsc[t + 1];
    // every stream load above is issued before anything waits (the
    // scheduler would otherwise put some of them behind the header's wait)
    __builtin_amdgcn_sched_barrier(0);
    const double *xb = X + (int64_t)h.z * ldx;
#pragma unroll
    for (int k = 0; k < V2; ++k) {
        const int64_t j0 = WIDE ? (int64_t)(int)(uint32_t)cc[k] : (int64_t)(o[k] & 0xFFFFu);
        const int64_t j1 = WIDE ? (int64_t)(int)(uint32_t)(cc[k] >> 32) : (int64_t)(o[k] >> 16);
        // pad slots gather nothing (a chunk of empty rows may sit on an empty X)
        const int e0 = 2 * (k * NT + t);
        const double x0 = e0 < h.w ? xb[j0 * ldx] : 0.0;
        const double x1 = e0 + 1 < h.w ? xb[j1 * ldx] : 0.0;
        chunk_d2 p;
        p.x = v[k].x * x0;
        p.y = v[k].y * x1;
        prod[k * NT + t] = p;
    }
    asm volatile("" ::"v"(a), "v"(b));  // the row starts are loaded now, not after the barrier
    __syncthreads();
    if (t < h.y) {
        const double *pr = reinterpret_cast<const double *>(prod);
        double acc = 0.0;
        int j = a;
        for (; j + 4 <= b; j += 4) {
            const double p0 = pr[j], p1 = pr[j + 1], p2 = pr[j + 2], p3 = pr[j + 3];
            acc = acc + p0;
            acc = acc + p1;
            acc = acc + p2;
            acc = acc + p3;
        }
        for (; j < b; ++j) acc = acc + pr[j];
        Y[(int64_t)(h.x + t) * ldy] = acc;
    }
}


// ---------------------------------------------------------------------------
// k_rows_mh: the production row kernel for K even and 16-byte aligned X/Y.
//
//  * a block of 256 lanes owns 256/TEAM consecutive rows; it stages its
//    row_ptr slice and its non-zero range (col, val) into LDS with one
//    coalesced pass (chunks of stage_cap(TEAM) non-zeros if it holds more), so the
//    dependent global round trips are row_ptr -> CSR -> X only;
//  * a team of TEAM lanes owns one row; lane t holds H double2 column groups
//    at columns 2t + 2*TEAM*h (h < H), i.e. each of the H 16-byte loads of a
//    team reads one contiguous 32*TEAM-byte segment of the X row -- full
//    coalescing while 64/TEAM rows share every per-non-zero instruction
//    (LDS read of col/val, address arithmetic, loop control);
//  * X is read through a buffer resource with a 32-bit byte offset
//    (col * ldx * 8 + lane column) and the column-group step as the
//    instruction's immediate offset (BUF = true, X < 4 GiB); BUF = false
//    is the 64-bit pointer path for larger X;
//  * U non-zeros' X rows are in flight per team before they are accumulated
//    in CSR order (separate multiply and add: bit-identical to the
//    reference's sequential loop).
// ---------------------------------------------------------------------------
// non-zeros staged per block pass: sized so a block's rows (256 / TEAM of
// them) usually fit one pass at ~22 non-zeros per row -- with a 1,024 cap a
// 128-row block (TEAM 2, a 4-column rank panel) ran three passes with a
// third of its teams live in each; 36 KiB at TEAM 2 still leaves 4 blocks
// (16 waves) per CU
constexpr int stage_cap(int team) { return team <= 1 ? 4096 : team == 2 ? 3072 : team == 4 ? 1536 : 1024; }
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int TEAM, int H, int U, bool BUF>
__global__ __launch_bounds__(256) void k_rows_mh(int row_begin, int nrows,
                                                 const int *__restrict__ rp,
                                                 const int *__restrict__ ci,
                                                 const double *__restrict__ va,
                                                 const double *__restrict__ X, int64_t ldx,
                                                 uint32_t xbytes, int K, double *__restrict__ Y,
                                                 int64_t ldy)
{
    constexpr int RPB = 256 / TEAM;
    constexpr int CP = 2 * TEAM * H;  // columns per pass
    constexpr int STAGE_CAP = stage_cap(TEAM);
    constexpr int PER_THREAD = STAGE_CAP / 256;
    __shared__ int s_rp[RPB + 1];
    __shared__ int s_ci[STAGE_CAP];
    __shared__ double s_va[STAGE_CAP];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int row0 = blk * RPB;
    const int nr = min(RPB, nrows - row0);
    const int tid = threadIdx.x;
    for (int i = tid; i <= nr; i += 256) s_rp[i] = rp[row_begin + row0 + i];  // nr + 1 entries
    __syncthreads();
    const int bs = s_rp[0], be = s_rp[nr];
    const int team = tid / TEAM, tl = tid & (TEAM - 1);
    const bool live = team < nr;
    const int js = live ? s_rp[team] : 0, je = live ? s_rp[team + 1] : 0;
    double *yrow = Y + (int64_t)(row0 + team) * ldy;
    // (BUF = false never reads xr; the descriptor is then an empty range)
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void *)X, 0, BUF ? (int)xbytes : 0, 0x00020000);
    const uint32_t ldxb = (uint32_t)(ldx * 8);
    const int npass = (K + CP - 1) / CP;
    for (int p = 0; p < npass; ++p) {
        const int cb = p * CP + 2 * tl;  // this lane's first column in the pass
        bool ok[H];
#pragma unroll
        for (int h = 0; h < H; ++h) ok[h] = cb + 2 * TEAM * h < K;
        double2 acc[H];
#pragma unroll
        for (int h = 0; h < H; ++h) acc[h] = make_double2(0.0, 0.0);
        for (int c0 = bs; c0 < be; c0 += STAGE_CAP) {
            const int cnt = min(STAGE_CAP, be - c0);
            if (c0 != bs || p != 0) __syncthreads();  // previous chunk fully consumed
            int rc[PER_THREAD];
            double rv[PER_THREAD];
#pragma unroll
            for (int u = 0; u < PER_THREAD; ++u) {
                const int idx = u * 256 + tid;
                rc[u] = 0;
                rv[u] = 0.0;
                if (idx < cnt) {
                    rc[u] = ci[c0 + idx];
                    rv[u] = va[c0 + idx];
                }
            }
#pragma unroll
            for (int u = 0; u < PER_THREAD; ++u) {
                const int idx = u * 256 + tid;
                if (idx < cnt) {
                    s_ci[idx] = rc[u];
                    s_va[idx] = rv[u];
                }
            }
            __syncthreads();
            if (!live) continue;
            const int a = max(js, c0) - c0, b = min(je, c0 + cnt) - c0;
            for (int j0 = a; j0 < b; j0 += U) {
                double2 x[U][H];
                double vv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    vv[u] = 0.0;
#pragma unroll
                    for (int h = 0; h < H; ++h) x[u][h] = make_double2(0.0, 0.0);
                    if (j0 + u < b) {
                        const int cc = s_ci[j0 + u];
                        vv[u] = s_va[j0 + u];
                        if constexpr (BUF) {
                            const int off = (int)((uint32_t)cc * ldxb + (uint32_t)cb * 8u);
#pragma unroll
                            for (int h = 0; h < H; ++h)
                                if (ok[h])
                                    x[u][h] = __builtin_bit_cast(
                                        double2, __builtin_amdgcn_raw_buffer_load_b128(
                                                     xr, off + h * 16 * TEAM, 0, 0));
                        } else {
                            const double *px = X + (int64_t)cc * ldx + cb;
#pragma unroll
                            for (int h = 0; h < H; ++h)
                                if (ok[h]) x[u][h] = *reinterpret_cast<const double2 *>(px + 2 * TEAM * h);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j0 + u < b)
#pragma unroll
                        for (int h = 0; h < H; ++h) acc[h] = VecT<2>::madd(acc[h], vv[u], x[u][h]);
            }
        }
        if (live)
#pragma unroll
            for (int h = 0; h < H; ++h)
                if (ok[h]) *reinterpret_cast<double2 *>(yrow + cb + 2 * TEAM * h) = acc[h];
    }
}

// ---------------------------------------------------------------------------
// k_rows_ws: the production tiled kernel (K % 32 == 0, plans with re-use).
// One persistent 1024-lane block per CU, warp-specialised:
//  * waves 8-15 (loaders) stage the next work unit into the other half of a
//    double-buffered LDS image by LDS-DMA (global_load_lds_dwordx4);
//  * waves 0-7 (compute) run 64 eight-lane teams, one row each, out of LDS:
//    per batch of 8 entries, one b64 read of 8 u8 image rows, four of 8 values,
//    16 b128 X reads; the next batch's meta is read behind this batch's X.
// A work unit is (tile, 32-column panel), panels innermost: a unit stages
// the tile's union of X rows for its panel (<= 255 x 256 B; image row 255
// stays zero) into X slot (unit & 1); the tile's values, u8 X-image rows
// (tile-ordered, interleaved per quad of teams, build_ws_plan) and 1 KiB
// record are staged once per tile, with its first panel, into meta slot
// (tile & 1) -- K = 128 reads them once, not four times.
// One barrier per unit.  An LDS-DMA stalls its wave while the CU's vector
// memory path drains, so compute waves never issue one.  Each row is summed
// over its non-zeros in CSR order with separate multiply and add; pads read
// the zero row with value -0.0, and acc + (-0.0 * +0.0) = acc exactly, so
// the result is bit-identical to the reference loop.  Values, offsets and
// records are read once (non-temporal); X rows are re-staged by later tiles
// and keep the default policy.  Tile order: XCD x = blockIdx.x % 8 owns
// tiles [ntiles*x/8, ntiles*(x+1)/8), its blocks sweep them together, so
// neighbouring tiles re-use X rows from the XCD's L2.  gridDim.x % 8 == 0.
// ---------------------------------------------------------------------------
namespace ws {
constexpr int XSLOT = (WS_UCAP + 1) * 256;  // X image: union rows + the zero row, 256 B each
constexpr int SL_M = 2 * XSLOT;             // meta slots follow the X slots
// values and offsets arrive in whole 1 KiB DMA pieces (128 doubles / 1,024 u8)
[[maybe_unused]] constexpr int M_V = 0, M_L = (WS_NCAP + 127) / 128 * 1024, M_R = M_L + (WS_NCAP + 1023) / 1024 * 1024,
              MSLOT = M_R + WS_LWORDS * 4;
static_assert(SL_M + 2 * MSLOT <= 160 * 1024, "two X and two meta slots must fit the CU's 160 KiB");
static_assert(XSLOT % 1024 == 0 && MSLOT % 1024 == 0, "1 KiB DMA pieces");
static_assert(WS_UCAP + 1 <= 4 * 8 * WS_LOADERS, "8 X pieces per loader wave cover the image");
typedef double d2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

// LDS-DMA of 16 B per lane to lds_dst + 16 * lane (M0 written in the same
// statement, MI355X guide recipe); NT: non-temporal source read.
template <bool NT> __device__ __forceinline__ void dma16(const void *g, unsigned lds_dst)
{
    unsigned keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
// The same with a scalar base + 32-bit per-lane byte offset (the global
// instructions' saddr form): the 64-bit address arithmetic per lane and
// piece disappears (one v_add per DMA at most instead of ~15 VALU).  The
// base must be wave-uniform; every byte addressed must lie within 4 GiB of it.
template <bool NT> __device__ __forceinline__ void dma16s(const void *base, unsigned voff, unsigned lds_dst)
{
    unsigned keep;
    const uint64_t b = (uint64_t)(uintptr_t)base;
    // (readfirstlane returns int: widen through uint32_t, never sign-extend)
    const uint64_t sb = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)b);
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(voff), "s"(sb), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(voff), "s"(sb), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
__device__ __forceinline__ void barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// (r5) The same through a buffer descriptor (SGPR quad) + 32-bit per-lane byte
// offset, non-temporal: the range check returns 0 for every dword at or past
// the descriptor's num_records (measured per dword on MI355X:
// scripts/micro/lds_dma_probe.hip), so a 16-byte piece that straddles the end
// of the caller's array reads no byte past it.  voff need only be 8-byte
// aligned (LDS-DMA of 8-byte aligned 16-byte pieces: exact, same probe).
typedef int bufrsrc __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void dma16b(bufrsrc r, unsigned voff, unsigned lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
// a raw buffer over [base, base + bytes) (bytes < 4 GiB), wave-uniform
__device__ __forceinline__ bufrsrc make_rsrc(const void *base, unsigned bytes)
{
    const uint64_t b = (uint64_t)(uintptr_t)base;
    return bufrsrc{__builtin_amdgcn_readfirstlane((int)(uint32_t)b),
                   __builtin_amdgcn_readfirstlane((int)((b >> 32) & 0xFFFF)),
                   __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}

// (r4) LDS layout of a k_rows_ws geometry (WsGeom, smfv_plan.h): two X
// images of UCAP + 1 rows (the last one zero), then two meta slots of values,
// u8 offsets and the tile's record ([0, R) rows, [R, 2R) L bases, [2R, 3R) V
// bases, (r5) [3R, 4R) second rows; 1 KiB for 64-team tiles, 512 B for 32)
template <int CW, int LW, int PPW, int UCAP, int NCAP> struct Lay {
    static constexpr int R = 8 * CW;
    static constexpr int XSLOT = (UCAP + 1) * 256;
    static constexpr int SL_M = 2 * XSLOT;
    static constexpr int M_V = 0, M_L = (NCAP + 127) / 128 * 1024, M_R = M_L + (NCAP + 1023) / 1024 * 1024;
    static constexpr int REC_LANES = CW == 8 ? 64 : R;  // 16 B per lane (4 words per team slot)
    static constexpr int RECB = CW == 8 ? 1024 : (REC_LANES * 16 + 255) / 256 * 256;
    static constexpr int MSLOT = M_R + RECB;
    static constexpr int BYTES = SL_M + 2 * MSLOT;
    static constexpr int ZOFF = UCAP * 256;
    static_assert(BYTES <= (CW == 8 ? 160 : 80) * 1024, "the blocks of one CU share its 160 KiB");
    static_assert(UCAP + 1 <= 4 * PPW * LW && PPW % 4 == 0, "PPW X pieces per loader wave cover the image");
    static_assert(UCAP <= 255, "u8 image offsets");
    static_assert(XSLOT % 16 == 0 && MSLOT % 16 == 0 && M_L % 1024 == 0, "16-byte DMA lanes");
};
}  // namespace ws

// SADDR: the loaders address X, the values and the offsets by scalar base +
// 32-bit byte offset (X and the plan's arrays each < 4 GiB; the host picks it).
struct WsXcd {
    int first[9];  // XCD x runs tiles [first[x], first[x + 1]) of the plan's order
};
// (r5) LIVE: the loaders DMA the value pairs straight from the caller's CSR
// values (tv = the block's first value, tv_bytes its bytes) at the CSR index
// vidx[t * vstride + slot] of each slot (WsPlan::live): no snapshot, no bind
// The body is shared by the two kernels below: k_rows_ws (the snapshot,
// with the r4 argument list) and k_rows_ws_live (r5, three more arguments).
template <int CW, int LW, int PPW, int UCAP, int NCAP, bool FMA, bool SADDR, bool NARROW, bool LIVE>
__device__ __forceinline__ void ws_body(int xfirst, int xend, int npanel, int chunked, const int *__restrict__ grec,
                                        const int *__restrict__ lrec, const uint8_t *__restrict__ loff,
                                        const double *__restrict__ tv, const double *__restrict__ X, int64_t ldx,
                                        double *__restrict__ Y, int64_t ldy, const int *__restrict__ vidx,
                                        int vstride, unsigned tv_bytes)
{
    using namespace ws;
    using L = Lay<CW, LW, PPW, UCAP, NCAP>;
    constexpr int XSLOT = L::XSLOT, SL_M = L::SL_M, M_V = L::M_V, M_L = L::M_L, M_R = L::M_R, MSLOT = L::MSLOT;
    __shared__ __attribute__((aligned(16))) char lds[L::BYTES];
    int t0, tstep, cnt;
    {
        // XCD x = blockIdx.x % 8 owns tiles [first, end) of the plan's order
        // (its row range, or an eighth of one wavefront: build_ws_plan);
        // its nb blocks take them strided (block j: first + j, + nb, ...) or,
        // chunked, as consecutive runs (block j: a run of q or q + 1 tiles),
        // so a block's next tile is the wavefront neighbour of its last one
        const int nb = gridDim.x >> 3;  // blocks per XCD
        const int j = blockIdx.x >> 3;
        const int first = xfirst, end = xend;
        if (chunked & 1) {
            const int S = end - first, q = S / nb, r = S % nb;
            t0 = first + j * q + min(j, r);
            cnt = q + (j < r ? 1 : 0);
            tstep = 1;
            if (cnt <= 0) return;  // block-uniform
        } else {
            t0 = first + j;
            tstep = nb;
            if (t0 >= end) return;  // block-uniform
            cnt = (end - 1 - t0) / nb + 1;
        }
    }
    const int tlast = t0 + (cnt - 1) * tstep;
    const int nunits = cnt * npanel;
    // (r4) NARROW: a narrow column window (chunked bits 16-23: K = 4, 8 or
    // 16, one panel).  The loaders stage the window's bytes of each union row
    // into BOTH 128-byte halves of its image row (lanes 8-15 of a row repeat
    // lanes 0-7: the same cache lines, one DMA), so every team reads its
    // columns from its own half as at K = 32 (conflict-free) and needs one
    // accumulator: half the X reads and FP64 of a full panel; the teams store
    // only the window's columns
    const int kwin = NARROW ? (chunked >> 16) & 0xFF : 0;
    constexpr int XLANE = NARROW ? 7 : 15;  // a loader lane's 16-byte column chunk: lane & XLANE
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned lds0 = (unsigned)(uintptr_t)lds;  // LDS byte address of the block's image
    if (wv >= CW) {
        // ---------------- loader waves ----------------
        // loaders win instruction arbitration on their SIMD: a DMA issued
        // late stretches the whole unit (30.1 -> 28.0 us on the surrogate)
        __builtin_amdgcn_s_setprio(3);
        const int wl = wv - CW;
        if (wl == 0 && lane < 32)  // zero row of both X slots
            reinterpret_cast<d2 *>(lds + (lane >> 4) * XSLOT + L::ZOFF)[lane & 15] = d2{0.0, 0.0};
        i4 ur[PPW / 4];                       // union ids of this lane's pieces
        int noff, tn, nu, voff, tnv;
        unsigned xo[PPW];                     // SADDR: byte offset of this lane's 16 B of union row uc[i]
        const unsigned ldxb = (unsigned)(ldx * 8);
        // LIVE: this lane's value slot in each of the wave's value pieces
        // (pieces wl, wl + LW, ...: VI at most), as byte offsets into tv
        constexpr int VI = (NCAP + 128 * LW - 1) / (128 * LW);
        unsigned vo[LIVE ? VI : 1] = {};
        bufrsrc vr{};
        if constexpr (LIVE) vr = make_rsrc(tv, tv_bytes);
        auto fetch_record = [&](int t) {
            const int *G = grec + (int64_t)t * WS_GWORDS;
            const i4 *gu = reinterpret_cast<const i4 *>(G + 4 * PPW * wl + PPW * (lane >> 4));
#pragma unroll
            for (int k = 0; k < PPW / 4; ++k) ur[k] = gu[k];
            noff = G[WS_G_NOFF + (lane & 15)];
            tn = G[WS_G_TN + (lane & 15)];
            nu = G[WS_G_NU + (lane & 15)];
            voff = G[WS_G_VOFF + (lane & 15)];
            tnv = G[WS_G_TNV + (lane & 15)];
            if constexpr (LIVE) {
                // the slots' CSR indices load beside the record, a unit before
                // their DMAs (no dependent round trip in front of the stage)
                const int *vt = vidx + (int64_t)t * vstride + 64 * wl + lane;
#pragma unroll
                for (int i = 0; i < VI; ++i)
                    if (64 * (wl + LW * i) < vstride) vo[i] = 8u * (unsigned)vt[64 * LW * i];
            }
        };
        // stage unit (tile t, panel p): X rows into X slot xs, and (first panel) the meta into slot ms
        auto stage = [&](int t, int p, int xs, int ms) {
            // hipcc does not count the asm DMAs: resolve the record registers
            // here, so no wait it places for them lands between two DMAs
#pragma unroll
            for (int k = 0; k < PPW / 4; ++k) asm volatile("" ::"v"(ur[k]));
            asm volatile("" ::"v"(noff), "v"(tn), "v"(nu), "v"(voff), "v"(tnv));
            if constexpr (LIVE)
                if (p == 0)
#pragma unroll
                    for (int i = 0; i < VI; ++i) asm volatile("" ::"v"(vo[i]));
            const unsigned xb = lds0 + xs * XSLOT;
            int uc[PPW];
#pragma unroll
            for (int k = 0; k < PPW / 4; ++k)
                uc[4 * k] = ur[k].x, uc[4 * k + 1] = ur[k].y, uc[4 * k + 2] = ur[k].z, uc[4 * k + 3] = ur[k].w;
            const int cp = p * TILE_KP;
            if constexpr (SADDR)
                if (p == 0)  // per tile: the union rows' byte offsets (panels add to the scalar base)
#pragma unroll
                    for (int i = 0; i < PPW; ++i) xo[i] = (unsigned)uc[i] * ldxb + 16u * (unsigned)(lane & XLANE);
            auto stage_meta = [&]() {
                const unsigned mb = lds0 + SL_M + ms * MSLOT;
                if constexpr (LIVE) {  // value pairs from the CSR values (SADDR for the rest)
#pragma unroll
                    for (int i = 0; i < VI; ++i) {
                        const int k = wl + LW * i;
                        if (k * 128 < tnv) dma16b(vr, vo[i], mb + M_V + k * 1024);
                    }
                    const uint8_t *lb = loff + __builtin_amdgcn_readfirstlane(noff);
                    for (int k = wl; k * 1024 < tn; k += LW)
                        dma16s<true>(lb, 1024u * k + 16u * lane, mb + M_L + k * 1024);
                    if (wl == LW - 1 && lane < L::REC_LANES)
                        dma16s<true>(lrec + (int64_t)t * WS_LWORDS, 16u * lane, mb + M_R);
                } else if constexpr (SADDR) {
                    const int nf = __builtin_amdgcn_readfirstlane(noff);
                    const double *tvb = tv + __builtin_amdgcn_readfirstlane(voff);
                    const uint8_t *lb = loff + nf;
                    for (int k = wl; k * 128 < tnv; k += LW)
                        dma16s<true>(tvb, 1024u * k + 16u * lane, mb + M_V + k * 1024);
                    for (int k = wl; k * 1024 < tn; k += LW)
                        dma16s<true>(lb, 1024u * k + 16u * lane, mb + M_L + k * 1024);
                    if (wl == LW - 1 && lane < L::REC_LANES)
                        dma16s<true>(lrec + (int64_t)t * WS_LWORDS, 16u * lane, mb + M_R);
                } else {
                    for (int k = wl; k * 128 < tnv; k += LW)
                        dma16<true>(tv + voff + 128 * k + 2 * lane, mb + M_V + k * 1024);
                    for (int k = wl; k * 1024 < tn; k += LW)
                        dma16<true>(loff + noff + 1024 * k + 16 * lane, mb + M_L + k * 1024);
                    if (wl == LW - 1 && lane < L::REC_LANES)
                        dma16<true>(lrec + (int64_t)t * WS_LWORDS + 4 * lane, mb + M_R);
                }
            };
#pragma unroll
            for (int i = 0; i < PPW; ++i) {
                const int piece = wl + LW * i;  // 1 KiB = union rows 4*piece .. +3 (pieces dealt round-robin)
                const int u = 4 * piece + (lane >> 4);
                if (4 * piece < nu && u < UCAP && (!NARROW || 2 * (lane & 7) < kwin)) {
                    if constexpr (SADDR)
                        dma16s<false>(X + cp, xo[i], xb + piece * 1024);
                    else
                        dma16<false>(X + (int64_t)uc[i] * ldx + cp + 2 * (lane & XLANE), xb + piece * 1024);
                }
            }
            if (p == 0) stage_meta();
        };
        // unit u = (tile index it, panel p); the record registers hold the
        // tile being staged until its last panel is issued, then the next one
        fetch_record(t0);
        stage(t0, 0, 0, 0);
        if (npanel == 1) fetch_record(min(t0 + tstep, tlast));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        int it = 0, p = 0;  // unit u + 1 to stage
        if (++p == npanel) p = 0, ++it;
        for (int u = 0; u < nunits; ++u) {
            if (u + 1 < nunits) {
                const int t = t0 + it * tstep;
                stage(t, p, (u + 1) & 1, it & 1);
                if (p == npanel - 1) fetch_record(min(t + tstep, tlast));
                if (++p == npanel) p = 0, ++it;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // unit u+1 has landed
            barrier_lds();
        }
        return;
    }
    // ---------------- compute waves ----------------
    // FMA (opt-in plan flag SMFV_PLAN_FMA): one fused multiply-add per term,
    // within the reference's 1e-6 tolerance but no longer bit-identical
    auto madd = [](d2 a, double v, d2 x) -> d2 {
        if constexpr (FMA)
            return d2{__builtin_fma(v, x.x, a.x), __builtin_fma(v, x.y, a.y)};
        else
            return a + v * x;
    };
    const int tw = (tid >> 3) & 7, tl = tid & 7, par = tw & 1;
    const int slot = tw * CW + wv;
    const int qk = tw & 3;  // position of the team in its quad
    barrier_lds();
    int it = 0, p = 0;
    for (int u = 0; u < nunits; ++u) {
        const char *xbase = lds + (u & 1) * XSLOT;
        const char *mbase = lds + SL_M + (it & 1) * MSLOT;
        const int *R = reinterpret_cast<const int *>(mbase + M_R);
        int row = R[slot];
        // (r5) a team may sum a second row after its first (row pairs: the
        // record's [3R, 4R), -1 none; its entries start at the batch after the
        // first row's last)
        const int pw = R[3 * L::R + slot];
        int info = R[L::R + slot], vw = R[2 * L::R + slot];
        for (; row >= 0;) {
            // the row runs nbat whole batches of 8, then rem (0, 2, 4 or 6)
            // entries of one more (its length rounded up to even)
            const int js = info & 0xFFFF, len = info >> 16, nbat = len >> 3, rem = len & 7;
            const int blast = nbat + (rem ? 1 : 0) - 1;
            const u2 *Lq = reinterpret_cast<const u2 *>(mbase + M_L) + js + qk;
            // (the LIVE flag bits sit above bit 16: a snapshot plan's word is the base itself)
            const d2 *Vq = reinterpret_cast<const d2 *>(mbase + M_V) + (LIVE ? (vw & 0xFFFF) : vw) + qk;
            if constexpr (LIVE)
                if (vw & (1 << 30)) {
                    // a row of odd length: its last pair's second half is the
                    // CSR value after the row (another row's, or 0 past the
                    // block); -0.0 there before the sums read it (in order:
                    // one wave's LDS operations execute in program order)
                    const unsigned a = (unsigned)(uintptr_t)(Vq + 4 * ((len >> 1) - 1)) + 8u;
                    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(-0.0) : "memory");
                }
            const char *xb0 = xbase + par * 128 + tl * 16;
            const char *xb1 = xbase + (par ^ 1) * 128 + tl * 16;
            d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
            // per batch of 8 entries: 8 offsets in one b128 read, 8 values in
            // four; X is read in halves of 4 entries, ping-pong: the reads of
            // the next half go out before the current half is summed, so each
            // half's LDS latency hides behind the other half's FP64 work
            // two entries' X reads from a word of four u8 image rows: one
            // v_perm_b32 spreads rows h, h+1 into the high bytes of two u16
            // halves (row * 256 = the byte offset), the address adds take
            // them as words (SDWA), as they did for u16 offsets
            const unsigned xo0 = (unsigned)(xb0 - lds), xo1 = (unsigned)(xb1 - lds);
            // (stored before the barrier, while the loaders wait for their
            // DMAs: stores deferred into the next unit, among the loaders'
            // DMA issue, measured 25.6 -> 28.1 us)
            auto store = [&](int r, d2 s0, d2 s1) {
                double *y = Y + (int64_t)r * ldy + p * TILE_KP + 2 * tl;
                if constexpr (NARROW) {
                    if (2 * tl < kwin)  // columns 2 tl, 2 tl + 1 of the window (from either image half)
                        __builtin_nontemporal_store(s0, reinterpret_cast<d2 *>(y));
                } else {
                    __builtin_nontemporal_store(s0, reinterpret_cast<d2 *>(y + 16 * par));
                    __builtin_nontemporal_store(s1, reinterpret_cast<d2 *>(y + 16 * (par ^ 1)));
                }
            };
            auto rdx = [&](unsigned w, unsigned sel, d2 &a0, d2 &a1, d2 &b0, d2 &b1) {
                const unsigned pw = __builtin_amdgcn_perm(0u, w, sel);
                unsigned r0, r1, r2, r3;
                asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                    : "=v"(r0) : "v"(xo0), "v"(pw));
                asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                    : "=v"(r1) : "v"(xo0), "v"(pw));
                asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                    : "=v"(r2) : "v"(xo1), "v"(pw));
                asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                    : "=v"(r3) : "v"(xo1), "v"(pw));
                a0 = *reinterpret_cast<const d2 *>(lds + r0);
                b0 = *reinterpret_cast<const d2 *>(lds + r1);
                if constexpr (!NARROW) {
                    a1 = *reinterpret_cast<const d2 *>(lds + r2);
                    b1 = *reinterpret_cast<const d2 *>(lds + r3);
                }
            };
            constexpr unsigned LO = 0x010c000cu, HI = 0x030c020cu;  // rows 0, 1 / rows 2, 3 of the word
            // offsets two batches ahead: ln (batch b), lnn (b + 1, read during
            // batch b - 1), ln2 (b + 2, read in batch b after its second-half X
            // reads) -- so the X reads of batch b + 1 wait only for an offsets
            // read a whole batch old, and the reads behind it stay in flight
            // (a counted lgkmcnt, no drain)
            u2 ln = Lq[0];
            u2 lnn = Lq[4 * min(1, max(blast, 0))];
            d2 vn[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) vn[q] = Vq[4 * q];
            d2 xa0[4], xa1[4], xc0[4], xc1[4];
            rdx(ln.x, LO, xa0[0], xa1[0], xa0[1], xa1[1]);
            rdx(ln.x, HI, xa0[2], xa1[2], xa0[3], xa1[3]);
            for (int b = 0; b < nbat; ++b) {
                const int bn = min(b + 1, blast);
                rdx(ln.y, LO, xc0[0], xc1[0], xc0[1], xc1[1]);  // second half of batch b
                rdx(ln.y, HI, xc0[2], xc1[2], xc0[3], xc1[3]);
                __builtin_amdgcn_sched_barrier(0);
                // offsets of batch b + 2 (the last batch re-reads itself)
                const u2 ln2 = *(const volatile __attribute__((address_space(3))) u2 *)(Lq + 4 * min(b + 2, blast));
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    acc0 = madd(acc0, (k & 1) ? vn[k >> 1].y : vn[k >> 1].x, xa0[k]);
                    if constexpr (!NARROW) acc1 = madd(acc1, (k & 1) ? vn[k >> 1].y : vn[k >> 1].x, xa1[k]);
                }
                __builtin_amdgcn_sched_barrier(0);
                // each value pair is re-read in place once its FP64 has issued
                // (no register copies of the batch's values)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    vn[q] = *(const volatile __attribute__((address_space(3))) d2 *)(Vq + 4 * (4 * bn + q));
                rdx(lnn.x, LO, xa0[0], xa1[0], xa0[1], xa1[1]);  // first half of batch b + 1
                rdx(lnn.x, HI, xa0[2], xa1[2], xa0[3], xa1[3]);
                __builtin_amdgcn_sched_barrier(0);  // keep them ahead of the second half's FP64
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    acc0 = madd(acc0, (k & 1) ? vn[2 + (k >> 1)].y : vn[2 + (k >> 1)].x, xc0[k]);
                    if constexpr (!NARROW) acc1 = madd(acc1, (k & 1) ? vn[2 + (k >> 1)].y : vn[2 + (k >> 1)].x, xc1[k]);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 2; q < 4; ++q)
                    vn[q] = *(const volatile __attribute__((address_space(3))) d2 *)(Vq + 4 * (4 * bn + q));
                ln = lnn;
                lnn = ln2;
            }
            // xa / vn / ln hold the first half of batch blast: its first rem
            // entries end the row (a wave runs a step if any of its teams needs it)
            if (rem >= 2) {
                acc0 = madd(acc0, vn[0].x, xa0[0]);
                if constexpr (!NARROW) acc1 = madd(acc1, vn[0].x, xa1[0]);
                acc0 = madd(acc0, vn[0].y, xa0[1]);
                if constexpr (!NARROW) acc1 = madd(acc1, vn[0].y, xa1[1]);
                if (rem >= 4) {
                    acc0 = madd(acc0, vn[1].x, xa0[2]);
                    if constexpr (!NARROW) acc1 = madd(acc1, vn[1].x, xa1[2]);
                    acc0 = madd(acc0, vn[1].y, xa0[3]);
                    if constexpr (!NARROW) acc1 = madd(acc1, vn[1].y, xa1[3]);
                    if (rem >= 6) {
                        rdx(ln.y, LO, xc0[0], xc1[0], xc0[1], xc1[1]);
                        acc0 = madd(acc0, vn[2].x, xc0[0]);
                        if constexpr (!NARROW) acc1 = madd(acc1, vn[2].x, xc1[0]);
                        acc0 = madd(acc0, vn[2].y, xc0[1]);
                        if constexpr (!NARROW) acc1 = madd(acc1, vn[2].y, xc1[1]);
                    }
                }
            }
            store(row, acc0, acc1);
            if (pw < 0 || row == (pw & 0xFFFFFF)) break;
            // the second row: from the batch after the first row's last (an
            // empty first row owns one batch); LIVE: its odd-length flag
            const int nb = max(1, (len + 7) >> 3);
            row = pw & 0xFFFFFF;
            info = (js + 4 * nb) | (((pw >> 24) & 63) << 16);
            vw = LIVE ? (((vw & 0xFFFF) + 16 * nb) | (pw & (1 << 30))) : vw + 16 * nb;
        }
        if (++p == npanel) p = 0, ++it;
        barrier_lds();  // X slot (u & 1) is free for unit u + 2, meta slot for tile it + 1
    }
}


// (r5) the second bound is HIP's minimum waves per EU: geometry 2
// runs two 512-lane blocks per CU = 4 waves per SIMD, so <= 128 VGPRs must
// be forced (a 1024-lane block forces it by its size; 768 lanes: 3 waves,
// 168 VGPRs allowed).  tests/test_host.py::test_ws_kernels_register_budget
// reads the code object's VGPR counts.
template <int CW, int LW, int PPW, int UCAP, int NCAP, bool FMA = false, bool SADDR = true, bool NARROW = false>
__global__ __launch_bounds__(64 * (CW + LW), CW == 4 ? 4 : 1) void k_rows_ws(WsXcd xr, int npanel, int chunked,
                                                     const int *__restrict__ grec,
                                                     const int *__restrict__ lrec,
                                                     const uint8_t *__restrict__ loff,
                                                     const double *__restrict__ tv,
                                                     const double *__restrict__ X, int64_t ldx,
                                                     double *__restrict__ Y, int64_t ldy)
{
    // (the XCD's tile range read here, from the kernel arguments: scalar loads)
    const int x = blockIdx.x & 7;
    ws_body<CW, LW, PPW, UCAP, NCAP, FMA, SADDR, NARROW, false>(xr.first[x], xr.first[x + 1], npanel, chunked, grec,
                                                               lrec, loff, tv, X, ldx, Y, ldy, nullptr, 0, 0u);
}
// (r5) live values: tv = the block's first CSR value, tv_bytes its bytes;
// vidx[t * vstride + slot] the CSR index of each value slot (WsPlan::live)
template <int CW, int LW, int PPW, int UCAP, int NCAP, bool FMA = false, bool NARROW = false>
__global__ __launch_bounds__(64 * (CW + LW), CW == 4 ? 4 : 1) void k_rows_ws_live(WsXcd xr, int npanel, int chunked,
                                                     const int *__restrict__ grec,
                                                     const int *__restrict__ lrec,
                                                     const uint8_t *__restrict__ loff,
                                                     const double *__restrict__ tv,
                                                     const double *__restrict__ X, int64_t ldx,
                                                     double *__restrict__ Y, int64_t ldy,
                                                     const int *__restrict__ vidx, int vstride, unsigned tv_bytes)
{
    const int x = blockIdx.x & 7;
    ws_body<CW, LW, PPW, UCAP, NCAP, FMA, true, NARROW, true>(xr.first[x], xr.first[x + 1], npanel, chunked, grec, lrec,
                                                             loff, tv, X, ldx, Y, ldy, vidx, vstride, tv_bytes);
}

// the product instances of k_rows_ws: geometry (smfv_plan.h WsGeom) x FMA x SADDR x NARROW
#define SMFV_WS_INST(G_) k_rows_ws<G_.cw, G_.lw, G_.ppw, G_.ucap, G_.ncap, FMA, SADDR, NARROW>
template <bool FMA, bool SADDR, bool NARROW> constexpr auto WS1 = SMFV_WS_INST(WS_GEOM1);
template <bool FMA, bool SADDR, bool NARROW> constexpr auto WS2 = SMFV_WS_INST(WS_GEOM2);
template <bool FMA, bool SADDR, bool NARROW> constexpr auto WS3 = SMFV_WS_INST(WS_GEOM3);
#undef SMFV_WS_INST
#define SMFV_WSL_INST(G_) k_rows_ws_live<G_.cw, G_.lw, G_.ppw, G_.ucap, G_.ncap, FMA, NARROW>
template <bool FMA, bool NARROW> constexpr auto WSL1 = SMFV_WSL_INST(WS_GEOM1);
template <bool FMA, bool NARROW> constexpr auto WSL2 = SMFV_WSL_INST(WS_GEOM2);
template <bool FMA, bool NARROW> constexpr auto WSL3 = SMFV_WSL_INST(WS_GEOM3);
#undef SMFV_WSL_INST
template <bool NARROW>
static auto pick_ws_n(int geom, bool fma, bool saddr)
{
    if (geom == 2)
        return fma ? (saddr ? WS2<true, true, NARROW> : WS2<true, false, NARROW>)
                   : (saddr ? WS2<false, true, NARROW> : WS2<false, false, NARROW>);
    if (geom == 3)
        return fma ? (saddr ? WS3<true, true, NARROW> : WS3<true, false, NARROW>)
                   : (saddr ? WS3<false, true, NARROW> : WS3<false, false, NARROW>);
    return fma ? (saddr ? WS1<true, true, NARROW> : WS1<true, false, NARROW>)
               : (saddr ? WS1<false, true, NARROW> : WS1<false, false, NARROW>);
}
// (r4) narrow: a K = 4 / 8 / 16 window (one accumulator per lane)
static auto pick_ws(int geom, bool fma, bool saddr, bool narrow = false)
{
    return narrow ? pick_ws_n<true>(geom, fma, saddr) : pick_ws_n<false>(geom, fma, saddr);
}
// (r5) the live-values kernel (value pairs DMA'd from the caller's CSR; scalar-base addressing always)
static auto pick_ws_live(int geom, bool fma, bool narrow)
{
    if (geom == 2)
        return fma ? (narrow ? WSL2<true, true> : WSL2<true, false>) : (narrow ? WSL2<false, true> : WSL2<false, false>);
    if (geom == 3)
        return fma ? (narrow ? WSL3<true, true> : WSL3<true, false>) : (narrow ? WSL3<false, true> : WSL3<false, false>);
    return fma ? (narrow ? WSL1<true, true> : WSL1<true, false>) : (narrow ? WSL1<false, true> : WSL1<false, false>);
}

// ---------------------------------------------------------------------------
// (r5) k_rows_wsn: the tiled row kernel for a NARROW column window of 4 or 8
// columns (a ColumnWise rank's K/p panel, SC/...ColumnWise.cpp:34-48) on the
// narrow-team plan (build_wsn_plan, smfv_plan.h WsnGeom).  One persistent
// 1024-lane block per CU, 8 loader + 8 compute waves, two-slot pipeline as
// k_rows_ws.  A team is KW/2 lanes (one double2 column pair each), so a
// compute wave sums TW = 128/KW rows at once and a tile holds 256 (KW = 4) /
// 128 (KW = 8) rows: 2-4 units per CU on cop20k where k_rows_ws's 64-row
// tiles make 8.  The X image holds only the window (32 / 64 B per union row,
// <= 1,023 / 639 rows, u16 image offsets).  Each row is summed in CSR order
// with a separate multiply and add (bit-identical to the reference); pads
// (zero image row, value -0.0) add +-0.
// ---------------------------------------------------------------------------
template <int KW> struct LayN {
    static constexpr WsnGeom G = wsn_geom(KW);
    static constexpr int TL = G.tl(), TW = G.tw(), R = G.rows(), XROW = G.xrow(), UCAP = G.ucap, NCAP = G.ncap;
    static constexpr int XSLOT = (UCAP + 1) * XROW;
    static constexpr int RP = 1024 / XROW;              // image rows per 1 KiB DMA piece
    static constexpr int XPIECES = (UCAP + 1) / RP;
    static constexpr int PPW = (XPIECES + WSN_LW - 1) / WSN_LW;
    static constexpr int M_V = 0, M_L = NCAP * 8, M_R = M_L + NCAP * 2;
    static constexpr int RECB = G.lwords() * 4;
    static constexpr int RECP = (RECB + 1023) / 1024;   // record DMA pieces
    static constexpr int MSLOT = (M_R + RECP * 1024 + 1023) / 1024 * 1024;
    static constexpr int SL_M = 2 * XSLOT;
    static constexpr int BYTES = SL_M + 2 * MSLOT;
    static_assert(BYTES <= 160 * 1024, "two X images and two meta slots fit the CU's 160 KiB");
    static_assert((UCAP + 1) % RP == 0 && XSLOT % 1024 == 0 && M_L % 1024 == 0 && M_R % 1024 == 0, "1 KiB pieces");
    static_assert(G.lwords() <= WSN_GWORDS, "record");
};

template <int KW, bool FMA>
__global__ __launch_bounds__(1024, 1) void k_rows_wsn(WsXcd xr, const int *__restrict__ grec,
                                                      const int *__restrict__ lrec,
                                                      const uint16_t *__restrict__ loff,
                                                      const double *__restrict__ tv,
                                                      const double *__restrict__ X, int64_t ldx,
                                                      double *__restrict__ Y, int64_t ldy)
{
    using namespace ws;
    using L = LayN<KW>;
    constexpr int TL = L::TL, TW = L::TW, R = L::R, XROW = L::XROW, UCAP = L::UCAP;
    __shared__ __attribute__((aligned(16))) char lds[L::BYTES];
    const int nb = gridDim.x >> 3, x = blockIdx.x & 7, jb = blockIdx.x >> 3;
    const int first = xr.first[x], end = xr.first[x + 1];
    const int t0 = first + jb;
    if (t0 >= end) return;  // block-uniform
    const int cnt = (end - 1 - t0) / nb + 1;
    const int tlast = t0 + (cnt - 1) * nb;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned lds0 = (unsigned)(uintptr_t)lds;
    if (wv >= 8) {
        // ---------------- loader waves ----------------
        __builtin_amdgcn_s_setprio(3);
        const int wl = wv - 8;
        if (wl == 0 && lane < 2 * (XROW / 16))  // the zero image row of both X slots
            reinterpret_cast<d2 *>(lds + (lane / (XROW / 16)) * L::XSLOT + UCAP * XROW)[lane % (XROW / 16)] =
                d2{0.0, 0.0};
        // (r5) a tile's record is read in two steps a unit apart: its header
        // (entry ranges, union size nu) two units ahead of its staging, its
        // union ids one unit ahead and only the first nu of them (a tile
        // stages ~420 of the 1,024 slots at K/p = 4), so no load waits on
        // another inside a unit; the first tile reads every slot (no extra
        // round trip before the pipeline fills)
        int uid[L::PPW];
        int noff, tn, nu, voff, tnv;       // the tile staged next
        int noff2, tn2, nu2, voff2, tnv2;  // the one after it
        const unsigned ldxb = (unsigned)(ldx * 8);
        auto fetch_ids = [&](int t, int n_u) {
            const int *Gr = grec + (int64_t)t * WSN_GWORDS;
#pragma unroll
            for (int i = 0; i < L::PPW; ++i) {
                const int piece = wl + WSN_LW * i;
                uid[i] = piece < L::XPIECES && L::RP * piece + lane / TL < n_u ? Gr[L::RP * piece + lane / TL] : 0;
            }
        };
        auto load_header = [&](int t, int &no, int &n, int &u, int &vo, int &nv) {
            const int *Gr = grec + (int64_t)t * WSN_GWORDS;
            no = Gr[WSN_G_NOFF + (lane & 15)];
            n = Gr[WSN_G_TN + (lane & 15)];
            u = Gr[WSN_G_NU + (lane & 15)];
            vo = Gr[WSN_G_VOFF + (lane & 15)];
            nv = Gr[WSN_G_TNV + (lane & 15)];
        };
        auto fetch_header = [&](int t) { load_header(t, noff2, tn2, nu2, voff2, tnv2); };
        auto advance = [&](int t) {  // the header after next becomes next; its ids and the next header go out
            noff = noff2, tn = tn2, nu = nu2, voff = voff2, tnv = tnv2;
            fetch_ids(t, nu);
            fetch_header(min(t + nb, tlast));
        };
        auto stage = [&](int t, int slot) {
#pragma unroll
            for (int i = 0; i < L::PPW; ++i) asm volatile("" ::"v"(uid[i]));
            asm volatile("" ::"v"(noff), "v"(tn), "v"(nu), "v"(voff), "v"(tnv));
            const unsigned xb = lds0 + slot * L::XSLOT;
#pragma unroll
            for (int i = 0; i < L::PPW; ++i) {
                const int piece = wl + WSN_LW * i;
                // a lane stages its 16 B of image row RP piece + lane / TL (never the zero row: nu <= UCAP)
                if (piece < L::XPIECES && L::RP * piece + lane / TL < nu)
                    dma16s<false>(X, (unsigned)uid[i] * ldxb + 16u * (unsigned)(lane % TL), xb + piece * 1024);
            }
            const unsigned mb = lds0 + L::SL_M + slot * L::MSLOT;
            const double *tvb = tv + __builtin_amdgcn_readfirstlane(voff);
            const uint16_t *lb = loff + __builtin_amdgcn_readfirstlane(noff);
            for (int k = wl; k * 128 < tnv; k += WSN_LW) dma16s<true>(tvb, 1024u * k + 16u * lane, mb + L::M_V + k * 1024);
            for (int k = wl; k * 512 < tn; k += WSN_LW) dma16s<true>(lb, 1024u * k + 16u * lane, mb + L::M_L + k * 1024);
#pragma unroll
            for (int k = 0; k < L::RECP; ++k)
                if (wl == WSN_LW - 1 - k && 16 * lane + 1024 * k < L::RECB)
                    dma16s<true>(lrec + (int64_t)t * L::G.lwords(), 1024u * k + 16u * lane, mb + L::M_R + k * 1024);
        };
        // the first tile in one round trip: its header and every id slot
        // together, the second tile's header beside them
        load_header(t0, noff, tn, nu, voff, tnv);
        fetch_ids(t0, L::UCAP + 1);
        fetch_header(min(t0 + nb, tlast));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stage(t0, 0);
        advance(min(t0 + nb, tlast));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        for (int u = 0; u < cnt; ++u) {
            if (u + 1 < cnt) {
                const int t = t0 + (u + 1) * nb;
                stage(t, (u + 1) & 1);
                advance(min(t + nb, tlast));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // unit u + 1 has landed
            barrier_lds();
        }
        return;
    }
    // ---------------- compute waves ----------------
    auto madd = [](d2 a, double v, d2 xx) -> d2 {
        if constexpr (FMA)
            return d2{__builtin_fma(v, xx.x, a.x), __builtin_fma(v, xx.y, a.y)};
        else
            return a + v * xx;
    };
    const int k = lane / TL, tli = lane % TL;
    barrier_lds();
    for (int u = 0; u < cnt; ++u) {
        const char *xbase = lds + (u & 1) * L::XSLOT + 16 * tli;
        const char *mbase = lds + L::SL_M + (u & 1) * L::MSLOT;
        const int *RR = reinterpret_cast<const int *>(mbase + L::M_R);
        const int word = RR[wv * TW + k];
        if (word != -1) {
            const int row = word & 0xFFFFFF, nbat = (int)((unsigned)word >> 24);
            // (r5) batches of WSN_B = 4 entries: 4 u16 image rows in one 8-byte
            // read, two value pairs; X of batch b + 1 is read before batch b
            // is summed.  Batches hold only the teams still running (a prefix
            // of the wave, smfv_plan.h): their count n_b is the lanes of
            // more than b batches, over TL -- a ballot among the lanes in
            // the loop, wave-uniform (scalar)
            const u2 *Lq = reinterpret_cast<const u2 *>(mbase + L::M_L) + RR[R + 2 * wv] + k;
            const d2 *Vq = reinterpret_cast<const d2 *>(mbase + L::M_V) + RR[R + 2 * wv + 1] + k;
            auto nact = [&](int b) { return (int)__builtin_popcountll(__builtin_amdgcn_ballot_w64(nbat > b)) / TL; };
            d2 acc = {0.0, 0.0};
            auto rdx = [&](u2 w, d2 (&x)[4]) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const unsigned w32 = e < 2 ? w.x : w.y;
                    const unsigned off = (e & 1) ? (w32 >> 16) : (w32 & 0xFFFFu);
                    x[e] = *reinterpret_cast<const d2 *>(xbase + off * XROW);
                }
            };
            d2 xa[4], xb[4];
            int n0 = nact(0), n1 = nact(1);  // teams in batches b, b + 1; Lq / Vq at batch b
            rdx(Lq[0], xa);
            u2 on = Lq[nbat > 1 ? n0 : 0];  // (a re-read of batch b when there is no next)
            for (int b = 0; b < nbat; b += 2) {
                // batch b in xa; batch b + 1's reads go out first
                d2 v0 = Vq[0], v1 = Vq[n0];
                rdx(on, xb);
                const int n2 = nact(b + 2);
                on = Lq[nbat > b + 2 ? n0 + n1 : 0];
                acc = madd(acc, v0.x, xa[0]);
                acc = madd(acc, v0.y, xa[1]);
                acc = madd(acc, v1.x, xa[2]);
                acc = madd(acc, v1.y, xa[3]);
                if (b + 1 < nbat) {
                    v0 = Vq[2 * n0], v1 = Vq[2 * n0 + n1];
                    rdx(on, xa);
                    const int n3 = nact(b + 3);
                    on = Lq[nbat > b + 3 ? n0 + n1 + n2 : n0];
                    acc = madd(acc, v0.x, xb[0]);
                    acc = madd(acc, v0.y, xb[1]);
                    acc = madd(acc, v1.x, xb[2]);
                    acc = madd(acc, v1.y, xb[3]);
                    Lq += n0 + n1;
                    Vq += 2 * (n0 + n1);
                    n0 = n2;
                    n1 = n3;
                }
            }
            __builtin_nontemporal_store(acc, reinterpret_cast<d2 *>(Y + (int64_t)row * ldy + 2 * tli));
        }
        barrier_lds();  // X slot (u & 1) and meta slot (u & 1) are free for unit u + 2
    }
}

// Rows the ws plan could not tile (over a cap alone): one 8-lane team per
// row, X gathered straight from HBM, CSR order (bit-identical).  `rows` are
// block-local (Y row), row_begin + row indexes the CSR; the values come from
// the plan's bound snapshot (tv + doff[team], CSR order), like the tiles'.
__global__ __launch_bounds__(256) void k_rows_list(int nrows, int kwin, const int *__restrict__ rows,
                                                   const int64_t *__restrict__ doff, int row_begin,
                                                   const int *__restrict__ rp, const int *__restrict__ ci,
                                                   const double *__restrict__ tv,
                                                   const double *__restrict__ X, int64_t ldx,
                                                   double *__restrict__ Y, int64_t ldy)
{
    const int team = blockIdx.x * 32 + (threadIdx.x >> 3);
    if (team >= nrows) return;
    const int tl = threadIdx.x & 7, par = (threadIdx.x >> 3) & 1;
    const int cp = blockIdx.y * TILE_KP;
    const int row = rows[team];
    const int j0 = rp[row_begin + row];
    const double *vrow = tv + doff[team] - j0;
    double2 acc0 = make_double2(0.0, 0.0), acc1 = make_double2(0.0, 0.0);
    if (kwin) {  // (r4) a narrow window (K = 4, 8, 16): columns 2 tl, 2 tl + 1 only
        if (2 * tl >= kwin) return;
        for (int jj = j0; jj < rp[row_begin + row + 1]; ++jj)
            acc0 = VecT<2>::madd(acc0, vrow[jj], *reinterpret_cast<const double2 *>(X + (int64_t)ci[jj] * ldx + 2 * tl));
        *reinterpret_cast<double2 *>(Y + (int64_t)row * ldy + 2 * tl) = acc0;
        return;
    }
    for (int jj = j0; jj < rp[row_begin + row + 1]; ++jj) {
        const double *px = X + (int64_t)ci[jj] * ldx + cp + 2 * tl;
        const double v = vrow[jj];
        acc0 = VecT<2>::madd(acc0, v, *reinterpret_cast<const double2 *>(px + 16 * par));
        acc1 = VecT<2>::madd(acc1, v, *reinterpret_cast<const double2 *>(px + 16 * (par ^ 1)));
    }
    double *y = Y + (int64_t)row * ldy + cp + 2 * tl;
    *reinterpret_cast<double2 *>(y + 16 * par) = acc0;
    *reinterpret_cast<double2 *>(y + 16 * (par ^ 1)) = acc1;
}

// ---------------------------------------------------------------------------
// k_rows_mfma: opt-in (SMFV_PLAN_MFMA) dense-block MFMA form of the tiled
// row kernel, the "MFMA K-panel" of BASELINE config 3, kept as a measured
// alternative.  One 256-lane workgroup per tile (build_mfma_plan): per
// 32-column panel the tile's union X rows are staged into LDS; wave g owns
// rows 16g..16g+15 and, for each non-zero 16 x 4 block of A (dense, A-operand
// lane order, zeros as pads), runs two v_mfma_f64_16x16x4f64 (columns 0-15 and
// 16-31 of the panel) with B read from the LDS image.  Sums are reassociated
// by the MFMA (4 terms at a time, union order): within tolerance, not
// bit-identical.  C/D lane map of the f64 MFMA: col = lane & 15,
// row = (lane >> 4) + 4 * reg (MI355X guide).
// ---------------------------------------------------------------------------
typedef double mf_d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_rows_mfma(int npanel, const int *__restrict__ rec,
                                                   const int *__restrict__ ucols, const int *__restrict__ bstep,
                                                   const double *__restrict__ av, const double *__restrict__ X,
                                                   int64_t ldx, double *__restrict__ Y, int64_t ldy)
{
    constexpr int UR = ((WS_UCAP + 3) / 4) * 4;  // image rows, padded to whole k-steps
    __shared__ double xs[UR * TILE_KP];           // 60 KiB: union rows x 32 doubles
    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
    const int *R = rec + (int64_t)t * MF_RWORDS;
    const int *U = ucols + (int64_t)t * WS_UCAP;
    const int nu = R[64 + 2 * MF_GROUPS];
    const int b0 = R[64 + 2 * g], nb = R[64 + 2 * g + 1];
    for (int p = 0; p < npanel; ++p) {
        const int cp = p * TILE_KP;
        if (p) __syncthreads();  // the previous panel's image is consumed
        for (int q = tid; q < UR * 16; q += 256) {  // 16 B pieces: row q >> 4, columns 2 (q & 15)
            const int u = q >> 4, c = 2 * (q & 15);
            double2 v = make_double2(0.0, 0.0);
            if (u < nu) v = *reinterpret_cast<const double2 *>(X + (int64_t)U[u] * ldx + cp + c);
            *reinterpret_cast<double2 *>(xs + u * TILE_KP + c) = v;
        }
        __syncthreads();
        mf_d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
        for (int b = 0; b < nb; ++b) {
            const double a = __builtin_nontemporal_load(av + (int64_t)(b0 + b) * 64 + lane);
            const int st = bstep[b0 + b];
            const double *xr = xs + (4 * st + (lane >> 4)) * TILE_KP + (lane & 15);
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, xr[0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, xr[16], acc1, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = R[16 * g + (lane >> 4) + 4 * r];
            if (row >= 0) {
                double *y = Y + (int64_t)row * ldy + cp + (lane & 15);
                y[0] = acc0[r];
                y[16] = acc1[r];
            }
        }
    }
}

// HBM streaming probe (bench only): 16-byte vector copy, one 16-KiB chunk
// per 256-lane block (4 loads in flight per lane), non-temporal both ways
// (6.2 TB/s on the box, against 5.8 with plain loads): the "measured
// STREAM-copy peak" next to the 8 TB/s spec.
__global__ __launch_bounds__(256) void k_copy16(int64_t n16, const ws::d2 *__restrict__ src,
                                                ws::d2 *__restrict__ dst)
{
    const int64_t base = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    ws::d2 a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + 256 * k < n16) a[k] = __builtin_nontemporal_load(src + base + 256 * k);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + 256 * k < n16) __builtin_nontemporal_store(a[k], dst + base + 256 * k);
}

// (r6) Floor probes of the SpMM's HBM mix (bench only; VERDICT r5 #2a).
// The headline moves ~2 bytes read per byte written (CSR + X in, Y out),
// which the 1:1 size-matched copy does not.  k_mix16: each lane reads two
// 16-B pieces (non-temporal) and writes their sum -- the plain-load floor of
// a 2:1 stream.  k_mix_lds: the same bytes through k_rows_ws's pipeline
// shape -- one persistent 1024-lane block per CU, 8 loader waves stage unit
// u + 1 (`ru` bytes) into one of two 64 KiB LDS slots by non-temporal
// LDS-DMA while 8 writer waves store unit u's `wu` bytes from LDS
// (non-temporal), one barrier per unit: the floor of the staged design at a
// given unit size.
__global__ __launch_bounds__(256) void k_mix16(int64_t w16, const ws::d2 *__restrict__ src,
                                               ws::d2 *__restrict__ dst)
{
    const int64_t base = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    ws::d2 a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + 256 * k < w16) {
            a[k] = __builtin_nontemporal_load(src + 2 * (base + 256 * k));
            b[k] = __builtin_nontemporal_load(src + 2 * (base + 256 * k) + 1);
        }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + 256 * k < w16) __builtin_nontemporal_store(a[k] + b[k], dst + base + 256 * k);
}

__global__ __launch_bounds__(1024, 1) void k_mix_lds(int64_t rbytes, int64_t wbytes, int nunits, int ru, int wu,
                                                     const char *__restrict__ src, char *__restrict__ dst)
{
    using namespace ws;
    constexpr int SLOT = 65536;
    __shared__ __attribute__((aligned(16))) char lds[2 * SLOT];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nb = gridDim.x;
    const int cnt = (int)blockIdx.x < nunits ? (nunits - 1 - (int)blockIdx.x) / nb + 1 : 0;
    if (cnt == 0) return;  // block-uniform
    const unsigned lds0 = (unsigned)(uintptr_t)lds;
    if (wv >= 8) {
        __builtin_amdgcn_s_setprio(3);
        const int wl = wv - 8;
        auto stage = [&](int u, int slot) {
            const int64_t base = (int64_t)u * ru;
            const char *sb = src + base;
            for (int k = wl; k * 1024 < ru; k += 8)
                if (base + k * 1024 + 16 * lane < rbytes) dma16s<true>(sb, 1024u * k + 16u * lane, lds0 + slot * SLOT + k * 1024);
        };
        stage((int)blockIdx.x, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        for (int i = 0; i < cnt; ++i) {
            if (i + 1 < cnt) stage((int)blockIdx.x + (i + 1) * nb, (i + 1) & 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            barrier_lds();
        }
        return;
    }
    barrier_lds();
    for (int i = 0; i < cnt; ++i) {
        const int u = (int)blockIdx.x + i * nb;
        const char *sl = lds + (i & 1) * SLOT;
        const int64_t wb = (int64_t)u * wu;
        for (int k = tid; k * 16 < wu; k += 512)
            if (wb + 16 * k < wbytes)
                __builtin_nontemporal_store(*reinterpret_cast<const d2 *>(sl + (16 * k) % ru),
                                            reinterpret_cast<d2 *>(dst + wb + 16 * k));
        barrier_lds();
    }
}

// smfv_device_init: loads the code object, computes nothing
__global__ void k_noop() {}

// plan value binding: tile-ordered copy of A's values (pads -> pad)
__global__ __launch_bounds__(256) void k_gather_vals(int64_t count, const int *__restrict__ tsrc,
                                                     const double *__restrict__ va,
                                                     double *__restrict__ tvals, double pad)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) {
        const int s = tsrc[i];
        tvals[i] = s >= 0 ? va[s] : pad;
    }
}

// (r4) The bind from "items": an item is up to 4 consecutive non-zeros of
// one row (tiled plans: entries 4g .. 4g + 3 of a quad's row k) or of one
// chunk (K = 1 plans).  Item i = {CSR index of its first value, (first value
// pair << 4) | (stride 4 ? 8 : 0) | real entries}: its values are one
// contiguous CSR run and land in two value pairs, 4 pairs apart in a tile's
// quad interleave (stride 4) or adjacent in a chunk.  Items are in snapshot
// order, so a wave's loads are 32-byte runs of a few rows and its stores
// fill whole 64-byte groups of pairs; the pads were written once when the
// plan was created (k_fill_f64).  One item per lane.
__global__ __launch_bounds__(256) void k_bind_items(int64_t n, const int2 *__restrict__ it,
                                                    const double *__restrict__ va, double *__restrict__ tv)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int2 d = it[i];
    const int cnt = d.y & 7;
    const int64_t p0 = (int64_t)((unsigned)d.y >> 4), p1 = p0 + ((d.y & 8) ? 4 : 1);
    const double *v = va + d.x;
    ws::d2 *o = reinterpret_cast<ws::d2 *>(tv);
    if (cnt == 4) {
        // two 16-byte loads (8-byte aligned: the global unaligned mode takes
        // them) instead of four 8-byte ones: half the load instructions
        ws::d2 lo, hi;
        __builtin_memcpy(&lo, v, 16);
        __builtin_memcpy(&hi, v + 2, 16);
        o[p0] = lo;
        o[p1] = hi;
        return;
    }
    const double a0 = v[0], a1 = cnt > 1 ? v[1] : 0.0, a2 = cnt > 2 ? v[2] : 0.0;
    if (cnt > 1) o[p0] = ws::d2{a0, a1};
    else reinterpret_cast<double *>(o + p0)[0] = a0;
    if (cnt > 2) reinterpret_cast<double *>(o + p1)[0] = a2;
}
// (r4) The cut rows of a NONZERO range (at most its first and last row):
// row i's partial sum over its entries [s[i], e[i]), one block per row.
// With K <= 256 the block's lanes are G = 256 / K groups of K columns; group g
// sums entries s + g, s + g + G, ... and the G partials are added in group
// order (deterministic; within the NonZeroElement tolerance, like the merge
// path it replaces for these rows).  K > 256: one group, columns looped.
struct CutRows {
    int n, row[2];
    int64_t s[2], e[2];
    int64_t yoff[2];  // the row's offset in Y (doubles)
};
__global__ __launch_bounds__(256) void k_cut_rows(CutRows cr, const int *__restrict__ ci, const double *__restrict__ va,
                                                  const double *__restrict__ X, int64_t ldx, int K,
                                                  double *__restrict__ Y)
{
    __shared__ double part[256];
    const int i = blockIdx.x, t = threadIdx.x;
    const int64_t s = cr.s[i], e = cr.e[i];
    double *y = Y + cr.yoff[i];
    if (K > 256) {
        for (int c = t; c < K; c += 256) {
            double acc = 0.0;
            for (int64_t j = s; j < e; ++j) acc = acc + va[j] * X[(int64_t)ci[j] * ldx + c];
            y[c] = acc;
        }
        return;
    }
    const int G = 256 / K, g = t / K, c = t % K;
    double acc = 0.0;
    if (g < G)
        for (int64_t j = s + g; j < e; j += G) acc = acc + va[j] * X[(int64_t)ci[j] * ldx + c];
    part[t] = acc;
    __syncthreads();
    if (t < K) {
        double sum = 0.0;
        for (int q = 0; q < G; ++q) sum = sum + part[q * K + t];
        y[t] = sum;
    }
}

__global__ __launch_bounds__(256) void k_fill_f64(int64_t n, double v, double *__restrict__ out)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = v;
}

// ---------------------------------------------------------------------------
// k_merge: nnz-balanced merge-path over the rows [row_first, row_first +
// nrows) restricted to nnz [s, e).  The merge list is {row ends} x {nnz};
// team t walks diagonals [t*ipt, (t+1)*ipt).  Rows whose end falls in the
// team's range are stored (possibly missing a prefix carried by earlier
// teams); the row still open at the range end is written to the team's
// carry slot, summed in team order by k_carry_fixup.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t merge_row_end(const int *rp, int row_first, int i, int64_t s,
                                                 int64_t e)
{
    int64_t v = rp[row_first + i + 1];
    return (v < e ? v : e) - s;
}

// number of rows i in [0, nrows) whose end event lies before diagonal d,
// i.e. end(i) + i < d (end(i) + i is strictly increasing in i)
__device__ __forceinline__ int merge_search(const int *rp, int row_first, int nrows, int64_t s,
                                            int64_t e, int64_t d)
{
    int lo = 0, hi = nrows;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (merge_row_end(rp, row_first, mid, s, e) + mid < d) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

template <int TEAM, int VEC>
__global__ __launch_bounds__(256) void k_merge(int row_first, int nrows, int64_t s, int64_t e,
                                               const int *__restrict__ rp,
                                               const int *__restrict__ ci,
                                               const double *__restrict__ va,
                                               const double *__restrict__ X, int64_t ldx, int K,
                                               double *__restrict__ Yc, int64_t ldy, int64_t ipt,
                                               int64_t nteams, int *__restrict__ carry_row,
                                               double *__restrict__ carry_val)
{
    using V = VecT<VEC>;
    constexpr int TPB = 256 / TEAM;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t t = (int64_t)blk * TPB + (threadIdx.x / TEAM);
    if (t >= nteams) return;
    const int tl = threadIdx.x & (TEAM - 1);
    const int64_t total = (int64_t)nrows + (e - s);
    const int64_t d0 = t * ipt;
    const int64_t d1 = d0 + ipt < total ? d0 + ipt : total;
    const int i0 = merge_search(rp, row_first, nrows, s, e, d0);
    const int i1 = merge_search(rp, row_first, nrows, s, e, d1);
    const int64_t j0 = d0 - i0, j1 = d1 - i1;  // relative nnz positions
    bool carried = false;
    const int npass = (K + TEAM * VEC - 1) / (TEAM * VEC);
    for (int p = 0; p < npass; ++p) {
        const int c = p * TEAM * VEC + tl * VEC;
        const bool cok = c < K;
        for (int i = i0; i <= i1 && i < nrows; ++i) {
            const int64_t rs0 = rp[row_first + i];
            const int64_t rs = (rs0 > s ? rs0 : s) - s;
            const int64_t js = rs > j0 ? rs : j0;
            const int64_t je = i < i1 ? merge_row_end(rp, row_first, i, s, e) : j1;
            if (i == i1 && je <= js) break;  // nothing open at the range end
            typename V::T acc = row_segment<TEAM, VEC>((int)(js + s), (int)(je + s), ci, va, X,
                                                       ldx, c, cok, V::zero());
            if (i < i1) {
                if (cok) V::store(Yc + (int64_t)i * ldy + c, acc);
            } else {
                carried = true;
                if (cok) V::store(carry_val + t * K + c, acc);
            }
        }
    }
    if (tl == 0) carry_row[t] = carried ? i1 : -1;
}

// k_merge_flat: k_merge for 16-byte columns and K % 32 == 0 with the team's
// non-zeros streamed flat, across row boundaries: 16 (col, val) pairs per
// coalesced load (one per lane, broadcast by shuffle), all 16 X-row gathers
// in flight, then summed in order; a row end met on the way stores the row
// (row ends of the next 16 rows are held one per lane).  Short rows (most of
// a power-law matrix) no longer cap the gathers in flight at their length.
// Same split, carries and per-row summation order as k_merge.
template <int TEAM>
__global__ __launch_bounds__(256) void k_merge_flat(int row_first, int nrows, int64_t s, int64_t e,
                                                    const int *__restrict__ rp, const int *__restrict__ ci,
                                                    const double *__restrict__ va,
                                                    const double *__restrict__ X, int64_t ldx, int K,
                                                    double *__restrict__ Yc, int64_t ldy, int64_t ipt,
                                                    int64_t nteams, int *__restrict__ carry_row,
                                                    double *__restrict__ carry_val)
{
    static_assert(TEAM == 16, "one 256-B X row per team gather (K panel of 32 doubles)");
    constexpr int TPB = 256 / TEAM, U = TEAM;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t t = (int64_t)blk * TPB + (threadIdx.x / TEAM);
    if (t >= nteams) return;
    const int lane = threadIdx.x & 63;
    const int tl = lane & (TEAM - 1), tbase = lane & ~(TEAM - 1);
    const int64_t total = (int64_t)nrows + (e - s);
    const int64_t d0 = t * ipt;
    const int64_t d1 = d0 + ipt < total ? d0 + ipt : total;
    const int i0 = merge_search(rp, row_first, nrows, s, e, d0);
    const int i1 = merge_search(rp, row_first, nrows, s, e, d1);
    const int64_t j0 = d0 - i0, j1 = d1 - i1;  // relative nnz positions
    // the row open at the range end is carried if this team holds >= 1 of its non-zeros
    bool carried = false;
    if (i1 < nrows) {
        const int64_t rs0 = rp[row_first + i1];
        const int64_t rs = (rs0 > s ? rs0 : s) - s;
        carried = j1 > (rs > j0 ? rs : j0);
    }
    for (int p = 0; p < K / 32; ++p) {
        const int c = p * 32 + 2 * tl;
        double2 acc = make_double2(0.0, 0.0);
        int i = i0;
        int wbase = i0;  // lane l holds the end of row wbase + l
        int64_t myend = wbase + tl < nrows ? merge_row_end(rp, row_first, wbase + tl, s, e) : INT64_MAX;
        auto row_end = [&](int r) -> int64_t {
            if (r - wbase >= TEAM) {  // team-uniform: slide the window
                wbase = r;
                myend = wbase + tl < nrows ? merge_row_end(rp, row_first, wbase + tl, s, e) : INT64_MAX;
            }
            return __shfl(myend, tbase + (r - wbase));
        };
        int64_t rend = i < i1 ? row_end(i) : INT64_MAX;
        auto flush_until = [&](int64_t j) {  // store every row (< i1) that ends at or before j
            while (i < i1 && rend <= j) {
                *reinterpret_cast<double2 *>(Yc + (int64_t)i * ldy + c) = acc;
                acc = make_double2(0.0, 0.0);
                ++i;
                rend = i < i1 ? row_end(i) : INT64_MAX;
            }
        };
        // (col, val) of the next chunk are loaded while this chunk's gathers fly
        int nc = 0;
        double nv = 0.0;
        if (j0 + tl < j1) {
            nc = ci[s + j0 + tl];
            nv = va[s + j0 + tl];
        }
        for (int64_t jb = j0; jb < j1; jb += U) {
            const int n = (int)(j1 - jb < U ? j1 - jb : U);
            const int myc = nc;
            const double myv = nv;
            double2 x[U];
            double vv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int cc = __shfl(myc, tbase + u);
                vv[u] = __shfl(myv, tbase + u);
                x[u] = make_double2(0.0, 0.0);
                if (u < n) x[u] = *reinterpret_cast<const double2 *>(X + (int64_t)cc * ldx + c);
            }
            if (jb + U + tl < j1) {
                nc = ci[s + jb + U + tl];
                nv = va[s + jb + U + tl];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u < n) {
                    flush_until(jb + u);
                    acc = VecT<2>::madd(acc, vv[u], x[u]);
                }
            }
        }
        flush_until(INT64_MAX - 1);  // rows ending at j1 (and empty rows before i1)
        if (carried) *reinterpret_cast<double2 *>(carry_val + t * K + c) = acc;
    }
    if (tl == 0) carry_row[t] = carried ? i1 : -1;
}

// one thread per (team, column): the first team of each run of equal carry
// rows sums the run in team order and adds it to the stored row.
__global__ __launch_bounds__(256) void k_carry_fixup(int64_t nteams, int K,
                                                     const int *__restrict__ carry_row,
                                                     const double *__restrict__ carry_val,
                                                     double *__restrict__ Yc, int64_t ldy)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t t = g / K;
    const int k = (int)(g - t * K);
    if (t >= nteams) return;
    const int r = carry_row[t];
    if (r < 0) return;
    if (t > 0 && carry_row[t - 1] == r) return;  // not the head of its run
    double sum = carry_val[t * K + k];
    for (int64_t u = t + 1; u < nteams && carry_row[u] == r; ++u) sum = sum + carry_val[u * K + k];
    double *y = Yc + (int64_t)r * ldy + k;
    *y = *y + sum;
}

// rank-major column panels -> row-major Y (SC/...ColumnWise.cpp:109-126)
__global__ __launch_bounds__(256) void k_panels_to_rowmajor(int m, int K, int p,
                                                            const double *__restrict__ panels,
                                                            double *__restrict__ Y, int64_t ldy)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (int64_t)m * K) return;
    const int64_t row = g / K;
    const int col = (int)(g - row * K);
    const int q = K / p;
    int r = q > 0 ? col / q : p - 1;
    if (r > p - 1) r = p - 1;
    const int c0 = r * q;
    const int kc = (r == p - 1) ? q + K % p : q;
    const int64_t off = (int64_t)m * c0;  // ranks before r hold q columns each
    Y[row * ldy + col] = panels[off + row * kc + (col - c0)];
}

struct BlockTable {
    int p;
    int rf[64];
    int rl[64];
    int64_t off[64];
};

// Y[row] = sum over ranks (in rank order) of their partial for row
__global__ __launch_bounds__(256) void k_combine_blocks(int m, int K, BlockTable tab,
                                                        const double *__restrict__ blocks,
                                                        double *__restrict__ Y, int64_t ldy)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (int64_t)m * K) return;
    const int row = (int)(g / K);
    const int k = (int)(g - (int64_t)row * K);
    double acc = 0.0;
    bool any = false;
    for (int r = 0; r < tab.p; ++r) {
        if (row >= tab.rf[r] && row <= tab.rl[r]) {
            const double v = blocks[tab.off[r] + (int64_t)(row - tab.rf[r]) * K + k];
            acc = any ? acc + v : v;
            any = true;
        }
    }
    Y[(int64_t)row * ldy + k] = acc;
}

// max |a-b| and max |a-b| / max(|b|, 1e-300) as order-preserving u64 bit
// patterns of non-negative doubles
__global__ __launch_bounds__(256) void k_compare(int m, int K, const double *__restrict__ A,
                                                 int64_t lda, const double *__restrict__ B,
                                                 int64_t ldb, unsigned long long *out)
{
    __shared__ double s_abs[256], s_rel[256];
    double mabs = 0.0, mrel = 0.0;
    const int64_t total = (int64_t)m * K;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = g / K;
        const int k = (int)(g - row * K);
        const double a = A[row * lda + k], b = B[row * ldb + k];
        double d = fabs(a - b);
        if (d != d) d = INFINITY;
        const double den = fabs(b) > 1e-300 ? fabs(b) : 1e-300;
        mabs = fmax(mabs, d);
        mrel = fmax(mrel, d / den);
    }
    s_abs[threadIdx.x] = mabs;
    s_rel[threadIdx.x] = mrel;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            s_abs[threadIdx.x] = fmax(s_abs[threadIdx.x], s_abs[threadIdx.x + w]);
            s_rel[threadIdx.x] = fmax(s_rel[threadIdx.x], s_rel[threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicMax(out, (unsigned long long)__double_as_longlong(s_abs[0]));
        atomicMax(out + 1, (unsigned long long)__double_as_longlong(s_rel[0]));
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill_x_hash(int64_t n, int K, uint64_t seed, double *X,
                                                     int64_t ldx)
{
    const int64_t total = n * K;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = g / K;
        const int k = (int)(g - i * K);
        X[i * ldx + k] = (double)(1 + splitmix64(seed ^ (uint64_t)g) % 100);
    }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
static bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

static int pick_vec(const double *X, int64_t ldx, const double *Y, int64_t ldy, int K)
{
    return (K % 2 == 0 && ldx % 2 == 0 && ldy % 2 == 0 && aligned16(X) && aligned16(Y)) ? 2 : 1;
}

static int pick_team(int K, int vec)
{
    int need = (K + vec - 1) / vec;
    int t = 1;
    while (t < need && t < 64) t <<= 1;
    return t;
}

#define SMFV_TEAM_SWITCH(team, vec, LAUNCH)                 \
    switch ((team) * 4 + (vec)) {                           \
    case 1 * 4 + 1: LAUNCH(1, 1); break;                    \
    case 1 * 4 + 2: LAUNCH(1, 2); break;                    \
    case 2 * 4 + 1: LAUNCH(2, 1); break;                    \
    case 2 * 4 + 2: LAUNCH(2, 2); break;                    \
    case 4 * 4 + 1: LAUNCH(4, 1); break;                    \
    case 4 * 4 + 2: LAUNCH(4, 2); break;                    \
    case 8 * 4 + 1: LAUNCH(8, 1); break;                    \
    case 8 * 4 + 2: LAUNCH(8, 2); break;                    \
    case 16 * 4 + 1: LAUNCH(16, 1); break;                  \
    case 16 * 4 + 2: LAUNCH(16, 2); break;                  \
    case 32 * 4 + 1: LAUNCH(32, 1); break;                  \
    case 32 * 4 + 2: LAUNCH(32, 2); break;                  \
    case 64 * 4 + 1: LAUNCH(64, 1); break;                  \
    case 64 * 4 + 2: LAUNCH(64, 2); break;                  \
    default: set_error("internal: team %d vec %d", (team), (vec)); return SMFV_ERR_INVALID; \
    }

// Row-kernel configuration (TEAM lanes per row, H column groups per lane,
// U gathers in flight per team) by K.
struct RowCfg {
    int team, h, u;
};

static RowCfg row_cfg_for(int K)
{
    const int pairs = K / 2;  // double2 columns
    if (pairs >= 64) return {16, 4, 4};
    if (pairs >= 16) return {8, 2, 8};
    if (pairs >= 8) return {8, 1, 8};
    if (pairs >= 4) return {4, 1, 8};
    if (pairs >= 2) return {2, 1, 8};
    return {1, 1, 8};
}

#define SMFV_MH_CONFIGS(X_) \
    X_(1, 1, 8) X_(2, 1, 8) X_(4, 1, 8) X_(8, 1, 8) X_(16, 1, 8) X_(16, 1, 16) X_(8, 2, 4)    \
    X_(8, 2, 8) X_(4, 4, 4) X_(4, 4, 2) X_(2, 8, 2) X_(16, 2, 4) X_(16, 4, 4) X_(32, 2, 4)   \
    X_(64, 1, 8) X_(8, 8, 2) X_(16, 4, 2) X_(32, 1, 8)

static int launch_rows_mh(int row_begin, int nrows, const int *rp, const int *ci, const double *va,
                          const double *X, int64_t ldx, int64_t xrows, int K, double *Y,
                          int64_t ldy, hipStream_t st)
{
    const RowCfg cfg = row_cfg_for(K);
    const int rpb = 256 / cfg.team;
    const int64_t nblk = ((int64_t)nrows + rpb - 1) / rpb;
    SMFV_REQUIRE(nblk <= 0x7fffffff, "too many rows for one launch");
    const int64_t xb = xrows * ldx * 8;
    const bool buf = xb > 0 && xb <= 0x7fffffffLL;
    const uint32_t xbytes = buf ? (uint32_t)xb : 0u;
#define L(T_, H_, U_)                                                                               \
    if (cfg.team == T_ && cfg.h == H_ && cfg.u == U_) {                                             \
        if (buf)                                                                                    \
            hipLaunchKernelGGL((k_rows_mh<T_, H_, U_, true>), dim3((unsigned)nblk), dim3(256), 0,   \
                               st, row_begin, nrows, rp, ci, va, X, ldx, xbytes, K, Y, ldy);        \
        else                                                                                        \
            hipLaunchKernelGGL((k_rows_mh<T_, H_, U_, false>), dim3((unsigned)nblk), dim3(256), 0,  \
                               st, row_begin, nrows, rp, ci, va, X, ldx, xbytes, K, Y, ldy);        \
        SMFV_LAUNCHED();                                                                            \
        return SMFV_OK;                                                                             \
    }
    SMFV_MH_CONFIGS(L)
#undef L
    set_error("row kernel configuration %d,%d,%d is not instantiated", cfg.team, cfg.h, cfg.u);
    return SMFV_ERR_INVALID;
}

static int launch_rows_simple(int row_begin, int nrows, const int *rp, const int *ci, const double *va,
                              const double *X, int64_t ldx, int K, double *Y, int64_t ldy, hipStream_t st);

static int launch_rows(int row_begin, int nrows, const int *rp, const int *ci, const double *va,
                       const double *X, int64_t ldx, int64_t xrows, int K, double *Y, int64_t ldy,
                       hipStream_t st)
{
    if (nrows <= 0 || K <= 0) return SMFV_OK;
    if (K == 1) {  // SpMV: coalesced CSR stream, products staged in LDS
        // 64 rows / 2,048-entry chunk per 256-lane block: one chunk per block
        // on cop20k (~1,390 non-zeros), 1,894 blocks.  Block-shape sweep on
        // the surrogate (cold us): 256 rows 19.5, 128 rows 12.6, 64 rows
        // 10.4-10.5, 32 rows 10.6-11.4, 512 lanes x 128 rows 10.4
        constexpr int NT = 256, RPB = 64, CH = 2048;
        const int64_t nblk = ((int64_t)nrows + RPB - 1) / RPB;
        SMFV_REQUIRE(nblk <= 0x7fffffff, "too many rows for one launch");
        hipLaunchKernelGGL((k_spmv_stream<NT, RPB, CH>), dim3((unsigned)nblk), dim3(NT), 0, st, row_begin, nrows,
                           rp, ci, va, X, ldx, Y, ldy);
        SMFV_LAUNCHED();
        return SMFV_OK;
    }
    const int vec = pick_vec(X, ldx, Y, ldy, K);
    if (vec == 2) return launch_rows_mh(row_begin, nrows, rp, ci, va, X, ldx, xrows, K, Y, ldy, st);
    return launch_rows_simple(row_begin, nrows, rp, ci, va, X, ldx, K, Y, ldy, st);
}

// odd K, unaligned X / Y, or a plan with SMFV_PLAN_SIMPLE_ROWS: one double
// per lane, the team's (col, val) pairs broadcast by shuffle (k_rows)
static int launch_rows_simple(int row_begin, int nrows, const int *rp, const int *ci, const double *va,
                              const double *X, int64_t ldx, int K, double *Y, int64_t ldy, hipStream_t st)
{
    if (nrows <= 0 || K <= 0) return SMFV_OK;
    const int team = pick_team(K, 1);
    const int rpb = 256 / team;
    const int64_t nblk = ((int64_t)nrows + rpb - 1) / rpb;
    SMFV_REQUIRE(nblk <= 0x7fffffff, "too many rows for one launch");
#define L(T_, V_) hipLaunchKernelGGL((k_rows<T_, V_>), dim3((unsigned)nblk), dim3(256), 0, st, \
                                     row_begin, nrows, rp, ci, va, X, ldx, K, Y, ldy)
    SMFV_TEAM_SWITCH(team, 1, L)
#undef L
    SMFV_LAUNCHED();
    return SMFV_OK;
}

MergeGeom merge_geom(int nrows, int64_t nnz, int K)
{
    MergeGeom g;
    g.items = (int64_t)nrows + nnz;
    // ~64 teams per CU on 256 CUs, at least 32 items per team
    const int64_t target = 256 * 64;  // (32-256 per CU measured equal on config 4)
    g.ipt = (g.items + target - 1) / target;
    if (g.ipt < 32) g.ipt = 32;
    (void)K;
    g.nteams = g.items > 0 ? (g.items + g.ipt - 1) / g.ipt : 0;
    return g;
}

size_t merge_workspace_bytes(int nrows, int64_t nnz, int K)
{
    const MergeGeom g = merge_geom(nrows, nnz, K);
    const size_t rows_b = ((size_t)g.nteams * sizeof(int) + 255) & ~(size_t)255;
    return rows_b + (size_t)g.nteams * (size_t)K * sizeof(double);
}

static int launch_merge(int row_first, int nrows, int64_t s, int64_t e, const int *rp,
                        const int *ci, const double *va, const double *X, int64_t ldx, int K,
                        double *Yc, int64_t ldy, void *ws, size_t ws_bytes, hipStream_t st)
{
    if (nrows <= 0 || K <= 0) return SMFV_OK;
    const MergeGeom g = merge_geom(nrows, e - s, K);
    const size_t need = merge_workspace_bytes(nrows, e - s, K);
    SMFV_REQUIRE(ws != nullptr || need == 0, "NONZERO variant needs %zu bytes of workspace", need);
    if (ws_bytes < need) {
        set_error("workspace too small: %zu < %zu bytes", ws_bytes, need);
        return SMFV_ERR_WORKSPACE;
    }
    SMFV_REQUIRE(aligned16(ws), "workspace must be 16-byte aligned");
    int *carry_row = static_cast<int *>(ws);
    const size_t rows_b = ((size_t)g.nteams * sizeof(int) + 255) & ~(size_t)255;
    double *carry_val = reinterpret_cast<double *>(static_cast<char *>(ws) + rows_b);
    const int vec = pick_vec(X, ldx, Yc, ldy, K);
    const int team = pick_team(K, vec);
    const int tpb = 256 / team;
    const int64_t nblk = (g.nteams + tpb - 1) / tpb;
    SMFV_REQUIRE(nblk <= 0x7fffffff, "too many merge teams for one launch");
    constexpr bool flat = true;
    if (flat && vec == 2 && K % 32 == 0) {
        const int64_t fblk_ = (g.nteams + 15) / 16;
        hipLaunchKernelGGL((k_merge_flat<16>), dim3((unsigned)fblk_), dim3(256), 0, st, row_first, nrows, s, e, rp,
                           ci, va, X, ldx, K, Yc, ldy, g.ipt, g.nteams, carry_row, carry_val);
    } else {
#define L(T_, V_) hipLaunchKernelGGL((k_merge<T_, V_>), dim3((unsigned)nblk), dim3(256), 0, st, \
                                     row_first, nrows, s, e, rp, ci, va, X, ldx, K, Yc, ldy,    \
                                     g.ipt, g.nteams, carry_row, carry_val)
        SMFV_TEAM_SWITCH(team, vec, L)
#undef L
    }
    SMFV_LAUNCHED();
    const int64_t nthr = g.nteams * (int64_t)K;
    const int64_t fblk = (nthr + 255) / 256;
    SMFV_REQUIRE(fblk <= 0x7fffffff, "too many carry slots for one launch");
    hipLaunchKernelGGL(k_carry_fixup, dim3((unsigned)fblk), dim3(256), 0, st, g.nteams, K,
                       carry_row, carry_val, Yc, ldy);
    SMFV_LAUNCHED();
    return SMFV_OK;
}

}  // namespace smfv

using namespace smfv;

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

SMFV_API const char *smfv_last_error(void) { return g_last_error.c_str(); }

SMFV_API const char *smfv_version(void) { return "smfv 0.1.0 gfx950"; }

SMFV_API int smfv_device_init(void *stream)
{
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, st);
    SMFV_LAUNCHED();
    // the runtime starts its host<->device copy path on the first transfer of
    // >= 1 MiB in the process (10-30 ms, whatever the memory; 4 KiB copies do
    // not start it: scripts/micro/h2d_reg_probe.cpp) -- one 1 MiB copy each
    // way here keeps that out of the first SpMM's H2D / D2H
    constexpr size_t warm = (size_t)1 << 20;
    std::vector<char> h(warm, 0);
    void *d = nullptr;
    SMFV_HIP(hipMalloc(&d, warm));
    hipError_t e = hipMemcpyAsync(d, h.data(), warm, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), d, warm, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(d);
    SMFV_HIP(e);
    SMFV_HIP(hipStreamSynchronize(st));
    return SMFV_OK;
}

SMFV_API void smfv_partition_rows(int m, int p, int r, int *start, int *end)
{
    const int q = m / p, extra = m % p;
    const int s = r * q + (r < extra ? r : extra);
    *start = s;
    *end = s + q + (r < extra ? 1 : 0);
}

SMFV_API void smfv_partition_cols(int K, int p, int r, int *start, int *end)
{
    const int q = K / p, extra = K % p;
    *start = r * q;
    *end = (r != p - 1) ? r * q + q : r * q + q + extra;
}

SMFV_API void smfv_partition_nnz(int64_t nnz, int p, int r, int64_t *start, int64_t *end)
{
    const int64_t q = nnz / p, extra = nnz % p;
    if (r < extra) {
        *start = (int64_t)r * (q + 1);
        *end = *start + q + 1;
    } else {
        *start = (int64_t)r * q + extra;
        *end = *start + q;
    }
}

SMFV_API int smfv_merge_geometry(int nrows, int64_t nnz, int K, int64_t out[3])
{
    SMFV_REQUIRE(out && nrows >= 0 && nnz >= 0 && K >= 0, "bad argument");
    const MergeGeom g = merge_geom(nrows, nnz, K);
    out[0] = g.items;
    out[1] = g.ipt;
    out[2] = g.nteams;
    return SMFV_OK;
}

SMFV_API int smfv_spmm_workspace_bytes(int variant, int m, int64_t nnz, int K, size_t *bytes)
{
    SMFV_REQUIRE(bytes != nullptr, "bytes is NULL");
    SMFV_REQUIRE(m >= 0 && nnz >= 0 && K >= 0, "negative size");
    SMFV_REQUIRE(variant >= SMFV_SEQUENTIAL && variant <= SMFV_NONZERO, "unknown variant %d", variant);
    *bytes = variant == SMFV_NONZERO ? merge_workspace_bytes(m, nnz, K) : 0;
    return SMFV_OK;
}

SMFV_API int smfv_spmm_csr_f64(int variant, int m, int n, int64_t nnz, const int *d_row_ptr,
                               const int *d_col_idx, const double *d_values, const double *d_X,
                               int64_t ldx, int K, double *d_Y, int64_t ldy, void *d_workspace,
                               size_t workspace_bytes, void *stream)
{
    SMFV_REQUIRE(variant >= SMFV_SEQUENTIAL && variant <= SMFV_NONZERO, "unknown variant %d", variant);
    SMFV_REQUIRE(m >= 0 && n >= 0 && nnz >= 0 && K >= 0, "negative size (m=%d n=%d nnz=%lld K=%d)",
                 m, n, (long long)nnz, K);
    SMFV_REQUIRE(nnz <= 0x7fffffff, "nnz %lld exceeds int32 row_ptr", (long long)nnz);
    SMFV_REQUIRE(ldx >= K && ldy >= K, "leading dimension smaller than K");
    if (m == 0 || K == 0) return SMFV_OK;
    SMFV_REQUIRE(d_row_ptr && d_Y, "null row_ptr / Y");
    SMFV_REQUIRE(nnz == 0 || (d_col_idx && d_values && d_X), "null col_idx / values / X");
    hipStream_t st = as_stream(stream);
    switch (variant) {
    case SMFV_SEQUENTIAL:
    case SMFV_ROWWISE:
        return launch_rows(0, m, d_row_ptr, d_col_idx, d_values, d_X, ldx, n, K, d_Y, ldy, st);
    case SMFV_COLUMNWISE:
        // The reference's ColumnWise splits the K columns into per-rank
        // panels (SC/...ColumnWise.cpp:25-48); each panel's entries are the
        // same per-row, CSR-ordered sums.  On one device every panel of a row
        // is computed by the row's team in ONE pass over its CSR segment
        // (the panels are the team's column groups / the tiled kernel's
        // 32-column units), so A is streamed once, not once per panel.
        // The per-rank panel of the distributed variant is
        // smfv_spmm_colpanel_f64 / a column-window plan (smfv_dist.cpp).
        return launch_rows(0, m, d_row_ptr, d_col_idx, d_values, d_X, ldx, n, K, d_Y, ldy, st);
    case SMFV_NONZERO:
        return launch_merge(0, m, 0, nnz, d_row_ptr, d_col_idx, d_values, d_X, ldx, K, d_Y, ldy,
                            d_workspace, workspace_bytes, st);
    }
    return SMFV_ERR_INVALID;
}

// ---- plans (analysed once per matrix pattern and K) ------------------------
}  // extern "C"

constexpr double SMFV_TILE_MIN_REUSE = 3.0;
// Tiles grown first (from the first rows, in the FULL pattern) to estimate
// re-use before the whole analysis is run; growing them in the full pattern
// makes the estimate independent of the row numbering (a sample of the first
// rows' own sub-pattern misjudges a permuted matrix).
constexpr int SMFV_TILE_SAMPLE_TILES = 128;  // (r3: 512 -> 128, 1/4 of the sample's time; 8k rows decide >= 3)
constexpr int SMFV_TILE_SAMPLE_MIN_ROWS = 16384;  // below this the full analysis runs directly
constexpr int SMFV_WS_BLOCKS_PER_XCD = 32;        // k_rows_ws blocks per XCD on MI355X (256 CUs), geometry 1
constexpr int SMFV_WS_DEFAULT_GEOM = 1;           // (r4) k_rows_ws geometry without SMFV_PLAN_WS_GEOM1 / GEOM2
constexpr int SMFV_WS_CHUNKED = 0;                // k_rows_ws tile order per block: 0 strided, 1 consecutive runs

// The tile caps a plan with these flags uses for the row block whose first
// row is global row col_base (its neighbour lookup), before the XCD parts.
static TileCaps plan_caps(int flags, int col_base)
{
    TileCaps caps;
    // (r4) the k_rows_ws geometry the tiles are cut for (WsGeom)
    const int g = (flags & SMFV_PLAN_WS_GEOM3)   ? 3
                  : (flags & SMFV_PLAN_WS_GEOM2) ? 2
                  : (flags & SMFV_PLAN_WS_GEOM1) ? 1
                                                 : SMFV_WS_DEFAULT_GEOM;
    caps.geom = ws_geom(g);
    caps.ucap = caps.geom.ucap;
    caps.ncap = caps.geom.ncap - 3 * caps.geom.rows();  // room for the quads' interleave padding
    caps.maxrows = caps.geom.rows();
    caps.xcd_blocks = caps.geom.xcd_blocks;
    caps.frontier = !(flags & SMFV_PLAN_NATURAL_SEEDS);
    caps.split_ends = (flags & SMFV_PLAN_SPLIT_ENDS) ? SMFV_WS_BLOCKS_PER_XCD : 0;
    caps.col_base = col_base;  // a row block's neighbours are its columns shifted by its first global row
    // (r5) row pairs: forced off / on, or the plan that runs fewer rounds
    caps.pairs = (flags & SMFV_PLAN_SINGLE_ROWS) ? 0 : (flags & SMFV_PLAN_ROW_PAIRS) ? 1 : 2;
    return caps;
}

// The XCD parts of a tiled plan (m rows; rp block-local, ci from the block's
// first non-zero): one part per XCD -- the row ranges or the breadth-first
// shares, whichever reads fewer X rows over the 8 L2s.  Run only once the
// plan is known to tile (the BFS and the footprints are O(nnz) passes with
// n-sized stamp arrays).
static void plan_parts(TileCaps &caps, int flags, int m, int n, const int *rp, const int *ci, double *footprint)
{
    *footprint = -1.0;
    if (!caps.frontier || m <= 0 || (flags & (SMFV_PLAN_ONE_WAVEFRONT | SMFV_PLAN_SPLIT_ENDS | SMFV_PLAN_MFMA)))
        return;
    std::vector<int> br, bs;
    range_parts(m, rp, 8, caps.part_rows, caps.part_start);
    double fr = 0.0;
    std::thread other([&] { fr = parts_footprint(m, n, rp, ci, caps.part_rows, caps.part_start); });
    bfs_parts(m, rp, ci, caps.col_base, 8, br, bs);
    const double fb = parts_footprint(m, n, rp, ci, br, bs);
    other.join();
    *footprint = std::min(fr, fb);
    if (fb < fr) {
        caps.part_rows.swap(br);
        caps.part_start.swap(bs);
    }
}

struct smfv_plan_s {
    int variant = 0, m = 0, n = 0, K = 0;
    int row_begin = 0;                     // first CSR row of the plan's row block
    int64_t nnz_base = 0, nnz_end = 0;     // the block's CSR range [row_ptr[row_begin], row_ptr[row_end])
    bool fma = false;  // SMFV_PLAN_FMA: fused multiply-add in the tiled kernel (not bit-identical)
    bool simple = false;  // SMFV_PLAN_SIMPLE_ROWS: untiled, one double per lane (k_rows<TEAM, 1>)
    int64_t nnz = 0;                       // non-zeros of the block
    bool tiled = false;
    int ntiles = 0, ndirect = 0;
    int64_t union_rows = 0, tiled_nnz = 0, padded_nnz = 0;
    int64_t snapshot = 0;                  // values gathered by bind (tile entries + slack + direct rows)
    double reuse = 0.0, est_reuse = -1.0, analysis_ms = 0.0;
    int ws_xcd[9] = {};            // XCD x runs tiles [ws_xcd[x], ws_xcd[x + 1])
    int ws_geom = 0;               // (r4) k_rows_ws geometry: WsGeom::id (1, 2, 3)
    int64_t paired = 0;            // (r5) rows summed as a team's second row
    int parts = 1;                 // 8: one part of the rows per XCD (build_ws_plan)
    double footprint = -1.0;       // parts_footprint of the 8 parts
    int *tsrc = nullptr;                   // snapshot entry -> CSR index of its value (-1: pad); NULL with descriptors
    int *bind_items = nullptr;             // (r4) 2 ints per bind item (k_bind_items)
    int64_t nbind_items = 0;
    bool bind_desc = false;                // bind by k_bind_items (pads filled at creation)
    bool wsn = false;                      // (r5) k_rows_wsn: narrow-team tiles for a 4 / 8-column window
    int *wsn_grec = nullptr, *wsn_lrec = nullptr;
    uint16_t *wsn_loff = nullptr;
    bool live = false;                     // (r5) k_rows_ws reads the live CSR values (ws_vidx): no snapshot
    int *ws_vidx = nullptr;                // live: per tile value slot, its first entry's block-local CSR index
    int ws_vstride = 0;
    double *tvals = nullptr;               // the bound values snapshot (tile order, pads -0.0, then direct rows)
    const double *bound_values = nullptr;  // d_values the snapshot came from
    int *ws_grec = nullptr, *ws_lrec = nullptr, *direct_rows = nullptr;
    int64_t *direct_off = nullptr;         // per direct row: its first value in tvals
    bool mfma = false;                     // SMFV_PLAN_MFMA: k_rows_mfma (dense blocks) instead of k_rows_ws
    int *mf_rec = nullptr, *mf_ucols = nullptr, *mf_bstep = nullptr;
    uint8_t *ws_loff = nullptr;
    bool k1 = false;                       // K = 1 chunk plan (k_spmv_chunks), ntiles = chunks
    int k1_cap = 0;                        // entry slots per chunk
    int *k1_hdr = nullptr;                 // 4 ints per chunk
    uint16_t *k1_rs = nullptr, *k1_off = nullptr;
    int *k1_col = nullptr;                 // wide layout: 32-bit columns (k1_off unused)
    bool k1_wide = false;
    int cs_xcd[9] = {};                    // XCD x runs tiles [cs_xcd[x], cs_xcd[x + 1])
    int *cs_bs = nullptr;                  // per block of the 8 x 32 grid: first chunk, chunks per panel
    int *cs_trow = nullptr, *cs_tlast = nullptr, *cs_crec = nullptr;
    uint8_t *cs_aux = nullptr;
    void *ws = nullptr;
    size_t ws_bytes = 0, dev_bytes = 0;
    hipEvent_t bind_ev = nullptr;          // recorded after the snapshot gather
    hipStream_t bind_stream = nullptr;
    // (r4) NONZERO over an nnz range that cuts rows (a rank's share): the
    // range's whole rows as a row-block plan (tiled / chunked), the cut first
    // and last rows on the merge path
    smfv_plan_s *sub = nullptr;
    int sub_row = 0;                       // the sub-plan's first row, block-local
    int ncut = 0, cut_row[2] = {0, 0};     // cut rows (global) and their nnz ranges
    int64_t cut_s[2] = {0, 0}, cut_e[2] = {0, 0};
    ~smfv_plan_s()
    {
        delete sub;
        for (void *q : {(void *)tsrc, (void *)bind_items, (void *)tvals, (void *)ws_vidx, (void *)wsn_grec, (void *)wsn_lrec,
                        (void *)wsn_loff, (void *)ws_grec, (void *)ws_lrec, (void *)direct_rows,
                        (void *)direct_off, (void *)ws_loff, ws, (void *)mf_rec, (void *)mf_ucols, (void *)mf_bstep,
                        (void *)k1_hdr, (void *)k1_rs, (void *)k1_off, (void *)k1_col, (void *)cs_bs,
                        (void *)cs_trow, (void *)cs_tlast, (void *)cs_crec, (void *)cs_aux})
            if (q) (void)hipFree(q);
        if (bind_ev) (void)hipEventDestroy(bind_ev);
    }
};

namespace {
template <class T> int upload(T **dst, const std::vector<T> &src, size_t &acc)
{
    const size_t b = std::max<size_t>(src.size(), 1) * sizeof(T);
    SMFV_HIP(hipMalloc(reinterpret_cast<void **>(dst), b));
    if (!src.empty()) SMFV_HIP(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    acc += b;
    return SMFV_OK;
}

}  // namespace

// (r4) The bind items (k_bind_items) from the snapshot's per-entry sources
// `ts` (CSR index or -1 for a pad): an item starts at every real entry whose
// CSR index begins a group of 4 (from its row start for a tiled plan, whose
// quads interleave rows; from its chunk start for a K = 1 plan, `group_base`
// gives the group origin of a CSR index), and the items are replayed on the
// host: they must write every real entry once, from its own source (else the
// plan keeps the per-entry gather, k_gather_vals).  The pads are written once.
template <class GroupBase, class Stride4>
static int setup_bind(smfv_plan_s *p, const std::vector<int> &ts, Stride4 stride4_at, GroupBase group_base, double pad)
{
    const int64_t n = (int64_t)ts.size();
    std::vector<int> items;
    bool ok = n / 2 < ((int64_t)1 << 27);
    for (int64_t e = 0; ok && e < n; ++e) {
        const int j = ts[(size_t)e];
        if (j < 0 || (j - group_base(j)) % 4 != 0) continue;
        ok = e % 2 == 0;  // a group starts a value pair
        const bool stride4 = stride4_at(e);
        // the group's real entries: consecutive sources at the layout's positions
        int cnt = 1;
        auto pos = [&](int h) { return 2 * (e / 2 + (h >= 2 ? (stride4 ? 4 : 1) : 0)) + (h & 1); };
        while (ok && cnt < 4 && pos(cnt) < n && ts[(size_t)pos(cnt)] == j + cnt && group_base(j + cnt) == group_base(j))
            ++cnt;
        items.push_back(j);
        items.push_back((int)(((e / 2) << 4) | (stride4 ? 8 : 0) | cnt));
    }
    // replay: every real entry written once, from its own source
    std::vector<int> chk((size_t)n, -1);
    for (size_t i = 0; ok && i < items.size(); i += 2) {
        const int j = items[i], d = items[i + 1], cnt = d & 7;
        const int64_t p0 = (unsigned)d >> 4, p1 = p0 + ((d & 8) ? 4 : 1);
        for (int h = 0; h < cnt && ok; ++h) {
            const int64_t e = 2 * (h < 2 ? p0 : p1) + (h & 1);
            ok = e < n && chk[(size_t)e] == -1;
            if (ok) chk[(size_t)e] = j + h;
        }
    }
    ok = ok && chk == ts;
    int rc = SMFV_OK;
    if (ok) {
        p->bind_desc = true;
        p->nbind_items = (int64_t)items.size() / 2;
        rc = upload(&p->bind_items, items, p->dev_bytes);
    } else {
        rc = upload(&p->tsrc, ts, p->dev_bytes);
    }
    if (!rc) {
        const size_t b = std::max<size_t>((size_t)n, 1) * sizeof(double);
        SMFV_HIP(hipMalloc(reinterpret_cast<void **>(&p->tvals), b));
        p->dev_bytes += b;
        if (ok && n > 0) {  // the pads, once, on a private stream (create is synchronous)
            hipStream_t fs = nullptr;
            SMFV_HIP(hipStreamCreateWithFlags(&fs, hipStreamNonBlocking));
            hipLaunchKernelGGL(k_fill_f64, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, fs,
                               n, pad, p->tvals);
            hipError_t e = hipGetLastError();
            if (e == hipSuccess) e = hipStreamSynchronize(fs);
            (void)hipStreamDestroy(fs);
            SMFV_HIP(e);
        }
    }
    return rc;
}

// Plan of rows [row_begin, row_begin + m) of a CSR matrix: h_rp / h_ci are the
// host arrays of the WHOLE matrix (or NULL: no tiling); the analysis runs on
// the block's own view (local row ids, its slice of col_idx), the snapshot
// indexes the whole matrix's values.  NONZERO plans cover the non-zeros
// [nnz_base, nnz_end) of the block's rows (a rank's nnz range).
int smfv::plan_create(smfv_plan_t *out, int variant, int row_begin, int m, int n, int64_t nnz_base, int64_t nnz_end,
                const int *h_rp, const int *h_ci, int K, int flags, int col_base)
{
    if (col_base < 0) col_base = row_begin;
    const auto t_start = std::chrono::steady_clock::now();
    auto *p = new smfv_plan_s;
    p->fma = (flags & SMFV_PLAN_FMA) != 0;
    p->simple = (flags & SMFV_PLAN_SIMPLE_ROWS) != 0 && variant != SMFV_NONZERO;
    if (p->simple) flags |= SMFV_PLAN_NO_TILES;
    p->variant = variant;
    p->row_begin = row_begin;
    p->m = m;
    p->n = n;
    p->K = K;
    p->nnz_base = nnz_base;
    p->nnz_end = nnz_end;
    p->nnz = nnz_end - nnz_base;
    int rc = SMFV_OK;
    auto fail_hip = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !rc) {
            set_error("%s: %s", what, hipGetErrorString(e));
            rc = SMFV_ERR_HIP;
        }
    };
    fail_hip(hipEventCreateWithFlags(&p->bind_ev, hipEventDisableTiming), "hipEventCreate");
    if (variant == SMFV_NONZERO) {
        // the merge-path workspace (the untiled path, and inputs the tiled
        // kernel cannot take: unaligned X / Y)
        p->ws_bytes = merge_workspace_bytes(m, p->nnz, K);
        if (p->ws_bytes) {
            fail_hip(hipMalloc(&p->ws, p->ws_bytes), "hipMalloc(workspace)");
            p->dev_bytes += p->ws_bytes;
        }
    }
    // NONZERO on whole rows (one device: the reference's NonZeroElement with
    // one rank sums every row in CSR order, SC/...NonZeroElement.cpp:56-67)
    // takes the tiled row kernel when the pattern has the re-use for it --
    // bit-identical to that; skewed or re-use-free patterns (config 4), nnz
    // ranges that cut rows (a rank's share) and SMFV_PLAN_NO_TILES keep the
    // nnz-balanced merge path
    const bool whole_rows = variant != SMFV_NONZERO ||
                            (h_rp && h_rp[row_begin] == nnz_base && h_rp[row_begin + m] == nnz_end);
    // (r4) K = 4 / 8 / 16 (a ColumnWise rank's panel): the same tiles, one
    // narrow column window (k_rows_ws stages and stores only its columns)
    const bool tile_k = K % TILE_KP == 0 || K == 4 || K == 8 || K == 16;
    if (!rc && whole_rows && h_rp && h_ci && m > 0 && p->nnz > 0 && K > 0 && tile_k &&
        !(flags & SMFV_PLAN_NO_TILES)) {  // (no non-zeros: nothing to stage)
        std::vector<int> rpl((size_t)m + 1);
        for (int i = 0; i <= m; ++i) rpl[i] = (int)(h_rp[row_begin + i] - nnz_base);
        const int *cil = h_ci + nnz_base;
        bool go = true;
        TileCaps caps = plan_caps(flags, col_base);
        // (r5) live values: the tiled kernel DMAs value pairs straight from the
        // CSR values through a buffer descriptor over the block's values
        caps.live = (flags & SMFV_PLAN_LIVE_VALUES) && !(flags & SMFV_PLAN_MFMA) && K != 1 &&
                    p->nnz * 8 < ((int64_t)1 << 32);
        if (!(flags & SMFV_PLAN_FORCE_TILES) && m > SMFV_TILE_SAMPLE_MIN_ROWS) {
            // estimate re-use on the first tiles (frontier-grown in the full
            // pattern, one part) before any O(nnz) pass of the full analysis
            TileCaps sc = caps;
            sc.max_tiles = SMFV_TILE_SAMPLE_TILES;
            TileAnalysis T;
            analyse_tiles(m, n, rpl.data(), cil, T, sc);
            p->est_reuse = T.union_rows ? (double)T.tiled_nnz / (double)T.union_rows : 0.0;
            go = p->est_reuse >= SMFV_TILE_MIN_REUSE;
        }
        if (go) plan_parts(caps, flags, m, n, rpl.data(), cil, &p->footprint);
        if (go && (flags & SMFV_PLAN_MFMA) && K % TILE_KP == 0) {
            MfmaPlan F;
            std::string err;
            if (!build_mfma_plan(m, n, rpl.data(), cil, F, &err, caps)) {
                set_error("%s", err.c_str());
                rc = SMFV_ERR_INVALID;
            } else {
                p->tiled = p->mfma = true;
                p->ntiles = F.ntiles;
                p->union_rows = F.union_rows;
                p->tiled_nnz = F.tiled_nnz;
                p->ndirect = (int)F.direct.size();
                p->reuse = F.union_rows ? (double)F.tiled_nnz / (double)F.union_rows : 0.0;
                std::vector<int> &ts = F.tsrc;
                for (int &q : ts)
                    if (q >= 0) q += (int)nnz_base;
                p->padded_nnz = (int64_t)ts.size();
                std::vector<int64_t> doff;
                for (int r : F.direct) {
                    doff.push_back((int64_t)ts.size());
                    for (int j = rpl[r]; j < rpl[r + 1]; ++j) ts.push_back((int)(nnz_base + j));
                }
                p->snapshot = (int64_t)ts.size();
                if (!rc) rc = upload(&p->mf_rec, F.rec, p->dev_bytes);
                if (!rc) rc = upload(&p->mf_ucols, F.ucols, p->dev_bytes);
                if (!rc) rc = upload(&p->mf_bstep, F.bstep, p->dev_bytes);
                if (!rc) rc = upload(&p->tsrc, ts, p->dev_bytes);
                if (!rc) rc = upload(&p->direct_rows, F.direct, p->dev_bytes);
                if (!rc) rc = upload(&p->direct_off, doff, p->dev_bytes);
                if (!rc) {
                    const size_t b = std::max<size_t>((size_t)p->snapshot, 1) * sizeof(double);
                    fail_hip(hipMalloc(reinterpret_cast<void **>(&p->tvals), b), "hipMalloc(tvals)");
                    p->dev_bytes += b;
                }
            }
        }
        // (r5) a 4- or 8-column window (a ColumnWise rank's panel): the
        // narrow-team tiles of k_rows_wsn, 2-4x the rows of a k_rows_ws tile
        // (SMFV_PLAN_WS keeps k_rows_ws's NARROW form, A/B)
        if (!rc && go && !p->mfma && !(flags & (SMFV_PLAN_MFMA | SMFV_PLAN_WS | SMFV_PLAN_LIVE_VALUES)) &&
            (K == 4 || K == 8)) {
            WsnPlan Wn;
            std::string err;
            TileCaps cn = caps;
            if (build_wsn_plan(m, n, rpl.data(), cil, K, Wn, &err, cn) && Wn.ntiles > 0 && Wn.union_rows > 0 &&
                ((double)Wn.tiled_nnz / (double)Wn.union_rows >= SMFV_TILE_MIN_REUSE ||
                 (flags & SMFV_PLAN_FORCE_TILES))) {
                p->tiled = p->wsn = true;
                p->ntiles = Wn.ntiles;
                for (int x = 0; x <= 8; ++x) p->ws_xcd[x] = Wn.xcd[x];
                p->parts = caps.part_start.size() > 2 ? (int)caps.part_start.size() - 1 : 1;
                p->union_rows = Wn.union_rows;
                p->tiled_nnz = Wn.tiled_nnz;
                p->padded_nnz = Wn.ventries;
                p->ndirect = (int)Wn.direct.size();
                p->reuse = (double)Wn.tiled_nnz / (double)Wn.union_rows;
                std::vector<int> &ts = Wn.tsrc;
                for (int &q : ts)
                    if (q >= 0) q += (int)nnz_base;
                std::vector<int64_t> doff;
                for (int r : Wn.direct) {
                    if (ts.size() % 2) ts.push_back(-1);
                    doff.push_back((int64_t)ts.size());
                    for (int j = rpl[r]; j < rpl[r + 1]; ++j) ts.push_back((int)(nnz_base + j));
                }
                p->snapshot = (int64_t)ts.size();
                if (!rc) rc = upload(&p->wsn_grec, Wn.grec, p->dev_bytes);
                if (!rc) rc = upload(&p->wsn_lrec, Wn.lrec, p->dev_bytes);
                if (!rc) rc = upload(&p->wsn_loff, Wn.loff, p->dev_bytes);
                if (!rc) rc = upload(&p->direct_rows, Wn.direct, p->dev_bytes);
                if (!rc) rc = upload(&p->direct_off, doff, p->dev_bytes);
                // (the per-entry gather binds it: a team's value pairs are TW
                // chunks apart, not the 4 / 1 the bind items know)
                if (!rc) rc = upload(&p->tsrc, ts, p->dev_bytes);
                if (!rc) {
                    const size_t b = std::max<size_t>((size_t)p->snapshot, 1) * sizeof(double);
                    fail_hip(hipMalloc(reinterpret_cast<void **>(&p->tvals), b), "hipMalloc(tvals)");
                    p->dev_bytes += b;
                }
            }
        }
        if (!rc && go && !p->mfma && !p->wsn && !(flags & SMFV_PLAN_MFMA)) {
            WsPlan W;
            std::string err;
            // a pattern the tile layout cannot take (the replayed plan fails its
            // checks) keeps the untiled plan rather than failing the create
            bool built = build_ws_plan(m, n, rpl.data(), cil, W, &err, caps);
            // (r4) a small plan (a rank's row block at p = 8: ~1 tile per CU
            // with 64-row tiles, one unit per block, all fill and drain) takes
            // geometry 2 unless the caller chose one: half-size tiles, two
            // blocks per CU (p = 8 on cop20k: 7.9 -> 7.1 us; at ~2 tiles per
            // CU, p = 4, geometry 1 stays ahead)
            if (built && W.ntiles > 0 &&
                !(flags & (SMFV_PLAN_WS_GEOM1 | SMFV_PLAN_WS_GEOM2 | SMFV_PLAN_WS_GEOM3))) {
                int dev = 0, ncu = 256;
                if (hipGetDevice(&dev) == hipSuccess) {
                    int v = 0;
                    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
                        ncu = v;
                }
                if (2 * W.ntiles < 3 * ncu) {
                    TileCaps c2 = plan_caps(flags | SMFV_PLAN_WS_GEOM2, col_base);
                    c2.live = caps.live;
                    c2.part_rows = caps.part_rows;
                    c2.part_start = caps.part_start;
                    WsPlan W2;
                    std::string err2;
                    // only where the smaller tiles keep the re-use and add no
                    // direct rows (rows over geometry 2's 125 X rows stay tiled in 1)
                    if (build_ws_plan(m, n, rpl.data(), cil, W2, &err2, c2) && W2.direct.size() == W.direct.size() &&
                        W2.union_rows > 0 && (double)W2.tiled_nnz / (double)W2.union_rows >= SMFV_TILE_MIN_REUSE)
                        W = std::move(W2);
                }
            }
            if (built) {
                p->ws_geom = W.geom.id;
                p->ntiles = W.ntiles;
                p->paired = W.paired;
                for (int x = 0; x <= 8; ++x) p->ws_xcd[x] = W.xcd[x];
                p->parts = caps.part_start.size() > 2 ? (int)caps.part_start.size() - 1 : 1;
                p->union_rows = W.union_rows;
                p->tiled_nnz = W.tiled_nnz;
                p->padded_nnz = W.ventries;
                p->ndirect = (int)W.direct.size();
                p->reuse = W.union_rows ? (double)W.tiled_nnz / (double)W.union_rows : 0.0;
                if ((p->reuse >= SMFV_TILE_MIN_REUSE || (flags & SMFV_PLAN_FORCE_TILES)) && W.live) {
                    // (r5) live values: no snapshot; direct rows read the CSR
                    // values too (their offset = their global CSR start)
                    p->tiled = p->live = true;
                    p->ws_vstride = W.vstride;
                    std::vector<int64_t> doff;
                    doff.reserve(W.direct.size());
                    for (int r : W.direct) doff.push_back(nnz_base + rpl[r]);
                    if (!rc) rc = upload(&p->ws_grec, W.grec, p->dev_bytes);
                    if (!rc) rc = upload(&p->ws_lrec, W.lrec, p->dev_bytes);
                    if (!rc) rc = upload(&p->ws_loff, W.loff, p->dev_bytes);
                    if (!rc) rc = upload(&p->ws_vidx, W.vidx, p->dev_bytes);
                    if (!rc) rc = upload(&p->direct_rows, W.direct, p->dev_bytes);
                    if (!rc) rc = upload(&p->direct_off, doff, p->dev_bytes);
                } else if (p->reuse >= SMFV_TILE_MIN_REUSE || (flags & SMFV_PLAN_FORCE_TILES)) {
                    p->tiled = true;
                    // snapshot sources: tile entries (+ DMA slack), then each direct row's values in CSR order
                    std::vector<int> &ts = W.tsrc;
                    for (int &s : ts)
                        if (s >= 0) s += (int)nnz_base;
                    std::vector<int64_t> doff;
                    doff.reserve(W.direct.size());
                    for (int r : W.direct) {
                        if (ts.size() % 2) ts.push_back(-1);  // (r4) each direct row starts a value pair (bind items)
                        doff.push_back((int64_t)ts.size());
                        for (int j = rpl[r]; j < rpl[r + 1]; ++j) ts.push_back((int)(nnz_base + j));
                    }
                    p->snapshot = (int64_t)ts.size();
                    if (!rc) rc = upload(&p->ws_grec, W.grec, p->dev_bytes);
                    if (!rc) rc = upload(&p->ws_lrec, W.lrec, p->dev_bytes);
                    if (!rc) rc = upload(&p->ws_loff, W.loff, p->dev_bytes);
                    if (!rc) rc = upload(&p->direct_rows, W.direct, p->dev_bytes);
                    if (!rc) rc = upload(&p->direct_off, doff, p->dev_bytes);
                    // bind items: groups of 4 from each row's start (global CSR index -> its row's start)
                    std::vector<int> rowstart;
                    rowstart.reserve((size_t)p->nnz);
                    for (int r = 0; r < m; ++r)
                        for (int j = rpl[r]; j < rpl[r + 1]; ++j) rowstart.push_back((int)nnz_base + rpl[r]);
                    const int64_t tiles_end = W.ventries;  // tile pairs interleave 4 rows; direct rows are contiguous
                    if (!rc)
                        rc = setup_bind(
                            p, ts, [&](int64_t e) { return e < tiles_end; },
                            [&](int j) { return rowstart[(size_t)(j - nnz_base)]; }, -0.0);
                }
            }
        }
    }
    // K = 1: the chunk plan (k_spmv_chunks) wherever the pattern fits its
    // layout (no row over a chunk, 16-bit column spans); otherwise the plan
    // stays untiled (k_spmv_stream on the live CSR)
    // ((r4) the same layout for 1 < K < 32 -- a ColumnWise rank's K/p window
    // -- with the products of 4 / 8 / 16 columns in LDS, k_panel_chunks, was
    // 1.0-7x slower than the untiled row kernel at K/p = 4 / 8 / 16 on cop20k
    // (profiles/r04/rank_plans) and was removed)
    if (!rc && whole_rows && h_rp && h_ci && m > 0 && K == 1 && !(flags & (SMFV_PLAN_NO_TILES | SMFV_PLAN_MFMA))) {
        std::vector<int> rpl((size_t)m + 1);
        for (int i = 0; i <= m; ++i) rpl[i] = (int)(h_rp[row_begin + i] - nnz_base);
        SpmvChunkPlan C;
        std::string err;
        if (build_spmv_chunks(m, n, rpl.data(), h_ci + nnz_base, spmv_chunk_cap(), K1_NT, C, &err)) {
            p->tiled = p->k1 = true;
            p->k1_cap = C.cap;
            p->k1_wide = C.wide;
            p->ntiles = C.nchunks;
            p->tiled_nnz = C.entries;
            p->padded_nnz = (int64_t)C.nchunks * C.cap;
            for (int &q : C.tsrc)
                if (q >= 0) q += (int)nnz_base;
            p->snapshot = (int64_t)C.tsrc.size();
            if (!rc) rc = upload(&p->k1_hdr, C.hdr, p->dev_bytes);
            if (!rc) rc = upload(&p->k1_rs, C.rs, p->dev_bytes);
            if (!rc) rc = C.wide ? upload(&p->k1_col, C.col, p->dev_bytes) : upload(&p->k1_off, C.off, p->dev_bytes);
            // bind items: groups of 4 from each chunk's start
            std::vector<int> chunkstart((size_t)p->nnz, 0);
            for (int c = 0; c < C.nchunks; ++c) {
                const int64_t cnt = C.hdr[(size_t)c * 4 + 3], s0 = C.tsrc[(size_t)c * C.cap];
                for (int64_t i = 0; i < cnt; ++i) chunkstart[(size_t)(s0 + i - nnz_base)] = (int)s0;
            }
            if (!rc)
                rc = setup_bind(
                    p, C.tsrc, [](int64_t) { return false; }, [&](int j) { return chunkstart[(size_t)(j - nnz_base)]; },
                    -0.0);
        }
    }
    // (r4) NONZERO over a range that cuts rows (SC/...NonZeroElement.cpp:24-67
    // at p > 1): its whole rows are summed in CSR order by the reference too,
    // so they run as a row-block plan (the tiled kernel / chunk panels,
    // bit-identical); only the cut rows' partial sums take the merge path
    if (!rc && variant == SMFV_NONZERO && !whole_rows && h_rp && h_ci && m > 0 && K > 0 &&
        !(flags & (SMFV_PLAN_NO_TILES | SMFV_PLAN_MFMA | SMFV_PLAN_SIMPLE_ROWS))) {
        const int f = row_begin, l = row_begin + m - 1;
        const int fi = h_rp[f] < nnz_base ? f + 1 : f, li = h_rp[l + 1] > nnz_end ? l - 1 : l;
        if (li >= fi) {
            smfv_plan_t sub = nullptr;
            if (plan_create(&sub, SMFV_ROWWISE, fi, li - fi + 1, n, h_rp[fi], h_rp[li + 1], h_rp, h_ci, K, flags, -1) ==
                    SMFV_OK &&
                sub->tiled) {
                p->sub = sub;
                p->sub_row = fi - f;
                if (fi > f) {
                    p->cut_row[p->ncut] = f;
                    p->cut_s[p->ncut] = nnz_base;
                    p->cut_e[p->ncut++] = std::min<int64_t>(nnz_end, h_rp[f + 1]);
                }
                if (li < l) {
                    p->cut_row[p->ncut] = l;
                    p->cut_s[p->ncut] = std::max<int64_t>(nnz_base, h_rp[l]);
                    p->cut_e[p->ncut++] = nnz_end;
                }
            } else {
                delete sub;  // no gain: the merge path keeps the whole range
            }
        }
    }
    if (rc) {
        delete p;
        return rc;
    }
    p->analysis_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    *out = p;
    return SMFV_OK;
}

extern "C" {

SMFV_API int smfv_plan_create(smfv_plan_t *out, int variant, int m, int n, int64_t nnz,
                              const int *h_row_ptr, const int *h_col_idx, int K, int flags)
{
    SMFV_REQUIRE(out, "null plan pointer");
    SMFV_REQUIRE(variant >= SMFV_SEQUENTIAL && variant <= SMFV_NONZERO, "unknown variant %d", variant);
    SMFV_REQUIRE(m >= 0 && n >= 0 && nnz >= 0 && nnz <= 0x7fffffff && K >= 0, "bad sizes");
    SMFV_REQUIRE(h_row_ptr == nullptr || (h_row_ptr[0] == 0 && h_row_ptr[m] == nnz), "row_ptr[0] != 0 or row_ptr[m] != nnz");
    return plan_create(out, variant, 0, m, n, 0, nnz, h_row_ptr, h_row_ptr ? h_col_idx : nullptr, K, flags);
}

SMFV_API int smfv_plan_create_rows(smfv_plan_t *out, int variant, int row_begin, int row_end, int n,
                                   const int *h_row_ptr, const int *h_col_idx, int K, int flags)
{
    SMFV_REQUIRE(out && h_row_ptr, "null plan pointer / row_ptr");
    SMFV_REQUIRE(variant >= SMFV_SEQUENTIAL && variant <= SMFV_NONZERO, "unknown variant %d", variant);
    SMFV_REQUIRE(row_begin >= 0 && row_end >= row_begin && n >= 0 && K >= 0, "bad row block [%d, %d)", row_begin,
                 row_end);
    const int64_t s = h_row_ptr[row_begin], e = h_row_ptr[row_end];
    SMFV_REQUIRE(0 <= s && s <= e && e <= 0x7fffffff, "bad row_ptr range [%lld, %lld)", (long long)s, (long long)e);
    return plan_create(out, variant, row_begin, row_end - row_begin, n, s, e, h_row_ptr, h_col_idx, K, flags);
}


SMFV_API int smfv_plan_analyse(int m, int n, const int *h_row_ptr, const int *h_col_idx,
                               double out[6])
{
    double o[9];
    const int rc = smfv_plan_analyse_rows(0, m, n, h_row_ptr, h_col_idx,
                                          SMFV_PLAN_NATURAL_SEEDS | SMFV_PLAN_ONE_WAVEFRONT, o);
    for (int i = 0; i < 6 && rc == SMFV_OK; ++i) out[i] = o[i];
    return rc;
}

SMFV_API int smfv_wsn_plan_analyse(int row_begin, int row_end, int n, const int *h_row_ptr_all,
                                   const int *h_col_idx_all, int kw, double out[9])
{
    SMFV_REQUIRE(row_begin >= 0 && row_end >= row_begin && n >= 0 && h_row_ptr_all && h_col_idx_all && out &&
                     (kw == 4 || kw == 8),
                 "bad argument");
    const int m = row_end - row_begin;
    std::vector<int> rpl((size_t)m + 1);
    for (int i = 0; i <= m; ++i) rpl[i] = h_row_ptr_all[row_begin + i] - h_row_ptr_all[row_begin];
    const int *cil = h_col_idx_all + h_row_ptr_all[row_begin];
    TileCaps caps = plan_caps(0, row_begin);
    caps.wsn_model = true;  // (r6) report the X reads' modelled LDS cycles
    double footprint = -1.0;
    plan_parts(caps, 0, m, n, rpl.data(), cil, &footprint);
    WsnPlan W;
    std::string err;
    if (!build_wsn_plan(m, n, rpl.data(), cil, kw, W, &err, caps)) {
        set_error("%s", err.c_str());
        return SMFV_ERR_INVALID;
    }
    int64_t most = 0;  // rows of the fullest tile
    for (int t = 0; t < W.ntiles; ++t) {
        int64_t r = 0;
        for (int s = 0; s < W.geom.rows(); ++s) r += W.lrec[(size_t)t * W.geom.lwords() + s] != -1;
        most = std::max(most, r);
    }
    out[0] = W.ntiles;
    out[1] = (double)W.union_rows;
    out[2] = W.union_rows ? (double)W.tiled_nnz / (double)W.union_rows : 0.0;
    out[3] = (double)W.direct.size();
    out[4] = (double)most;
    out[5] = (double)W.entries;
    out[6] = (double)W.x_groups;
    out[7] = (double)W.x_cycles;
    out[8] = (double)W.x_cycles_plain;
    return SMFV_OK;
}

SMFV_API int smfv_plan_analyse_rows(int row_begin, int row_end, int n, const int *h_row_ptr_all,
                                    const int *h_col_idx_all, int flags, double out[9])
{
    SMFV_REQUIRE(row_begin >= 0 && row_end >= row_begin && n >= 0 && h_row_ptr_all &&
                     (h_row_ptr_all[row_end] == h_row_ptr_all[row_begin] || h_col_idx_all) && out,
                 "bad argument");
    const int m = row_end - row_begin;
    std::vector<int> rpl((size_t)m + 1);
    for (int i = 0; i <= m; ++i) rpl[i] = h_row_ptr_all[row_begin + i] - h_row_ptr_all[row_begin];
    const int *h_row_ptr = rpl.data();
    const int *h_col_idx = h_col_idx_all ? h_col_idx_all + h_row_ptr_all[row_begin] : nullptr;
    double footprint = -1.0;
    TileCaps caps = plan_caps(flags, row_begin);
    plan_parts(caps, flags, m, n, h_row_ptr, h_col_idx, &footprint);
    caps.live = (flags & SMFV_PLAN_LIVE_VALUES) != 0;  // (r5) the live-values layout (WsPlan::vidx)
    TileAnalysis T;
    analyse_tiles(m, n, h_row_ptr, h_col_idx, T, caps);
    // invariants of the clustered analysis the plan is built from
    std::vector<char> seen((size_t)std::max(m, 1), 0);
    int64_t nd = 0;
    for (const TileMeta &tm : T.meta) {
        SMFV_REQUIRE(tm.nrows >= 1 && tm.nrows <= caps.maxrows, "tile rows out of range");
        SMFV_REQUIRE(tm.noff % 8 == 0, "tile segment not 16-byte aligned");
        if (tm.direct) {
            ++nd;
            SMFV_REQUIRE(tm.nrows == 1, "direct tile with several rows");
        } else {
            SMFV_REQUIRE(tm.nu <= caps.ucap && tm.tn <= caps.ncap, "tile over a cap");
        }
        int local = 0;
        for (int k = 0; k < tm.nrows; ++k) {
            const int r = T.trows[tm.roff + k];
            SMFV_REQUIRE(r >= 0 && r < m && !seen[r], "row %d missing or in two tiles", r);
            seen[r] = 1;
            const int info = T.rbeg[tm.roff + k];
            SMFV_REQUIRE((info & 0xFFFF) == (local & 0xFFFF) && local % 8 == 0 &&
                             (tm.direct || (info >> 16) == h_row_ptr[r + 1] - h_row_ptr[r]),
                         "row offsets inconsistent");
            for (int j = h_row_ptr[r]; j < h_row_ptr[r + 1]; ++j, ++local) {
                const int64_t e = (int64_t)tm.noff + local;
                SMFV_REQUIRE(T.tsrc[e] == j, "tile order is not CSR order inside a row");
                if (!tm.direct)
                    SMFV_REQUIRE(T.ucols[tm.uoff + T.tlidx[e]] == h_col_idx[j], "bad union position");
            }
            for (; local % 8; ++local) SMFV_REQUIRE(T.tsrc[(int64_t)tm.noff + local] == -1, "bad pad");
        }
        SMFV_REQUIRE(local == tm.tn, "tile non-zero count");
    }
    for (int r = 0; r < m; ++r) SMFV_REQUIRE(seen[r], "row %d in no tile", r);
    (void)nd;
    // the production (k_rows_ws) plan: built from the same analysis with its
    // own caps and verified by replaying the kernel's reads
    WsPlan W;
    std::string err;
    if (!build_ws_plan(m, n, h_row_ptr, h_col_idx, W, &err, caps)) {
        set_error("%s", err.c_str());
        return SMFV_ERR_INVALID;
    }
    out[0] = (double)W.ntiles;
    out[1] = (double)W.union_rows;
    out[2] = W.union_rows ? (double)W.tiled_nnz / (double)W.union_rows : 0.0;
    out[3] = (double)W.direct.size();
    out[4] = (double)W.ventries;
    out[5] = (double)W.tiled_nnz;
    out[6] = caps.part_start.size() > 2 ? (double)caps.part_start.size() - 1 : 1.0;
    out[7] = footprint;
    // X rows the XCDs' tile ranges read, summed over the XCDs, over the
    // block's distinct X rows (the compulsory X traffic of the XCD split)
    std::vector<int> stamp((size_t)std::max(n, 1), -1);
    int64_t sum = 0, total = 0;
    for (int x = 0; x < 8; ++x)
        for (int t = W.xcd[x]; t < W.xcd[x + 1]; ++t) {
            const int *G = &W.grec[(size_t)t * WS_GWORDS];
            for (int u = 0; u < G[WS_G_NU]; ++u) {
                const int c = G[W.geom.gword((u / 4) % W.geom.lw, u % 4, (u / 4) / W.geom.lw)];
                if (stamp[c] != x) stamp[c] = x, ++sum;
            }
        }
    std::fill(stamp.begin(), stamp.end(), -1);
    for (int j = 0; j < h_row_ptr[m]; ++j)
        if (stamp[h_col_idx[j]] != 0) stamp[h_col_idx[j]] = 0, ++total;
    out[8] = total ? (double)sum / (double)total : 0.0;
    return SMFV_OK;
}


SMFV_API int smfv_spmv_chunks_analyse(int row_begin, int row_end, int n, const int *h_row_ptr_all,
                                      const int *h_col_idx_all, int cap, double out[6])
{
    SMFV_REQUIRE(row_begin >= 0 && row_end >= row_begin && n >= 0 && h_row_ptr_all && out &&
                     (h_row_ptr_all[row_end] == h_row_ptr_all[row_begin] || h_col_idx_all),
                 "bad argument");
    SMFV_REQUIRE(cap == 0 || cap == 512 || cap == 1024 || cap == 2048, "chunk cap must be 512, 1024 or 2048");
    const int m = row_end - row_begin, base = h_row_ptr_all[row_begin];
    std::vector<int> rpl((size_t)m + 1);
    for (int i = 0; i <= m; ++i) rpl[i] = h_row_ptr_all[row_begin + i] - base;
    SpmvChunkPlan C;
    std::string err;
    const bool fits = build_spmv_chunks(m, n, rpl.data(), h_col_idx_all ? h_col_idx_all + base : nullptr,
                                        cap ? cap : spmv_chunk_cap(), K1_NT, C, &err);
    int most = 0;
    for (int c = 0; c < C.nchunks && fits; ++c) most = std::max(most, C.hdr[(size_t)c * 4 + 1]);
    out[0] = fits ? 1.0 : 0.0;
    out[1] = fits ? C.nchunks : 0;
    out[2] = fits ? (double)C.entries : 0.0;
    out[3] = most;
    out[4] = fits && C.nchunks ? (double)C.entries / ((double)C.nchunks * C.cap) : 0.0;
    out[5] = fits && C.wide ? 1.0 : 0.0;
    return SMFV_OK;
}

SMFV_API void smfv_set_analysis_threads(int threads) { smfv::analysis_threads = threads > 0 ? threads : 0; }

SMFV_API int smfv_plan_bind_values(smfv_plan_t plan, const double *d_values, void *stream)
{
    SMFV_REQUIRE(plan, "null plan");
    if (plan->sub) return smfv_plan_bind_values(plan->sub, d_values, stream);  // (the cut rows read live values)
    if (!plan->tiled || plan->live) return SMFV_OK;  // (r5) live plans read the values at execute
    SMFV_REQUIRE(d_values || plan->nnz == 0, "null values");
    hipStream_t st = as_stream(stream);
    const int64_t cnt = plan->snapshot;
    if (plan->bind_desc) {
        // (r4) the real entries from the bind items (pads written at creation)
        if (plan->nbind_items > 0) {
            hipLaunchKernelGGL(k_bind_items, dim3((unsigned)((plan->nbind_items + 255) / 256)), dim3(256), 0, st,
                               plan->nbind_items, reinterpret_cast<const int2 *>(plan->bind_items), d_values,
                               plan->tvals);
            SMFV_LAUNCHED();
        }
    } else if (cnt > 0) {
        hipLaunchKernelGGL(k_gather_vals, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, cnt, plan->tsrc,
                           d_values, plan->tvals, plan->mfma ? 0.0 : -0.0);
        SMFV_LAUNCHED();
    }
    // executes on another stream wait for this gather (smfv_plan_execute)
    SMFV_HIP(hipEventRecord(plan->bind_ev, st));
    plan->bind_stream = st;
    plan->bound_values = d_values;
    return SMFV_OK;
}


SMFV_API int smfv_stream_copy(void *d_dst, const void *d_src, size_t bytes, void *stream)
{
    SMFV_REQUIRE(d_dst && d_src && aligned16(d_dst) && aligned16(d_src) && bytes % 16 == 0,
                 "copy needs 16-byte aligned pointers and size");
    if (bytes == 0) return SMFV_OK;
    const int64_t n16 = (int64_t)(bytes / 16), nblk = (n16 + 1023) / 1024;
    SMFV_REQUIRE(nblk <= 0x7fffffff, "copy too large");
    hipLaunchKernelGGL(k_copy16, dim3((unsigned)nblk), dim3(256), 0, as_stream(stream), n16, static_cast<const ws::d2 *>(d_src), static_cast<ws::d2 *>(d_dst));
    SMFV_LAUNCHED();
    return SMFV_OK;
}

SMFV_API int smfv_stream_mix(void *d_dst, size_t wbytes, const void *d_src, size_t rbytes, int unit_kib,
                             void *stream)
{
    SMFV_REQUIRE(d_dst && d_src && aligned16(d_dst) && aligned16(d_src) && wbytes % 16 == 0 && rbytes % 16 == 0,
                 "mix probe needs 16-byte aligned pointers and sizes");
    if (wbytes == 0) return SMFV_OK;
    hipStream_t st = as_stream(stream);
    if (unit_kib <= 0) {
        SMFV_REQUIRE(rbytes == 2 * wbytes, "plain mix probe reads exactly twice the bytes it writes");
        const int64_t w16 = (int64_t)(wbytes / 16), nblk = (w16 + 1023) / 1024;
        SMFV_REQUIRE(nblk <= 0x7fffffff, "mix too large");
        hipLaunchKernelGGL(k_mix16, dim3((unsigned)nblk), dim3(256), 0, st, w16, static_cast<const ws::d2 *>(d_src),
                           static_cast<ws::d2 *>(d_dst));
        SMFV_LAUNCHED();
        return SMFV_OK;
    }
    SMFV_REQUIRE(unit_kib <= 64 && rbytes >= wbytes, "LDS mix probe: units of at most 64 KiB, reads >= writes");
    SMFV_REQUIRE(rbytes < (1ull << 31), "LDS mix probe: under 2 GiB read");
    const int ru = unit_kib * 1024;
    const int64_t nunits = ((int64_t)rbytes + ru - 1) / ru;
    // the unit's write share, rounded up to 16 B so the units cover wbytes
    const int wu = (int)((((int64_t)wbytes + nunits - 1) / nunits + 15) / 16 * 16);
    SMFV_REQUIRE(wu <= ru, "LDS mix probe: a unit writes more than it stages");
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
    }
    const int blocks = (int)std::min<int64_t>(nunits, ncu);
    hipLaunchKernelGGL(k_mix_lds, dim3((unsigned)blocks), dim3(1024), 0, st, (int64_t)rbytes, (int64_t)wbytes,
                       (int)nunits, ru, wu, static_cast<const char *>(d_src), static_cast<char *>(d_dst));
    SMFV_LAUNCHED();
    return SMFV_OK;
}

SMFV_API int smfv_plan_destroy(smfv_plan_t plan)
{
    delete plan;
    return SMFV_OK;
}

SMFV_API int smfv_plan_stats(smfv_plan_t plan, double out[SMFV_PLAN_STATS])
{
    SMFV_REQUIRE(plan && out, "null argument");
    if (plan->sub) {  // a NONZERO range: its whole rows' plan describes it
        smfv_plan_stats(plan->sub, out);
        out[6] = plan->row_begin;
        out[8] = plan->analysis_ms;
        return SMFV_OK;
    }
    out[0] = plan->tiled ? 1.0 : 0.0;
    out[1] = plan->ntiles;
    out[2] = (double)plan->union_rows;
    out[3] = plan->reuse;
    out[4] = (double)plan->dev_bytes;
    out[5] = plan->ndirect;
    out[6] = plan->row_begin;
    out[7] = plan->est_reuse;
    out[8] = plan->analysis_ms;
    out[9] = (double)plan->snapshot;
    out[10] = plan->mfma ? 1.0 : 0.0;
    out[11] = plan->parts;
    out[12] = plan->footprint;
    out[13] = !plan->tiled ? 0.0 : plan->k1 ? 3.0 : plan->mfma ? 2.0 : plan->wsn ? 5.0 : 1.0;
    out[14] = plan->live ? 1.0 : 0.0;  // (r5) live values (k_rows_cs, which used this slot, is retired)
    out[15] = plan->tiled && !plan->k1 && !plan->mfma && !plan->wsn ? plan->ws_geom : 0;
    out[16] = plan->bind_desc ? 1.0 : 0.0;
    out[17] = (double)plan->paired;
    return SMFV_OK;
}

SMFV_API int smfv_plan_execute(smfv_plan_t plan, const int *d_row_ptr, const int *d_col_idx,
                               const double *d_values, const double *d_X, int64_t ldx,
                               double *d_Y, int64_t ldy, void *stream)
{
    SMFV_REQUIRE(plan, "null plan");
    const int m = plan->m, K = plan->K;
    SMFV_REQUIRE(ldx >= K && ldy >= K, "leading dimension smaller than K");
    if (m == 0 || K == 0) return SMFV_OK;
    SMFV_REQUIRE(d_row_ptr && d_Y, "null row_ptr / Y");
    SMFV_REQUIRE(plan->nnz == 0 || (d_col_idx && d_values && d_X), "null col_idx / values / X");
    hipStream_t st = as_stream(stream);
    if (plan->sub) {
        // (r4) the whole rows by their plan, then the cut rows' partial sums
        // (each alone on the merge path: one row, its part of the range)
        const int rc = smfv_plan_execute(plan->sub, d_row_ptr, d_col_idx, d_values, d_X, ldx,
                                         d_Y + (int64_t)plan->sub_row * ldy, ldy, stream);
        if (rc) return rc;
        if (plan->ncut > 0) {  // one launch for both cut rows
            CutRows cr{};
            cr.n = plan->ncut;
            for (int i = 0; i < plan->ncut; ++i) {
                cr.row[i] = plan->cut_row[i];
                cr.s[i] = plan->cut_s[i];
                cr.e[i] = plan->cut_e[i];
                cr.yoff[i] = (int64_t)(plan->cut_row[i] - plan->row_begin) * ldy;
            }
            hipLaunchKernelGGL(k_cut_rows, dim3((unsigned)plan->ncut), dim3(256), 0, st, cr, d_col_idx, d_values, d_X,
                               ldx, K, d_Y);
            SMFV_LAUNCHED();
        }
        return SMFV_OK;
    }
    if (!plan->tiled || (!plan->k1 && pick_vec(d_X, ldx, d_Y, ldy, K) != 2)) {
        // untiled: the row / merge kernels on the live values
        if (plan->variant == SMFV_NONZERO)
            return launch_merge(plan->row_begin, m, plan->nnz_base, plan->nnz_end, d_row_ptr, d_col_idx, d_values,
                                d_X, ldx, K, d_Y, ldy, plan->ws, plan->ws_bytes, st);
        if (plan->simple)
            return launch_rows_simple(plan->row_begin, m, d_row_ptr, d_col_idx, d_values, d_X, ldx, K, d_Y, ldy, st);
        return launch_rows(plan->row_begin, m, d_row_ptr, d_col_idx, d_values, d_X, ldx, plan->n, K, d_Y, ldy, st);
    }
    if (!plan->live && d_values != plan->bound_values) {
        set_error("tiled plan: values not bound (call smfv_plan_bind_values with these d_values)");
        return SMFV_ERR_INVALID;
    }
    if (!plan->live && st != plan->bind_stream) {
        // the snapshot was gathered on another stream: order this launch after it
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        SMFV_HIP(hipStreamIsCapturing(st, &cs));
        if (cs == hipStreamCaptureStatusNone) {
            SMFV_HIP(hipStreamWaitEvent(st, plan->bind_ev, 0));
        } else if (hipEventQuery(plan->bind_ev) != hipSuccess) {
            set_error("tiled plan: the values snapshot (bound on another stream) is still in flight while "
                      "capturing; synchronize the bind stream before capture");
            return SMFV_ERR_INVALID;
        }
    }
    if (plan->k1) {
        if (plan->ntiles > 0) {
            auto kern = plan->k1_wide ? k_spmv_chunks<K1_NT, 1024, true> : k_spmv_chunks<K1_NT, 1024, false>;
            hipLaunchKernelGGL(kern, dim3((unsigned)plan->ntiles), dim3(K1_NT), 0, st,
                               reinterpret_cast<const int4 *>(plan->k1_hdr), plan->k1_rs, plan->k1_off, plan->k1_col,
                               plan->tvals, d_X, ldx, d_Y, ldy);
            SMFV_LAUNCHED();
        }
        return SMFV_OK;
    }
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
    }
    if (plan->mfma) {
        if (plan->ntiles > 0) {
            hipLaunchKernelGGL(k_rows_mfma, dim3((unsigned)plan->ntiles), dim3(256), 0, st, K / TILE_KP, plan->mf_rec,
                               plan->mf_ucols, plan->mf_bstep, plan->tvals, d_X, ldx, d_Y, ldy);
            SMFV_LAUNCHED();
        }
    } else if (plan->wsn && plan->ntiles > 0) {
        // (r5) narrow-team tiles: one persistent 1024-lane block per CU
        if ((uint64_t)plan->n * (uint64_t)ldx * 8u >= (1ull << 32) || (uint64_t)plan->snapshot * 8u >= (1ull << 32))
            return launch_rows(plan->row_begin, m, d_row_ptr, d_col_idx, d_values, d_X, ldx, plan->n, K, d_Y, ldy, st);
        WsXcd xr;
        for (int x = 0; x <= 8; ++x) xr.first[x] = plan->ws_xcd[x];
        const int blocks = std::max(8, (std::min(plan->ntiles, ncu) + 7) & ~7);
        auto kern = K == 4 ? (plan->fma ? k_rows_wsn<4, true> : k_rows_wsn<4, false>)
                           : (plan->fma ? k_rows_wsn<8, true> : k_rows_wsn<8, false>);
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(1024), 0, st, xr, plan->wsn_grec, plan->wsn_lrec,
                           plan->wsn_loff, plan->tvals, d_X, ldx, d_Y, ldy);
        SMFV_LAUNCHED();
    } else if (plan->ntiles > 0) {
        // persistent blocks: one (geometry 1) or two (geometry 2) per CU; a
        // multiple of 8 (>= 8) so every XCD's tile range has blocks
        const int per_cu = ws_geom(plan->ws_geom).cw == 4 ? 2 : 1;
        const int blocks = std::max(8, (std::min(plan->ntiles, per_cu * ncu) + 7) & ~7);
        int chunked = SMFV_WS_CHUNKED;
        // scalar-base addressing when X (n rows of ldx doubles) and the
        // snapshot each span < 4 GiB
        const bool saddr = (uint64_t)plan->n * (uint64_t)ldx * 8u < (1ull << 32) &&
                           (uint64_t)plan->snapshot * 8u < (1ull << 32);
        auto kern = pick_ws(plan->ws_geom, plan->fma, saddr);
        WsXcd xr;
        for (int x = 0; x <= 8; ++x) xr.first[x] = plan->ws_xcd[x];
        const int threads = ws_geom(plan->ws_geom).threads();
        // (r4) K = 4 / 8 / 16: one panel, a narrow column window (chunked bits 16-23)
        const bool narrow = K < TILE_KP;
        if (narrow) {
            kern = pick_ws(plan->ws_geom, plan->fma, saddr, true);
            chunked = (chunked & 1) | (K << 16);
        }
        if (plan->live) {
            if (!saddr || (uint64_t)plan->nnz * 8u >= (1ull << 32)) {
                // (r6) X (or the block's values) spanning 4 GiB or
                // more: the untiled row kernel on the same live values, as the
                // wsn branch does (bit-identical: each row in CSR order)
                return launch_rows(plan->row_begin, m, d_row_ptr, d_col_idx, d_values, d_X, ldx, plan->n, K, d_Y,
                                   ldy, st);
            }
            // the value pairs come from the block's CSR values through a
            // range-checked buffer (the last odd row's read past the end gives 0)
            hipLaunchKernelGGL(pick_ws_live(plan->ws_geom, plan->fma, narrow), dim3((unsigned)blocks),
                               dim3((unsigned)threads), 0, st, xr, narrow ? 1 : K / TILE_KP, chunked, plan->ws_grec,
                               plan->ws_lrec, plan->ws_loff, d_values + plan->nnz_base, d_X, ldx, d_Y, ldy,
                               plan->ws_vidx, plan->ws_vstride, (unsigned)(plan->nnz * 8));
        } else {
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3((unsigned)threads), 0, st, xr,
                               narrow ? 1 : K / TILE_KP, chunked, plan->ws_grec, plan->ws_lrec, plan->ws_loff,
                               plan->tvals, d_X, ldx, d_Y, ldy);
        }
        SMFV_LAUNCHED();
    }
    if (plan->ndirect > 0) {
        hipLaunchKernelGGL(k_rows_list, dim3((unsigned)((plan->ndirect + 31) / 32), (unsigned)std::max(1, K / TILE_KP)),
                           dim3(256), 0, st, plan->ndirect, K < TILE_KP ? K : 0, plan->direct_rows, plan->direct_off, plan->row_begin,
                           d_row_ptr, d_col_idx, plan->live ? d_values : plan->tvals, d_X, ldx, d_Y, ldy);
        SMFV_LAUNCHED();
    }
    return SMFV_OK;
}


SMFV_API int smfv_spmm_rowblock_f64(int row_begin, int row_end, int n, const int *d_row_ptr,
                                    const int *d_col_idx, const double *d_values,
                                    const double *d_X, int64_t ldx, int K, double *d_Yblock,
                                    int64_t ldy, void *stream)
{
    SMFV_REQUIRE(row_begin >= 0 && row_end >= row_begin && K >= 0, "bad row block [%d, %d)",
                 row_begin, row_end);
    SMFV_REQUIRE(ldx >= K && ldy >= K, "leading dimension smaller than K");
    SMFV_REQUIRE(n >= 0, "negative n");
    return launch_rows(row_begin, row_end - row_begin, d_row_ptr, d_col_idx, d_values, d_X, ldx, n,
                       K, d_Yblock, ldy, as_stream(stream));
}

SMFV_API int smfv_spmm_colpanel_f64(int m, int n, int col_begin, int col_end, const int *d_row_ptr,
                                    const int *d_col_idx, const double *d_values,
                                    const double *d_X, int64_t ldx, double *d_panel, int64_t ldp,
                                    void *stream)
{
    const int kc = col_end - col_begin;
    SMFV_REQUIRE(m >= 0 && col_begin >= 0 && kc >= 0 && col_end <= ldx, "bad column panel");
    SMFV_REQUIRE(ldp >= kc, "panel leading dimension smaller than panel width");
    SMFV_REQUIRE(n >= 0, "negative n");
    return launch_rows(0, m, d_row_ptr, d_col_idx, d_values, d_X + col_begin, ldx, n, kc, d_panel,
                       ldp, as_stream(stream));
}

SMFV_API int smfv_nnz_range_rows(int m, const int *h_row_ptr, int64_t nnz_begin, int64_t nnz_end,
                                 int *row_first, int *row_last)
{
    SMFV_REQUIRE(h_row_ptr && row_first && row_last, "null argument");
    SMFV_REQUIRE(0 <= nnz_begin && nnz_begin <= nnz_end && nnz_end <= h_row_ptr[m],
                 "bad nnz range");
    if (nnz_begin == nnz_end) {
        *row_first = 0;
        *row_last = -1;
        return SMFV_OK;
    }
    // row containing nnz_begin: last i with row_ptr[i] <= nnz_begin and row non-empty
    const int *b = h_row_ptr, *e = h_row_ptr + m + 1;
    const int rf = (int)(std::upper_bound(b, e, (int)nnz_begin) - b) - 1;
    const int rl = (int)(std::upper_bound(b, e, (int)(nnz_end - 1)) - b) - 1;
    *row_first = rf;
    *row_last = rl;
    return SMFV_OK;
}

SMFV_API int smfv_spmm_nnzrange_workspace_bytes(int nrows, int64_t nnz_count, int K, size_t *bytes)
{
    SMFV_REQUIRE(bytes && nrows >= 0 && nnz_count >= 0 && K >= 0, "bad argument");
    *bytes = merge_workspace_bytes(nrows, nnz_count, K);
    return SMFV_OK;
}

SMFV_API int smfv_spmm_nnzrange_f64(int row_first, int row_last, int64_t nnz_begin,
                                    int64_t nnz_end, int n, const int *d_row_ptr, const int *d_col_idx,
                                    const double *d_values, const double *d_X, int64_t ldx, int K,
                                    double *d_Ypart, int64_t ldy, void *d_workspace,
                                    size_t workspace_bytes, void *stream)
{
    SMFV_REQUIRE(nnz_begin >= 0 && nnz_end >= nnz_begin && K >= 0, "bad nnz range");
    SMFV_REQUIRE(ldx >= K && ldy >= K, "leading dimension smaller than K");
    const int nrows = row_last - row_first + 1;
    if (nrows <= 0) return SMFV_OK;
    return launch_merge(row_first, nrows, nnz_begin, nnz_end, d_row_ptr, d_col_idx, d_values, d_X,
                        ldx, K, d_Ypart, ldy, d_workspace, workspace_bytes, as_stream(stream));
}

SMFV_API int smfv_panels_to_rowmajor_f64(int m, int K, int p, const double *d_panels, double *d_Y,
                                         int64_t ldy, void *stream)
{
    SMFV_REQUIRE(m >= 0 && K >= 0 && p > 0 && ldy >= K, "bad argument");
    const int64_t total = (int64_t)m * K;
    if (total == 0) return SMFV_OK;
    const int64_t nblk = (total + 255) / 256;
    SMFV_REQUIRE(nblk <= 0x7fffffff, "too large");
    hipLaunchKernelGGL(k_panels_to_rowmajor, dim3((unsigned)nblk), dim3(256), 0, as_stream(stream),
                       m, K, p, d_panels, d_Y, ldy);
    SMFV_LAUNCHED();
    return SMFV_OK;
}

SMFV_API int smfv_combine_row_blocks_f64(int m, int K, int p, const int *h_row_first,
                                         const int *h_row_last, const double *d_blocks,
                                         double *d_Y, int64_t ldy, void *stream)
{
    SMFV_REQUIRE(m >= 0 && K >= 0 && p > 0 && p <= 64 && ldy >= K, "bad argument (p <= 64)");
    BlockTable tab;
    std::memset(&tab, 0, sizeof tab);
    tab.p = p;
    int64_t off = 0;
    for (int r = 0; r < p; ++r) {
        tab.rf[r] = h_row_first[r];
        tab.rl[r] = h_row_last[r];
        tab.off[r] = off;
        const int nr = h_row_last[r] - h_row_first[r] + 1;
        if (nr > 0) off += (int64_t)nr * K;
    }
    const int64_t total = (int64_t)m * K;
    if (total == 0) return SMFV_OK;
    const int64_t nblk = (total + 255) / 256;
    SMFV_REQUIRE(nblk <= 0x7fffffff, "too large");
    hipLaunchKernelGGL(k_combine_blocks, dim3((unsigned)nblk), dim3(256), 0, as_stream(stream), m,
                       K, tab, d_blocks, d_Y, ldy);
    SMFV_LAUNCHED();
    return SMFV_OK;
}

SMFV_API int smfv_compare_f64(int m, int K, const double *d_A, int64_t lda, const double *d_B,
                              int64_t ldb, double *h_out, void *stream)
{
    SMFV_REQUIRE(h_out && m >= 0 && K >= 0 && lda >= K && ldb >= K, "bad argument");
    hipStream_t st = as_stream(stream);
    // a checker, synchronous by contract: plain allocation and a blocking
    // read-back after the stream has drained (no pageable async copy)
    unsigned long long *d_out = nullptr;
    SMFV_HIP(hipMalloc(reinterpret_cast<void **>(&d_out), 2 * sizeof(unsigned long long)));
    unsigned long long h[2] = {0, 0};
    hipError_t e = hipMemsetAsync(d_out, 0, 2 * sizeof(unsigned long long), st);
    if (e == hipSuccess && (int64_t)m * K > 0) {
        hipLaunchKernelGGL(k_compare, dim3(1024), dim3(256), 0, st, m, K, d_A, lda, d_B, ldb, d_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    SMFV_HIP(e);
    std::memcpy(h_out, h, sizeof h);
    return SMFV_OK;
}

SMFV_API int smfv_fill_x_hash_f64(int64_t n, int K, uint64_t seed, double *d_X, int64_t ldx,
                                  void *stream)
{
    SMFV_REQUIRE(n >= 0 && K >= 0 && ldx >= K && (n == 0 || K == 0 || d_X), "bad argument");
    if (n * K == 0) return SMFV_OK;
    hipLaunchKernelGGL(k_fill_x_hash, dim3(4096), dim3(256), 0, as_stream(stream), n, K, seed, d_X,
                       ldx);
    SMFV_LAUNCHED();
    return SMFV_OK;
}

}  // extern "C"
