// Lab (not part of the product): candidate tiled row kernels for the
// cop20k_A surrogate at K = 32, timed cold (rotated copies) and warm, and
// checked bit-for-bit against the production ROWWISE result.
//   lab_spmm <matrix.smfvcsr> [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "smfv.h"
#include "smfv_host.h"
#include "smfv_plan.h"

using namespace smfv;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);     \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

#pragma clang fp contract(off)

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));

// Workgroup barrier that orders LDS only: __syncthreads() also drains every
// outstanding global load (vmcnt(0)), which would serialise the prefetch of
// the next tile behind each barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------------------
// k_rows_dbuf: persistent, 2 blocks per CU, each block owns TWO LDS slots
// (tile t computed from one while tile t+1 is written into the other from
// registers), one barrier per tile.  8-lane teams, swizzled halves, CSR
// order, separate multiply / add (bit-identical).
// ---------------------------------------------------------------------------
constexpr int UC = 128, NC = 768, KP = 32;

struct Pref {
    d2 x[8];   // X rows (tid>>4) + 16k, 16-B chunk tid&15
    d2 v[2];   // values 2*tid + 512k
    u2 l;      // local columns 4*tid..+3
    int ri;    // row / info word (tid < 64)
    int hdr;   // record word tid (tid < 72): header, rows, info
    int tn, nu, direct;
};

__device__ __forceinline__ void hdr_of(const int *__restrict__ rec, int t, int &noff, int &tn, int &nu,
                                       int &direct)
{
    const int4 h0 = *reinterpret_cast<const int4 *>(rec + (int64_t)t * TREC_WORDS);
    const int4 h1 = *reinterpret_cast<const int4 *>(rec + (int64_t)t * TREC_WORDS + 4);
    noff = h0.x;
    tn = h0.y;
    nu = h0.w;
    direct = h1.z;  // word 6 = direct (TileMeta: noff tn uoff nu roff nrows direct pad)
    (void)h1;
}

template <int MODE>  // 0 full, 1 no compute, 2 no staging
__global__ __launch_bounds__(256, 2) void k_rows_dbuf(int ntiles, const int *__restrict__ rec,
                                                      const uint16_t *__restrict__ tlidx,
                                                      const double *__restrict__ tvals,
                                                      const double *__restrict__ X, double *__restrict__ Y)
{
    __shared__ __attribute__((aligned(16))) double s_x[2][UC * KP];
    __shared__ __attribute__((aligned(16))) double s_va[2][NC];
    __shared__ __attribute__((aligned(16))) uint16_t s_li[2][NC];
    __shared__ __attribute__((aligned(16))) int s_ri[2][72];  // [0..7] header, [8..39] rows, [40..71] info
    int t0, tstep, tlast;
    {
        const int G = gridDim.x;
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
        const int nb = (G >> 3) + (x < (G & 7) ? 1 : 0);
        const int first = (int)((int64_t)ntiles * x / 8), end = (int)((int64_t)ntiles * (x + 1) / 8);
        t0 = first + j;
        tstep = nb;
        if (t0 >= end) return;
        tlast = t0 + ((end - 1 - t0) / nb) * nb;
    }
    const int tid = threadIdx.x, team = tid >> 3, tl = tid & 7, par = team & 1;
    const int xr = tid >> 4, xs = tid & 15;
    Pref P;
    // record of the tile after the one in P: header, rows/info word, union ids
    struct Rec {
        i4 c0, c1;
        int hdr, noff, tn, nu, direct;
    } Rn;
    auto loadrec = [&](int t) {
        const int *R = rec + (int64_t)t * TREC_WORDS;
        hdr_of(rec, t, Rn.noff, Rn.tn, Rn.nu, Rn.direct);
        Rn.hdr = tid < 72 ? R[tid] : 0;
        Rn.c0 = *reinterpret_cast<const i4 *>(R + TREC_UCOLS + 8 * xr);
        Rn.c1 = *reinterpret_cast<const i4 *>(R + TREC_UCOLS + 8 * xr + 4);
    };
    // tile data into P, from the record in Rn
    auto load = [&]() {
        P.tn = Rn.tn;
        P.nu = Rn.nu;
        P.direct = Rn.direct;
        P.hdr = Rn.hdr;
        const int uc[8] = {Rn.c0.x, Rn.c0.y, Rn.c0.z, Rn.c0.w, Rn.c1.x, Rn.c1.y, Rn.c1.z, Rn.c1.w};
        const int tn = Rn.tn, nu = Rn.nu, noff = Rn.noff;
        if (MODE == 2) return;
        if (Rn.direct) return;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (xr + 16 * k < nu) P.x[k] = *reinterpret_cast<const d2 *>(X + (int64_t)uc[k] * KP + 2 * xs);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int e = 2 * tid + 512 * k;
            if (e < tn) P.v[k] = *reinterpret_cast<const d2 *>(tvals + noff + e);
        }
        if (4 * tid < tn) P.l = *reinterpret_cast<const u2 *>(tlidx + noff + 4 * tid);
    };
    // prologue: tile t0 -> slot 0
    loadrec(t0);
    load();
    loadrec(min(t0 + tstep, tlast));
    {
        const int *R = rec + (int64_t)t0 * TREC_WORDS;
        const int tn = R[1], nu = R[3], direct = R[6];
        if (tid < 72) s_ri[0][tid] = P.hdr;
        if (MODE != 2 && !direct) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (xr + 16 * k < nu) reinterpret_cast<d2 *>(s_x[0])[(xr + 16 * k) * (KP / 2) + xs] = P.x[k];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int e = 2 * tid + 512 * k;
                if (e < tn) reinterpret_cast<d2 *>(s_va[0])[e / 2] = P.v[k];
            }
            if (4 * tid < tn) reinterpret_cast<u2 *>(s_li[0])[tid] = P.l;
        }
    }
    load();  // tile t0 + tstep (or t0 again: clamped, never stored)
    loadrec(min(t0 + 2 * tstep, tlast));
    lds_barrier();
    const d2 *sx0b = reinterpret_cast<const d2 *>(s_x[0]) + par * 8 + tl;
    for (int t = t0, it = 0; t <= tlast; t += tstep, ++it) {
        const int c = it & 1, n = c ^ 1;
        // phase 1: registers (tile t + tstep) -> slot n
        const int tn1 = t + tstep;
        if (tn1 <= tlast) {
            const int tn = P.tn, nu = P.nu, direct = P.direct;
            if (tid < 72) s_ri[n][tid] = P.hdr;
            if (MODE != 2 && !direct) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (xr + 16 * k < nu)
                        reinterpret_cast<d2 *>(s_x[n])[(xr + 16 * k) * (KP / 2) + xs] = P.x[k];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int e = 2 * tid + 512 * k;
                    if (e < tn) reinterpret_cast<d2 *>(s_va[n])[e / 2] = P.v[k];
                }
                if (4 * tid < tn) reinterpret_cast<u2 *>(s_li[n])[tid] = P.l;
            }
            // phase 2: loads for tile t + 2 tstep (record of t + 3 tstep)
            load();
            loadrec(min(tn1 + 2 * tstep, tlast));
        }
        // phase 3: compute tile t from slot c
        if (MODE != 1) {
            const int *ri = s_ri[c];
            const int nrows = ri[5], direct = ri[6];
            if (team < nrows && !direct) {
                const int row = ri[8 + team];
                const int info = ri[40 + team];
                const int js = info & 0xFFFF, je = js + (info >> 16);
                const d2 *sx0 = sx0b + c * (UC * KP / 2);
                const d2 *sx1 = reinterpret_cast<const d2 *>(s_x[c]) + (par ^ 1) * 8 + tl;
                d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
                const uint16_t *li = s_li[c];
                const double *va = s_va[c];
                int j = js;
                for (; j + 4 <= je; j += 4) {
                    const u2 lq = *reinterpret_cast<const u2 *>(li + j);
                    const d2 va0 = *reinterpret_cast<const d2 *>(va + j);
                    const d2 va1 = *reinterpret_cast<const d2 *>(va + j + 2);
                    const int l[4] = {(int)(lq.x & 0xFFFF), (int)(lq.x >> 16), (int)(lq.y & 0xFFFF),
                                      (int)(lq.y >> 16)};
                    const double v[4] = {va0.x, va0.y, va1.x, va1.y};
                    d2 x0[4], x1[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        x0[u] = sx0[l[u] * (KP / 2)];
                        x1[u] = sx1[l[u] * (KP / 2)];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        acc0 = acc0 + v[u] * x0[u];
                        acc1 = acc1 + v[u] * x1[u];
                    }
                }
                for (; j < je; ++j) {
                    const int l = li[j];
                    const double v = va[j];
                    acc0 = acc0 + v * sx0[l * (KP / 2)];
                    acc1 = acc1 + v * sx1[l * (KP / 2)];
                }
                double *y = Y + (int64_t)row * KP + 2 * tl;
                *reinterpret_cast<d2 *>(y + 16 * par) = acc0;
                *reinterpret_cast<d2 *>(y + 16 * (par ^ 1)) = acc1;
            }
        }
        lds_barrier();
    }
}


// ---------------------------------------------------------------------------
// k_rows_db2: k_rows_dbuf without any wait the pipeline does not need:
// every prefetch load is unconditional (indices clamped, arrays padded), all
// record words are VECTOR loads (an SMEM load shares lgkmcnt with LDS and
// would be waited for by the first LDS wait), the barrier orders LDS only,
// and the rows of a tile are dealt round-robin to the 4 waves.
// Record words used: [0..71] header / rows / info (word tid), [72..199]
// union ids, [200..215] noff replicated (word 200 + (tid & 15)).
// DEPTH = tiles of register prefetch (1: tile t+1 in flight while t computes).
// ---------------------------------------------------------------------------
constexpr int REC_NOFF = 200;
template <int MODE>
__global__ __launch_bounds__(256, 2) void k_rows_db2(int ntiles, const int *__restrict__ rec,
                                                     const uint16_t *__restrict__ tlidx,
                                                     const double *__restrict__ tvals,
                                                     const double *__restrict__ X, double *__restrict__ Y)
{
    __shared__ __attribute__((aligned(16))) double s_x[2][UC * KP];
    __shared__ __attribute__((aligned(16))) double s_va[2][NC];
    __shared__ __attribute__((aligned(16))) uint16_t s_li[2][NC];
    __shared__ __attribute__((aligned(16))) int s_ri[2][72];
    int t0, tstep, cnt;
    {
        const int G = gridDim.x;
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
        const int nb = (G >> 3) + (x < (G & 7) ? 1 : 0);
        const int first = (int)((int64_t)ntiles * x / 8), end = (int)((int64_t)ntiles * (x + 1) / 8);
        t0 = first + j;
        tstep = nb;
        if (t0 >= end) return;
        cnt = (end - 1 - t0) / nb + 1;  // tiles of this block
    }
    const int tlast = t0 + (cnt - 1) * tstep;
    const int tid = threadIdx.x, tl = tid & 7, wv = tid >> 6, tw = (tid >> 3) & 7, par = tw & 1;
    const int xr = tid >> 4, xs = tid & 15;
    const int rowslot = tw * 4 + wv;  // round-robin: tile row i -> wave i % 4, team i / 4
    // prefetch registers
    i4 c0, c1;
    int noff;
    d2 px[8], pv[2];
    u2 pl;
    int ph;
    auto loadrec = [&](int t) {
        const int *R = rec + (int64_t)t * TREC_WORDS;
        c0 = *reinterpret_cast<const i4 *>(R + TREC_UCOLS + 8 * xr);
        c1 = *reinterpret_cast<const i4 *>(R + TREC_UCOLS + 8 * xr + 4);
        noff = R[REC_NOFF + xs];
    };
    auto load = [&](int t) {
        const int *R = rec + (int64_t)t * TREC_WORDS;
        ph = R[tid < 72 ? tid : 0];
        const int uc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        if (MODE == 2) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) px[k] = *reinterpret_cast<const d2 *>(X + (int64_t)uc[k] * KP + 2 * xs);
#pragma unroll
        for (int k = 0; k < 2; ++k) pv[k] = *reinterpret_cast<const d2 *>(tvals + noff + 2 * tid + 512 * k);
        pl = *reinterpret_cast<const u2 *>(tlidx + noff + 4 * tid);
    };
    auto store = [&](int s) {
        if (tid < 72) s_ri[s][tid] = ph;
        if (MODE == 2) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) reinterpret_cast<d2 *>(s_x[s])[(xr + 16 * k) * (KP / 2) + xs] = px[k];
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (2 * tid + 512 * k < NC) reinterpret_cast<d2 *>(s_va[s])[tid + 256 * k] = pv[k];
        if (4 * tid < NC) reinterpret_cast<u2 *>(s_li[s])[tid] = pl;
    };
    loadrec(t0);
    load(t0);
    loadrec(min(t0 + tstep, tlast));
    store(0);
    load(min(t0 + tstep, tlast));
    loadrec(min(t0 + 2 * tstep, tlast));
    lds_barrier();
    for (int it = 0; it < cnt; ++it) {
        const int c = it & 1;
        const int t = t0 + it * tstep;
        // phase 1: tile t + tstep (registers) -> the other slot
        store(c ^ 1);
        // phase 2: tile t + 2 tstep -> registers; record of t + 3 tstep
        load(min(t + 2 * tstep, tlast));
        loadrec(min(t + 3 * tstep, tlast));
        // phase 3: compute tile t
        if (MODE != 1) {
            const int *ri = s_ri[c];
            const int nrows = ri[5];
            if (rowslot < nrows) {
                const int row = ri[8 + rowslot];
                const int info = ri[40 + rowslot];
                const int js = info & 0xFFFF, je = js + (info >> 16);
                const d2 *sx0 = reinterpret_cast<const d2 *>(s_x[c]) + par * 8 + tl;
                const d2 *sx1 = reinterpret_cast<const d2 *>(s_x[c]) + (par ^ 1) * 8 + tl;
                d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
                const uint16_t *li = s_li[c];
                const double *va = s_va[c];
                int j = js;
                for (; j + 4 <= je; j += 4) {
                    const u2 lq = *reinterpret_cast<const u2 *>(li + j);
                    const d2 va0 = *reinterpret_cast<const d2 *>(va + j);
                    const d2 va1 = *reinterpret_cast<const d2 *>(va + j + 2);
                    const int l[4] = {(int)(lq.x & 0xFFFF), (int)(lq.x >> 16), (int)(lq.y & 0xFFFF),
                                      (int)(lq.y >> 16)};
                    const double v[4] = {va0.x, va0.y, va1.x, va1.y};
                    d2 x0[4], x1[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        x0[u] = sx0[l[u] * (KP / 2)];
                        x1[u] = sx1[l[u] * (KP / 2)];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        acc0 = acc0 + v[u] * x0[u];
                        acc1 = acc1 + v[u] * x1[u];
                    }
                }
                for (; j < je; ++j) {
                    const int l = li[j];
                    const double v = va[j];
                    acc0 = acc0 + v * sx0[l * (KP / 2)];
                    acc1 = acc1 + v * sx1[l * (KP / 2)];
                }
                double *y = Y + (int64_t)row * KP + 2 * tl;
                *reinterpret_cast<d2 *>(y + 16 * par) = acc0;
                *reinterpret_cast<d2 *>(y + 16 * (par ^ 1)) = acc1;
            }
        }
        lds_barrier();
    }
}


// ---------------------------------------------------------------------------
// k_rows_db3: k_rows_db2 with a cheaper inner loop: local columns are stored
// as byte offsets of the X row inside the slot's image (u16), each row is
// walked in batches of 8 (meta: 1 + 4 b128 reads, then 16 X reads in
// flight), and pad entries (value +0.0, offset of a zero row) make the walk
// over the padded length exact: acc + (+0.0) == acc for every acc the
// reference can hold (a sum that starts at +0.0 is never -0.0), and the
// zero row keeps a pad from multiplying an Inf / NaN of X.
// TAIL4: the last 4 of a row's padded-to-8 length are skipped when the
// row's length rounded up to 4 ends there (team-divergent).
// FMA (lab only): fused multiply-add (not bit-identical).
// ---------------------------------------------------------------------------
constexpr int NC3 = 752;
constexpr int ZROW = UC * KP * 8;  // byte offset of the zero row in a slot
template <int MODE, bool TAIL4, bool FMA>
__global__ __launch_bounds__(256, 2) void k_rows_db3(int ntiles, const int *__restrict__ rec,
                                                     const uint16_t *__restrict__ tlidx,
                                                     const double *__restrict__ tvals,
                                                     const double *__restrict__ X, double *__restrict__ Y)
{
    __shared__ __attribute__((aligned(16))) double s_x[2][(UC + 1) * KP];
    __shared__ __attribute__((aligned(16))) double s_va[2][NC3];
    __shared__ __attribute__((aligned(16))) uint16_t s_li[2][NC3];
    __shared__ __attribute__((aligned(16))) int s_ri[2][72];
    int t0, tstep, cnt;
    {
        const int G = gridDim.x;
        const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
        const int nb = (G >> 3) + (x < (G & 7) ? 1 : 0);
        const int first = (int)((int64_t)ntiles * x / 8), end = (int)((int64_t)ntiles * (x + 1) / 8);
        t0 = first + j;
        tstep = nb;
        if (t0 >= end) return;
        cnt = (end - 1 - t0) / nb + 1;
    }
    const int tlast = t0 + (cnt - 1) * tstep;
    const int tid = threadIdx.x, tl = tid & 7, wv = tid >> 6, tw = (tid >> 3) & 7, par = tw & 1;
    const int xr = tid >> 4, xs = tid & 15;
    const int rowslot = tw * 4 + wv;
    if (tid < 64) {  // zero rows of both slots
        reinterpret_cast<d2 *>(s_x[0] + UC * KP)[tid & 15] = d2{0.0, 0.0};
        reinterpret_cast<d2 *>(s_x[1] + UC * KP)[tid & 15] = d2{0.0, 0.0};
    }
    i4 c0, c1;
    int noff;
    d2 px[8], pv[2];
    u2 pl;
    int ph;
    auto loadrec = [&](int t) {
        const int *R = rec + (int64_t)t * TREC_WORDS;
        c0 = *reinterpret_cast<const i4 *>(R + TREC_UCOLS + 8 * xr);
        c1 = *reinterpret_cast<const i4 *>(R + TREC_UCOLS + 8 * xr + 4);
        noff = R[REC_NOFF + xs];
    };
    auto load = [&](int t) {
        const int *R = rec + (int64_t)t * TREC_WORDS;
        ph = R[tid < 72 ? tid : 0];
        const int uc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        if (MODE >= 2) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) px[k] = *reinterpret_cast<const d2 *>(X + (int64_t)uc[k] * KP + 2 * xs);
#pragma unroll
        for (int k = 0; k < 2; ++k) pv[k] = *reinterpret_cast<const d2 *>(tvals + noff + 2 * tid + 512 * k);
        pl = *reinterpret_cast<const u2 *>(tlidx + noff + 4 * tid);
    };
    auto store = [&](int s) {
        if (tid < 72) s_ri[s][tid] = ph;
        if (MODE >= 2) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) reinterpret_cast<d2 *>(s_x[s])[(xr + 16 * k) * (KP / 2) + xs] = px[k];
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (2 * tid + 512 * k < NC3) reinterpret_cast<d2 *>(s_va[s])[tid + 256 * k] = pv[k];
        if (4 * tid < NC3) reinterpret_cast<u2 *>(s_li[s])[tid] = pl;
    };
    auto madd = [&](d2 a, double v, d2 x) -> d2 {
        if constexpr (FMA)
            return d2{__builtin_fma(v, x.x, a.x), __builtin_fma(v, x.y, a.y)};
        else
            return a + v * x;
    };
    loadrec(t0);
    load(t0);
    loadrec(min(t0 + tstep, tlast));
    store(0);
    load(min(t0 + tstep, tlast));
    loadrec(min(t0 + 2 * tstep, tlast));
    lds_barrier();
    for (int it = 0; it < cnt; ++it) {
        const int c = it & 1;
        const int t = t0 + it * tstep;
        store(c ^ 1);
        load(min(t + 2 * tstep, tlast));
        loadrec(min(t + 3 * tstep, tlast));
        if (MODE != 1) {
            const int *ri = s_ri[c];
            const int nrows = ri[5];
            if (rowslot < nrows) {
                const int row = ri[8 + rowslot];
                const int info = ri[40 + rowslot];
                const int js = info & 0xFFFF, len = info >> 16;
                const int je8 = MODE == 3 ? js : js + ((len + 7) & ~7);
                const char *sb0 = reinterpret_cast<const char *>(s_x[c]) + par * 128 + tl * 16;
                const char *sb1 = reinterpret_cast<const char *>(s_x[c]) + (par ^ 1) * 128 + tl * 16;
                d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
                const uint16_t *li = s_li[c];
                const double *va = s_va[c];
                for (int j = js; j < je8; j += 8) {
                    uint4 lq;
                    double v[8];
                    if constexpr (MODE == 4) {  // lab: no meta reads
                        const unsigned b = (unsigned)(j * 37 + rowslot * 11) & 127;
                        lq = uint4{(b << 8) | (((b + 5) & 127) << 24), (((b + 9) & 127) << 8) | (((b + 17) & 127) << 24),
                                   (((b + 33) & 127) << 8) | (((b + 65) & 127) << 24), (((b + 3) & 127) << 8) | (((b + 7) & 127) << 24)};
#pragma unroll
                        for (int q = 0; q < 8; ++q) v[q] = 1.0 + q;
                    } else {
                        lq = *reinterpret_cast<const uint4 *>(li + j);
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const d2 t2 = *reinterpret_cast<const d2 *>(va + j + 2 * q);
                            v[2 * q] = t2.x;
                            v[2 * q + 1] = t2.y;
                        }
                    }
                    const unsigned lw[4] = {lq.x, lq.y, lq.z, lq.w};
                    const bool half = TAIL4 && j + 4 >= js + ((len + 3) & ~3);
                    d2 x0[8], x1[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const unsigned off = (lw[u >> 1] >> (16 * (u & 1))) & 0xFFFF;
                        x0[u] = *reinterpret_cast<const d2 *>(sb0 + off);
                        x1[u] = *reinterpret_cast<const d2 *>(sb1 + off);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        acc0 = madd(acc0, v[u], x0[u]);
                        acc1 = madd(acc1, v[u], x1[u]);
                    }
                    if (!half) {
#pragma unroll
                        for (int u = 4; u < 8; ++u) {
                            acc0 = madd(acc0, v[u], x0[u]);
                            acc1 = madd(acc1, v[u], x1[u]);
                        }
                    }
                }
                double *y = Y + (int64_t)row * KP + 2 * tl;
                *reinterpret_cast<d2 *>(y + 16 * par) = acc0;
                *reinterpret_cast<d2 *>(y + 16 * (par ^ 1)) = acc1;
            }
        }
        lds_barrier();
    }
}

// ---------------------------------------------------------------------------
struct Copy {
    double *X, *Y, *tvals;
    uint16_t *tlidx;
    int *rec, *rec2;
    uint16_t *tl3;
};

int main(int argc, char **argv)
{
    int m, n, *rp, *ci;
    int64_t nnz;
    double *va;
    if (argc < 2 || smfv_csr_read_bin(argv[1], &m, &n, &nnz, &rp, &ci, &va) != SMFV_OK) {
        printf("usage / read error\n");
        return 1;
    }
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    const int K = 32;
    TileCaps caps;
    caps.ucap = UC;
    caps.ncap = NC3;
    TileAnalysis T;
    analyse_tiles(m, n, rp, ci, T, caps);
    for (auto &tm : T.meta)
        if (tm.direct) {
            printf("direct tiles unsupported in lab\n");
            return 1;
        }
    std::vector<int> rec = pack_tile_records(T);
    // db2 records: rows / info at slot (i / 4) * 4 + i % 4 -> rowslot = team*4 + wave ... (identity: row i
    // sits at index i; the kernel's rowslot = tw * 4 + wv reads row i = rowslot), noff replicated
    std::vector<uint16_t> tl3(T.tlidx.size() + 1024, (uint16_t)ZROW);
    for (int64_t i = 0; i < T.padded_nnz; ++i)
        if (T.tsrc[i] >= 0) tl3[i] = (uint16_t)(T.tlidx[i] * 256);
    std::vector<int> rec2 = rec;
    for (size_t t = 0; t < T.meta.size(); ++t)
        for (int k = 0; k < 16; ++k) rec2[t * TREC_WORDS + 200 + k] = T.meta[t].noff;
    const int ntiles = (int)T.meta.size();
    std::vector<double> tv(T.padded_nnz + 1024, 0.0);
    T.tlidx.resize(T.padded_nnz + 1024, 0);
    for (int64_t i = 0; i < T.padded_nnz; ++i) tv[i] = T.tsrc[i] >= 0 ? va[T.tsrc[i]] : 0.0;
    {
        double wb = 0, ideal = 0;  // wave-batches (of 4) with one row per team, all 4 waves to the longest
        for (auto &tm : T.meta) {
            int lmax = 0;
            for (int k = 0; k < tm.nrows; ++k) {
                const int r = T.trows[tm.roff + k], L = rp[r + 1] - rp[r];
                lmax = std::max(lmax, L);
                ideal += (L + 3) / 4 / 8.0;
            }
            wb += 4.0 * ((lmax + 3) / 4);
        }
        printf("wave-batches: barrier-coupled %.0f, ideal %.0f (utilisation %.2f)\n", wb, ideal, ideal / wb);
    }
    printf("m %d nnz %lld tiles %d staged rows %lld reuse %.2f padded %lld\n", m, (long long)nnz, ntiles,
           (long long)T.union_rows, (double)T.tiled_nnz / T.union_rows, (long long)T.padded_nnz);

    // X: reference fat vector values 1..100 via hash fill; reference Y by production kernel
    int *d_rp, *d_ci;
    double *d_va;
    CK(hipMalloc(&d_rp, (m + 1) * 4));
    CK(hipMalloc(&d_ci, nnz * 4));
    CK(hipMalloc(&d_va, nnz * 8));
    CK(hipMemcpy(d_rp, rp, (m + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ci, ci, nnz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_va, va, nnz * 8, hipMemcpyHostToDevice));
    const int NCOPY = 12;
    std::vector<Copy> cp(NCOPY);
    for (auto &c : cp) {
        CK(hipMalloc(&c.X, (size_t)n * K * 8));
        CK(hipMalloc(&c.Y, (size_t)m * K * 8));
        CK(hipMalloc(&c.tvals, tv.size() * 8));
        CK(hipMalloc(&c.tlidx, T.tlidx.size() * 2));
        CK(hipMalloc(&c.rec, rec.size() * 4));
        CK(hipMalloc(&c.rec2, rec2.size() * 4));
        CK(hipMalloc(&c.tl3, tl3.size() * 2));
        CK(hipMemcpy(c.tl3, tl3.data(), tl3.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.rec2, rec2.data(), rec2.size() * 4, hipMemcpyHostToDevice));
        smfv_fill_x_hash_f64(n, K, 1, c.X, K, nullptr);
        CK(hipMemcpy(c.tvals, tv.data(), tv.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.tlidx, T.tlidx.data(), T.tlidx.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.rec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
    }
    double *d_ref;
    CK(hipMalloc(&d_ref, (size_t)m * K * 8));
    if (smfv_spmm_csr_f64(SMFV_ROWWISE, m, n, nnz, d_rp, d_ci, d_va, cp[0].X, K, K, d_ref, K, nullptr, 0,
                          nullptr) != SMFV_OK) {
        printf("ref: %s\n", smfv_last_error());
        return 1;
    }
    std::vector<double> href((size_t)m * K), hy((size_t)m * K);
    CK(hipMemcpy(href.data(), d_ref, href.size() * 8, hipMemcpyDeviceToHost));
    int ncu = 256;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double algo = 12.0 * nnz + 4.0 * (m + 1) + 16.0 * (double)n * K;

    auto run = [&](const char *name, auto launch, bool check) {
        CK(hipMemset(cp[0].Y, 0, (size_t)m * K * 8));
        launch(cp[0]);
        CK(hipDeviceSynchronize());
        bool ok = true;
        if (check) {
            CK(hipMemcpy(hy.data(), cp[0].Y, hy.size() * 8, hipMemcpyDeviceToHost));
            ok = memcmp(hy.data(), href.data(), hy.size() * 8) == 0;
            if (!ok) {
                int64_t bad = 0, first = -1;
                double md = 0;
                for (size_t i = 0; i < hy.size(); ++i)
                    if (memcmp(&hy[i], &href[i], 8)) {
                        if (first < 0) first = (int64_t)i;
                        ++bad;
                        md = std::max(md, fabs(hy[i] - href[i]) / std::max(fabs(href[i]), 1e-300));
                    }
                printf("  %lld mismatches, first at row %lld col %lld (got %g want %g), max rel %g\n", (long long)bad,
                       (long long)(first / K), (long long)(first % K), hy[first], href[first], md);
            }
        }
        float ms[2];
        for (int warm = 0; warm < 2; ++warm) {
            for (int i = 0; i < 20; ++i) launch(cp[warm ? 0 : i % NCOPY]);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) launch(cp[warm ? 0 : i % NCOPY]);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[warm], e0, e1));
        }
        const double cold = ms[0] * 1e3 / reps, warm = ms[1] * 1e3 / reps;
        printf("%-28s cold %7.2f us (%6.0f GB/s)  warm %7.2f us  %s\n", name, cold, algo / cold / 1e3, warm,
               check ? (ok ? "bit-exact" : "MISMATCH") : "-");
    };
    // production kernels for reference
    smfv_plan_t plan;
    if (smfv_plan_create(&plan, SMFV_ROWWISE, m, n, nnz, rp, ci, K, SMFV_PLAN_FORCE_TILES) != SMFV_OK) {
        printf("plan: %s\n", smfv_last_error());
        return 1;
    }
    // (the production plan binds to one values pointer: warm only)
    smfv_plan_bind_values(plan, d_va, nullptr);
    run("prod k_rows_mh", [&](Copy &c) {
        smfv_spmm_csr_f64(SMFV_ROWWISE, m, n, nnz, d_rp, d_ci, d_va, c.X, K, K, c.Y, K, nullptr, 0, nullptr);
    }, true);
    run("prod plan (X/Y rotate)", [&](Copy &c) {
        smfv_plan_execute(plan, d_rp, d_ci, d_va, c.X, K, c.Y, K, nullptr);
    }, true);
    const int blocks = 2 * ncu;
    run("db2", [&](Copy &c) {
        hipLaunchKernelGGL(k_rows_db2<0>, dim3(blocks), dim3(256), 0, 0, ntiles, c.rec2, c.tlidx, c.tvals, c.X, c.Y);
    }, true);
#define DB3(name, M, T4, F, chk)                                                                              \
    run(name, [&](Copy &c) {                                                                                \
        hipLaunchKernelGGL((k_rows_db3<M, T4, F>), dim3(blocks), dim3(256), 0, 0, ntiles, c.rec2, c.tl3, c.tvals, \
                           c.X, c.Y);                                                                        \
    }, chk)
    DB3("db3 skeleton", 3, true, false, false);
    DB3("db3 no-staging no-meta", 4, true, false, false);
    DB3("db3 b8+tail4", 0, true, false, true);
    DB3("db3 b8+tail4 no-staging", 2, true, false, false);
    DB3("db3 b8+tail4 no-compute", 1, true, false, false);
    DB3("db3 b8+tail4 FMA", 0, true, true, false);
    DB3("db3 b8+tail4 FMA no-staging", 2, true, true, false);
    return 0;
}
