// Lab (not part of the product): "one block per CU" tiled row kernel.
//   lab_cu <matrix.smfvcsr> [reps]
// Tiles: <= 255 distinct X rows (64 KiB LDS image + a zero row), <= 64 rows,
// <= NCAP padded non-zeros; rows dealt to 32 eight-lane teams by LPT on their
// padded length (a team walks 1-4 rows back to back).  Staging by LDS-DMA
// into two slots (tile t+1 lands while tile t is computed), one barrier per
// tile.  Checked bit-for-bit against the production ROWWISE kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "smfv.h"
#include "smfv_host.h"
#include "smfv_plan.h"

using namespace smfv;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

#pragma clang fp contract(off)

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

constexpr int KP = 32;              // columns per panel
constexpr int UCAP = 255;           // union rows (row 255 of the image = zeros)
constexpr int NCAP = 1536;          // padded entries per tile
constexpr int NTEAM = 32;           // 8-lane teams per block
constexpr int RMAX = 4;             // rows per team
constexpr int ZOFF = UCAP * 256;    // byte offset of the zero row
// LDS slot layout (bytes)
// (V and L regions are whole 1 KiB DMA pieces: 128 doubles / 512 u16 each)
constexpr int SL_X = 0, SL_V = 65536, SL_L = SL_V + (NCAP + 127) / 128 * 1024,
              SL_R = SL_L + (NCAP + 511) / 512 * 1024, SL_BYTES = SL_R + 1024;
static_assert(2 * SL_BYTES <= 163840, "LDS");
// LDS record words
constexpr int R_TS = 0, R_ROW = 33, R_END = 97, R_T0 = 161;
// global record words (per tile): [0..255] union ids (per-lane order), [256..] replicated header
constexpr int G_U = 0, G_NOFF = 256, G_TN = 272, G_NU = 288, G_WORDS = 320;

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void glds16(const void *g, void *l)
{
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}
// The same LDS-DMA hidden from hipcc: the builtin makes hipcc wait vmcnt(0)
// before every later LDS read (it cannot tell the slots apart), which would
// serialise staging and compute.  Its completion is waited for by hand
// (s_waitcnt vmcnt(0) before the barrier that publishes the slot).
__device__ __forceinline__ void glds16_m0(const void *g, const void *l)
{
    const unsigned dst = (unsigned)(uintptr_t)l;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g), "s"(__builtin_amdgcn_readfirstlane(dst))
                 : "memory");
}
__device__ __forceinline__ void glds16_nt(const void *g, const void *l)
{
    unsigned keep;
    const unsigned dst = (unsigned)(uintptr_t)l;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(__builtin_amdgcn_readfirstlane(dst))
                 : "memory");
}
__device__ __forceinline__ void glds16_asm(const void *g, const void *l)
{
    unsigned keep;
    const unsigned dst = (unsigned)(uintptr_t)l;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(__builtin_amdgcn_readfirstlane(dst))
                 : "memory");
}
template <int V> __device__ __forceinline__ void glds_v(const void *g, void *l)
{
    if constexpr (V == 0) glds16_asm(g, l);
    else if constexpr (V == 1) glds16_m0(g, l);
    else glds16(g, l);
}


template <int MODE>  // 0 full; 1 staging only; 2 compute only (slot 0 staged once)
__global__ __launch_bounds__(256, 1) void k_rows_cu(int ntiles, const int *__restrict__ grec,
                                                    const int *__restrict__ lrec, const uint16_t *__restrict__ tlo,
                                                    const double *__restrict__ tv, const double *__restrict__ X,
                                                    int64_t ldx, double *__restrict__ Y, int64_t ldy, int m)
{
    __shared__ __attribute__((aligned(16))) char lds[2 * SL_BYTES];
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
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int team = tid >> 3, tl = tid & 7, par = team & 1;
    const int cp = blockIdx.y * KP;
    // zero rows of both slots
    if (tid < 32) reinterpret_cast<d2 *>(lds + (tid >> 4) * SL_BYTES + ZOFF)[tid & 15] = d2{0.0, 0.0};
    // per-lane record of the next tile to stage
    i4 u0, u1, u2v, u3;
    int noff, tn, nu;
    auto prefetch = [&](int t) {
        const int *G = grec + (int64_t)t * G_WORDS;
        const i4 *gu = reinterpret_cast<const i4 *>(G + G_U + wv * 64 + (lane >> 4) * 16);
        u0 = gu[0];
        u1 = gu[1];
        u2v = gu[2];
        u3 = gu[3];
        noff = G[G_NOFF + (lane & 15)];
        tn = G[G_TN + (lane & 15)];
        nu = G[G_NU + (lane & 15)];
    };
    auto stage = [&](int t, int s) {
        char *base = lds + s * SL_BYTES;
        const int uc[16] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w,
                            u2v.x, u2v.y, u2v.z, u2v.w, u3.x, u3.y, u3.z, u3.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int u = 4 * (16 * wv + i) + (lane >> 4);
            if (4 * (16 * wv + i) < nu && u < UCAP)
                glds16(X + (int64_t)uc[i] * ldx + cp + 2 * (lane & 15), base + SL_X + (16 * wv + i) * 1024);
        }
        for (int k = wv; k * 128 < tn; k += 4) glds16(tv + noff + 128 * k + 2 * lane, base + SL_V + k * 1024);
        for (int k = wv; k * 512 < tn; k += 4) glds16(tlo + noff + 512 * k + 8 * lane, base + SL_L + k * 1024);
        if (wv == 0) glds16(lrec + (int64_t)t * 256 + 4 * lane, base + SL_R);
    };
    prefetch(t0);
    stage(t0, 0);
    prefetch(min(t0 + tstep, tlast));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    const int nit = MODE == 2 ? cnt : cnt;
    for (int it = 0; it < nit; ++it) {
        const int c = MODE == 2 ? 0 : (it & 1);
        const int t = t0 + it * tstep;
        if (MODE != 2 && it + 1 < cnt) {
            stage(t + tstep, c ^ 1);
            prefetch(min(t + 2 * tstep, tlast));
        }
        if (MODE != 1) {
            const char *base = lds + c * SL_BYTES;
            const int *R = reinterpret_cast<const int *>(base + SL_R);
            const int ts = R[R_TS + team], te = R[R_TS + team + 1];
            const int r0 = R[R_T0 + team], r1 = R[R_T0 + team + 1];
            int rows[RMAX], ends[RMAX];
#pragma unroll
            for (int k = 0; k < RMAX; ++k) {
                rows[k] = R[R_ROW + min(r0 + k, 63)];
                ends[k] = r0 + k < r1 ? R[R_END + min(r0 + k, 63)] : 1 << 30;
            }
            const uint16_t *L = reinterpret_cast<const uint16_t *>(base + SL_L);
            const double *V = reinterpret_cast<const double *>(base + SL_V);
            const char *xb0 = base + SL_X + par * 128 + tl * 16;
            const char *xb1 = base + SL_X + (par ^ 1) * 128 + tl * 16;
            d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
            auto rdx = [&](u2 lq, d2 (&x0)[4], d2 (&x1)[4]) {
                const unsigned o[4] = {lq.x & 0xFFFF, lq.x >> 16, lq.y & 0xFFFF, lq.y >> 16};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    x0[u] = *reinterpret_cast<const d2 *>(xb0 + o[u]);
                    x1[u] = *reinterpret_cast<const d2 *>(xb1 + o[u]);
                }
            };
            auto rdl = [&](int j) { return *reinterpret_cast<const u2 *>(L + min(j, NCAP - 4)); };
            auto rdv = [&](int j, d2 &a, d2 &b) {
                a = *reinterpret_cast<const d2 *>(V + min(j, NCAP - 4));
                b = *reinterpret_cast<const d2 *>(V + min(j, NCAP - 4) + 2);
            };
            auto comp = [&](const d2 (&x0)[4], const d2 (&x1)[4], d2 va, d2 vb) {
                const double v[4] = {va.x, va.y, vb.x, vb.y};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc0 = acc0 + v[u] * x0[u];
                    acc1 = acc1 + v[u] * x1[u];
                }
            };
            int k = 0;
            auto boundary = [&](int jn) {  // after the batch ending at entry jn
                if (jn == ends[0]) {
                    if ((unsigned)rows[0] < (unsigned)m) {
                    double *y = Y + (int64_t)rows[0] * ldy + cp + 2 * tl;
                    *reinterpret_cast<d2 *>(y + 16 * par) = acc0;
                    *reinterpret_cast<d2 *>(y + 16 * (par ^ 1)) = acc1;
                    }
                    acc0 = d2{0.0, 0.0};
                    acc1 = d2{0.0, 0.0};
#pragma unroll
                    for (int q = 0; q + 1 < RMAX; ++q) {
                        rows[q] = rows[q + 1];
                        ends[q] = ends[q + 1];
                    }
                }
            };
            (void)k;
            // the team's stream is an even number of batches (planner): two
            // batches per iteration, no exit in between, so hipcc's LDS wait
            // counts stay exact and batch j+4's reads fly during batch j's math
            {
                d2 xA0[4], xA1[4], xB0[4], xB1[4], vA0, vA1, vB0, vB1;
                u2 lA = rdl(ts), lB;
                lB = rdl(ts + 4);
                rdx(lA, xA0, xA1);
                rdv(ts, vA0, vA1);
#define SB __builtin_amdgcn_sched_barrier(0)
                for (int j = ts; j < te; j += 8) {
                    lA = rdl(j + 8);
                    SB;
                    rdx(lB, xB0, xB1);
                    rdv(j + 4, vB0, vB1);
                    SB;
                    comp(xA0, xA1, vA0, vA1);
                    boundary(j + 4);
                    SB;
                    lB = rdl(j + 12);
                    SB;
                    rdx(lA, xA0, xA1);
                    rdv(j + 8, vA0, vA1);
                    SB;
                    comp(xB0, xB1, vB0, vB1);
                    boundary(j + 8);
                    SB;
                }
#undef SB
            }
        }
        if (MODE != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
    }
}


// ---------------------------------------------------------------------------
// k_rows_cu64: 512 threads (8 waves, 2 per SIMD), 64 eight-lane teams, one
// row per team per tile (rows dealt round-robin to the waves), rows padded
// to 8 entries.  Per 8 entries: the next 8 entries' meta (8 offsets in one
// b128, 8 values in four) is read right after this batch's 16 X reads, so
// the only value carried across the loop back-edge is meta that has had a
// whole batch to land (hipcc waits lgkmcnt(0) there, which then costs
// nothing).  FMA: lab only.
// LDS record (per tile, 1 KiB): [0..63] row id per team slot (-1 = none),
// [64..127] start | (padded length << 16) per team slot.
// ---------------------------------------------------------------------------
constexpr int NT64 = 64;
template <int MODE, bool FMA, bool IL = false>
__global__ __launch_bounds__(512, 1) void k_rows_cu64(int ntiles, const int *__restrict__ grec,
                                                      const int *__restrict__ lrec, const uint16_t *__restrict__ tlo,
                                                      const double *__restrict__ tv, const double *__restrict__ X,
                                                      int64_t ldx, double *__restrict__ Y, int64_t ldy, int m,
                                                      long long *__restrict__ prof = nullptr)
{
    __shared__ __attribute__((aligned(16))) char lds[2 * SL_BYTES];
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
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int tw = (tid >> 3) & 7, tl = tid & 7, par = tw & 1;
    long long *pw = MODE == 5 ? prof + ((int64_t)blockIdx.x * 16 * 8 + wv) * 5 : nullptr;  // [block][step][wave][5]
    auto stamp = [&](int it, int k) {
        if constexpr (MODE == 5)
            if (lane == 0 && it < 16) pw[(it * 8) * 5 + k] = __builtin_amdgcn_s_memtime();
    };
    const int slot = tw * 8 + wv;  // team slot: tile row i -> wave i % 8
    const int cp = blockIdx.y * KP;
    if (tid < 32) reinterpret_cast<d2 *>(lds + (tid >> 4) * SL_BYTES + ZOFF)[tid & 15] = d2{0.0, 0.0};
    i4 u0, u1;
    int noff, tn, nu;
    auto prefetch = [&](int t) {
        const int *G = grec + (int64_t)t * G_WORDS;
        const i4 *gu = reinterpret_cast<const i4 *>(G + G_U + wv * 32 + (lane >> 4) * 8);
        u0 = gu[0];
        u1 = gu[1];
        noff = G[G_NOFF + (lane & 15)];
        tn = G[G_TN + (lane & 15)];
        nu = G[G_NU + (lane & 15)];
    };
    auto stage = [&](int t, int s) {
        asm volatile("" ::"v"(u0), "v"(u1), "v"(noff), "v"(tn), "v"(nu));
        char *base = lds + s * SL_BYTES;
        const int uc[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int u = 4 * (8 * wv + i) + (lane >> 4);
            if (4 * (8 * wv + i) < nu && u < UCAP)
                glds16_asm(X + (int64_t)uc[i] * ldx + cp + 2 * (lane & 15), base + SL_X + (8 * wv + i) * 1024);
        }
        for (int k = wv; k * 128 < tn; k += 8) glds16_asm(tv + noff + 128 * k + 2 * lane, base + SL_V + k * 1024);
        for (int k = wv; k * 512 < tn; k += 8) glds16_asm(tlo + noff + 512 * k + 8 * lane, base + SL_L + k * 1024);
        if (wv == 7) glds16_asm(lrec + (int64_t)t * 256 + 4 * lane, base + SL_R);
    };
    auto madd = [&](d2 a, double v, d2 x) -> d2 {
        if constexpr (FMA)
            return d2{__builtin_fma(v, x.x, a.x), __builtin_fma(v, x.y, a.y)};
        else
            return a + v * x;
    };
    prefetch(t0);
    stage(t0, 0);
    prefetch(min(t0 + tstep, tlast));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    for (int it = 0; it < cnt; ++it) {
        const int c = MODE == 2 ? 0 : (it & 1);
        const int t = t0 + it * tstep;
        stamp(it, 0);
        if (MODE != 2 && it + 1 < cnt) {
            stage(t + tstep, c ^ 1);
            prefetch(min(t + 2 * tstep, tlast));
        }
        stamp(it, 1);
        if (MODE != 1) {
            const char *base = lds + c * SL_BYTES;
            const int *R = reinterpret_cast<const int *>(base + SL_R);
            const int row = R[slot];
            const int info = R[64 + slot];
            // IL: info = quad base chunk (16-B units) | len << 16; chunk q of this team at (base + 4q + k) * 16 B
            const int js = info & 0xFFFF, je = js + (info >> 16);
            const int qk = (tw & 3);
            const uint16_t *L = reinterpret_cast<const uint16_t *>(base + SL_L);
            const double *V = reinterpret_cast<const double *>(base + SL_V);
            const char *xb0 = base + SL_X + par * 128 + tl * 16;
            const char *xb1 = base + SL_X + (par ^ 1) * 128 + tl * 16;
            d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
            if (row >= 0) {
                // IL offsets: L chunk b (8 entries) at Lq + 4b + k; V chunk c (2 entries) at Vq + 4c + k (16-B units)
                const u4 *Lq = reinterpret_cast<const u4 *>(L) + (IL ? js + qk : 0);
                const d2 *Vq = reinterpret_cast<const d2 *>(V) + (IL ? (R[128 + slot] + qk) : 0);
                auto lrd = [&](int j) -> u4 {
                    if constexpr (IL) return Lq[4 * ((j - js) >> 3)];
                    else return *reinterpret_cast<const u4 *>(L + j);
                };
                u4 ln = lrd(js);
                d2 vn[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if constexpr (IL) vn[q] = Vq[4 * q];
                    else vn[q] = reinterpret_cast<const d2 *>(V + js)[q];
                }
                for (int j = js; j < je; j += 8) {
                    const unsigned lw[4] = {ln.x, ln.y, ln.z, ln.w};
                    const double v[8] = {vn[0].x, vn[0].y, vn[1].x, vn[1].y, vn[2].x, vn[2].y, vn[3].x, vn[3].y};
                    d2 x0[8], x1[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const unsigned o = (lw[u >> 1] >> (16 * (u & 1))) & 0xFFFF;
                        x0[u] = *reinterpret_cast<const d2 *>(xb0 + o);
                        x1[u] = *reinterpret_cast<const d2 *>(xb1 + o);
                    }
                    const int jn = min(j + 8, NCAP - 8);
                    // volatile: keeps the next batch's meta reads here, behind this batch's X reads
                    if constexpr (IL) {
                        const int b = min((j - js) / 8 + 1, (je - js) / 8 - 1);
                        ln = *(const volatile __attribute__((address_space(3))) u4 *)(Lq + 4 * b);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            vn[q] = *(const volatile __attribute__((address_space(3))) d2 *)(Vq + 4 * (4 * b + q));
                    } else {
                        ln = *(const volatile __attribute__((address_space(3))) u4 *)(L + jn);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            vn[q] = ((const volatile __attribute__((address_space(3))) d2 *)(V + jn))[q];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        acc0 = madd(acc0, v[u], x0[u]);
                        acc1 = madd(acc1, v[u], x1[u]);
                    }
                }
                if ((unsigned)row < (unsigned)m) {
                    double *y = Y + (int64_t)row * ldy + cp + 2 * tl;
                    *reinterpret_cast<d2 *>(y + 16 * par) = acc0;
                    *reinterpret_cast<d2 *>(y + 16 * (par ^ 1)) = acc1;
                }
            }
        }
        stamp(it, 2);
        if (MODE != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(it, 3);
        lds_barrier();
        stamp(it, 4);
    }
}


// ---------------------------------------------------------------------------
// k_rows_ws: k_rows_cu64<IL> with warp specialisation: waves 0-7 compute
// (64 eight-lane teams), waves 8-11 only stage the next tile by LDS-DMA
// (an LDS-DMA issue stalls its wave while the CU's texture path drains, so
// compute waves must not issue it).  One barrier per tile.
// ---------------------------------------------------------------------------
template <int MODE, bool FMA, bool PF = false, int DV = 0, int NLW = 4, bool RS = false, bool NT = false>
__global__ __launch_bounds__(512 + 64 * NLW, 1) void k_rows_ws(int ntiles, const int *__restrict__ grec,
                                                    const int *__restrict__ lrec, const uint16_t *__restrict__ tlo,
                                                    const double *__restrict__ tv, const double *__restrict__ X,
                                                    int64_t ldx, double *__restrict__ Y, int64_t ldy, int m,
                                                    long long *__restrict__ prof = nullptr)
{
    __shared__ __attribute__((aligned(16))) char lds[2 * SL_BYTES];
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
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int cp = blockIdx.y * KP;
    // MODE 5: stamps [block][step < 16][wave 0 / loader 8][4]
    auto stamp = [&](int it, int k) {
        if constexpr (MODE == 5)
            if (lane == 0 && it < 16 && (wv == 0 || wv == 8))
                prof[(((int64_t)blockIdx.x * 16 + it) * 2 + (wv >> 3)) * 4 + k] = __builtin_amdgcn_s_memtime();
    };
    if (wv >= 8) {
        // ---------------- loader waves ----------------
        const int wl = wv - 8;
        constexpr int IPW = 64 / NLW;  // X pieces (4 rows = 1 KiB) per loader wave
        if (wl == 0 && lane < 32) reinterpret_cast<d2 *>(lds + (lane >> 4) * SL_BYTES + ZOFF)[lane & 15] = d2{0.0, 0.0};
        i4 u0, u1, u2v, u3;
        int noff, tn, nu;
        auto prefetch = [&](int t) {
            const int *G = grec + (int64_t)t * G_WORDS;
            const i4 *gu = reinterpret_cast<const i4 *>(G + G_U + wl * 4 * IPW + (lane >> 4) * IPW);
            u0 = gu[0];
            u1 = gu[1];
            if constexpr (IPW == 16) {
                u2v = gu[2];
                u3 = gu[3];
            }
            noff = G[G_NOFF + (lane & 15)];
            tn = G[G_TN + (lane & 15)];
            nu = G[G_NU + (lane & 15)];
        };
        // hipcc cannot see the asm DMAs: any wait it places for these
        // registers at their first use (between two DMAs) would be counted
        // without them and stall on the DMAs just issued.  Resolving the
        // registers up front (all older loads are done) keeps its waits here.
        auto settle = [&]() {
            if constexpr (IPW == 16) asm volatile("" ::"v"(u0), "v"(u1), "v"(u2v), "v"(u3), "v"(noff), "v"(tn), "v"(nu));
            else asm volatile("" ::"v"(u0), "v"(u1), "v"(noff), "v"(tn), "v"(nu));
        };
        // RS: register staging.  Loader wave wl holds X pieces IPW*wl .. +IPW-1
        // (1 KiB each), value pieces wl and wl + NLW, and one more 1 KiB piece:
        // offsets (wl < 3) or the tile record (wl == 3).
        d2 rx[IPW];
        d2 rv[2];
        u4 rl;
        auto stage_regs_load = [&](int t) {
            settle();
            const int uc[16] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w,
                                u2v.x, u2v.y, u2v.z, u2v.w, u3.x, u3.y, u3.z, u3.w};
#pragma unroll
            for (int i = 0; i < IPW; ++i)
                rx[i] = *reinterpret_cast<const d2 *>(X + (int64_t)uc[i] * ldx + cp + 2 * (lane & 15));
#pragma unroll
            for (int q = 0; q < 2; ++q)
                rv[q] = *reinterpret_cast<const d2 *>(tv + noff + 128 * (wl + NLW * q) + 2 * lane);
            if (wl < 3) rl = *reinterpret_cast<const u4 *>(tlo + noff + 512 * wl + 8 * lane);
            else rl = *reinterpret_cast<const u4 *>(lrec + (int64_t)t * 256 + 4 * lane);
        };
        auto stage_regs_store = [&](int s) {
            char *base = lds + s * SL_BYTES;
#pragma unroll
            for (int i = 0; i < IPW; ++i)
                if (IPW * wl + i < 63 || lane < 48)  // row 255 of the image stays zero
                    reinterpret_cast<d2 *>(base + SL_X + (IPW * wl + i) * 1024)[lane] = rx[i];
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (wl + NLW * q < 12) reinterpret_cast<d2 *>(base + SL_V + (wl + NLW * q) * 1024)[lane] = rv[q];
            if (wl < 3) reinterpret_cast<u4 *>(base + SL_L + wl * 1024)[lane] = rl;
            else if (wl == 3) reinterpret_cast<u4 *>(base + SL_R)[lane] = rl;
        };
        auto stage = [&](int t, int s) {
            settle();
            char *base = lds + s * SL_BYTES;
            const int uc[16] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w,
                                u2v.x, u2v.y, u2v.z, u2v.w, u3.x, u3.y, u3.z, u3.w};
#pragma unroll
            for (int i = 0; i < IPW; ++i) {
                const int u = 4 * (IPW * wl + i) + (lane >> 4);
                if (4 * (IPW * wl + i) < nu && u < UCAP)
                    glds_v<DV>(X + (int64_t)uc[i] * ldx + cp + 2 * (lane & 15), base + SL_X + (IPW * wl + i) * 1024);
            }
            // meta and record are read once: non-temporal, so they do not push the
            // X rows (re-staged by ~6 tiles) out of the XCD's L2
            auto gm = [&](const void *g, void *l) {
                if constexpr (NT) glds16_nt(g, l);
                else glds_v<DV>(g, l);
            };
            for (int k = wl; k * 128 < tn; k += NLW) gm(tv + noff + 128 * k + 2 * lane, base + SL_V + k * 1024);
            for (int k = wl; k * 512 < tn; k += NLW) gm(tlo + noff + 512 * k + 8 * lane, base + SL_L + k * 1024);
            if (wl == NLW - 1) gm(lrec + (int64_t)t * 256 + 4 * lane, base + SL_R);
        };
        // PF: software L2 prefetch of the tile after next: one 4-byte load per
        // 128-B line (X rows of its union, its meta and record), results
        // discarded; its union ids come in natural order (id u of loader lane
        // wl*64 + lane at the permuted record position).
        unsigned dummy = 0;
        int pf_id = 0, pf_noff = 0, pf_tn = 0;
        auto pf_load = [&](int t) {
            const int *G = grec + (int64_t)t * G_WORDS;
            pf_id = G[G_U + wl * 64 + (lane & 3) * 16 + (lane >> 2)];
            pf_noff = G[G_NOFF + (lane & 15)];
            pf_tn = G[G_TN + (lane & 15)];
        };
        auto pf_issue = [&](int t) {
            asm volatile("" ::"v"(pf_id), "v"(pf_noff), "v"(pf_tn));
            const char *xr = reinterpret_cast<const char *>(X + (int64_t)pf_id * ldx + cp);
            asm volatile("global_load_dword %0, %1, off" : "+v"(dummy) : "v"(xr) : "memory");
            asm volatile("global_load_dword %0, %1, off offset:128" : "+v"(dummy) : "v"(xr) : "memory");
            // meta lines: V (tn*8 B), L (tn*2 B), record (1 KiB)
            const int line = wl * 64 + lane;
            const int nv = (pf_tn * 8 + 127) / 128, nl = (pf_tn * 2 + 127) / 128;
            const char *a;
            if (line < nv) a = reinterpret_cast<const char *>(tv + pf_noff) + line * 128;
            else if (line < nv + nl) a = reinterpret_cast<const char *>(tlo + pf_noff) + (line - nv) * 128;
            else a = reinterpret_cast<const char *>(lrec + (int64_t)t * 256) + ((line - nv - nl) & 7) * 128;
            asm volatile("global_load_dword %0, %1, off" : "+v"(dummy) : "v"(a) : "memory");
        };
        if constexpr (RS) {
            static_assert(NLW == 8, "RS layout assumes 8 loader waves");
            prefetch(t0);
            stage_regs_load(t0);
            prefetch(min(t0 + tstep, tlast));
            stage_regs_store(0);
            stage_regs_load(min(t0 + tstep, tlast));
            prefetch(min(t0 + 2 * tstep, tlast));
            lds_barrier();
            for (int it = 0; it < cnt; ++it) {
                const int c = it & 1;
                const int t = t0 + it * tstep;
                if (MODE != 2) {
                    stage_regs_store(c ^ 1);  // tile t + tstep (loaded one step ago)
                    stage_regs_load(min(t + 2 * tstep, tlast));
                    prefetch(min(t + 3 * tstep, tlast));
                }
                lds_barrier();
            }
            return;
        }
        prefetch(t0);
        stage(t0, 0);
        prefetch(min(t0 + tstep, tlast));
        if (PF) pf_load(min(t0 + 2 * tstep, tlast));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (PF) pf_issue(min(t0 + tstep, tlast));
        lds_barrier();
        for (int it = 0; it < cnt; ++it) {
            const int c = it & 1;
            const int t = t0 + it * tstep;
            stamp(it, 0);
            if (PF) asm volatile("s_waitcnt vmcnt(0)" : "+v"(dummy) :: "memory");
            if (MODE != 2 && it + 1 < cnt) {
                stage(t + tstep, c ^ 1);
                stamp(it, 1);
                if (PF) pf_issue(min(t + 2 * tstep, tlast));
                prefetch(min(t + 2 * tstep, tlast));
                if (PF) pf_load(min(t + 3 * tstep, tlast));
            }
            // DMAs are older than the prefetches (3) and the id loads (PF: 8 + 3 dwords, else 7)
            if (PF) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp(it, 2);
            lds_barrier();
            stamp(it, 3);
        }
        if (PF) asm volatile("s_waitcnt vmcnt(0)" : "+v"(dummy) :: "memory");
        return;
    }
    // ---------------- compute waves ----------------
    const int tw = (tid >> 3) & 7, tl = tid & 7, par = tw & 1;
    const int slot = tw * 8 + wv;
    const int qk = tw & 3;
    auto madd = [&](d2 a, double v, d2 x) -> d2 {
        if constexpr (FMA)
            return d2{__builtin_fma(v, x.x, a.x), __builtin_fma(v, x.y, a.y)};
        else
            return a + v * x;
    };
    lds_barrier();
    for (int it = 0; it < cnt; ++it) {
        const int c = MODE == 2 ? 0 : (it & 1);
        stamp(it, 0);
        if (MODE != 1) {
            const char *base = lds + c * SL_BYTES;
            const int *R = reinterpret_cast<const int *>(base + SL_R);
            const int row = R[slot];
            const int info = R[64 + slot];
            const int js = info & 0xFFFF, je = js + (info >> 16);
            const uint16_t *L = reinterpret_cast<const uint16_t *>(base + SL_L);
            const double *V = reinterpret_cast<const double *>(base + SL_V);
            const char *xb0 = base + SL_X + par * 128 + tl * 16;
            const char *xb1 = base + SL_X + (par ^ 1) * 128 + tl * 16;
            d2 acc0 = {0.0, 0.0}, acc1 = {0.0, 0.0};
            if (row >= 0) {
                const u4 *Lq = reinterpret_cast<const u4 *>(L) + js + qk;
                const d2 *Vq = reinterpret_cast<const d2 *>(V) + R[128 + slot] + qk;
                u4 ln = Lq[0];
                d2 vn[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) vn[q] = Vq[4 * q];
                for (int j = js; j < je; j += 8) {
                    const unsigned lw[4] = {ln.x, ln.y, ln.z, ln.w};
                    const double v[8] = {vn[0].x, vn[0].y, vn[1].x, vn[1].y, vn[2].x, vn[2].y, vn[3].x, vn[3].y};
                    d2 x0[8], x1[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const unsigned o = (lw[u >> 1] >> (16 * (u & 1))) & 0xFFFF;
                        x0[u] = *reinterpret_cast<const d2 *>(xb0 + o);
                        x1[u] = *reinterpret_cast<const d2 *>(xb1 + o);
                    }
                    const int b = min((j - js) / 8 + 1, (je - js) / 8 - 1);
                    ln = *(const volatile __attribute__((address_space(3))) u4 *)(Lq + 4 * b);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        vn[q] = *(const volatile __attribute__((address_space(3))) d2 *)(Vq + 4 * (4 * b + q));
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        acc0 = madd(acc0, v[u], x0[u]);
                        acc1 = madd(acc1, v[u], x1[u]);
                    }
                }
                if ((unsigned)row < (unsigned)m) {
                    double *y = Y + (int64_t)row * ldy + cp + 2 * tl;
                    if constexpr (NT) {
                        __builtin_nontemporal_store(acc0, reinterpret_cast<d2 *>(y + 16 * par));
                        __builtin_nontemporal_store(acc1, reinterpret_cast<d2 *>(y + 16 * (par ^ 1)));
                    } else {
                        *reinterpret_cast<d2 *>(y + 16 * par) = acc0;
                        *reinterpret_cast<d2 *>(y + 16 * (par ^ 1)) = acc1;
                    }
                }
            }
        }
        stamp(it, 1);
        stamp(it, 2);
        lds_barrier();
        stamp(it, 3);
    }
}

// ---------------------------------------------------------------------------
// host planner
// ---------------------------------------------------------------------------
struct CuPlan {
    int ntiles = 0;
    std::vector<int> grec, lrec;
    std::vector<uint16_t> tl;
    std::vector<int> tsrc;  // entry -> CSR index or -1
    double util = 0;
};

static bool build_cu_plan(int m, int n, const int *rp, const int *ci, CuPlan &P)
{
    TileCaps caps;
    caps.ucap = UCAP;
    caps.ncap = NCAP - 4 - 4 * NTEAM;  // rows padded to 4, + even batches per team, + tile closed at 8
    caps.pad = 4;
    caps.maxrows = 64;
    TileAnalysis T;
    analyse_tiles(m, n, rp, ci, T, caps);
    P = CuPlan();
    double ideal = 0, used = 0;
    for (size_t ti = 0; ti < T.meta.size(); ++ti) {
        const TileMeta &tm = T.meta[ti];
        if (tm.direct) {
            printf("direct tile unsupported in lab\n");
            return false;
        }
        // union position of each column
        std::vector<int> rows(T.trows.begin() + tm.roff, T.trows.begin() + tm.roff + tm.nrows);
        std::sort(rows.begin(), rows.end(), [&](int a, int b) {
            const int la = rp[a + 1] - rp[a], lb = rp[b + 1] - rp[b];
            return la != lb ? la > lb : a < b;
        });
        std::vector<std::vector<int>> team(NTEAM);
        std::vector<int> load(NTEAM, 0);
        for (int r : rows) {
            const int b = std::max(1, (rp[r + 1] - rp[r] + 3) / 4);
            int best = 0;
            for (int q = 1; q < NTEAM; ++q)
                if (load[q] < load[best] || (load[q] == load[best] && team[q].size() < team[best].size())) best = q;
            if ((int)team[best].size() >= RMAX) {
                printf("team over RMAX\n");
                return false;
            }
            team[best].push_back(r);
            load[best] += b;
            ideal += b;
        }
        used += (double)*std::max_element(load.begin(), load.end()) * NTEAM;
        // union map from the analysis (ucols in first-use order)
        std::vector<int> ucols(T.ucols.begin() + tm.uoff, T.ucols.begin() + tm.uoff + tm.nu);
        std::vector<int> lrec(256, 0), grec(G_WORDS, 0);
        const int noff = (int)P.tl.size();
        int e = 0, ri = 0;
        for (int q = 0; q < NTEAM; ++q) {
            lrec[R_TS + q] = e;
            lrec[R_T0 + q] = ri;
            for (int r : team[q]) {
                const int rs = e;
                for (int j = rp[r]; j < rp[r + 1]; ++j) {
                    const int u = (int)(std::find(ucols.begin(), ucols.end(), ci[j]) - ucols.begin());
                    P.tl.push_back((uint16_t)(u * 256));
                    P.tsrc.push_back(j);
                    ++e;
                }
                while (e % 4 || e == rs) {  // pad to a whole batch; an empty row gets one batch of pads
                    P.tl.push_back((uint16_t)ZOFF);
                    P.tsrc.push_back(-1);
                    ++e;
                }
                lrec[R_ROW + ri] = r;
                lrec[R_END + ri] = e;
                ++ri;
            }
            while ((e - lrec[R_TS + q]) % 8) {  // even number of batches per team
                P.tl.push_back((uint16_t)ZOFF);
                P.tsrc.push_back(-1);
                ++e;
            }
        }
        lrec[R_TS + NTEAM] = e;
        lrec[R_T0 + NTEAM] = ri;
        while (e % 8) {
            P.tl.push_back((uint16_t)ZOFF);
            P.tsrc.push_back(-1);
            ++e;
        }
        if (e > NCAP) {
            printf("tile over NCAP (%d)\n", e);
            return false;
        }
        for (int w = 0; w < 4; ++w)
            for (int q = 0; q < 4; ++q)
                for (int i = 0; i < 16; ++i) {
                    const int u = 4 * (16 * w + i) + q;
                    grec[G_U + w * 64 + q * 16 + i] = u < tm.nu ? ucols[u] : 0;
                }
        for (int q = 0; q < 16; ++q) {
            grec[G_NOFF + q] = noff;
            grec[G_TN + q] = e;
            grec[G_NU + q] = tm.nu;
        }
        P.grec.insert(P.grec.end(), grec.begin(), grec.end());
        P.lrec.insert(P.lrec.end(), lrec.begin(), lrec.end());
    }
    P.ntiles = (int)T.meta.size();
    P.util = ideal / used;
    // host-side validation of every address the kernel derives from the plan
    for (int t = 0; t < P.ntiles; ++t) {
        const int *g = &P.grec[(size_t)t * G_WORDS];
        const int *l = &P.lrec[(size_t)t * 256];
        const int noff = g[G_NOFF], tn = g[G_TN], nu = g[G_NU];
        if (tn > NCAP || nu > UCAP || noff % 8) { printf("bad tile header %d\n", t); return false; }
        for (int q = 0; q < 256; ++q)
            if (g[q] < 0 || g[q] >= n) { printf("bad ucol\n"); return false; }
        for (int q = 0; q < NTEAM; ++q) {
            if (l[R_TS + q] > l[R_TS + q + 1] || l[R_TS + q] % 4) { printf("bad team range\n"); return false; }
            if (l[R_T0 + q + 1] - l[R_T0 + q] > RMAX) { printf("bad team rows\n"); return false; }
            for (int k = l[R_T0 + q]; k < l[R_T0 + q + 1]; ++k) {
                if (l[R_ROW + k] < 0 || l[R_ROW + k] >= m) { printf("bad row\n"); return false; }
                if (l[R_END + k] > l[R_TS + q + 1] || l[R_END + k] <= (k == l[R_T0 + q] ? l[R_TS + q] : l[R_END + k - 1]) ||
                    l[R_END + k] % 4) {
                    printf("bad row end\n");
                    return false;
                }
            }
            if ((l[R_TS + q + 1] - l[R_TS + q]) % 8 ||
                (l[R_T0 + q + 1] > l[R_T0 + q] && l[R_END + l[R_T0 + q + 1] - 1] + 4 < l[R_TS + q + 1])) {
                printf("team stream end mismatch\n");
                return false;
            }
        }
        for (int j = 0; j < l[R_TS + NTEAM]; ++j)
            if (P.tl[noff + j] > ZOFF || P.tl[noff + j] % 256) { printf("bad offset\n"); return false; }
    }
    // DMA over-read slack
    P.tl.resize(P.tl.size() + 2048, (uint16_t)ZOFF);
    P.tsrc.resize(P.tsrc.size() + 2048, -1);
    for (int t = 0; t < P.ntiles; ++t) {
        const int noff = P.grec[(size_t)t * G_WORDS + G_NOFF], tn = P.grec[(size_t)t * G_WORDS + G_TN];
        if ((size_t)(noff + (tn + 511) / 512 * 512) > P.tl.size()) { printf("DMA over-read\n"); return false; }
    }
    printf("cu plan: tiles %d staged rows %lld reuse %.2f entries %zu util %.3f\n", P.ntiles,
           (long long)T.union_rows, (double)T.tiled_nnz / T.union_rows, P.tl.size(), P.util);
    return true;
}


static bool build_cu64_plan(int m, int n, const int *rp, const int *ci, CuPlan &P)
{
    TileCaps caps;
    caps.ucap = UCAP;
    caps.ncap = NCAP - 8;
    caps.maxrows = NT64;
    caps.pad = 8;
    TileAnalysis T;
    analyse_tiles(m, n, rp, ci, T, caps);
    P = CuPlan();
    double ideal = 0, used = 0;
    for (size_t ti = 0; ti < T.meta.size(); ++ti) {
        const TileMeta &tm = T.meta[ti];
        if (tm.direct) { printf("direct tile unsupported in lab\n"); return false; }
        std::vector<int> rows(T.trows.begin() + tm.roff, T.trows.begin() + tm.roff + tm.nrows);
        std::sort(rows.begin(), rows.end(), [&](int a, int b) {
            const int la = rp[a + 1] - rp[a], lb = rp[b + 1] - rp[b];
            return la != lb ? la > lb : a < b;
        });
        std::vector<int> ucols(T.ucols.begin() + tm.uoff, T.ucols.begin() + tm.uoff + tm.nu);
        std::vector<int> pos(n, -1);
        for (int u = 0; u < tm.nu; ++u) pos[ucols[u]] = u;
        std::vector<int> lrec(256, 0), grec(G_WORDS, 0);
        for (int q = 0; q < NT64; ++q) lrec[q] = -1;
        const int noff = (int)P.tl.size();
        int e = 0;
        std::vector<int> wmax(8, 0);
        for (int i = 0; i < (int)rows.size(); ++i) {
            const int r = rows[i];
            // row i -> wave i % 8, team i / 8 -> slot = team * 8 + wave = i
            const int rs = e;
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                P.tl.push_back((uint16_t)(pos[ci[j]] * 256));
                P.tsrc.push_back(j);
                ++e;
            }
            while (e % 8 || e == rs) { P.tl.push_back((uint16_t)ZOFF); P.tsrc.push_back(-1); ++e; }
            lrec[i] = r;
            lrec[64 + i] = rs | ((e - rs) << 16);
            ideal += (rp[r + 1] - rp[r] + 3) / 4;
            wmax[i % 8] = std::max(wmax[i % 8], (e - rs) / 4);
        }
        for (int w = 0; w < 8; ++w) used += 8.0 * wmax[w];
        if (e > NCAP) { printf("tile over NCAP (%d)\n", e); return false; }
        for (int w = 0; w < 8; ++w)
            for (int q = 0; q < 4; ++q)
                for (int i = 0; i < 8; ++i) {
                    const int u = 4 * (8 * w + i) + q;
                    grec[G_U + w * 32 + q * 8 + i] = u < tm.nu ? ucols[u] : 0;
                }
        for (int q = 0; q < 16; ++q) { grec[G_NOFF + q] = noff; grec[G_TN + q] = e; grec[G_NU + q] = tm.nu; }
        P.grec.insert(P.grec.end(), grec.begin(), grec.end());
        P.lrec.insert(P.lrec.end(), lrec.begin(), lrec.end());
    }
    P.ntiles = (int)T.meta.size();
    P.util = ideal / used;
    P.tl.resize(P.tl.size() + 2048, (uint16_t)ZOFF);
    P.tsrc.resize(P.tsrc.size() + 2048, -1);
    for (int t = 0; t < P.ntiles; ++t) {
        const int *g = &P.grec[(size_t)t * G_WORDS];
        const int *l = &P.lrec[(size_t)t * 256];
        if (g[G_TN] > NCAP || g[G_NU] > UCAP || g[G_NOFF] % 8) { printf("bad header\n"); return false; }
        if ((size_t)(g[G_NOFF] + (g[G_TN] + 511) / 512 * 512) > P.tl.size()) { printf("DMA over-read\n"); return false; }
        for (int q = 0; q < 256; ++q) if (g[q] < 0 || g[q] >= n) { printf("bad ucol\n"); return false; }
        for (int q = 0; q < NT64; ++q) {
            if (l[q] < -1 || l[q] >= m) { printf("bad row\n"); return false; }
            if (l[q] >= 0) {
                const int js = l[64 + q] & 0xFFFF, len = l[64 + q] >> 16;
                if (js % 8 || len % 8 || len == 0 || js + len > g[G_TN]) { printf("bad segment\n"); return false; }
                for (int j = js; j < js + len; ++j)
                    if (P.tl[g[G_NOFF] + j] > ZOFF || P.tl[g[G_NOFF] + j] % 256) { printf("bad offset\n"); return false; }
            }
        }
    }
    printf("cu64 plan: tiles %d staged rows %lld reuse %.2f entries %zu util %.3f\n", P.ntiles,
           (long long)T.union_rows, (double)T.tiled_nnz / T.union_rows, P.tl.size(), P.util);
    return true;
}

// interleaved meta: the 4 teams of a lane group (a "quad": wave w, teams 4h..4h+3)
// store batch b of team k at L chunk Lbase + 4b + k and value pair c at V
// chunk Vbase + 4c + k (16-B chunks), so one meta read of a lane group hits
// four different bank quarters.
static bool build_cu64i_plan(int m, int n, const int *rp, const int *ci, CuPlan &P, int LW = 8)
{
    const int IPW = 64 / LW;  // X DMA instructions per loader wave
    TileCaps caps;
    caps.ucap = UCAP;
    caps.ncap = NCAP - 96;
    caps.maxrows = NT64;
    caps.pad = 8;
    TileAnalysis T;
    analyse_tiles(m, n, rp, ci, T, caps);
    P = CuPlan();
    double ideal = 0, used = 0;
    int64_t padwaste = 0;
    for (size_t ti = 0; ti < T.meta.size(); ++ti) {
        const TileMeta &tm = T.meta[ti];
        if (tm.direct) { printf("direct tile unsupported in lab\n"); return false; }
        std::vector<int> rows(T.trows.begin() + tm.roff, T.trows.begin() + tm.roff + tm.nrows);
        std::sort(rows.begin(), rows.end(), [&](int a, int b) {
            const int la = rp[a + 1] - rp[a], lb = rp[b + 1] - rp[b];
            return la != lb ? la > lb : a < b;
        });
        std::vector<int> ucols(T.ucols.begin() + tm.uoff, T.ucols.begin() + tm.uoff + tm.nu);
        std::vector<int> pos(n, -1);
        for (int u = 0; u < tm.nu; ++u) pos[ucols[u]] = u;
        std::vector<int> lrec(256, 0), grec(G_WORDS, 0);
        for (int q = 0; q < NT64; ++q) lrec[q] = -1;
        // quad q = sorted rows 4q..4q+3 (similar lengths: little interleave padding) -> wave q % 8,
        // teams 4 (q / 8) .. +3; team slot = tw * 8 + w
        auto len8 = [&](int i) { return i < (int)rows.size() ? std::max(8, (rp[rows[i] + 1] - rp[rows[i]] + 7) & ~7) : 0; };
        std::vector<uint16_t> Lt;  // in 16-B chunks of 8 u16
        std::vector<int> Vt;       // CSR index per value slot (-1 pad), 2 per chunk
        std::vector<int> wmax(8, 0);
        for (int q = 0; q < 16; ++q) {
            const int w = q % 8, h = q / 8;
            int nb = 0;
            for (int k = 0; k < 4; ++k) nb = std::max(nb, len8(4 * q + k) / 8);
            if (nb == 0) continue;
            const int lbase = (int)Lt.size() / 8, vbase = (int)Vt.size() / 2;
            Lt.resize(Lt.size() + 32 * nb, (uint16_t)ZOFF);
            Vt.resize(Vt.size() + 32 * nb, -1);
            for (int k = 0; k < 4; ++k) {
                const int i = 4 * q + k;
                if (i >= (int)rows.size()) continue;
                const int r = rows[i], slot = (4 * h + k) * 8 + w;
                for (int j = rp[r]; j < rp[r + 1]; ++j) {
                    const int e = j - rp[r];
                    Lt[(lbase + 4 * (e / 8) + k) * 8 + e % 8] = (uint16_t)(pos[ci[j]] * 256);
                    Vt[(vbase + 4 * (e / 2) + k) * 2 + e % 2] = j;
                }
                lrec[slot] = r;
                lrec[64 + slot] = lbase | (len8(i) << 16);
                lrec[128 + slot] = vbase;
                ideal += (rp[r + 1] - rp[r] + 3) / 4;
                wmax[w] = std::max(wmax[w], len8(i) / 4);
                padwaste += 8 * nb - len8(i);
            }
        }
        for (int w = 0; w < 8; ++w) used += 8.0 * wmax[w];
        const int e = (int)Lt.size();  // entries (L and V hold the same count)
        if (e > NCAP) { printf("tile over NCAP (%d)\n", e); return false; }
        const int noff = (int)P.tl.size();
        // L and V are separate streams with their own layouts but the same entry count
        P.tl.insert(P.tl.end(), Lt.begin(), Lt.end());
        P.tsrc.insert(P.tsrc.end(), Vt.begin(), Vt.end());
        for (int w = 0; w < LW; ++w)
            for (int q = 0; q < 4; ++q)
                for (int i = 0; i < IPW; ++i) {
                    const int u = 4 * (IPW * w + i) + q;
                    grec[G_U + w * 4 * IPW + q * IPW + i] = u < tm.nu ? ucols[u] : 0;
                }
        for (int q = 0; q < 16; ++q) { grec[G_NOFF + q] = noff; grec[G_TN + q] = e; grec[G_NU + q] = tm.nu; }
        P.grec.insert(P.grec.end(), grec.begin(), grec.end());
        P.lrec.insert(P.lrec.end(), lrec.begin(), lrec.end());
    }
    P.ntiles = (int)T.meta.size();
    P.util = ideal / used;
    P.tl.resize(P.tl.size() + 2048, (uint16_t)ZOFF);
    P.tsrc.resize(P.tsrc.size() + 2048, -1);
    for (int t = 0; t < P.ntiles; ++t) {
        const int *g = &P.grec[(size_t)t * G_WORDS];
        const int *l = &P.lrec[(size_t)t * 256];
        if (g[G_TN] > NCAP || g[G_NU] > UCAP || g[G_NOFF] % 8) { printf("bad header\n"); return false; }
        if ((size_t)(g[G_NOFF] + (g[G_TN] + 511) / 512 * 512) > P.tl.size()) { printf("DMA over-read\n"); return false; }
        for (int q = 0; q < 256; ++q) if (g[q] < 0 || g[q] >= n) { printf("bad ucol\n"); return false; }
        for (int q = 0; q < NT64; ++q) {
            if (l[q] < -1 || l[q] >= m) { printf("bad row\n"); return false; }
            if (l[q] >= 0) {
                const int lb = l[64 + q] & 0xFFFF, len = l[64 + q] >> 16, vb = l[128 + q];
                const int k = (q / 8) & 3;
                if (len % 8 || len == 0) { printf("bad len\n"); return false; }
                if ((lb + 4 * (len / 8 - 1) + k + 1) * 8 > g[G_TN] || (vb + 4 * (len / 2 - 1) + k + 1) * 2 > g[G_TN]) {
                    printf("segment out of tile\n");
                    return false;
                }
            }
        }
        for (int j = 0; j < g[G_TN]; ++j)
            if (P.tl[g[G_NOFF] + j] > ZOFF || P.tl[g[G_NOFF] + j] % 256) { printf("bad offset\n"); return false; }
    }
    printf("cu64i plan: tiles %d staged rows %lld reuse %.2f entries %zu util %.3f quad pad %lld\n", P.ntiles,
           (long long)T.union_rows, (double)T.tiled_nnz / T.union_rows, P.tl.size(), P.util, (long long)padwaste);
    return true;
}

// ---------------------------------------------------------------------------
struct Copy {
    double *X, *Y, *tv;
    uint16_t *tl;
    int *grec, *lrec;
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
    CuPlan P;
    if (!build_cu_plan(m, n, rp, ci, P)) return 1;
    CuPlan Q;
    if (!build_cu64_plan(m, n, rp, ci, Q)) return 1;
    CuPlan Qi, Qw;
    if (!build_cu64i_plan(m, n, rp, ci, Qi)) return 1;
    if (!build_cu64i_plan(m, n, rp, ci, Qw, 4)) return 1;
    std::vector<double> tvh(P.tsrc.size());
    for (size_t i = 0; i < tvh.size(); ++i) tvh[i] = P.tsrc[i] >= 0 ? va[P.tsrc[i]] : 0.0;

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
        CK(hipMalloc(&c.tv, tvh.size() * 8));
        CK(hipMalloc(&c.tl, P.tl.size() * 2));
        CK(hipMalloc(&c.grec, P.grec.size() * 4));
        CK(hipMalloc(&c.lrec, P.lrec.size() * 4));
        smfv_fill_x_hash_f64(n, K, 1, c.X, K, nullptr);
        CK(hipMemcpy(c.tv, tvh.data(), tvh.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.tl, P.tl.data(), P.tl.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.grec, P.grec.data(), P.grec.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.lrec, P.lrec.data(), P.lrec.size() * 4, hipMemcpyHostToDevice));
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
                for (size_t i = 0; i < hy.size(); ++i)
                    if (memcmp(&hy[i], &href[i], 8)) {
                        if (first < 0) first = (int64_t)i;
                        ++bad;
                    }
                printf("  %lld mismatches, first at row %lld col %lld (got %g want %g)\n", (long long)bad,
                       (long long)(first / K), (long long)(first % K), hy[first], href[first]);
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
        printf("%-30s cold %7.2f us (%6.0f GB/s)  warm %7.2f us  %s\n", name, cold, algo / cold / 1e3, warm,
               check ? (ok ? "bit-exact" : "MISMATCH") : "-");
    };
    run("prod k_rows_mh", [&](Copy &c) {
        smfv_spmm_csr_f64(SMFV_ROWWISE, m, n, nnz, d_rp, d_ci, d_va, c.X, K, K, c.Y, K, nullptr, 0, nullptr);
    }, true);
    const int blocks = std::min(ncu, P.ntiles);
    std::vector<double> tvq(Q.tsrc.size());
    for (size_t i = 0; i < tvq.size(); ++i) tvq[i] = Q.tsrc[i] >= 0 ? va[Q.tsrc[i]] : 0.0;
    std::vector<Copy> cq(NCOPY);
    for (int i = 0; i < NCOPY; ++i) {
        Copy &c = cq[i];
        c.X = cp[i].X;
        c.Y = cp[i].Y;
        CK(hipMalloc(&c.tv, tvq.size() * 8));
        CK(hipMalloc(&c.tl, Q.tl.size() * 2));
        CK(hipMalloc(&c.grec, Q.grec.size() * 4));
        CK(hipMalloc(&c.lrec, Q.lrec.size() * 4));
        CK(hipMemcpy(c.tv, tvq.data(), tvq.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.tl, Q.tl.data(), Q.tl.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.grec, Q.grec.data(), Q.grec.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.lrec, Q.lrec.data(), Q.lrec.size() * 4, hipMemcpyHostToDevice));
    }
    const int blocks64 = std::min(ncu, Q.ntiles);
    std::vector<double> tvi(Qi.tsrc.size());
    for (size_t i = 0; i < tvi.size(); ++i) tvi[i] = Qi.tsrc[i] >= 0 ? va[Qi.tsrc[i]] : 0.0;
    std::vector<Copy> ci_(NCOPY);
    for (int i = 0; i < NCOPY; ++i) {
        Copy &c = ci_[i];
        c.X = cp[i].X;
        c.Y = cp[i].Y;
        CK(hipMalloc(&c.tv, tvi.size() * 8));
        CK(hipMalloc(&c.tl, Qi.tl.size() * 2));
        CK(hipMalloc(&c.grec, Qi.grec.size() * 4));
        CK(hipMalloc(&c.lrec, Qi.lrec.size() * 4));
        CK(hipMemcpy(c.tv, tvi.data(), tvi.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.tl, Qi.tl.data(), Qi.tl.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.grec, Qi.grec.data(), Qi.grec.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(c.lrec, Qi.lrec.data(), Qi.lrec.size() * 4, hipMemcpyHostToDevice));
    }
    const int blocks64i = std::min(ncu, Qi.ntiles);
    std::vector<Copy> cw_(NCOPY);
    for (int i = 0; i < NCOPY; ++i) {
        Copy &c = cw_[i];
        c = ci_[i];
        CK(hipMalloc(&c.grec, Qw.grec.size() * 4));
        CK(hipMemcpy(c.grec, Qw.grec.data(), Qw.grec.size() * 4, hipMemcpyHostToDevice));
    }
#define CU64I(name, M, F, chk)                                                                                 \
    run(name, [&](Copy &cc) {                                                                                \
        Copy &c = ci_[&cc - &cp[0]];                                                                         \
        hipLaunchKernelGGL((k_rows_cu64<M, F, true>), dim3(blocks64i), dim3(512), 0, 0, Qi.ntiles, c.grec, c.lrec, \
                           c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m);                                 \
    }, chk)
    CU64I("cu64i", 0, false, true);
    CU64I("cu64i staging only", 1, false, false);
    CU64I("cu64i compute only", 2, false, false);
    CU64I("cu64i FMA", 0, true, false);
    CU64I("cu64i FMA compute only", 2, true, false);
#define PFX false
#define WS(name, M, F, chk)                                                                                    \
    run(name, [&](Copy &cc) {                                                                                \
        Copy &c = cw_[&cc - &cp[0]];                                                                         \
        hipLaunchKernelGGL((k_rows_ws<M, F, PFX>), dim3(blocks64i), dim3(768), 0, 0, Qi.ntiles, c.grec, c.lrec,       \
                           c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m);                                 \
    }, chk)
    WS("ws", 0, false, true);
    WS("ws staging only", 1, false, false);
    WS("ws compute only", 2, false, false);
    WS("ws FMA", 0, true, false);
#undef PFX
#define PFX true
    run("ws8 (8 loader waves)", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<0, false, false, 0, 8>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles, c.grec, c.lrec,
                           c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, true);
    run("ws8 staging only", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<1, false, false, 0, 8>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles, c.grec, c.lrec,
                           c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, false);
    run("ws8 RS (register staging)", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<0, false, false, 0, 8, true>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles, c.grec,
                           c.lrec, c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, true);
    run("ws8 RS staging only", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<1, false, false, 0, 8, true>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles, c.grec,
                           c.lrec, c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, false);
    run("ws8 RS FMA", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<0, true, false, 0, 8, true>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles, c.grec,
                           c.lrec, c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, false);
    run("ws8 NT", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<0, false, false, 0, 8, false, true>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles,
                           c.grec, c.lrec, c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, true);
    run("ws8 NT staging only", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<1, false, false, 0, 8, false, true>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles,
                           c.grec, c.lrec, c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, false);
    run("ws8 NT FMA", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<0, true, false, 0, 8, false, true>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles,
                           c.grec, c.lrec, c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, false);
    run("ws8 FMA", [&](Copy &cc) {
        Copy &c = ci_[&cc - &cp[0]];
        hipLaunchKernelGGL((k_rows_ws<0, true, false, 0, 8>), dim3(blocks64i), dim3(1024), 0, 0, Qi.ntiles, c.grec, c.lrec,
                           c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, nullptr);
    }, false);
    {
        long long *d_prof;
        const size_t pn = (size_t)blocks64i * 16 * 2 * 4;
        CK(hipMalloc(&d_prof, pn * 8));
        CK(hipMemset(d_prof, 0, pn * 8));
        for (int r = 0; r < 30; ++r) {
            Copy &c = cw_[r % NCOPY];
            hipLaunchKernelGGL((k_rows_ws<5, false, false>), dim3(blocks64i), dim3(768), 0, 0, Qi.ntiles, c.grec, c.lrec,
                               c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, d_prof);
        }
        CK(hipDeviceSynchronize());
        std::vector<long long> h(pn);
        CK(hipMemcpy(h.data(), d_prof, pn * 8, hipMemcpyDeviceToHost));
        for (int who = 0; who < 2; ++who) {
            const char *names[2][3] = {{"compute", "-", "barrier"}, {"DMA issue", "DMA land", "barrier"}};
            for (int k = 0; k < 3; ++k) {
                std::vector<long long> d;
                for (int b = 0; b < blocks64i; ++b)
                    for (int it = 1; it < 15; ++it) {
                        const long long *e = &h[(((size_t)b * 16 + it) * 2 + who) * 4];
                        if (e[0] && e[3] && e[k] && e[k + 1]) d.push_back(e[k + 1] - e[k]);
                    }
                std::sort(d.begin(), d.end());
                if (!d.empty() && names[who][k][0] != '-')
                    printf("  ws %s %-10s median %6lld p10 %6lld p90 %6lld\n", who ? "loader " : "compute", names[who][k],
                           d[d.size() / 2], d[d.size() / 10], d[d.size() * 9 / 10]);
            }
        }
    }
    {
        long long *d_prof;
        const size_t pn = (size_t)blocks64i * 16 * 8 * 5;
        CK(hipMalloc(&d_prof, pn * 8));
        CK(hipMemset(d_prof, 0, pn * 8));
        for (int r = 0; r < 30; ++r) {
            Copy &c = ci_[r % NCOPY];
            hipLaunchKernelGGL((k_rows_cu64<5, false, true>), dim3(blocks64i), dim3(512), 0, 0, Qi.ntiles, c.grec, c.lrec,
                               c.tl, c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m, d_prof);
        }
        CK(hipDeviceSynchronize());
        std::vector<long long> h(pn);
        CK(hipMemcpy(h.data(), d_prof, pn * 8, hipMemcpyDeviceToHost));
        // per phase: median over (block, step>=1, wave) of stamp deltas (s_memtime ticks)
        const char *names[4] = {"stage issue", "compute", "vmcnt wait", "barrier"};
        for (int k = 0; k < 4; ++k) {
            std::vector<long long> d;
            for (int b = 0; b < blocks64i; ++b)
                for (int it = 1; it < 16; ++it)
                    for (int w = 0; w < 8; ++w) {
                        const long long *e = &h[(((size_t)b * 16 + it) * 8 + w) * 5];
                        if (e[0] && e[4]) d.push_back(e[k + 1] - e[k]);
                    }
            std::sort(d.begin(), d.end());
            if (!d.empty())
                printf("  phase %-12s median %6lld p10 %6lld p90 %6lld ticks (n=%zu)\n", names[k], d[d.size() / 2],
                       d[d.size() / 10], d[d.size() * 9 / 10], d.size());
        }
        std::vector<long long> tot;
        for (int b = 0; b < blocks64i; ++b) {
            const long long *e0 = &h[((size_t)b * 16 * 8) * 5];
            long long last = 0;
            for (int it = 0; it < 16; ++it) { const long long *e = &h[(((size_t)b * 16 + it) * 8) * 5]; if (e[4]) last = e[4]; }
            if (e0[0] && last) tot.push_back(last - e0[0]);
        }
        std::sort(tot.begin(), tot.end());
        if (!tot.empty()) printf("  block loop span median %lld max %lld ticks\n", tot[tot.size() / 2], tot.back());
    }
#define CU64(name, M, F, chk)                                                                                  \
    run(name, [&](Copy &cc) {                                                                                \
        Copy &c = cq[&cc - &cp[0]];                                                                          \
        hipLaunchKernelGGL((k_rows_cu64<M, F>), dim3(blocks64), dim3(512), 0, 0, Q.ntiles, c.grec, c.lrec, c.tl, \
                           c.tv, c.X, (int64_t)K, c.Y, (int64_t)K, m);                                       \
    }, chk)
    CU64("cu64", 0, false, true);
    CU64("cu64 staging only", 1, false, false);
    CU64("cu64 compute only", 2, false, false);
    CU64("cu64 FMA", 0, true, false);
    CU64("cu64 FMA compute only", 2, true, false);
#define CU(name, M, chk)                                                                                       \
    run(name, [&](Copy &c) {                                                                                 \
        hipLaunchKernelGGL((k_rows_cu<M>), dim3(blocks), dim3(256), 0, 0, P.ntiles, c.grec, c.lrec, c.tl, c.tv, \
                           c.X, (int64_t)K, c.Y, (int64_t)K, m);                                                \
    }, chk)

    return 0;
}
