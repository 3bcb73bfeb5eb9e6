// Lab micro-benchmarks (not part of the product): f64 VALU rate, LDS b128
// latency and team-pattern LDS read throughput on the box's GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_valu(double *out, int iters, double a, long long *stamps)
{
    long long c0 = clock64(), w0 = wall_clock64();
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3 + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { double p = x[k] * a; x[k] = p + 1e-9; }  // mul + add
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k];
    if (s == 12345.678) out[0] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { stamps[0] = clock64() - c0; stamps[1] = wall_clock64() - w0; }
}

// one wave, pointer chase through LDS with ds_read_b128
__global__ __launch_bounds__(64) void k_lds_lat(long long *out, int iters)
{
    __shared__ __attribute__((aligned(16))) int4 buf[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) buf[i] = make_int4((i * 97 + 13) & 2047, 0, 0, 0);
    __syncthreads();
    int p = threadIdx.x;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) p = buf[p].x;
    long long t1 = clock64();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

// team pattern: 8-lane teams read 128-B halves of 256-B rows (parity swizzled), U rows in flight
template <int U>
__global__ __launch_bounds__(256) void k_lds_team(double *out, int iters)
{
    __shared__ __attribute__((aligned(16))) double s_x[128 * 32];
    for (int i = threadIdx.x; i < 128 * 32; i += 256) s_x[i] = i;
    __syncthreads();
    const int tid = threadIdx.x, team = tid >> 3, tl = tid & 7, par = team & 1;
    const double2 *sx0 = reinterpret_cast<const double2 *>(s_x) + par * 8 + tl;
    const double2 *sx1 = reinterpret_cast<const double2 *>(s_x) + (par ^ 1) * 8 + tl;
    double2 a0 = make_double2(0, 0), a1 = a0;
    unsigned l = (team * 37) & 127;
    for (int i = 0; i < iters; ++i) {
        double2 x0[U], x1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned lu = (l + u * 29) & 127;
            x0[u] = sx0[lu * 16];
            x1[u] = sx1[lu * 16];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { a0.x += x0[u].x; a0.y += x0[u].y; a1.x += x1[u].x; a1.y += x1[u].y; }
        l = (l + 11) & 127;
    }
    if (a0.x + a0.y + a1.x + a1.y == 1.2345) out[0] = a0.x;
}

int main()
{
    double *d;
    long long *dl;
    CK(hipMalloc(&d, 64));
    CK(hipMalloc(&dl, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int dev = 0, ncu = 0, clk = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
    printf("CUs %d clock %d kHz\n", ncu, clk);
    // VALU: blocks x 256 threads x iters x 8 x 2 f64 ops
    for (int bpc : {1, 2, 3, 4}) {
        const int blocks = ncu * bpc, iters = 20000;
        hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, d, 100, 1.0000001, dl);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0000001, dl);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double winst = (double)blocks * 4 * iters * 16;  // wave-instructions (f64)
        const double per_simd = winst / (ncu * 4.0);
        printf("valu f64 waves/SIMD=%d: %.3f ms, %.2f clk per wave-instr per SIMD, %.1f TFLOP/s (mul+add)\n", bpc, ms,
               (ms * 1e-3 * clk * 1e3) / per_simd, (double)blocks * 256 * iters * 16 / (ms * 1e-3) / 1e12);
        long long st[2];
        CK(hipMemcpy(st, dl, 16, hipMemcpyDeviceToHost));
        int wr = 0;
        CK(hipDeviceGetAttribute(&wr, hipDeviceAttributeWallClockRate, dev));
        printf("   block0: clock64 %lld ticks, wall_clock64 %lld ticks (%d kHz) -> %.1f us wall, clock64 rate %.3f GHz\n",
               st[0], st[1], wr, st[1] / (wr * 1e-3), st[0] / (st[1] / (wr * 1e3)) / 1e9);
    }
    {
        hipLaunchKernelGGL(k_lds_lat, dim3(1), dim3(64), 0, 0, dl, 10000);
        CK(hipDeviceSynchronize());
        long long h[2];
        CK(hipMemcpy(h, dl, 16, hipMemcpyDeviceToHost));
        printf("lds b128 dependent latency: %.1f clk (clock64 units)\n", h[0] / 10000.0);
    }
    auto team = [&](auto kern, int U, int bpc) -> int {
        const int blocks = ncu * bpc, iters = 4000;
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 10);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double bytes = (double)blocks * 256 * iters * U * 32;  // 2 x 16 B per lane per u
        printf("lds team U=%d blocks/CU=%d: %.3f ms, %.1f B/clk/CU, %.1f TB/s\n", U, bpc, ms,
               bytes / ncu / (ms * 1e-3 * clk * 1e3), bytes / (ms * 1e-3) / 1e12);
        return 0;
    };
    for (int bpc : {1, 3}) {
        team(k_lds_team<1>, 1, bpc);
        team(k_lds_team<4>, 4, bpc);
        team(k_lds_team<8>, 8, bpc);
    }
    return 0;
}
