#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef double d2 __attribute__((ext_vector_type(2)));
// 1) global_load_lds_dwordx4 from an 8-byte (not 16-byte) aligned source
__global__ void k_mis(const double *src, double *out)
{
    __shared__ __attribute__((aligned(16))) double lds[128];
    const int lane = threadIdx.x;
    for (int i = lane; i < 128; i += 64) lds[i] = -1.0;
    __syncthreads();
    const double *g = src + 1 + 2 * lane;  // 8-byte aligned
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds)) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = lane; i < 128; i += 64) out[i] = lds[i];
}
// 2) buffer_load_dwordx4 ... lds with a range-checked descriptor: bytes [0, nrec)
__global__ void k_buf(const double *src, int nrec, double *out)
{
    __shared__ __attribute__((aligned(16))) double lds[128];
    const int lane = threadIdx.x;
    for (int i = lane; i < 128; i += 64) lds[i] = -1.0;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, nrec, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)lds, 16, 16 * lane, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = lane; i < 128; i += 64) out[i] = lds[i];
}
// 3) the same into VGPRs
__global__ void k_bufv(const double *src, int nrec, double *out)
{
    const int lane = threadIdx.x;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, nrec, 0x00020000);
    d2 v = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, 16 * lane, 0, 0));
    out[2 * lane] = v.x;
    out[2 * lane + 1] = v.y;
}
int main()
{
    double h[260], *d, *o, ho[128];
    for (int i = 0; i < 260; ++i) h[i] = i + 1;
    hipMalloc(&d, sizeof h);
    hipMalloc(&o, sizeof ho);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mis, 1, 64, 0, 0, d, o);
    hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 128; ++i) bad += ho[i] != h[1 + i];
    printf("misaligned global_load_lds_dwordx4: %s (lane0 %g %g, lane1 %g %g)\n", bad ? "WRONG" : "exact", ho[0], ho[1], ho[2], ho[3]);
    for (int nrec : {24, 40, 8 * 127}) {
        hipLaunchKernelGGL(k_buf, 1, 64, 0, 0, d, nrec, o);
        hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
        printf("buffer lds nrec %d: lane0 %g %g lane1 %g %g lane2 %g %g | last %g %g\n", nrec, ho[0], ho[1], ho[2], ho[3], ho[4], ho[5], ho[126], ho[127]);
        hipLaunchKernelGGL(k_bufv, 1, 64, 0, 0, d, nrec, o);
        hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
        printf("buffer vgpr nrec %d: lane0 %g %g lane1 %g %g lane2 %g %g | last %g %g\n", nrec, ho[0], ho[1], ho[2], ho[3], ho[4], ho[5], ho[126], ho[127]);
    }
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
