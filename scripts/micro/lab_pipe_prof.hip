// Lab (not part of the product): per-wave phase timestamps of the pipelined
// tiled kernel.  Includes the kernel TU so it can launch the instrumented
// instantiation k_rows_pipe<0, 4> directly.
//   lab_pipe_prof <matrix.smfvcsr> <K> <out.bin>
// out.bin: int64 [blocks][16 steps][4 waves][4 phases] clock64 stamps:
// 0 step start, 1 compute done, 2 after barrier 1, 3 LDS staging written.
#include "../../sparsematrixmultiplicationmpi_amd/csrc/smfv_kernels.hip"
#include "smfv_host.h"

#include <cstdio>
#include <cstdlib>

int main(int argc, char **argv)
{
    if (argc < 4) return 2;
    int m, n, *rp, *ci;
    int64_t nnz;
    double *va;
    if (smfv_csr_read_bin(argv[1], &m, &n, &nnz, &rp, &ci, &va) != SMFV_OK) {
        printf("read: %s\n", smfv_last_error());
        return 1;
    }
    const int K = atoi(argv[2]);
    int *d_rp, *d_ci;
    double *d_va, *d_X, *d_Y;
    long long *d_prof;
    (void)hipMalloc(&d_rp, (m + 1) * 4);
    (void)hipMalloc(&d_ci, nnz * 4);
    (void)hipMalloc(&d_va, nnz * 8);
    (void)hipMalloc(&d_X, (size_t)n * K * 8);
    (void)hipMalloc(&d_Y, (size_t)m * K * 8);
    (void)hipMemcpy(d_rp, rp, (m + 1) * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ci, ci, nnz * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_va, va, nnz * 8, hipMemcpyHostToDevice);
    smfv_fill_x_hash_f64(n, K, 1, d_X, K, nullptr);
    smfv_plan_t plan;
    if (smfv_plan_create(&plan, SMFV_ROWWISE, m, n, nnz, rp, ci, K, 2) != SMFV_OK) {
        printf("plan: %s\n", smfv_last_error());
        return 1;
    }
    smfv_plan_bind_values(plan, d_va, nullptr);
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = std::min(plan->ntiles, 3 * ncu);
    const size_t pn = (size_t)blocks * 16 * 4 * 4;
    (void)hipMalloc(&d_prof, pn * 8);
    (void)hipMemset(d_prof, 0, pn * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 20; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_rows_pipe<0, 4>), dim3(blocks), dim3(256), 0, 0, plan->ntiles, plan->rec,
                           plan->tlidx, plan->tvals, d_rp, d_ci, d_va, d_X, (int64_t)K, K, d_Y, (int64_t)K, 1,
                           d_prof);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
    }
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("blocks %d tiles %d last launch %.2f us\n", blocks, plan->ntiles, ms * 1e3);
    std::vector<long long> h(pn);
    (void)hipMemcpy(h.data(), d_prof, pn * 8, hipMemcpyDeviceToHost);
    FILE *f = fopen(argv[3], "wb");
    fwrite(h.data(), 8, pn, f);
    fclose(f);
    smfv_plan_destroy(plan);
    return 0;
}
