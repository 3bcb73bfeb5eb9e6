// First-use cost of staging 64 MB for an H2D copy on this box: pageable 4 KiB
// pages, pageable huge pages (MADV_HUGEPAGE), and huge pages registered with
// hipHostRegister (pinned) -- each timed as fill + (register) + copy + sync, a
// fresh buffer every trial, and the copy alone on the second use.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char **argv)
{
    // trial order: argv[1] 'p' 4 KiB pages first, 't' huge pages first, 'g' registered first
    const int shift = argc > 1 ? (argv[1][0] == 't' ? 1 : argv[1][0] == 'g' ? 2 : 0) : 0;
    // argv[2]: MiB of a first warm-up copy (argv[3] 'r': from registered memory)
    const size_t warm = argc > 2 ? (size_t)std::atoi(argv[2]) << 20 : 0;
    const bool warm_reg = argc > 3 && argv[3][0] == 'r';
    const size_t n = 64ull << 20;
    void *d = nullptr;
    CK(hipMalloc(&d, n));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    {
        // the process's first copies: a 4 KiB pageable H2D and D2H (what a
        // device start-up can absorb), then the 64 MB trials below
        static char small[4096];
        for (int k = 0; k < 2; ++k) {
            double a = now();
            CK(hipMemcpyAsync(d, small, sizeof small, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            double b = now();
            CK(hipMemcpyAsync(small, d, sizeof small, hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            double c = now();
            std::printf("{\"small_copy\": %d, \"h2d_ms\": %.3f, \"d2h_ms\": %.3f}\n", k, 1e3 * (b - a), 1e3 * (c - b));
        }
    }
    if (warm) {
        char *w = (char *)mmap(nullptr, warm, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        std::memset(w, 1, warm);
        if (warm_reg) CK(hipHostRegister(w, warm, hipHostRegisterDefault));
        double a = now();
        CK(hipMemcpyAsync(d, w, warm, hipMemcpyHostToDevice, st));
        CK(hipStreamSynchronize(st));
        std::printf("{\"warm_MiB\": %zu, \"registered\": %d, \"ms\": %.3f}\n", warm >> 20, (int)warm_reg, 1e3 * (now() - a));
        if (warm_reg) CK(hipHostUnregister(w));
        munmap(w, warm);
    }
    const char *names[3] = {"pageable_4k", "pageable_thp", "registered_thp"};
    for (int trial = 0; trial < 2; ++trial)
        for (int mi = 0; mi < 3; ++mi) {
            const int mode = (mi + shift) % 3;
            double t0 = now();
            char *h = (char *)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (h == MAP_FAILED) return 1;
            if (mode >= 1) madvise(h, n, MADV_HUGEPAGE);
            std::memset(h, 1, n);
            double t1 = now();
            if (mode == 2) CK(hipHostRegister(h, n, hipHostRegisterDefault));
            double t2 = now();
            CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            double t3 = now();
            CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            double t4 = now();
            if (mode == 2) CK(hipHostUnregister(h));
            double t5 = now();
            munmap(h, n);
            std::printf("{\"trial\": %d, \"mode\": \"%s\", \"fill_ms\": %.3f, \"register_ms\": %.3f, \"first_copy_ms\": %.3f, "
                        "\"second_copy_ms\": %.3f, \"unregister_ms\": %.3f, \"first_GBps\": %.1f, \"second_GBps\": %.1f}\n",
                        trial, names[mode], 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3),
                        1e3 * (t5 - t4), n / (t3 - t2) / 1e9, n / (t4 - t3) / 1e9);
        }
    return 0;
}
