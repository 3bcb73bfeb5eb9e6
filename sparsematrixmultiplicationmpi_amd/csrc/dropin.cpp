// dropin.cpp -- the reference's C++ call surface over the libsmfv C ABI
// (libsmfv_mpi.so).  Callers written against SC/SparseMatrixFatVectorMultiply*.h
// and SC/utils.h link this instead of the reference's .cpp files.
//
//   sparseMatrixFatVectorMultiply*   SC/SparseMatrixFatVectorMultiply*.cpp
//   areMatricesEqual                 SC/utils.cpp:38-63
//   readMatrixMarketFile             SC/utils.cpp:70-185   (-> smfv_mtx_read)
//   generateLargeFatVector           SC/utils.cpp:193-209  (rand() % 100 + 1)
//   serialize / deserialize          SC/utils.cpp:216-253
// plus the extensions of include/smfv_dropin.h (device-resident inputs,
// device-side result check).
//
// Every call goes through a PLAN cached by matrix pattern (variant, sizes,
// K, world size and a 64-bit hash of rowPtr and colIndices): the first call
// on a pattern analyses it (the tiled kernel's row tiles, or the rank's
// share of a distributed variant); later calls only bind the values and
// launch.  A call therefore runs the same kernels the bench times
// (k_rows_ws where the pattern re-uses X rows).
//
// Device placement: rank r of MPI_COMM_WORLD uses GPU (local rank % devices).
// The RCCL communicator is created on first collective use (rank 0 makes the
// unique id, MPI_Bcast hands it out: MPI is only the bootstrap, every data
// movement of the SpMM itself is RCCL over xGMI).
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "SparseMatrixFatVectorMultiply.h"
#include "SparseMatrixFatVectorMultiplyColumnWise.h"
#include "SparseMatrixFatVectorMultiplyNonZeroElement.h"
#include "SparseMatrixFatVectorMultiplyRowWise.h"
#include "smfv.h"
#include "smfv_dropin.h"
#include "smfv_host.h"
#include "utils.h"

#define DROPIN_API __attribute__((visibility("default")))

namespace {

struct Context {
    bool init = false;
    bool mpi = false;
    int rank = 0, size = 1;
    smfv_comm_t comm = nullptr;
    hipStream_t stream = nullptr;
};

Context g_ctx;

[[noreturn]] void fail(const std::string &what)
{
    int mpi_on = 0, fin = 0;
    MPI_Initialized(&mpi_on);
    MPI_Finalized(&fin);
    if (mpi_on && !fin) {
        std::fprintf(stderr, "smfv: %s\n", what.c_str());
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    throw std::runtime_error("smfv: " + what);
}

void check(int rc, const char *where)
{
    if (rc != SMFV_OK) fail(std::string(where) + ": " + smfv_last_error());
}

void hip_check(hipError_t e, const char *where)
{
    if (e != hipSuccess) fail(std::string(where) + ": " + hipGetErrorString(e));
}

Context &ctx()
{
    if (g_ctx.init) return g_ctx;
    int on = 0;
    MPI_Initialized(&on);
    g_ctx.mpi = on != 0;
    int local = 0;
    if (g_ctx.mpi) {
        MPI_Comm_rank(MPI_COMM_WORLD, &g_ctx.rank);
        MPI_Comm_size(MPI_COMM_WORLD, &g_ctx.size);
        MPI_Comm node;
        MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, g_ctx.rank, MPI_INFO_NULL, &node);
        MPI_Comm_rank(node, &local);
        MPI_Comm_free(&node);
    }
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev <= 0) fail("no HIP device");
    hip_check(hipSetDevice(local % ndev), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking), "hipStreamCreate");
    g_ctx.init = true;
    return g_ctx;
}

smfv_comm_t comm_world()
{
    Context &c = ctx();
    if (c.comm || c.size == 1) return c.comm;
    char id[SMFV_UNIQUE_ID_BYTES] = {0};
    if (c.rank == 0) check(smfv_comm_unique_id(id), "smfv_comm_unique_id");
    MPI_Bcast(id, SMFV_UNIQUE_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
    check(smfv_comm_init(&c.comm, c.size, c.rank, id), "smfv_comm_init");
    return c.comm;
}

// Buffers reused across calls (grow-only): device copies of A, X, Y, the
// kept reference result, and pinned host staging for X (in) and Y (out), so
// a call pays no hipMalloc and its X / Y transfers run at pinned-copy speed
// (the FatVector <-> flat conversion and the rank-0
// rebuild are a large share of the reference's RowWise time).
struct Cached {
    void *p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    void *get(size_t bytes)
    {
        if (bytes <= cap) return p;
        release();
        const size_t b = std::max<size_t>(bytes, 256);
        if (pinned)
            hip_check(hipHostMalloc(&p, b, hipHostMallocDefault), "hipHostMalloc");
        else
            hip_check(hipMalloc(&p, b), "hipMalloc");
        cap = b;
        return p;
    }
    void release()
    {
        if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        cap = 0;
    }
};

struct Buffers {
    Cached rp, ci, va, X, Y, ref, hX{nullptr, 0, true}, hY{nullptr, 0, true};
    // the result of the last call on this rank (device) and the kept reference
    const double *lastY = nullptr;
    int last_m = -1, last_K = -1, ref_m = -1, ref_K = -1;
};

Buffers &bufs()
{
    static Buffers *b = new Buffers;  // process lifetime (freed with the context at exit)
    return *b;
}

// host rows [0, rows) processed in parallel (plain threads: the copies are
// memory-bound and the FatVector side is m separate allocations)
template <class F> void par_rows(int64_t rows, F f)
{
    const int nt = rows < 4096 ? 1 : (int)std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency()));
    if (nt == 1) {
        f((int64_t)0, rows);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(f, rows * t / nt, rows * (t + 1) / nt);
    for (auto &x : th) x.join();
}

// 64-bit hash of a byte range (8-byte words, multiply-xorshift; chunks in parallel)
uint64_t hash_bytes(const void *data, size_t bytes)
{
    const size_t nw = bytes / 8;
    const uint64_t *w = static_cast<const uint64_t *>(data);
    const int nchunk = nw < (1u << 16) ? 1 : 8;  // one chunk per thread
    std::vector<uint64_t> part((size_t)nchunk, 0);
    auto work = [&](int64_t a, int64_t b) {
        for (int64_t c = a; c < b; ++c) {
            const size_t i0 = nw * (size_t)c / (size_t)nchunk;
            const size_t i1 = nw * (size_t)(c + 1) / (size_t)nchunk;
            uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)c;
            for (size_t i = i0; i < i1; ++i) {
                uint64_t x;
                std::memcpy(&x, w + i, 8);
                h = (h ^ x) * 0xBF58476D1CE4E5B9ull;
                h ^= h >> 29;
            }
            part[(size_t)c] = h;
        }
    };
    std::vector<std::thread> th;
    for (int c = 1; c < nchunk; ++c) th.emplace_back(work, c, c + 1);
    work(0, 1);
    for (auto &t : th) t.join();
    uint64_t h = bytes;
    for (uint64_t x : part) h = (h ^ x) * 0x94D049BB133111EBull, h ^= h >> 31;
    const unsigned char *tail = static_cast<const unsigned char *>(data) + nw * 8;
    for (size_t i = 0; i < bytes % 8; ++i) h = (h ^ tail[i]) * 0x100000001B3ull;
    return h;
}

// inputs distributed by smfvDistributeInputs: device copies kept resident
// (own buffers: a call with other inputs does not overwrite them)
struct Resident {
    bool on = false;
    const SparseMatrix *A = nullptr;
    const FatVector *fat = nullptr;
    const double *va_host = nullptr;
    const int *ci_host = nullptr, *rp_host = nullptr;
    size_t nnz = 0, rows = 0;
    int m = 0, n = 0, K = 0;
    uint64_t hrp = 0, hci = 0;
    Cached rp, ci, va, X;
    bool matches(const SparseMatrix &Am, const FatVector &f, int K_) const
    {
        return on && &Am == A && &f == fat && K_ == K && Am.values.data() == va_host &&
               Am.colIndices.data() == ci_host && Am.rowPtr.data() == rp_host && Am.values.size() == nnz &&
               Am.numRows == m && Am.numCols == n && f.size() == rows;
    }
};

Resident &resident()
{
    static Resident *r = new Resident;
    return *r;
}

// A and X on the device for one call
struct Problem {
    int m, n, K;
    int64_t nnz;
    int *rp, *ci;
    double *va, *X, *Y;
    uint64_t hrp = 0, hci = 0;  // pattern hashes (plan cache key)
    Problem(const SparseMatrix &A, const FatVector &fat, int K_, hipStream_t st)
        : m(A.numRows), n(A.numCols), K(K_), nnz((int64_t)A.values.size())
    {
        if ((int)A.rowPtr.size() != m + 1 || (int64_t)A.colIndices.size() != nnz ||
            (m >= 0 && A.rowPtr.size() && A.rowPtr[m] != nnz))
            fail("malformed SparseMatrix (rowPtr / colIndices / values sizes)");
        if ((int)fat.size() != n)
            fail("fatVector has " + std::to_string(fat.size()) + " rows, matrix has " + std::to_string(n) + " columns");
        Buffers &B = bufs();
        Y = static_cast<double *>(B.Y.get((size_t)m * K * sizeof(double)));
        Resident &R = resident();
        if (R.matches(A, fat, K)) {  // device-resident inputs: nothing to upload
            rp = static_cast<int *>(R.rp.p);
            ci = static_cast<int *>(R.ci.p);
            va = static_cast<double *>(R.va.p);
            X = static_cast<double *>(R.X.p);
            hrp = R.hrp;
            hci = R.hci;
            return;
        }
        for (const auto &r : fat)
            if ((int)r.size() != K) fail("fatVector rows must have vecCols entries");
        rp = static_cast<int *>(B.rp.get(A.rowPtr.size() * sizeof(int)));
        ci = static_cast<int *>(B.ci.get(A.colIndices.size() * sizeof(int)));
        va = static_cast<double *>(B.va.get(A.values.size() * sizeof(double)));
        X = static_cast<double *>(B.X.get((size_t)n * K * sizeof(double)));
        // serialize (SC/utils.cpp:216-228) straight into pinned staging
        double *hx = static_cast<double *>(B.hX.get((size_t)n * K * sizeof(double)));
        par_rows(n, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) std::copy(fat[i].begin(), fat[i].end(), hx + (size_t)i * K);
        });
        auto up = [&](void *d, const void *h, size_t bytes) {
            if (bytes) hip_check(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
        };
        up(rp, A.rowPtr.data(), A.rowPtr.size() * sizeof(int));
        up(ci, A.colIndices.data(), A.colIndices.size() * sizeof(int));
        up(va, A.values.data(), A.values.size() * sizeof(double));
        up(X, hx, (size_t)n * K * sizeof(double));
        hrp = hash_bytes(A.rowPtr.data(), A.rowPtr.size() * sizeof(int));
        hci = hash_bytes(A.colIndices.data(), A.colIndices.size() * sizeof(int));
    }
    FatVector download(hipStream_t st)
    {
        double *hy = static_cast<double *>(bufs().hY.get((size_t)m * K * sizeof(double)));
        if ((size_t)m * K)
            hip_check(hipMemcpyAsync(hy, Y, (size_t)m * K * sizeof(double), hipMemcpyDeviceToHost, st),
                      "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
        // deserialize (SC/utils.cpp:238-253): the m row vectors built in parallel
        FatVector out((size_t)m);
        par_rows(m, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) out[i].assign(hy + (size_t)i * K, hy + (size_t)(i + 1) * K);
        });
        return out;
    }
    void note_result()
    {
        Buffers &B = bufs();
        B.lastY = Y;
        B.last_m = m;
        B.last_K = K;
    }
};

// plan cache (least recently used out; a plan holds device memory)
struct PlanKey {
    int variant, m, n, K, world;
    int64_t nnz;
    uint64_t hrp, hci;
    bool operator==(const PlanKey &o) const
    {
        return variant == o.variant && m == o.m && n == o.n && K == o.K && world == o.world && nnz == o.nnz &&
               hrp == o.hrp && hci == o.hci;
    }
};
struct PlanEntry {
    PlanKey key;
    smfv_plan_t local = nullptr;
    smfv_dist_plan_t dist = nullptr;
    uint64_t used = 0;
};
constexpr size_t kMaxPlans = 8;

std::vector<PlanEntry> &plans()
{
    static auto *v = new std::vector<PlanEntry>;
    return *v;
}

PlanEntry &plan_for(int variant, const SparseMatrix &A, const Problem &P, int world)
{
    static uint64_t tick = 0;
    // on one rank SEQUENTIAL / ROWWISE / COLUMNWISE are the same computation
    // (bit-identical per-row sums): they share one plan
    if (world == 1 && variant != SMFV_NONZERO) variant = SMFV_ROWWISE;
    const PlanKey key{variant, P.m, P.n, P.K, world, P.nnz, P.hrp, P.hci};
    auto &v = plans();
    for (auto &e : v)
        if (e.key == key) {
            e.used = ++tick;
            return e;
        }
    if (v.size() >= kMaxPlans) {
        auto lru = std::min_element(v.begin(), v.end(), [](const PlanEntry &a, const PlanEntry &b) { return a.used < b.used; });
        if (lru->local) smfv_plan_destroy(lru->local);
        if (lru->dist) smfv_dist_plan_destroy(lru->dist);
        v.erase(lru);
    }
    PlanEntry e;
    e.key = key;
    e.used = ++tick;
    if (world == 1)
        check(smfv_plan_create(&e.local, variant, P.m, P.n, P.nnz, A.rowPtr.data(), A.colIndices.data(), P.K, 0),
              "smfv_plan_create");
    else
        check(smfv_dist_plan_create(&e.dist, comm_world(), variant, SMFV_TO_ROOT, 0, P.m, P.n, P.nnz, A.rowPtr.data(),
                                    A.colIndices.data(), P.K, 0),
              "smfv_dist_plan_create");
    v.push_back(e);
    return v.back();
}

FatVector local_run(int variant, const SparseMatrix &A, const FatVector &fat, int K)
{
    Context &c = ctx();
    Problem P(A, fat, K, c.stream);
    PlanEntry &e = plan_for(variant, A, P, 1);
    check(smfv_plan_bind_values(e.local, P.va, c.stream), "smfv_plan_bind_values");
    check(smfv_plan_execute(e.local, P.rp, P.ci, P.va, P.X, K, P.Y, K, c.stream), "smfv_plan_execute");
    P.note_result();
    return P.download(c.stream);
}

FatVector collective_run(int variant, const SparseMatrix &A, const FatVector &fat, int K)
{
    Context &c = ctx();
    if (c.size == 1) return local_run(variant, A, fat, K);
    Problem P(A, fat, K, c.stream);
    PlanEntry &e = plan_for(variant, A, P, c.size);
    check(smfv_dist_plan_bind_values(e.dist, P.va, c.stream), "smfv_dist_plan_bind_values");
    check(smfv_dist_plan_execute(e.dist, P.rp, P.ci, P.va, P.X, P.Y, c.stream), "smfv_dist_plan_execute");
    if (c.rank != 0) {
        hip_check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
        return FatVector{};
    }
    P.note_result();
    return P.download(c.stream);
}

}  // namespace

DROPIN_API FatVector sparseMatrixFatVectorMultiply(const SparseMatrix &sparseMatrix,
                                                   const FatVector &fatVector, int vecCols)
{
    return local_run(SMFV_SEQUENTIAL, sparseMatrix, fatVector, vecCols);
}

DROPIN_API FatVector sparseMatrixFatVectorMultiplyRowWise(const SparseMatrix &sparseMatrix,
                                                          const FatVector &fatVector, int vecCols)
{
    return collective_run(SMFV_ROWWISE, sparseMatrix, fatVector, vecCols);
}

DROPIN_API FatVector sparseMatrixFatVectorMultiplyColumnWise(const SparseMatrix &sparseMatrix,
                                                             const FatVector &fatVector, int vecCols)
{
    return collective_run(SMFV_COLUMNWISE, sparseMatrix, fatVector, vecCols);
}

DROPIN_API FatVector sparseMatrixFatVectorMultiplyNonZeroElement(const SparseMatrix &sparseMatrix,
                                                                 const FatVector &fatVector, int vecCols)
{
    return collective_run(SMFV_NONZERO, sparseMatrix, fatVector, vecCols);
}

// ---- extensions (include/smfv_dropin.h) -------------------------------------

DROPIN_API double smfvDistributeInputs(SparseMatrix &A, FatVector &fat, int k)
{
    Context &c = ctx();
    const double t0 = MPI_Wtime();
    // sizes (the control plane) go by MPI as SC/main.cpp:110-112 does; the
    // data goes GPU to GPU
    long long dims[4] = {A.numRows, A.numCols, (long long)A.values.size(), k};
    if (c.mpi) MPI_Bcast(dims, 4, MPI_LONG_LONG, 0, MPI_COMM_WORLD);
    const int m = (int)dims[0], n = (int)dims[1], K = (int)dims[3];
    const int64_t nnz = dims[2];
    if (m < 0 || n < 0 || nnz < 0 || K < 0) fail("smfvDistributeInputs: bad sizes");
    Resident &R = resident();
    R.on = false;
    int *rp = static_cast<int *>(R.rp.get(((size_t)m + 1) * sizeof(int)));
    int *ci = static_cast<int *>(R.ci.get((size_t)nnz * sizeof(int)));
    double *va = static_cast<double *>(R.va.get((size_t)nnz * sizeof(double)));
    double *X = static_cast<double *>(R.X.get((size_t)n * K * sizeof(double)));
    Buffers &B = bufs();
    double *hx = static_cast<double *>(B.hX.get((size_t)n * K * sizeof(double)));
    hipStream_t st = c.stream;
    if (c.rank == 0) {
        if ((int)A.rowPtr.size() != m + 1 || (int64_t)A.colIndices.size() != nnz || (int)fat.size() != n)
            fail("smfvDistributeInputs: malformed inputs on rank 0");
        for (const auto &r : fat)
            if ((int)r.size() != K) fail("fatVector rows must have k entries");
        par_rows(n, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) std::copy(fat[i].begin(), fat[i].end(), hx + (size_t)i * K);
        });
        hip_check(hipMemcpyAsync(rp, A.rowPtr.data(), ((size_t)m + 1) * sizeof(int), hipMemcpyHostToDevice, st), "H2D");
        if (nnz) {
            hip_check(hipMemcpyAsync(ci, A.colIndices.data(), nnz * sizeof(int), hipMemcpyHostToDevice, st), "H2D");
            hip_check(hipMemcpyAsync(va, A.values.data(), nnz * sizeof(double), hipMemcpyHostToDevice, st), "H2D");
        }
        if ((size_t)n * K)
            hip_check(hipMemcpyAsync(X, hx, (size_t)n * K * sizeof(double), hipMemcpyHostToDevice, st), "H2D");
    }
    if (c.size > 1) {
        smfv_comm_t comm = comm_world();
        check(smfv_comm_bcast(comm, rp, ((size_t)m + 1) * sizeof(int), 0, st), "smfv_comm_bcast");
        check(smfv_comm_bcast(comm, ci, (size_t)nnz * sizeof(int), 0, st), "smfv_comm_bcast");
        check(smfv_comm_bcast(comm, va, (size_t)nnz * sizeof(double), 0, st), "smfv_comm_bcast");
        check(smfv_comm_bcast(comm, X, (size_t)n * K * sizeof(double), 0, st), "smfv_comm_bcast");
    }
    if (c.rank != 0) {  // the host copies every rank holds after SC/main.cpp:106-143
        A.numRows = m;
        A.numCols = n;
        A.rowPtr.resize((size_t)m + 1);
        A.colIndices.resize((size_t)nnz);
        A.values.resize((size_t)nnz);
        hip_check(hipMemcpyAsync(A.rowPtr.data(), rp, ((size_t)m + 1) * sizeof(int), hipMemcpyDeviceToHost, st), "D2H");
        if (nnz) {
            hip_check(hipMemcpyAsync(A.colIndices.data(), ci, nnz * sizeof(int), hipMemcpyDeviceToHost, st), "D2H");
            hip_check(hipMemcpyAsync(A.values.data(), va, nnz * sizeof(double), hipMemcpyDeviceToHost, st), "D2H");
        }
        if ((size_t)n * K)
            hip_check(hipMemcpyAsync(hx, X, (size_t)n * K * sizeof(double), hipMemcpyDeviceToHost, st), "D2H");
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
        fat.assign((size_t)n, std::vector<double>());
        par_rows(n, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) fat[i].assign(hx + (size_t)i * K, hx + (size_t)(i + 1) * K);
        });
    }
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    R.A = &A;
    R.fat = &fat;
    R.va_host = A.values.data();
    R.ci_host = A.colIndices.data();
    R.rp_host = A.rowPtr.data();
    R.nnz = (size_t)nnz;
    R.rows = fat.size();
    R.m = m;
    R.n = n;
    R.K = K;
    R.hrp = hash_bytes(A.rowPtr.data(), A.rowPtr.size() * sizeof(int));
    R.hci = hash_bytes(A.colIndices.data(), A.colIndices.size() * sizeof(int));
    R.on = true;
    return MPI_Wtime() - t0;
}

DROPIN_API void smfvReleaseInputs() { resident().on = false; }

DROPIN_API void smfvKeepResultAsReference()
{
    Buffers &B = bufs();
    if (!B.lastY || B.last_m < 0) return;
    const size_t bytes = (size_t)B.last_m * B.last_K * sizeof(double);
    void *dst = B.ref.get(bytes);
    if (bytes) hip_check(hipMemcpyAsync(dst, B.lastY, bytes, hipMemcpyDeviceToDevice, ctx().stream), "D2D");
    hip_check(hipStreamSynchronize(ctx().stream), "hipStreamSynchronize");
    B.ref_m = B.last_m;
    B.ref_K = B.last_K;
}

DROPIN_API bool smfvCompareWithReference(double tolerance, double *max_abs_diff)
{
    Buffers &B = bufs();
    if (max_abs_diff) *max_abs_diff = INFINITY;
    if (!B.lastY || B.ref_m < 0 || B.ref_m != B.last_m || B.ref_K != B.last_K) return false;
    double out[2] = {0.0, 0.0};
    check(smfv_compare_f64(B.last_m, B.last_K, static_cast<const double *>(B.ref.p), B.last_K, B.lastY, B.last_K, out,
                           ctx().stream),
          "smfv_compare_f64");
    if (max_abs_diff) *max_abs_diff = out[0];
    return out[0] <= tolerance;  // NaN differences are +inf (k_compare)
}

// ---- SC/utils.cpp helpers ---------------------------------------------------

DROPIN_API bool areMatricesEqual(const FatVector &mat1, const FatVector &mat2, double tolerance)
{
    if (mat1.size() != mat2.size()) return false;
    for (size_t i = 0; i < mat1.size(); ++i) {
        if (mat1[i].size() != mat2[i].size()) return false;
        for (size_t j = 0; j < mat1[i].size(); ++j)
            if (std::fabs(mat1[i][j] - mat2[i][j]) > tolerance) return false;
    }
    return true;
}

DROPIN_API SparseMatrix readMatrixMarketFile(const std::string &filename)
{
    int m = 0, n = 0;
    int64_t nnz = 0;
    int *rp = nullptr, *ci = nullptr;
    double *va = nullptr;
    if (smfv_mtx_read(filename.c_str(), &m, &n, &nnz, &rp, &ci, &va) != SMFV_OK)
        throw std::runtime_error(smfv_last_error());
    SparseMatrix A;
    A.numRows = m;
    A.numCols = n;
    A.rowPtr.assign(rp, rp + m + 1);
    A.colIndices.assign(ci, ci + nnz);
    A.values.assign(va, va + nnz);
    smfv_free(rp);
    smfv_free(ci);
    smfv_free(va);
    return A;
}

DROPIN_API FatVector generateLargeFatVector(int n, int k)
{
    // the process-global rand() stream, exactly as SC/utils.cpp:203
    FatVector v((size_t)n, std::vector<double>((size_t)k));
    for (auto &row : v)
        for (auto &x : row) x = rand() % 100 + 1;
    return v;
}

DROPIN_API std::vector<double> serialize(const FatVector &denseVec)
{
    size_t total = 0;
    for (const auto &r : denseVec) total += r.size();
    std::vector<double> flat;
    flat.reserve(total);
    for (const auto &r : denseVec) flat.insert(flat.end(), r.begin(), r.end());
    return flat;
}

DROPIN_API FatVector deserialize(const std::vector<double> &flat, int rows, int cols)
{
    FatVector out((size_t)rows, std::vector<double>((size_t)cols));
    for (int i = 0; i < rows; ++i)
        std::copy(flat.begin() + (size_t)i * cols, flat.begin() + (size_t)(i + 1) * cols, out[i].begin());
    return out;
}
