// smfv_host.cpp -- host-side inputs: Matrix Market reader, glibc-rand fat
// vector, synthetic CSR generators, SMFV binary containers (smfv_host.h).
//
// Reader semantics follow SC/utils.cpp:70-185; the fat vector follows
// SC/utils.cpp:193-209.  Generators are counter-hash based so that any row
// block (one GPU's shard) can be produced independently and in parallel.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "smfv.h"
#include "smfv_host.h"
#include "smfv_internal.h"

using smfv::set_error;

namespace {

inline uint64_t splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline uint64_t hash3(uint64_t seed, uint64_t a, uint64_t b)
{
    return splitmix64(splitmix64(seed ^ splitmix64(a)) ^ b);
}
inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

int nthreads_for(int64_t work)
{
    unsigned hc = std::thread::hardware_concurrency();
    int t = (int)std::min<unsigned>(hc ? hc : 1, 16u);
    if (work < (1 << 16)) t = 1;
    return std::max(1, t);
}

template <class F> void parallel_rows(int64_t begin, int64_t end, F f)
{
    const int nt = nthreads_for(end - begin);
    if (nt == 1) {
        f(begin, end);
        return;
    }
    std::vector<std::thread> th;
    const int64_t chunk = (end - begin + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t a = begin + t * chunk, b = std::min(end, a + chunk);
        if (a >= b) break;
        th.emplace_back(f, a, b);
    }
    for (auto &x : th) x.join();
}

// Parses the entry lines of [p, end) in parallel (see smfv_mtx_read).  True
// when every line of the region holds exactly one valid entry and there are
// exactly nz of them; rows / ent then hold them in file order (mirrored
// entries right after their source, as the sequential reader stores them).
bool parse_entries_parallel(const char *p, const char *end, long long m, long long n, long long nz, bool sym,
                            bool pat, std::vector<int> &rows, std::vector<std::pair<int, double>> &ent, int64_t &t)
{
    const int nt = nthreads_for(end - p);
    if (nt == 1 || nz == 0) return false;
    // chunk boundaries at line starts
    std::vector<const char *> cut(nt + 1, end);
    cut[0] = p;
    for (int k = 1; k < nt; ++k) {
        const char *q = p + (end - p) * k / nt;
        if (q < cut[k - 1]) q = cut[k - 1];
        while (q < end && q[-1] != '\n') ++q;
        cut[k] = q;
    }
    // one line -> one entry: parse into per-thread buffers
    struct Part {
        std::vector<int> r;
        std::vector<std::pair<int, double>> e;
        bool ok = true;
    };
    std::vector<Part> part(nt);
    auto work = [&](int k) {
        Part &P = part[k];
        const char *q = cut[k], *qe = cut[k + 1];
        while (q < qe) {
            const char *le = static_cast<const char *>(std::memchr(q, '\n', qe - q));
            if (!le) le = qe;
            const char *a = q;
            while (a < le && (*a == ' ' || *a == '\t' || *a == '\r')) ++a;
            if (a == le) {  // blank line: the sequential reader would skip it too
                q = le + 1;
                continue;
            }
            char *x;
            const long r = std::strtol(a, &x, 10);
            if (x == a) { P.ok = false; return; }
            const char *b = x;
            const long c = std::strtol(b, &x, 10);
            if (x == b) { P.ok = false; return; }
            double v = 1.0;
            if (!pat) {
                const char *d = x;
                v = std::strtod(d, &x);
                if (x == d) { P.ok = false; return; }
            }
            for (const char *z = x; z < le; ++z)  // nothing else on the line
                if (!(*z == ' ' || *z == '\t' || *z == '\r')) { P.ok = false; return; }
            if (r < 1 || r > m || c < 1 || c > n || (sym && r != c && c > m)) { P.ok = false; return; }
            P.r.push_back((int)(r - 1));
            P.e.push_back({(int)(c - 1), v});
            if (sym && r != c) {
                P.r.push_back((int)(c - 1));
                P.e.push_back({(int)(r - 1), v});
            }
            q = le + 1;
        }
    };
    {
        std::vector<std::thread> th;
        for (int k = 0; k < nt; ++k) th.emplace_back(work, k);
        for (auto &x : th) x.join();
    }
    int64_t total = 0, entries = 0;
    for (const Part &P : part) {
        if (!P.ok) return false;
        total += (int64_t)P.r.size();
    }
    // the file's entry count (a mirrored pair counts once)
    for (const Part &P : part)
        for (size_t i = 0; i < P.r.size(); ++i) {
            ++entries;
            if (sym && P.r[i] != P.e[i].first) ++i;  // skip the mirror
        }
    if (entries != nz || total > (int64_t)rows.size()) return false;
    std::vector<int64_t> off(nt + 1, 0);
    for (int k = 0; k < nt; ++k) off[k + 1] = off[k] + (int64_t)part[k].r.size();
    std::vector<std::thread> th;
    for (int k = 0; k < nt; ++k)
        th.emplace_back([&, k] {
            std::copy(part[k].r.begin(), part[k].r.end(), rows.begin() + off[k]);
            std::copy(part[k].e.begin(), part[k].e.end(), ent.begin() + off[k]);
        });
    for (auto &x : th) x.join();
    t = total;
    return true;
}

template <class T> T *xmalloc(size_t count)
{
    return static_cast<T *>(std::malloc(sizeof(T) * (count ? count : 1)));
}

}  // namespace

extern "C" {

SMFV_API void smfv_free(void *p) { std::free(p); }

// ---------------------------------------------------------------------------
// glibc rand() stream, default seed 1 (TYPE_3: r[i] = r[i-3] + r[i-31])
// ---------------------------------------------------------------------------
SMFV_API void smfv_fatvector_rand(int64_t n, int K, double *X)
{
    int32_t r[34];
    r[0] = 1;
    for (int i = 1; i < 31; ++i) {
        // 16807 * r[i-1] % (2^31 - 1) via Schrage, as glibc's srandom_r
        const int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int32_t w = 16807 * lo - 2836 * hi;
        if (w < 0) w += 2147483647;
        r[i] = w;
    }
    uint32_t ring[34];
    for (int i = 0; i < 31; ++i) ring[i] = (uint32_t)r[i];
    for (int i = 31; i < 34; ++i) ring[i] = ring[i - 31];
    // r[i] for i >= 34 = r[i-31] + r[i-3]; outputs start at i = 344
    int64_t idx = 34;
    auto next = [&]() {
        const uint32_t v = ring[(idx - 31) % 34] + ring[(idx - 3) % 34];
        ring[idx % 34] = v;
        ++idx;
        return v;
    };
    while (idx < 344) next();
    const int64_t total = n * (int64_t)K;
    for (int64_t i = 0; i < total; ++i) X[i] = (double)((int32_t)(next() >> 1) % 100 + 1);
}

// ---------------------------------------------------------------------------
// Matrix Market (SC/utils.cpp:70-185)
// ---------------------------------------------------------------------------
SMFV_API int smfv_mtx_read(const char *path, int *out_m, int *out_n, int64_t *out_nnz,
                           int **out_rp, int **out_ci, double **out_va)
{
    SMFV_REQUIRE(path && out_m && out_n && out_nnz && out_rp && out_ci && out_va, "null argument");
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        set_error("Unable to open file: %s", path);
        return SMFV_ERR_HOST;
    }
    std::string buf;
    {
        std::fseek(f, 0, SEEK_END);
        long sz = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        buf.resize(sz > 0 ? (size_t)sz : 0);
        if (sz > 0 && std::fread(&buf[0], 1, (size_t)sz, f) != (size_t)sz) {
            std::fclose(f);
            set_error("read error: %s", path);
            return SMFV_ERR_HOST;
        }
        std::fclose(f);
    }
    // comment / header lines: first char '%' (utils.cpp:84-105)
    size_t pos = 0;
    bool sym = false, pat = false;
    std::string line;
    bool have = false;
    while (pos <= buf.size()) {
        size_t nl = buf.find('\n', pos);
        if (nl == std::string::npos) nl = buf.size();
        line.assign(buf, pos, nl - pos);
        pos = nl + 1;
        if (!line.empty() && line[0] == '%') {
            if (line.find("symmetric") != std::string::npos) sym = true;
            if (line.find("pattern") != std::string::npos) pat = true;
            continue;
        }
        have = true;
        break;
    }
    long long m = -1, n = -1, nz = -1;
    if (!have || std::sscanf(line.c_str(), "%lld %lld %lld", &m, &n, &nz) != 3 || m < 0 || n < 0 ||
        nz < 0 || m > 0x7fffffff || n > 0x7fffffff) {
        set_error("Failed to read matrix dimensions from file: %s", path);
        return SMFV_ERR_HOST;
    }
    const int64_t cap = sym ? 2 * nz : nz;
    std::vector<int> rows((size_t)cap);
    std::vector<std::pair<int, double>> ent((size_t)cap);
    const char *p = buf.c_str() + std::min(pos, buf.size());
    int64_t t = 0;
    // Parallel parse (one entry per line, the layout every writer uses): the
    // data region is cut at line starts into one chunk per thread, each chunk
    // counted and parsed on its own, results placed by a prefix sum.  Any
    // chunk that does not parse cleanly, or a total other than nz, falls back
    // to the sequential token reader below (the reference's semantics: nz
    // entries, whitespace-separated, the rest of the file ignored).
    if (parse_entries_parallel(p, buf.c_str() + buf.size(), m, n, nz, sym, pat, rows, ent, t)) goto assemble;
    t = 0;
    for (long long i = 0; i < nz; ++i) {
        char *endp;
        errno = 0;
        long r = std::strtol(p, &endp, 10);
        if (endp == p) goto bad;
        p = endp;
        {
            long c = std::strtol(p, &endp, 10);
            if (endp == p) goto bad;
            p = endp;
            double v = 1.0;  // pattern (utils.cpp:130)
            if (!pat) {
                v = std::strtod(p, &endp);
                if (endp == p) goto bad;
                p = endp;
            }
            r -= 1;
            c -= 1;  // 1-based -> 0-based (utils.cpp:143-144)
            if (r < 0 || r >= m || c < 0 || c >= n) goto bad;
            rows[t] = (int)r;
            ent[t] = {(int)c, v};
            ++t;
            if (sym && r != c) {  // mirror (utils.cpp:149-152)
                if (c >= m) goto bad;
                rows[t] = (int)c;
                ent[t] = {(int)r, v};
                ++t;
            }
        }
    }
assemble:
    {
        int *rp = xmalloc<int>((size_t)m + 1);
        int *ci = xmalloc<int>((size_t)t);
        double *va = xmalloc<double>((size_t)t);
        if (!rp || !ci || !va) {
            std::free(rp);
            std::free(ci);
            std::free(va);
            set_error("out of memory");
            return SMFV_ERR_HOST;
        }
        std::vector<int64_t> cnt((size_t)m + 1, 0);
        for (int64_t i = 0; i < t; ++i) cnt[(size_t)rows[i] + 1]++;
        for (long long i = 0; i < m; ++i) cnt[i + 1] += cnt[i];
        if (cnt[m] > 0x7fffffff) {
            std::free(rp);
            std::free(ci);
            std::free(va);
            set_error("nnz exceeds int32 row_ptr");
            return SMFV_ERR_HOST;
        }
        std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
        std::vector<std::pair<int, double>> sorted((size_t)t);
        for (int64_t i = 0; i < t; ++i) sorted[fill[rows[i]]++] = ent[i];
        parallel_rows(0, m, [&](int64_t a, int64_t b) {  // per-row sort by (col, value) (utils.cpp:156-159)
            for (int64_t i = a; i < b; ++i) std::sort(sorted.begin() + cnt[i], sorted.begin() + cnt[i + 1]);
        });
        for (long long i = 0; i <= m; ++i) rp[i] = (int)cnt[i];
        parallel_rows(0, t, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) {
                ci[i] = sorted[i].first;
                va[i] = sorted[i].second;
            }
        });
        *out_m = (int)m;
        *out_n = (int)n;
        *out_nnz = t;
        *out_rp = rp;
        *out_ci = ci;
        *out_va = va;
        return SMFV_OK;
    }
bad:
    set_error("Failed to read data from file: %s", path);
    return SMFV_ERR_HOST;
}

SMFV_API int smfv_mtx_write(const char *path, int m, int n, const int *rp, const int *ci,
                            const double *va, int symmetric)
{
    SMFV_REQUIRE(path && rp && m >= 0 && n >= 0, "bad argument");
    FILE *f = std::fopen(path, "w");
    if (!f) {
        set_error("cannot write %s", path);
        return SMFV_ERR_HOST;
    }
    int64_t cnt = 0;
    for (int i = 0; i < m; ++i)
        for (int j = rp[i]; j < rp[i + 1]; ++j)
            if (!symmetric || ci[j] <= i) ++cnt;
    std::fprintf(f, "%%%%MatrixMarket matrix coordinate real %s\n", symmetric ? "symmetric" : "general");
    std::fprintf(f, "%d %d %lld\n", m, n, (long long)cnt);
    for (int i = 0; i < m; ++i)
        for (int j = rp[i]; j < rp[i + 1]; ++j)
            if (!symmetric || ci[j] <= i) std::fprintf(f, "%d %d %.17g\n", i + 1, ci[j] + 1, va[j]);
    const bool ok = std::fclose(f) == 0;
    if (!ok) {
        set_error("write error on %s", path);
        return SMFV_ERR_HOST;
    }
    return SMFV_OK;
}

// ---------------------------------------------------------------------------
// SMFV binary containers
// ---------------------------------------------------------------------------
SMFV_API int smfv_csr_write_bin(const char *path, int m, int n, const int *rp, const int *ci,
                                const double *va)
{
    SMFV_REQUIRE(path && rp && m >= 0 && n >= 0, "bad argument");
    FILE *f = std::fopen(path, "wb");
    if (!f) {
        set_error("cannot write %s", path);
        return SMFV_ERR_HOST;
    }
    const int64_t nnz = rp[m];
    bool ok = std::fwrite("SMFVCSR1", 1, 8, f) == 8 && std::fwrite(&m, 4, 1, f) == 1 &&
              std::fwrite(&n, 4, 1, f) == 1 && std::fwrite(&nnz, 8, 1, f) == 1 &&
              std::fwrite(rp, 4, (size_t)m + 1, f) == (size_t)m + 1 &&
              (nnz == 0 || (std::fwrite(ci, 4, (size_t)nnz, f) == (size_t)nnz &&
                            std::fwrite(va, 8, (size_t)nnz, f) == (size_t)nnz));
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        set_error("write error on %s", path);
        return SMFV_ERR_HOST;
    }
    return SMFV_OK;
}

SMFV_API int smfv_csr_read_bin(const char *path, int *out_m, int *out_n, int64_t *out_nnz,
                               int **out_rp, int **out_ci, double **out_va)
{
    SMFV_REQUIRE(path && out_m && out_n && out_nnz && out_rp && out_ci && out_va, "null argument");
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        set_error("Unable to open file: %s", path);
        return SMFV_ERR_HOST;
    }
    char magic[8];
    int32_t m = 0, n = 0;
    int64_t nnz = 0;
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "SMFVCSR1", 8) == 0 &&
              std::fread(&m, 4, 1, f) == 1 && std::fread(&n, 4, 1, f) == 1 &&
              std::fread(&nnz, 8, 1, f) == 1 && m >= 0 && n >= 0 && nnz >= 0;
    int *rp = nullptr, *ci = nullptr;
    double *va = nullptr;
    if (ok) {
        rp = xmalloc<int>((size_t)m + 1);
        ci = xmalloc<int>((size_t)nnz);
        va = xmalloc<double>((size_t)nnz);
        ok = rp && ci && va && std::fread(rp, 4, (size_t)m + 1, f) == (size_t)m + 1 &&
             (nnz == 0 || (std::fread(ci, 4, (size_t)nnz, f) == (size_t)nnz &&
                           std::fread(va, 8, (size_t)nnz, f) == (size_t)nnz));
    }
    std::fclose(f);
    if (!ok) {
        std::free(rp);
        std::free(ci);
        std::free(va);
        set_error("bad SMFV CSR file %s", path);
        return SMFV_ERR_HOST;
    }
    *out_m = m;
    *out_n = n;
    *out_nnz = nnz;
    *out_rp = rp;
    *out_ci = ci;
    *out_va = va;
    return SMFV_OK;
}

SMFV_API int smfv_dense_write_bin(const char *path, int64_t rows, int64_t cols, const double *data)
{
    SMFV_REQUIRE(path && rows >= 0 && cols >= 0 && (rows * cols == 0 || data), "bad argument");
    FILE *f = std::fopen(path, "wb");
    if (!f) {
        set_error("cannot write %s", path);
        return SMFV_ERR_HOST;
    }
    bool ok = std::fwrite("SMFVDNS1", 1, 8, f) == 8 && std::fwrite(&rows, 8, 1, f) == 1 &&
              std::fwrite(&cols, 8, 1, f) == 1 &&
              (rows * cols == 0 || std::fwrite(data, 8, (size_t)(rows * cols), f) == (size_t)(rows * cols));
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        set_error("write error on %s", path);
        return SMFV_ERR_HOST;
    }
    return SMFV_OK;
}

// ---------------------------------------------------------------------------
// fem27: symmetric 27-point-stencil surrogate
// ---------------------------------------------------------------------------
// Irregular FEM-like surrogate: m points in the unit cube, 70 % uniform and
// 30 % in 48 Gaussian clusters (so the neighbour distance varies ~5x), each
// joined to its k_i nearest points (see below)
// scale s, the graph symmetrised (union) plus the diagonal, rows numbered in
// Morton (Z) order of the points -- a mesh-like numbering with locality but
// no stencil regularity.  s is bisected so that nnz lands on target_nnz.
// Row degrees spread from ~4 to ~80 (k_i in [3, 48] x s, log-graded along
// the cube's diagonal with noise, at most 64 out-neighbours).  Values as fem27 (symmetric,
// off-diagonal in [-1, 1), diagonal in [1, 2)).
SMFV_API int smfv_gen_knn3d(int m, int64_t target_nnz, uint64_t seed, int64_t *out_nnz, int **out_rp, int **out_ci,
                            double **out_va)
{
    SMFV_REQUIRE(m >= 2 && target_nnz >= m && out_nnz && out_rp && out_ci && out_va, "bad knn3d parameters");
    constexpr int KMAX = 64, NCL = 48;
    // points (hash-based, independent of the thread count)
    std::vector<double> P((size_t)m * 3);
    std::vector<double> cen(NCL * 3);
    for (int c = 0; c < NCL * 3; ++c) cen[c] = 0.1 + 0.8 * u01(hash3(seed, 0xC1u, (uint64_t)c));
    auto gauss = [](uint64_t h1, uint64_t h2) {
        const double u = std::max(u01(h1), 1e-300), v = u01(h2);
        return std::sqrt(-2.0 * std::log(u)) * std::cos(6.283185307179586 * v);
    };
    parallel_rows(0, m, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const uint64_t h = hash3(seed, 0xA0u, (uint64_t)i);
            if (u01(h) < 0.7) {
                for (int d = 0; d < 3; ++d) P[(size_t)i * 3 + d] = u01(hash3(seed, 0xB0u + d, (uint64_t)i));
            } else {
                const int c = (int)(splitmix64(h) % NCL);
                for (int d = 0; d < 3; ++d) {
                    double x = cen[c * 3 + d] + 0.035 * gauss(hash3(seed, 0xD0u + d, (uint64_t)i),
                                                              hash3(seed, 0xE0u + d, (uint64_t)i));
                    P[(size_t)i * 3 + d] = std::min(1.0 - 1e-9, std::max(0.0, x));
                }
            }
        }
    });
    // Morton order
    auto morton = [&](int64_t i) {
        uint64_t code = 0;
        for (int d = 0; d < 3; ++d) {
            uint64_t q = (uint64_t)(P[(size_t)i * 3 + d] * 2097152.0);  // 21 bits
            for (int b = 0; b < 21; ++b) code |= ((q >> b) & 1ull) << (3 * b + d);
        }
        return code;
    };
    std::vector<std::pair<uint64_t, int>> ord((size_t)m);
    for (int i = 0; i < m; ++i) ord[i] = {morton(i), i};
    std::sort(ord.begin(), ord.end());
    {
        std::vector<double> Q((size_t)m * 3);
        for (int i = 0; i < m; ++i)
            for (int d = 0; d < 3; ++d) Q[(size_t)i * 3 + d] = P[(size_t)ord[i].second * 3 + d];
        P.swap(Q);
    }
    // grid buckets (about two points per cell)
    const int G = std::max(1, (int)std::cbrt((double)m / 2.0));
    std::vector<int> cstart((size_t)G * G * G + 1, 0), cell((size_t)m), cpts((size_t)m);
    auto cell_of = [&](int i, int d) { return std::min(G - 1, (int)(P[(size_t)i * 3 + d] * G)); };
    for (int i = 0; i < m; ++i) {
        cell[i] = (cell_of(i, 2) * G + cell_of(i, 1)) * G + cell_of(i, 0);
        ++cstart[(size_t)cell[i] + 1];
    }
    for (size_t c = 0; c + 1 < cstart.size(); ++c) cstart[c + 1] += cstart[c];
    {
        std::vector<int> fill(cstart.begin(), cstart.end() - 1);
        for (int i = 0; i < m; ++i) cpts[(size_t)fill[(size_t)cell[i]]++] = i;
    }
    // the KMAX nearest points of every point, nearest first (ties by index)
    std::vector<int> nn((size_t)m * KMAX);
    parallel_rows(0, m, [&](int64_t a, int64_t b) {
        std::vector<std::pair<double, int>> cand;
        for (int64_t i = a; i < b; ++i) {
            const int cx = cell_of((int)i, 0), cy = cell_of((int)i, 1), cz = cell_of((int)i, 2);
            for (int r = 1;; ++r) {
                cand.clear();
                for (int z = std::max(0, cz - r); z <= std::min(G - 1, cz + r); ++z)
                    for (int y = std::max(0, cy - r); y <= std::min(G - 1, cy + r); ++y)
                        for (int x = std::max(0, cx - r); x <= std::min(G - 1, cx + r); ++x) {
                            const int c = (z * G + y) * G + x;
                            for (int q = cstart[c]; q < cstart[(size_t)c + 1]; ++q) {
                                const int j = cpts[q];
                                if (j == i) continue;
                                double d2 = 0;
                                for (int d = 0; d < 3; ++d) {
                                    const double t = P[(size_t)i * 3 + d] - P[(size_t)j * 3 + d];
                                    d2 += t * t;
                                }
                                cand.push_back({d2, j});
                            }
                        }
                // complete once KMAX candidates lie within the searched radius r / G
                // (every closer point is inside the searched cube) or the cube is the grid
                const double reach = (double)r / G;
                int inside = 0;
                for (auto &c : cand) inside += c.first <= reach * reach;
                if (inside >= KMAX || r >= G) break;
            }
            const size_t k = std::min<size_t>(KMAX, cand.size());
            std::partial_sort(cand.begin(), cand.begin() + k, cand.end());
            for (size_t q = 0; q < (size_t)KMAX; ++q) nn[(size_t)i * KMAX + q] = q < k ? cand[q].second : -1;
        }
    });
    // per-point base k in [3, 48], log-graded across the cube (a refined
    // region's points all have many neighbours); symmetrised degree for a scale s
    std::vector<double> kb((size_t)m);
    for (int i = 0; i < m; ++i) {  // spatially graded (neighbours have similar k) plus noise
        const double g = (P[(size_t)i * 3] + P[(size_t)i * 3 + 1] + P[(size_t)i * 3 + 2]) / 3.0;
        const double u = std::min(1.0, std::max(0.0, 1.6 * (g - 0.5) + 0.5 + 0.3 * (u01(hash3(seed, 0xF0u, (uint64_t)i)) - 0.5)));
        kb[i] = 3.0 * std::pow(16.0, u);
    }
    std::vector<std::vector<int>> adj;
    auto build = [&](double s) {
        adj.assign((size_t)m, {});
        for (int i = 0; i < m; ++i) {
            const int k = std::max(1, std::min(KMAX, (int)std::lround(kb[i] * s)));
            for (int q = 0; q < k; ++q) {
                const int j = nn[(size_t)i * KMAX + q];
                if (j < 0) break;
                adj[i].push_back(j);
                adj[j].push_back(i);
            }
        }
        int64_t t = 0;
        for (int i = 0; i < m; ++i) {
            adj[i].push_back(i);
            std::sort(adj[i].begin(), adj[i].end());
            adj[i].erase(std::unique(adj[i].begin(), adj[i].end()), adj[i].end());
            t += (int64_t)adj[i].size();
        }
        return t;
    };
    double lo = 0.05, hi = 2.0;
    for (int it = 0; it < 40 && hi - lo > 1e-6; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (build(mid) < target_nnz) lo = mid;
        else hi = mid;
    }
    // of the two bracketing scales, the one closer to the target
    const int64_t tl = build(lo), th = build(hi);
    const int64_t nnz = std::llabs(tl - target_nnz) <= std::llabs(th - target_nnz) ? build(lo) : th;
    SMFV_REQUIRE(nnz <= 0x7fffffff, "knn3d nnz exceeds int32");
    int *rp = xmalloc<int>((size_t)m + 1);
    int *ci = xmalloc<int>((size_t)nnz);
    double *va = xmalloc<double>((size_t)nnz);
    if (!rp || !ci || !va) {
        std::free(rp);
        std::free(ci);
        std::free(va);
        set_error("out of memory");
        return SMFV_ERR_HOST;
    }
    rp[0] = 0;
    for (int i = 0; i < m; ++i) rp[i + 1] = rp[i] + (int)adj[i].size();
    parallel_rows(0, m, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            int o = rp[i];
            for (int j : adj[i]) {
                ci[o] = j;
                if (j == i) {
                    va[o] = 1.0 + u01(hash3(seed, (uint64_t)i, (uint64_t)i));
                } else {
                    const uint64_t x = (uint64_t)std::min<int64_t>(i, j), y = (uint64_t)std::max<int64_t>(i, j);
                    va[o] = 2.0 * u01(splitmix64(hash3(seed, x, y) ^ 0xA5A5A5A5ull)) - 1.0;
                }
                ++o;
            }
        }
    });
    *out_nnz = nnz;
    *out_rp = rp;
    *out_ci = ci;
    *out_va = va;
    return SMFV_OK;
}

SMFV_API int smfv_gen_fem27(int m, int nx, int ny, double keep, uint64_t seed, int64_t *out_nnz,
                            int **out_rp, int **out_ci, double **out_va)
{
    SMFV_REQUIRE(m >= 0 && nx >= 3 && ny >= 3 && keep >= 0 && keep <= 1, "bad fem27 parameters");
    SMFV_REQUIRE(out_nnz && out_rp && out_ci && out_va, "null argument");
    const int64_t plane = (int64_t)nx * ny;
    auto visit = [&](int64_t i, auto &&emit) {
        const int64_t x = i % nx, y = (i / nx) % ny, z = i / plane;
        for (int dz = -1; dz <= 1; ++dz)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    if (x + dx < 0 || x + dx >= nx || y + dy < 0 || y + dy >= ny || z + dz < 0) continue;
                    const int64_t j = i + dx + (int64_t)nx * dy + plane * dz;
                    if (j < 0 || j >= m) continue;
                    if (j == i) {
                        emit(j, 1.0 + u01(hash3(seed, (uint64_t)i, (uint64_t)i)));
                        continue;
                    }
                    const uint64_t a = (uint64_t)std::min(i, j), b = (uint64_t)std::max(i, j);
                    const uint64_t h = hash3(seed, a, b);
                    if (u01(h) < keep) emit(j, 2.0 * u01(splitmix64(h ^ 0xA5A5A5A5ull)) - 1.0);
                }
    };
    std::vector<int64_t> cnt((size_t)m + 1, 0);
    parallel_rows(0, m, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            int64_t c = 0;
            visit(i, [&](int64_t, double) { ++c; });
            cnt[i + 1] = c;
        }
    });
    for (int i = 0; i < m; ++i) cnt[i + 1] += cnt[i];
    SMFV_REQUIRE(cnt[m] <= 0x7fffffff, "fem27 nnz exceeds int32");
    int *rp = xmalloc<int>((size_t)m + 1);
    int *ci = xmalloc<int>((size_t)cnt[m]);
    double *va = xmalloc<double>((size_t)cnt[m]);
    if (!rp || !ci || !va) {
        std::free(rp);
        std::free(ci);
        std::free(va);
        set_error("out of memory");
        return SMFV_ERR_HOST;
    }
    for (int i = 0; i <= m; ++i) rp[i] = (int)cnt[i];
    parallel_rows(0, m, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            int64_t o = cnt[i];
            visit(i, [&](int64_t j, double v) {
                ci[o] = (int)j;
                va[o] = v;
                ++o;
            });
        }
    });
    *out_nnz = cnt[m];
    *out_rp = rp;
    *out_ci = ci;
    *out_va = va;
    return SMFV_OK;
}

// ---------------------------------------------------------------------------
// random rows: truncated power-law (alpha > 1) or fixed length (alpha <= 0)
// ---------------------------------------------------------------------------
static double powerlaw_raw(uint64_t seed, int64_t row, double alpha)
{
    // Pareto(x_m = 1): P(L >= x) = x^(1 - alpha)
    const double u = 1.0 - u01(hash3(seed, (uint64_t)row, 0x5EEDull));  // (0, 1]
    return std::pow(u, -1.0 / (alpha - 1.0));
}

static int64_t row_len(uint64_t seed, int64_t row, double alpha, double scale, int cap, int64_t n)
{
    int64_t L;
    if (alpha <= 0) L = (int64_t)std::llround(scale);
    else L = (int64_t)std::floor(powerlaw_raw(seed, row, alpha) * scale);
    L = std::max<int64_t>(1, std::min<int64_t>(L, cap));
    return std::min<int64_t>(L, n);
}

SMFV_API int smfv_gen_random_rows(int64_t m, int64_t n, int64_t row_begin, int64_t row_end,
                                  double mean, double alpha, int cap, uint64_t seed,
                                  int64_t *out_nnz, int **out_rp, int **out_ci, double **out_va)
{
    SMFV_REQUIRE(m >= 0 && n > 0 && 0 <= row_begin && row_begin <= row_end && row_end <= m,
                 "bad row range");
    SMFV_REQUIRE(mean >= 1 && cap >= 1 && (alpha <= 0 || alpha > 1), "bad distribution");
    SMFV_REQUIRE(out_nnz && out_rp && out_ci && out_va, "null argument");
    double scale = mean;
    if (alpha > 0) {
        // scale so that E[row length] == mean, estimated on a fixed sample of
        // 2^16 hashed rows (independent of m and of the block): bisection
        double lo = 0.01, hi = 4.0 * mean;
        for (int it = 0; it < 60; ++it) {
            const double mid = 0.5 * (lo + hi);
            double s = 0;
            for (int64_t r = 0; r < (1 << 16); ++r) s += (double)row_len(seed, r, alpha, mid, cap, n);
            if (s / (1 << 16) < mean) lo = mid;
            else hi = mid;
        }
        scale = 0.5 * (lo + hi);
    }
    const int64_t nr = row_end - row_begin;
    std::vector<int64_t> cnt((size_t)nr + 1, 0);
    parallel_rows(0, nr, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) cnt[i + 1] = row_len(seed, row_begin + i, alpha, scale, cap, n);
    });
    for (int64_t i = 0; i < nr; ++i) cnt[i + 1] += cnt[i];
    SMFV_REQUIRE(cnt[nr] <= 0x7fffffff, "block nnz exceeds int32 row_ptr");
    int *rp = xmalloc<int>((size_t)nr + 1);
    int *ci = xmalloc<int>((size_t)cnt[nr]);
    double *va = xmalloc<double>((size_t)cnt[nr]);
    if (!rp || !ci || !va) {
        std::free(rp);
        std::free(ci);
        std::free(va);
        set_error("out of memory");
        return SMFV_ERR_HOST;
    }
    for (int64_t i = 0; i <= nr; ++i) rp[i] = (int)cnt[i];
    parallel_rows(0, nr, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const int64_t row = row_begin + i;
            int *c = ci + cnt[i];
            const int64_t L = cnt[i + 1] - cnt[i];
            for (int64_t k = 0; k < L; ++k)
                c[k] = (int)(hash3(seed ^ 0xC0FFEEull, (uint64_t)row, (uint64_t)k) % (uint64_t)n);
            std::sort(c, c + L);
            for (int64_t k = 1; k < L; ++k)  // make distinct: bump forward ...
                if (c[k] <= c[k - 1]) c[k] = c[k - 1] + 1;
            for (int64_t k = L - 1; k >= 0; --k) {  // ... and pull back below n
                const int64_t lim = n - (L - k);
                if (c[k] > lim) c[k] = (int)lim;
                else break;
            }
            for (int64_t k = 1; k < L; ++k)
                if (c[k] <= c[k - 1]) c[k] = c[k - 1] + 1;
            double *v = va + cnt[i];
            for (int64_t k = 0; k < L; ++k)
                v[k] = 2.0 * u01(hash3(seed ^ 0xBEEFull, (uint64_t)row, (uint64_t)k)) - 1.0;
        }
    });
    *out_nnz = cnt[nr];
    *out_rp = rp;
    *out_ci = ci;
    *out_va = va;
    return SMFV_OK;
}

}  // extern "C"
