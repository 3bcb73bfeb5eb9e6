// Lab (host only, not part of the product): how many X rows a block must
// stage into LDS when its LDS holds a software cache of S X rows and it
// walks a stream of row tiles, under two row orders.
//   plan_sim <matrix.smfvcsr> <streams G> <slots S> <rows per tile R>
#include "smfv.h"
#include "smfv_host.h"
#include "smfv_plan.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <queue>
#include <set>
#include <vector>

using namespace smfv;

// Belady (furthest next use) over a sequence of tiles, each needing a set of
// rows; rows used by the next W tiles (in flight) are never evicted.
static long long simulate(const std::vector<std::vector<int>> &tiles, int S, int W)
{
    // next-use index for each (tile, row)
    std::map<int, std::vector<int>> uses;
    for (int t = 0; t < (int)tiles.size(); ++t)
        for (int r : tiles[t]) uses[r].push_back(t);
    std::map<int, int> ptr;
    std::set<int> cache;
    long long loads = 0;
    auto next_use = [&](int r, int after) {
        auto &v = uses[r];
        auto it = std::upper_bound(v.begin(), v.end(), after);
        return it == v.end() ? 1 << 30 : *it;
    };
    for (int t = 0; t < (int)tiles.size(); ++t) {
        for (int r : tiles[t]) {
            if (cache.count(r)) continue;
            ++loads;
            if ((int)cache.size() >= S) {
                int victim = -1, far = -1;
                for (int c : cache) {
                    int nu = next_use(c, t - 1);
                    bool needed_now = nu <= t + W;
                    if (needed_now) continue;
                    if (nu > far) { far = nu; victim = c; }
                }
                if (victim < 0) { return -1; }  // window does not fit
                cache.erase(victim);
            }
            cache.insert(r);
        }
    }
    return loads;
}

int main(int argc, char **argv)
{
    int m, n, *rp, *ci;
    int64_t nnz;
    double *va;
    if (argc < 5 || smfv_csr_read_bin(argv[1], &m, &n, &nnz, &rp, &ci, &va) != SMFV_OK) return 1;
    const int G = atoi(argv[2]), S = atoi(argv[3]), R = atoi(argv[4]);
    // order A: natural; order B: clustered tile order (analyse_tiles)
    TileAnalysis T;
    analyse_tiles(m, n, rp, ci, T);
    std::vector<int> clus;
    for (auto &tm : T.meta)
        for (int k = 0; k < tm.nrows; ++k) clus.push_back(T.trows[tm.roff + k]);
    std::vector<int> nat(m);
    for (int i = 0; i < m; ++i) nat[i] = i;
    for (int which = 0; which < 2; ++which) {
        const std::vector<int> &ord = which ? clus : nat;
        long long tot = 0, uniq = 0;
        int worst = 0;
        for (int g = 0; g < G; ++g) {
            const int a = (int)((long long)m * g / G), b = (int)((long long)m * (g + 1) / G);
            std::vector<std::vector<int>> tiles;
            std::set<int> u;
            for (int s = a; s < b; s += R) {
                std::set<int> tu;
                for (int i = s; i < std::min(b, s + R); ++i)
                    for (int j = rp[ord[i]]; j < rp[ord[i] + 1]; ++j) tu.insert(ci[j]);
                tiles.emplace_back(tu.begin(), tu.end());
                u.insert(tu.begin(), tu.end());
                worst = std::max(worst, (int)tu.size());
            }
            uniq += u.size();
            long long l = simulate(tiles, S, 2);
            if (l < 0) { printf("order %d: window does not fit S=%d\n", which, S); tot = -1; break; }
            tot += l;
        }
        printf("order %s G=%d S=%d R=%d: loads %lld (reuse %.2f) unique-per-stream %lld (reuse %.2f) max tile union %d\n",
               which ? "cluster" : "natural", G, S, R, tot, (double)nnz / tot, uniq, (double)nnz / uniq, worst);
    }
    return 0;
}
