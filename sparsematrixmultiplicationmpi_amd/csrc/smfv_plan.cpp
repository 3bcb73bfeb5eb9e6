// smfv_plan.cpp -- clustered row-tile analysis of a CSR pattern (host).
//
// The LDS-tiled row kernel processes a tile of rows in one workgroup: the
// distinct X rows the tile touches are staged into LDS once and every
// non-zero of the tile reads its X row from LDS.  Its speed is set by how
// many non-zeros share each staged row (re-use), so tiles are grown as
// clusters: starting from the first unassigned row, repeatedly add the
// candidate row that brings the fewest new columns into the tile's union.
// Candidates are the rows named by the tile's columns (for a square pattern,
// graph neighbours), which for mesh-like matrices grows compact 3-D blocks
// (re-use ~4.3 at a 128-row union on the cop20k_A surrogate, against ~2.1
// for runs of consecutive rows).  Each row is still summed over its
// non-zeros in CSR order, so results are bit-identical.
#include "smfv_plan.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

namespace smfv {

void analyse_tiles(int m, int n, const int *rp, const int *ci, TileAnalysis &A)
{
    A = TileAnalysis();
    const int ncol = std::max(n, 1);
    std::vector<char> assigned((size_t)std::max(m, 1), 0);
    std::vector<int> ustamp((size_t)ncol, -1);      // column in current tile union
    std::vector<int> upos((size_t)ncol, 0);         // its position in the union
    std::vector<int> cstamp((size_t)std::max(m, 1), -1);  // row already a candidate
    std::vector<int64_t> probe((size_t)ncol, -1);   // column counted in a probe
    std::vector<int> cand, rows;
    int64_t probe_id = 0;
    int tile = 0;

    int next_free = 0;
    for (int seed = 0; seed < m; ++seed) {
        if (assigned[seed]) continue;
        next_free = seed + 1;
        int ucount = 0;
        int64_t tnnz = 0, tpad = 0;  // real and row-padded non-zeros
        rows.clear();
        cand.clear();
        const size_t ubase = A.ucols.size();
        auto add_row = [&](int r) {
            assigned[r] = 1;
            rows.push_back(r);
            tnnz += rp[r + 1] - rp[r];
            tpad += (rp[r + 1] - rp[r] + 7) & ~7;
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                const int c = ci[j];
                if (ustamp[c] != tile) {
                    ustamp[c] = tile;
                    upos[c] = ucount++;
                    A.ucols.push_back(c);
                }
                if (c < m && !assigned[c] && cstamp[c] != tile) {
                    cstamp[c] = tile;
                    cand.push_back(c);
                }
            }
        };
        add_row(seed);
        const bool over = ucount > TILE_UCAP || tpad > TILE_NCAP;
        while (!over && (int)rows.size() < TILE_MAXROWS) {
            int best = -1, best_fresh = 1 << 30;
            for (int r : cand) {
                if (assigned[r]) continue;
                ++probe_id;
                int fresh = 0;
                for (int j = rp[r]; j < rp[r + 1]; ++j) {
                    const int c = ci[j];
                    if (ustamp[c] != tile && probe[c] != probe_id) {
                        probe[c] = probe_id;
                        ++fresh;
                    }
                }
                if (fresh < best_fresh || (fresh == best_fresh && r < best)) {
                    best_fresh = fresh;
                    best = r;
                }
            }
            if (best < 0) {
                // no neighbour left (e.g. a diagonal or block-diagonal pattern):
                // continue with the next unassigned row in natural order
                while (next_free < m && assigned[next_free]) ++next_free;
                if (next_free >= m) break;
                best = next_free;
                ++probe_id;
                best_fresh = 0;
                for (int j = rp[best]; j < rp[best + 1]; ++j) {
                    const int c = ci[j];
                    if (ustamp[c] != tile && probe[c] != probe_id) {
                        probe[c] = probe_id;
                        ++best_fresh;
                    }
                }
            }
            if (ucount + best_fresh > TILE_UCAP ||
                tpad + ((rp[best + 1] - rp[best] + 7) & ~7) > TILE_NCAP)
                break;
            add_row(best);
        }
        // rows by decreasing length: the 8 rows of a wave (one per 8-lane
        // team) have similar lengths, so less of the wave idles on the
        // longest row (lane-slot waste 25% -> 15% on the cop20k_A surrogate)
        static const bool by_index = [] {  // lab toggle: SMFV_TILE_SORT=index
            const char *e = std::getenv("SMFV_TILE_SORT");
            return e && std::string(e) == "index";
        }();
        if (by_index)
            std::sort(rows.begin(), rows.end());
        else
            std::sort(rows.begin(), rows.end(), [&](int a, int b) {
                const int la = rp[a + 1] - rp[a], lb = rp[b + 1] - rp[b];
                return la != lb ? la > lb : a < b;
            });

        TileMeta tm{};
        tm.roff = (int)A.trows.size();
        tm.nrows = (int)rows.size();
        tm.noff = (int)A.padded_nnz;
        tm.tn = (int)tnnz;
        tm.direct = over ? 1 : 0;
        if (over) {
            A.ucols.resize(ubase);
            tm.uoff = (int)ubase;
            tm.nu = 0;
        } else {
            tm.uoff = (int)ubase;
            tm.nu = ucount;
            A.union_rows += ucount;
            A.tiled_nnz += tnnz;
        }
        // tile-ordered non-zeros; every ROW segment starts at a multiple of 8
        // entries, so the kernel's 8-wide batches of u16 / f64 LDS reads are
        // 16-byte aligned (unaligned wide LDS reads are replayed); pads
        // (tsrc = -1) are never summed: loops stop at the row's real length
        int local = 0;
        for (int r : rows) {
            A.trows.push_back(r);
            // packed (tile-local start, length); a direct tile's lengths are
            // not used (the kernel reads row_ptr there)
            const int len = rp[r + 1] - rp[r];
            A.rbeg.push_back(over ? local : (local | (len << 16)));
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                A.tsrc.push_back(j);
                A.tlidx.push_back(over ? 0 : (uint16_t)upos[ci[j]]);
                ++local;
            }
            while (local % 8) {
                A.tsrc.push_back(-1);
                A.tlidx.push_back(0);
                ++local;
            }
        }
        tm.tn = local;  // padded segment length (row ends come from rbeg / rp)
        A.padded_nnz += local;
        A.meta.push_back(tm);
        ++tile;
    }
}

std::vector<int> pack_tile_records(const TileAnalysis &A)
{
    std::vector<int> rec(A.meta.size() * TREC_WORDS, 0);
    for (size_t t = 0; t < A.meta.size(); ++t) {
        int *r = rec.data() + t * TREC_WORDS;
        const TileMeta &tm = A.meta[t];
        static_assert(sizeof(TileMeta) == 8 * sizeof(int), "TileMeta is 8 words");
        std::memcpy(r, &tm, sizeof tm);
        for (int k = 0; k < tm.nrows; ++k) {
            r[TREC_ROWS + k] = A.trows[tm.roff + k];
            r[TREC_INFO + k] = A.rbeg[tm.roff + k];
        }
        // union id u at (u % 16) * 8 + u / 16: the staging thread for rows
        // u = xr + 16k finds its 8 ids contiguous
        for (int u = 0; u < tm.nu; ++u) r[TREC_UCOLS + (u % 16) * 8 + u / 16] = A.ucols[tm.uoff + u];
    }
    return rec;
}

}  // namespace smfv
