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
// (re-use 5.8 with <= 64 rows and <= 255 union rows on the cop20k_A
// surrogate, against ~2.1 for runs of consecutive rows).  Each row is still summed over its
// non-zeros in CSR order, so results are bit-identical.
#include "smfv_plan.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <functional>
#include <thread>

namespace smfv {

thread_local int analysis_threads = 0;

namespace {

// Rows that hold each column (the pattern's transpose, O(nnz) to build):
// `all` lists a row once per entry (multiplicity kept: the in-tile
// neighbour count of a candidate counts entries), `dist` once per column.
struct ColumnRows {
    std::vector<int64_t> ptr, dptr;
    std::vector<int> all, dist;
    void build(int m, int n, const int *rp, const int *ci)
    {
        const int nc = std::max(n, 1);
        ptr.assign((size_t)nc + 1, 0);
        dptr.assign((size_t)nc + 1, 0);
        // a row is listed once per column in `dist` even when its repeats of
        // the column are not adjacent (unsorted rows): last row stamp per column
        std::vector<int> last((size_t)nc, -1);
        for (int r = 0; r < m; ++r)
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                ++ptr[(size_t)ci[j] + 1];
                if (last[(size_t)ci[j]] != r) last[(size_t)ci[j]] = r, ++dptr[(size_t)ci[j] + 1];
            }
        for (int c = 0; c < nc; ++c) ptr[c + 1] += ptr[c], dptr[c + 1] += dptr[c];
        all.resize((size_t)ptr[(size_t)nc]);
        dist.resize((size_t)dptr[(size_t)nc]);
        std::vector<int64_t> fa(ptr.begin(), ptr.end() - 1), fd(dptr.begin(), dptr.end() - 1);
        std::fill(last.begin(), last.end(), -1);
        for (int r = 0; r < m; ++r)
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                all[(size_t)fa[(size_t)ci[j]]++] = r;
                if (last[(size_t)ci[j]] != r) last[(size_t)ci[j]] = r, dist[(size_t)fd[(size_t)ci[j]]++] = r;
            }
    }
};

// Per-thread state of the greedy (column- and row-indexed stamps).
struct TileScratch {
    std::vector<int> ustamp, upos, cstamp, rstamp, fresh, inner;
    std::vector<int> hist, fit, small;  // (r5) row-pair check (analyse_part)
    std::vector<int64_t> probe;
    int64_t probe_id = 0;
    TileScratch(int m, int n)
        : ustamp((size_t)std::max(n, 1), -1), upos((size_t)std::max(n, 1), 0), cstamp((size_t)std::max(m, 1), -1),
          rstamp((size_t)std::max(m, 1), -1), fresh((size_t)std::max(m, 1), 0), inner((size_t)std::max(m, 1), 0),
          probe((size_t)std::max(n, 1), -1)
    {
    }
};

// The tiles of one part (positions [lo, hi) of the row order P), appended to
// A with tile ids starting at `tile`; stops after max_tiles tiles in all
// (> 0).  Candidate scores are kept up to date as the tile grows (the union
// gains a column: its rows' fresh counts drop; the tile gains a row: the
// rows naming it gain an in-tile neighbour), so a step costs a scan of the
// candidates' scores, not of their rows.  Returns false when max_tiles ended it.
bool analyse_part(int part, int lo, int hi, const int *P, int m, const int *rp, const int *ci, const ColumnRows &T,
                  const std::vector<int> &pid, const std::vector<int> &ppos, std::vector<char> &assigned,
                  TileScratch &S, TileAnalysis &A, int &tile, const TileCaps &caps)
{
    std::vector<int> cand, rows, front;
    size_t fhead = 0;
    int next_free = 0;
    for (int scan = lo; scan < hi;) {
        int seed = -1;
        if (caps.frontier)
            while (fhead < front.size() && seed < 0) {
                const int r = front[fhead++];
                if (!assigned[r]) seed = r;
            }
        if (seed < 0) {
            while (scan < hi && assigned[P[scan]]) ++scan;
            if (scan >= hi) break;
            seed = P[scan];
        }
        if (caps.max_tiles > 0 && tile >= caps.max_tiles) return false;
        next_free = ppos[(size_t)seed] + 1;  // position after the seed in its part
        int ucount = 0;
        int64_t tnnz = 0, tpad = 0;  // real and row-padded non-zeros
        rows.clear();
        cand.clear();
        const size_t ubase = A.ucols.size();
        // a row's score terms against the current tile, from scratch
        auto score_terms = [&](int r) {
            ++S.probe_id;
            int fresh = 0, inner = 0;
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                const int c = ci[j];
                const int cr = c - caps.col_base;
                if (cr >= 0 && cr < m && S.rstamp[cr] == tile) ++inner;
                if (S.ustamp[c] != tile && S.probe[c] != S.probe_id) {
                    S.probe[c] = S.probe_id;
                    ++fresh;
                }
            }
            S.fresh[r] = fresh;
            S.inner[r] = inner;
        };
        auto add_row = [&](int r) {
            assigned[r] = 1;
            S.rstamp[r] = tile;
            rows.push_back(r);
            tnnz += rp[r + 1] - rp[r];
            tpad += (rp[r + 1] - rp[r] + caps.pad - 1) & ~(caps.pad - 1);
            // union grows: the candidates holding a new column need one fresh row less
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                const int c = ci[j];
                if (S.ustamp[c] == tile) continue;
                S.ustamp[c] = tile;
                S.upos[c] = ucount++;
                A.ucols.push_back(c);
                for (int64_t q = T.dptr[(size_t)c]; q < T.dptr[(size_t)c + 1]; ++q) {
                    const int x = T.dist[(size_t)q];
                    if (S.cstamp[x] == tile && !assigned[x]) --S.fresh[x];
                }
            }
            // r joins the tile: the candidates naming it gain an in-tile neighbour
            const int64_t gc = (int64_t)r + caps.col_base;  // r as a column
            if (gc >= 0 && gc < (int64_t)T.ptr.size() - 1)
                for (int64_t q = T.ptr[(size_t)gc]; q < T.ptr[(size_t)gc + 1]; ++q) {
                    const int x = T.all[(size_t)q];
                    if (S.cstamp[x] == tile && !assigned[x]) ++S.inner[x];
                }
            // new candidates: r's columns as rows of this part
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                const int cr = ci[j] - caps.col_base;  // the column's row in this block
                if (cr >= 0 && cr < m && pid[(size_t)cr] == part && !assigned[cr] && S.cstamp[cr] != tile) {
                    S.cstamp[cr] = tile;
                    cand.push_back(cr);
                    score_terms(cr);
                }
            }
        };
        add_row(seed);
        const bool over = ucount > caps.ucap || tpad > caps.ncap;
        // (r5) row pairs: a tile of n > team_rows rows sums its 2 np = 2 (n -
        // team_rows) shortest rows two to a team, the i-th longest of them
        // with the i-th shortest (build_ws_plan).  A row may join only if that
        // pairing keeps every pair within the whole batches of the tile's
        // longest row (which paces its unit) and every second row within
        // pair_len non-zeros.  The check depends on the joining row's batch
        // count only: computed once per count per step, on a histogram
        auto nbat = [&](int r) { return std::max(1, (rp[r + 1] - rp[r] + 7) >> 3); };
        constexpr int HB = 256;  // batch counts kept (longer rows never pair)
        if (caps.team_rows > 0) {
            S.hist.assign(HB + 1, 0);
            S.hist[std::min(nbat(seed), HB)]++;
        }
        int bmax = nbat(seed);
        const int bpair = std::max(1, caps.pair_len / 8);  // a second row: at most this many whole batches
        int fit_step = -1;
        auto pairs_fit = [&](int b) -> bool {  // rows + 1 (a row of b batches): do the pairs fit?
            const int np = (int)rows.size() + 1 - caps.team_rows;
            if (caps.team_rows <= 0 || np <= 0) return true;
            if (fit_step != (int)rows.size()) fit_step = (int)rows.size(), S.fit.assign(HB + 1, -1);
            const int bc = std::min(b, HB);
            if (S.fit[bc] >= 0) return S.fit[bc] != 0;
            // the 2 np shortest batch counts, ascending
            S.small.clear();
            for (int v = 1; v <= HB && (int)S.small.size() < 2 * np; ++v)
                for (int c = S.hist[v] + (v == bc ? 1 : 0); c > 0 && (int)S.small.size() < 2 * np; --c)
                    S.small.push_back(v);
            bool ok = (int)S.small.size() == 2 * np;
            const int lim = std::max(bmax, b) + caps.pair_slack;
            for (int i = 0; ok && i < np; ++i)
                ok = S.small[i] <= bpair && S.small[i] + S.small[2 * np - 1 - i] <= lim;
            S.fit[bc] = ok ? 1 : 0;
            return ok;
        };
        while (!over && (int)rows.size() < caps.maxrows) {
            int best = -1, best_fresh = 1 << 30;
            long best_score = 1L << 40;
            for (int r : cand) {
                if (assigned[r]) continue;
                // fewest new union rows first; among those, the row with more
                // neighbours already in the tile (compact blobs) and more
                // non-zeros (re-use 5.73 -> 5.80 on the cop20k_A surrogate)
                const int len = rp[r + 1] - rp[r];
                const long score = (long)S.fresh[r] * 64 - S.inner[r] * 16 - len;
                if ((score < best_score || (score == best_score && r < best)) && pairs_fit(nbat(r))) {
                    best_score = score;
                    best_fresh = S.fresh[r];
                    best = r;
                }
            }
            if (best < 0) {
                // no neighbour left (e.g. a diagonal or block-diagonal pattern):
                // continue with the next unassigned row of the part
                while (next_free < hi && assigned[P[next_free]]) ++next_free;
                if (next_free >= hi) break;
                best = P[next_free];
                if (!pairs_fit(nbat(best))) break;
                score_terms(best);
                best_fresh = S.fresh[best];
            }
            if (ucount + best_fresh > caps.ucap ||
                tpad + ((rp[best + 1] - rp[best] + caps.pad - 1) & ~(caps.pad - 1)) > caps.ncap)
                break;
            add_row(best);
            if (caps.team_rows > 0) S.hist[std::min(nbat(best), HB)]++;
            bmax = std::max(bmax, nbat(best));
        }
        if (caps.frontier)
            for (int r : cand)
                if (!assigned[r]) front.push_back(r);
        A.grow.insert(A.grow.end(), rows.begin(), rows.end());
        // rows by decreasing length (build_ws_plan deals them to waves in
        // this order, so the rows of a wave have similar lengths)
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
                A.tlidx.push_back(over ? 0 : (uint16_t)S.upos[ci[j]]);
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
    return true;
}

// B's tiles appended to A (offsets shifted)
void append_analysis(TileAnalysis &A, const TileAnalysis &B)
{
    const int roff = (int)A.trows.size(), uoff = (int)A.ucols.size();
    const int64_t noff = A.padded_nnz;
    for (TileMeta tm : B.meta) {
        tm.roff += roff;
        tm.uoff += uoff;
        tm.noff += (int)noff;
        A.meta.push_back(tm);
    }
    A.trows.insert(A.trows.end(), B.trows.begin(), B.trows.end());
    A.grow.insert(A.grow.end(), B.grow.begin(), B.grow.end());
    A.rbeg.insert(A.rbeg.end(), B.rbeg.begin(), B.rbeg.end());
    A.ucols.insert(A.ucols.end(), B.ucols.begin(), B.ucols.end());
    A.tsrc.insert(A.tsrc.end(), B.tsrc.begin(), B.tsrc.end());
    A.tlidx.insert(A.tlidx.end(), B.tlidx.begin(), B.tlidx.end());
    A.union_rows += B.union_rows;
    A.tiled_nnz += B.tiled_nnz;
    A.padded_nnz += B.padded_nnz;
}

}  // namespace

void analyse_tiles(int m, int n, const int *rp, const int *ci, TileAnalysis &A, const TileCaps &caps)
{
    A = TileAnalysis();
    // caps.part_rows / part_start: row sets tiled one after the other (a tile
    // takes rows of one part only); default one part of all rows in order
    std::vector<int> own_rows, own_start;
    const std::vector<int> *prow = &caps.part_rows, *pst = &caps.part_start;
    if (caps.part_start.size() < 2) {
        own_rows.resize((size_t)m);
        for (int r = 0; r < m; ++r) own_rows[(size_t)r] = r;
        own_start = {0, m};
        prow = &own_rows;
        pst = &own_start;
    }
    const int np = (int)pst->size() - 1;
    std::vector<int> pid((size_t)std::max(m, 1), -1), ppos((size_t)std::max(m, 1), 0);
    for (int x = 0; x < np; ++x)
        for (int k = (*pst)[(size_t)x]; k < (*pst)[(size_t)x + 1]; ++k) {
            pid[(size_t)(*prow)[(size_t)k]] = x;
            ppos[(size_t)(*prow)[(size_t)k]] = k;
        }
    ColumnRows T;
    T.build(m, n, rp, ci);
    std::vector<char> assigned((size_t)std::max(m, 1), 0);  // parts own disjoint rows: shared safely
    // parts are independent (a tile takes the rows of one part; candidates
    // are filtered by part): with several parts and no tile cap they run on
    // threads, each with its own stamps, and are appended in part order --
    // the result does not depend on the thread count
    const int64_t scratch_bytes = ((int64_t)std::max(n, 1) * 16 + (int64_t)std::max(m, 1) * 16);
    int threads = np > 1 && caps.max_tiles <= 0
                      ? (int)std::min<int64_t>({(int64_t)np, 8, std::max<int64_t>(1, ((int64_t)1 << 31) / scratch_bytes)})
                      : 1;
    threads = std::max(1, std::min<int>(threads, (int)std::max(1u, std::thread::hardware_concurrency())));
    if (analysis_threads > 0) threads = std::min(threads, analysis_threads);
    if (threads <= 1) {
        TileScratch S(m, n);
        int tile = 0;
        for (int part = 0; part < np; ++part) {
            A.part_tile.push_back(tile);
            if (!analyse_part(part, (*pst)[(size_t)part], (*pst)[(size_t)part + 1], prow->data(), m, rp, ci, T, pid,
                              ppos, assigned, S, A, tile, caps))
                break;
        }
        while ((int)A.part_tile.size() <= np) A.part_tile.push_back(tile);
        return;
    }
    std::vector<TileAnalysis> out((size_t)np);
    std::atomic<int> next{0};
    auto worker = [&]() {
        TileScratch S(m, n);
        for (int part; (part = next++) < np;) {
            int tile = 0;
            analyse_part(part, (*pst)[(size_t)part], (*pst)[(size_t)part + 1], prow->data(), m, rp, ci, T, pid, ppos,
                         assigned, S, out[(size_t)part], tile, caps);
            // stamps are per tile id: the next part on this thread starts clean
            std::fill(S.ustamp.begin(), S.ustamp.end(), -1);
            std::fill(S.cstamp.begin(), S.cstamp.end(), -1);
            std::fill(S.rstamp.begin(), S.rstamp.end(), -1);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(worker);
    worker();
    for (auto &t : pool) t.join();
    for (int part = 0; part < np; ++part) {
        A.part_tile.push_back((int)A.meta.size());
        append_analysis(A, out[(size_t)part]);
    }
    A.part_tile.push_back((int)A.meta.size());
}

// ---------------------------------------------------------------------------
// k_rows_ws plan
// ---------------------------------------------------------------------------
namespace {

// Replays the reads k_rows_ws makes for every tile and checks that each row's
// entries come out as its CSR non-zeros in order, then pads (zero row).
bool verify_ws_plan(int m, int n, const int *rp, const int *ci, const WsPlan &P, std::string *err)
{
    auto fail = [&](const std::string &msg) {
        if (err) *err = "ws plan: " + msg;
        return false;
    };
    const WsGeom G = P.geom;
    const int R = G.rows();
    std::vector<char> seen((size_t)std::max(m, 1), 0);
    for (int r : P.direct) {
        if (r < 0 || r >= m || seen[r]) return fail("direct row out of range or repeated");
        seen[r] = 1;
    }
    if ((int64_t)P.loff.size() != P.entries + WS_SLACK ||
        (P.live ? (P.vstride != G.ncap / 2 || (int64_t)P.vidx.size() != (int64_t)P.ntiles * P.vstride + WS_SLACK ||
                   !P.tsrc.empty())
                : (int64_t)P.tsrc.size() != P.ventries + WS_SLACK))
        return fail("entry arrays");
    // headers and row ownership (sequential: every row in exactly one place)
    for (int t = 0; t < P.ntiles; ++t) {
        const int *g = &P.grec[(size_t)t * WS_GWORDS];
        const int *l = &P.lrec[(size_t)t * WS_LWORDS];
        const int noff = g[WS_G_NOFF], tn = g[WS_G_TN], nu = g[WS_G_NU], voff = g[WS_G_VOFF], tnv = g[WS_G_TNV];
        for (int q = 0; q < 16; ++q)
            if (g[WS_G_NOFF + q] != noff || g[WS_G_TN + q] != tn || g[WS_G_NU + q] != nu ||
                g[WS_G_VOFF + q] != voff || g[WS_G_TNV + q] != tnv)
                return fail("record header not replicated");
        if (noff % 32 || tn % 32 || tn <= 0 || tn > G.ncap || nu < 0 || nu > G.ucap ||
            (int64_t)noff + tn > P.entries || voff % 8 || tnv % 8 || tnv < 0 || tnv > tn ||
            (int64_t)voff + tnv > P.ventries)
            return fail("tile header out of range");
        for (int slot = 0; slot < R; ++slot) {
            const int r = l[slot], pw = l[3 * R + slot];
            if (r == -1) {
                if (pw != -1) return fail("second row in an empty team");
                continue;
            }
            if (r < 0 || r >= m || seen[r]) return fail("tile row out of range or repeated");
            seen[r] = 1;
            if (pw == -1) continue;
            const int r2 = pw & 0xFFFFFF;
            if (pw < 0 || r2 >= m || seen[r2]) return fail("second row out of range or repeated");
            seen[r2] = 1;
        }
    }
    for (int r = 0; r < m; ++r)
        if (!seen[r]) return fail("row " + std::to_string(r) + " in no tile");
    if (P.xcd[0] != 0 || P.xcd[8] != P.ntiles) return fail("XCD ranges do not cover the tiles");
    for (int x = 0; x < 8; ++x)
        if (P.xcd[x] > P.xcd[x + 1]) return fail("XCD ranges out of order");
    // every tile's entries, replayed as the kernel reads them (tiles in parallel)
    auto check_tile = [&](int t) -> const char * {
        const int *g = &P.grec[(size_t)t * WS_GWORDS];
        const int *l = &P.lrec[(size_t)t * WS_LWORDS];
        const int noff = g[WS_G_NOFF], tn = g[WS_G_TN], nu = g[WS_G_NU], voff = g[WS_G_VOFF], tnv = g[WS_G_TNV];
        for (int q = 0; q < 256; ++q)
            if (g[q] < 0 || g[q] >= n) return "union id out of range";
        for (int e = noff; e < noff + tn; ++e)
            if (P.loff[e] != G.ucap && P.loff[e] >= nu)
                return "entry offset outside the tile's union";
        // one row of a team: L base lb, V base vb, summed length len
        auto check_row = [&](int r, int lb, int len, int vb, int k) -> const char * {
            const int rl = rp[r + 1] - rp[r];
            if (len % 2 || len < rl || len > rl + 1) return "row segment length";
            if (P.live)  // each value slot the row sums starts at its pair of CSR values
                for (int c = 0; c < len / 2; ++c) {
                    const int64_t s = (int64_t)t * P.vstride + vb + 4 * c + k;
                    if (vb + 4 * c + k >= P.vstride || 2 * (vb + 4 * c + k) >= tnv) return "value slot leaves its tile";
                    if (P.vidx[(size_t)s] != rp[r] + 2 * c) return "value slot is not its row's CSR pair";
                }
            // the entries the kernel sums (len: the row's, rounded up to even);
            // past them its reads only prefetch (never summed), so a quad's
            // last batch may store fewer value pairs than offsets
            for (int b = 0; b < (len + 7) / 8; ++b)
                for (int u = 0; u < 8; ++u) {
                    const int el = 8 * b + u;
                    const int64_t le = (int64_t)noff + (int64_t)(lb + 4 * b + k) * 8 + u;
                    const int64_t ve = (int64_t)voff + (int64_t)(vb + 4 * (4 * b + u / 2) + k) * 2 + u % 2;
                    if (le >= noff + tn) return "segment leaves its tile";
                    if (el >= len) {  // never summed: the offset only has to stay on the zero row
                        if (P.loff[le] != G.ucap) return "prefetched pad offset not on the zero row";
                        continue;
                    }
                    if (ve >= voff + tnv) return "segment leaves its tile";
                    if (el < rl) {
                        const int j = rp[r] + el;
                        const int u_ = P.loff[le];
                        const int w = (u_ / 4) % G.lw, i = (u_ / 4) / G.lw, qq = u_ % 4;
                        if ((!P.live && P.tsrc[ve] != j) || P.loff[le] == G.ucap || u_ >= nu ||
                            g[G.gword(w, qq, i)] != ci[j])
                            return "row entry is not its CSR non-zero";
                    } else if ((!P.live && P.tsrc[ve] != -1) || P.loff[le] != G.ucap) {
                        return "pad entry does not read the zero row";
                    }
                }
            return nullptr;
        };
        for (int slot = 0; slot < R; ++slot) {
            const int r = l[slot];
            if (r == -1) continue;
            const int lb = l[R + slot] & 0xFFFF, len = l[R + slot] >> 16, vb = l[2 * R + slot] & 0xFFFF;
            const int k = (slot / G.cw) & 3;  // the team's position in its quad
            const int rl = rp[r + 1] - rp[r];
            if ((l[2 * R + slot] & ~0xFFFF) != (P.live && rl % 2 ? 1 << 30 : 0)) return "row value flags";
            if (const char *e = check_row(r, lb, len, vb, k)) return e;
            const int pw = l[3 * R + slot];
            if (pw != -1) {
                // the second row starts at the batch after the first row's
                // last (an empty first row still owns one batch)
                const int nb = std::max(1, (len + 7) / 8), r2 = pw & 0xFFFFFF;
                if ((pw & (1 << 30)) != (P.live && (rp[r2 + 1] - rp[r2]) % 2 ? 1 << 30 : 0)) return "second row value flags";
                if (const char *e = check_row(r2, lb + 4 * nb, (pw >> 24) & 63, vb + 16 * nb, k)) return e;
            }
        }
        return nullptr;
    };
    const int nt = P.ntiles;
    const int nth = std::max(1, std::min({8, (nt + 63) / 64, (int)std::max(1u, std::thread::hardware_concurrency()),
                                          analysis_threads > 0 ? analysis_threads : 8}));
    std::vector<const char *> bad((size_t)nth, nullptr);
    auto work = [&](int w) {
        for (int t = (int)((int64_t)nt * w / nth); t < (int)((int64_t)nt * (w + 1) / nth) && !bad[(size_t)w]; ++t)
            bad[(size_t)w] = check_tile(t);
    };
    std::vector<std::thread> pool;
    for (int w = 1; w < nth; ++w) pool.emplace_back(work, w);
    work(0);
    for (auto &x : pool) x.join();
    for (const char *b : bad)
        if (b) return fail(b);
    return true;
}

}  // namespace

void range_parts(int m, const int *rp, int parts, std::vector<int> &rows, std::vector<int> &start)
{
    rows.resize((size_t)m);
    for (int r = 0; r < m; ++r) rows[(size_t)r] = r;
    start.assign((size_t)parts + 1, m);
    start[0] = 0;
    for (int x = 1, r = 0; x < parts; ++x) {
        const int64_t target = (int64_t)rp[m] * x / parts;
        while (r < m && rp[r] < target) ++r;
        start[(size_t)x] = r;
    }
}

void bfs_parts(int m, const int *rp, const int *ci, int col_base, int parts, std::vector<int> &rows,
               std::vector<int> &start)
{
    // rows in breadth-first order from row 0 (restarting at the first
    // unvisited row), cut into shares of equal non-zero count
    rows.clear();
    rows.reserve((size_t)m);
    std::vector<char> seen((size_t)std::max(m, 1), 0);
    for (int s = 0; s < m; ++s) {
        if (seen[s]) continue;
        seen[s] = 1;
        rows.push_back(s);
        for (size_t h = rows.size() - 1; h < rows.size(); ++h) {
            const int r = rows[h];
            for (int j = rp[r]; j < rp[r + 1]; ++j) {
                const int c = ci[j] - col_base;
                if (c >= 0 && c < m && !seen[c]) seen[c] = 1, rows.push_back(c);
            }
        }
    }
    start.assign((size_t)parts + 1, m);
    start[0] = 0;
    int64_t acc = 0;
    for (int k = 0, x = 1; k < m && x < parts; ++k) {
        while (x < parts && acc >= (int64_t)rp[m] * x / parts) start[(size_t)x++] = k;
        const int r = rows[(size_t)k];
        acc += rp[r + 1] - rp[r];
    }
}

double parts_footprint(int m, int n, const int *rp, const int *ci, const std::vector<int> &rows,
                       const std::vector<int> &start)
{
    if (m <= 0 || rp[m] <= 0) return 1.0;
    std::vector<int> stamp((size_t)std::max(n, 1), -1);
    int64_t total = 0, sum = 0;
    for (int j = 0; j < rp[m]; ++j)
        if (stamp[ci[j]] != 0) stamp[ci[j]] = 0, ++total;
    std::fill(stamp.begin(), stamp.end(), -1);
    for (size_t x = 0; x + 1 < start.size(); ++x)
        for (int k = start[x]; k < start[x + 1]; ++k) {
            const int r = rows[(size_t)k];
            for (int j = rp[r]; j < rp[r + 1]; ++j)
                if (stamp[ci[j]] != (int)x) stamp[ci[j]] = (int)x, ++sum;
        }
    return (double)sum / (double)total;
}

namespace {
// one k_rows_ws plan: one row per team or row pairs (caps.pairs 0 / 1),
// tiles laid out within tcap entries
bool build_ws_plan_one(int m, int n, const int *rp, const int *ci, WsPlan &P, std::string *err, const TileCaps &caps,
                       int tcap)
{
    // SMFV_PLAN_TIMING=1: the phases' host times on stderr (diagnostic)
    static const bool timing = std::getenv("SMFV_PLAN_TIMING") != nullptr;
    auto tick = [t = std::chrono::steady_clock::now()](const char *what) mutable {
        const auto now = std::chrono::steady_clock::now();
        if (timing)
            std::fprintf(stderr, "[smfv plan] %s %.1f ms\n", what,
                         std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    };
    P = WsPlan();
    const WsGeom G = caps.geom;
    P.geom = G;
    P.live = caps.live;
    P.vstride = caps.live ? G.ncap / 2 : 0;
    if ((G.cw != 8 && G.cw != 4) || G.ucap + 1 > 4 * G.lw * G.ppw || 4 * G.ppw * G.lw > WS_G_NOFF) {
        if (err) *err = "ws plan: unsupported geometry";
        return false;
    }
    // (r5) row pairs: a tile may hold up to twice the kernel's teams in rows;
    // the rows past one per team go, shortest first, as second rows to the
    // teams of the next-shortest (the row index and its even length share
    // one record word: < 2^24 rows, second rows of <= 62 entries, bit 30 the
    // live-values odd-length flag)
    const bool pairs = caps.pairs == 1 && m < (1 << 24);
    TileAnalysis T;
    {
        TileCaps ac = caps;  // ucap / ncap / maxrows follow caps.geom (plan_caps)
        if (pairs) ac.maxrows = 2 * G.rows(), ac.team_rows = G.rows(), ac.pair_len = caps.pair_len;
        analyse_tiles(m, n, rp, ci, T, ac);
    }
    tick("analyse_tiles");

    auto len8 = [&](int r) { return std::max(8, (rp[r + 1] - rp[r] + 7) & ~7); };
    // the length a team computes: its row's, rounded up to even (the kernel
    // ends a row on 0, 2, 4 or 6 entries of a last batch); its storage stays
    // whole batches (quad layout, len8)
    auto len2 = [&](int r) { return (rp[r + 1] - rp[r] + 1) & ~1; };
    // a team (its first row r): second row, whole-batch and summed lengths --
    // the second row's entries follow the first's last batch
    std::vector<int> partner(pairs ? (size_t)m : 0, -1);
    auto second = [&](int r) { return pairs ? partner[(size_t)r] : -1; };
    auto tlen8 = [&](int r) {
        const int b = second(r);
        return len8(r) + (b >= 0 ? len8(b) : 0);
    };
    auto tlen2 = [&](int r) {
        const int b = second(r);
        return b >= 0 ? len8(r) + len2(b) : len2(r);
    };
    // a tile's rows -> its teams (first rows, by decreasing length); false if
    // the rows cannot be teamed (too many, or a second row too long)
    auto make_teams = [&](std::vector<int> &R) -> bool {
        const int NR = G.rows();
        if ((int)R.size() > (pairs ? 2 * NR : NR)) return false;
        std::sort(R.begin(), R.end(), [&](int a, int b) {
            const int la = rp[a + 1] - rp[a], lb = rp[b + 1] - rp[b];
            return la != lb ? la > lb : a < b;
        });
        if (!pairs) return true;
        for (int r : R) partner[(size_t)r] = -1;
        if ((int)R.size() > NR) {
            // the 2 np shortest rows in np teams, the i-th longest with the
            // i-th shortest (even team lengths)
            const size_t n = R.size(), np = n - (size_t)NR, b = n - 2 * np;
            for (size_t i = 0; i < np; ++i)  // (no pair longer than the longest row; 6-bit second lengths)
                if (len2(R[n - 1 - i]) > 62 || std::min(len8(R[b + i]), 8 * 256) + len8(R[n - 1 - i]) >
                                                      len8(R[0]) + 8 * caps.pair_slack)
                    return false;
            for (size_t i = 0; i < np; ++i) partner[(size_t)R[b + i]] = R[n - 1 - i];
            R.resize(n - np);
            std::sort(R.begin(), R.end(), [&](int a, int b) {
                const int la = tlen8(a), lb = tlen8(b), sa = tlen2(a), sb = tlen2(b);
                return la != lb ? la > lb : sa != sb ? sa > sb : a < b;
            });
        }
        return true;
    };
    // entries of a team set sorted by decreasing length: a quad takes 4x its first (longest) team
    auto layout = [&](const std::vector<int> &rows) {
        int64_t e = 0;
        for (size_t q = 0; q < rows.size(); q += 4) e += 4 * (int64_t)tlen8(rows[q]);
        return e;
    };
    auto fits = [&](const std::vector<int> &R) {
        std::vector<int> h = R;
        return make_teams(h) && layout(h) <= tcap;
    };
    // value entries of a quad: its offsets' 32 per batch, less the value
    // pairs of its last batch that no row sums (pair groups q >= qmax of a
    // batch sit last in the quad's value range: rows of 27 store 28, not 32)
    auto vquad = [&](const std::vector<int> &rows, size_t q0) {
        const int nb = tlen8(rows[q0]) / 8;
        int qmax = 0;
        for (size_t k = q0; k < q0 + 4 && k < rows.size(); ++k)
            if (tlen8(rows[k]) / 8 == nb) qmax = std::max(qmax, (tlen2(rows[k]) - 8 * (nb - 1) + 1) / 2);
        return 32 * (int64_t)nb - 8 * (int64_t)(4 - qmax);
    };
    auto vlayout = [&](const std::vector<int> &rows) {
        int64_t e = 0;
        for (size_t q = 0; q < rows.size(); q += 4) e += vquad(rows, q);
        return e;
    };
    // one tile into the plan at entry offset noff, record index t (the
    // tiles are independent: run in parallel, each with its own pos stamps)
    std::vector<std::vector<int>> tunion;  // each tile's union rows (filled before the emit)
    auto emit = [&](const std::vector<int> &R, int64_t noff, int64_t vnoff, int t, std::vector<int> &pos,
                    std::vector<int> &stamp, std::vector<int> &ucols, int64_t &tiled, int64_t &unions) {
        ucols.clear();
        for (int r0 : R)
            for (int r = r0; r >= 0; r = r == r0 ? second(r0) : -1)
                for (int j = rp[r]; j < rp[r + 1]; ++j)
                    if (pos[ci[j]] < 0) {
                        pos[ci[j]] = (int)ucols.size();
                        ucols.push_back(ci[j]);
                    }
        const int nu = (int)ucols.size();
        // issue order: loader wave w stages pieces w, w + 8, ... (4 union
        // rows each) in that order, so positions go out in ascending order;
        // the union rows no tile of the XCD's previous two strides staged
        // (likely HBM, not L2) take the first ones
        if (nu > 4) {
            int x = 0;
            while (x < 7 && t >= P.xcd[x + 1]) ++x;
            const int first = P.xcd[x], nb = std::max(1, caps.xcd_blocks);
            const int lo = std::max(first, t - (t - first) % nb - 2 * nb), hi = t - (t - first) % nb;
            for (int t2 = lo; t2 < hi; ++t2)
                for (int c : tunion[(size_t)t2]) stamp[c] = t;
            std::vector<int> cold, warm;
            for (int c : ucols) (stamp[c] == t ? warm : cold).push_back(c);
            cold.insert(cold.end(), warm.begin(), warm.end());
            ucols.swap(cold);
            for (int u = 0; u < nu; ++u) pos[ucols[(size_t)u]] = u;
        }
        int *lrec = &P.lrec[(size_t)t * WS_LWORDS];
        int *grec = &P.grec[(size_t)t * WS_GWORDS];
        const int NR = G.rows();
        for (int s = 0; s < NR; ++s) lrec[s] = lrec[3 * NR + s] = -1;
        int64_t e = 0, ev = 0;
        for (int q = 0; 4 * q < (int)R.size(); ++q) {
            // 8 compute waves: octet o = quads 2o, 2o + 1 -> one wave, and SIMD s
            // runs octets s and 7 - s (a long and a short one); 4 compute waves
            // (geometry 2, tiles often of 24 rows): quad q -> wave q % 4, half
            // q / 4, so a tile of fewer than 32 rows still keeps all 4 waves busy
            const int o = q / 2;
            const int w = G.cw == 8 ? (o < 4 ? o : 11 - o) : q % 4, h = G.cw == 8 ? q % 2 : q / 4;
            const int nb = tlen8(R[4 * q]) / 8;
            const int lbase = (int)(e / 8), vbase = (int)(ev / 2);
            for (int k = 0; k < 4 && 4 * q + k < (int)R.size(); ++k) {
                const int r = R[4 * q + k], slot = (4 * h + k) * G.cw + w, r2 = second(r);
                // the team's entries: its first row's, then (from the batch
                // after the first row's last) its second row's
                for (int r1 = r, e0 = 0; r1 >= 0; e0 = len8(r), r1 = r1 == r ? r2 : -1)
                    for (int j = rp[r1]; j < rp[r1 + 1]; ++j) {
                        const int el = e0 + j - rp[r1];
                        P.loff[(size_t)(noff + (int64_t)(lbase + 4 * (el / 8) + k) * 8 + el % 8)] =
                            (uint8_t)pos[ci[j]];
                        if (!P.live) P.tsrc[(size_t)(vnoff + (int64_t)(vbase + 4 * (el / 2) + k) * 2 + el % 2)] = j;
                    }
                const int rl = rp[r + 1] - rp[r];
                if (P.live) {  // (r5) value slot of pair c: its first entry's CSR index
                    for (int c = 0; c < len2(r) / 2; ++c) P.vidx[(size_t)t * P.vstride + vbase + 4 * c + k] = rp[r] + 2 * c;
                    if (r2 >= 0)  // the second row's pairs from the batch after the first row's last
                        for (int c = 0; c < len2(r2) / 2; ++c)
                            P.vidx[(size_t)t * P.vstride + vbase + 2 * len8(r) + 4 * c + k] = rp[r2] + 2 * c;
                }
                lrec[slot] = r;
                lrec[NR + slot] = lbase | (len2(r) << 16);
                lrec[2 * NR + slot] = vbase | (P.live && rl % 2 ? 1 << 30 : 0);
                tiled += rl;
                if (r2 >= 0) {
                    lrec[3 * NR + slot] = r2 | (len2(r2) << 24) | (P.live && (rp[r2 + 1] - rp[r2]) % 2 ? 1 << 30 : 0);
                    tiled += rp[r2 + 1] - rp[r2];
                }
            }
            e += 32 * nb;
            ev += vquad(R, (size_t)(4 * q));
        }
        for (int w = 0; w < G.lw; ++w)
            for (int q = 0; q < 4; ++q)
                for (int i = 0; i < G.ppw; ++i) {
                    const int u = 4 * (w + G.lw * i) + q;
                    grec[G.gword(w, q, i)] = u < nu ? ucols[u] : 0;
                }
        for (int q = 0; q < 16; ++q) {
            grec[WS_G_NOFF + q] = (int)noff;
            grec[WS_G_TN + q] = (int)e;
            grec[WS_G_NU + q] = nu;
            grec[WS_G_VOFF + q] = (int)vnoff;
            grec[WS_G_TNV + q] = (int)ev;
        }
        for (int c : ucols) pos[c] = -1;
        unions += nu;
    };

    auto by_length = [&](std::vector<int> &R) {
        std::sort(R.begin(), R.end(), [&](int a, int b) {
            const int la = rp[a + 1] - rp[a], lb = rp[b + 1] - rp[b];
            return la != lb ? la > lb : a < b;
        });
    };
    // final tiles (growth order kept for the end-halving), in wavefront order
    std::vector<std::vector<int>> tiles, stack;
    const int np = (int)T.part_tile.size() - 1;
    std::vector<int> first_tile((size_t)np + 1, 0);  // final tiles: first of each part
    for (size_t t = 0, part = 0; t < T.meta.size(); ++t) {
        while ((int)part < np && (int)t >= T.part_tile[part + 1]) first_tile[++part] = (int)tiles.size();
        const TileMeta &tm = T.meta[t];
        std::vector<int> rows(T.grow.begin() + tm.roff, T.grow.begin() + tm.roff + tm.nrows);
        if (tm.direct) {
            P.direct.insert(P.direct.end(), rows.begin(), rows.end());
            continue;
        }
        if (fits(rows)) {
            tiles.push_back(std::move(rows));
            continue;
        }
        ++P.split;
        std::vector<int> sorted = rows;
        by_length(sorted);
        stack.assign(1, sorted);
        while (!stack.empty()) {
            std::vector<int> R = std::move(stack.back());
            stack.pop_back();
            if (fits(R)) {
                tiles.push_back(std::move(R));
            } else if (R.size() == 1) {
                P.direct.push_back(R[0]);
            } else {
                const size_t h = R.size() / 2;
                stack.emplace_back(R.begin() + h, R.end());
                stack.emplace_back(R.begin(), R.begin() + h);
            }
        }
    }
    for (int x = 1; x <= np; ++x)  // parts after the last tile (and empty ones) start at the end
        if (x == np || T.part_tile[x] >= (int)T.meta.size()) first_tile[x] = std::max(first_tile[x], (int)tiles.size());
    const int nb = caps.split_ends;
    const int64_t N = (int64_t)tiles.size();
    // XCD x runs tiles [xcd[x], xcd[x + 1]): the 8 parts, or 8 equal shares
    // of the order.  Each XCD's blocks run its tiles in rounds of
    // caps.xcd_blocks; a part over the rounds every XCD needs (its first or
    // last tiles, the part's edge) moves to the neighbouring XCD, so no block
    // runs a round more than the tile count requires
    for (int x = 0; x <= 8; ++x) P.xcd[x] = np == 8 ? first_tile[x] : (int)(N * x / 8);
    if (np == 8 && N > 0) {
        const int64_t nbk = std::max(1, caps.xcd_blocks);
        const int64_t cap = nbk * ((N + 8 * nbk - 1) / (8 * nbk));  // tiles per XCD in the fewest rounds
        for (int x = 1; x < 8; ++x)
            P.xcd[x] = (int)std::max<int64_t>(std::min<int64_t>(P.xcd[x], P.xcd[x - 1] + cap),
                                              std::max<int64_t>(N - cap * (8 - x), P.xcd[x - 1]));
    }
    if (nb > 0 && np == 1 && N >= 8 * 3 * (int64_t)nb) {
        // per XCD range [N x / 8, N (x + 1) / 8): its first nb tiles are cut in
        // halves; the range grows by nb, which keeps the kernel's boundaries
        // (N + 8 nb) x / 8 = N x / 8 + nb x aligned with the per-XCD rebuild
        std::vector<std::vector<int>> out;
        out.reserve((size_t)(N + 8 * nb));
        for (int x = 0; x < 8; ++x) {
            const int64_t a = N * x / 8, b = N * (x + 1) / 8, S = b - a + nb;
            std::vector<std::vector<int>> range((size_t)S);
            std::vector<char> used((size_t)S, 0);
            for (int j = 0; j < nb; ++j) {
                std::vector<int> &t = tiles[(size_t)(a + j)];
                const size_t h = (t.size() + 1) / 2;
                const int64_t last = j + ((S - 1 - j) / nb) * nb;  // block j's last unit
                range[(size_t)j].assign(t.begin(), t.begin() + h);
                range[(size_t)last].assign(t.begin() + h, t.end());
                used[(size_t)j] = used[(size_t)last] = 1;
            }
            int64_t k = a + nb;
            for (int64_t q = 0; q < S; ++q)
                if (!used[(size_t)q]) range[(size_t)q] = std::move(tiles[(size_t)k++]);
            for (auto &t : range)
                if (!t.empty()) out.push_back(std::move(t));
        }
        tiles = std::move(out);
        for (int x = 0; x <= 8; ++x) P.xcd[x] = (int)((int64_t)tiles.size() * x / 8);
    }
    tick("split / order tiles");
    // each tile's entry offset (a prefix sum of its quad layout), then the
    // tiles emitted in parallel into their own ranges
    const int nt = (int)tiles.size();
    std::vector<int64_t> toff((size_t)nt + 1, 0), tvoff((size_t)nt + 1, 0);
    for (int t = 0; t < nt; ++t) {
        std::vector<int> &R = tiles[(size_t)t];
        const size_t rows = R.size();
        if (!make_teams(R)) {  // (a half of split_ends: fewer rows than a tile that fit)
            if (err) *err = "ws plan: a tile's rows do not form teams";
            return false;
        }
        P.paired += (int64_t)(rows - R.size());
        toff[(size_t)t + 1] = toff[(size_t)t] + layout(R);
        tvoff[(size_t)t + 1] = tvoff[(size_t)t] + vlayout(R);
    }
    P.ntiles = nt;
    P.entries = toff[(size_t)nt];
    P.ventries = tvoff[(size_t)nt];
    if (P.entries + WS_SLACK > 0x7fffffff) {
        if (err) *err = "ws plan: too many tile entries for int32 offsets";
        return false;
    }
    P.loff.assign((size_t)(P.entries + WS_SLACK), (uint8_t)G.ucap);
    if (P.live)
        P.vidx.assign((size_t)nt * P.vstride + WS_SLACK, 0);
    else
        P.tsrc.assign((size_t)(P.ventries + WS_SLACK), -1);
    P.grec.assign((size_t)nt * WS_GWORDS, 0);
    P.lrec.assign((size_t)nt * WS_LWORDS, 0);
    {
        const int nth = std::max(1, std::min({8, (nt + 63) / 64, (int)std::max(1u, std::thread::hardware_concurrency()),
                                              analysis_threads > 0 ? analysis_threads : 8}));
        std::vector<int64_t> tiled((size_t)nth, 0), unions((size_t)nth, 0);
        tunion.assign((size_t)nt, {});
        auto unite = [&](int w) {
            std::vector<int> seen((size_t)std::max(n, 1), -1);
            for (int t = (int)((int64_t)nt * w / nth); t < (int)((int64_t)nt * (w + 1) / nth); ++t)
                for (int r0 : tiles[(size_t)t])
                    for (int r = r0; r >= 0; r = r == r0 ? second(r0) : -1)
                        for (int j = rp[r]; j < rp[r + 1]; ++j)
                            if (seen[ci[j]] != t) seen[ci[j]] = t, tunion[(size_t)t].push_back(ci[j]);
        };
        auto work = [&](int w) {
            std::vector<int> pos((size_t)std::max(n, 1), -1), stamp((size_t)std::max(n, 1), -1), ucols;
            for (int t = (int)((int64_t)nt * w / nth); t < (int)((int64_t)nt * (w + 1) / nth); ++t)
                emit(tiles[(size_t)t], toff[(size_t)t], tvoff[(size_t)t], t, pos, stamp, ucols, tiled[(size_t)w],
                     unions[(size_t)w]);
        };
        for (auto fn : {std::function<void(int)>(unite), std::function<void(int)>(work)}) {
            std::vector<std::thread> pool;
            for (int w = 1; w < nth; ++w) pool.emplace_back(fn, w);
            fn(0);
            for (auto &x : pool) x.join();
        }
        for (int w = 0; w < nth; ++w) P.tiled_nnz += tiled[(size_t)w], P.union_rows += unions[(size_t)w];
    }
    tick("emit");
    std::sort(P.direct.begin(), P.direct.end());
    const bool ok = verify_ws_plan(m, n, rp, ci, P, err);
    tick("verify");
    return ok;
}
}  // namespace

bool build_ws_plan(int m, int n, const int *rp, const int *ci, WsPlan &P, std::string *err, const TileCaps &caps)
{
    // caps.ncap leaves the quads' interleave room below geom.ncap; a plan of
    // one row per team keeps the same room below geom.ncap1
    const WsGeom G = caps.geom;
    auto one = [&](WsPlan &Q, int pairs, std::string *e) {
        TileCaps c = caps;
        c.pairs = pairs;
        const int tcap = pairs ? G.ncap : G.ncap1;
        c.ncap = caps.ncap - (G.ncap - tcap);
        return build_ws_plan_one(m, n, rp, ci, Q, e, c, tcap);
    };
    if (caps.pairs != 2) return one(P, caps.pairs, err);
    // (r5) both, and the one whose busiest block runs fewer tiles: a round
    // of units costs about the same whatever the tiles hold, and bigger
    // tiles make longer units (measured: row pairs 27.6 -> 25.7 us on the
    // irregular stand-in, 10 -> 8 rounds; 23.5 -> 24.0 us on the stencil
    // one, 8 rounds either way)
    auto rounds = [&](const WsPlan &Q) {
        int r = 0;
        for (int x = 0; x < 8; ++x)
            r = std::max(r, (Q.xcd[x + 1] - Q.xcd[x] + std::max(1, caps.xcd_blocks) - 1) / std::max(1, caps.xcd_blocks));
        return r;
    };
    // the two plans are built side by side (the pair plan on a second
    // thread, with the caller's analysis-thread budget split between them)
    WsPlan Q;
    std::string e2;  // (a pair plan that fails its checks is not taken)
    bool q_ok = false;
    const int budget = analysis_threads > 0 ? analysis_threads : 8;
    const int half = std::max(1, budget / 2);
    std::thread other([&, half] {
        analysis_threads = half;
        q_ok = one(Q, 1, &e2);
    });
    const int saved = analysis_threads;
    analysis_threads = std::max(1, budget - half);
    const bool p_ok = one(P, 0, err);
    analysis_threads = saved;
    other.join();
    if (!p_ok) return false;
    if (q_ok && rounds(Q) < rounds(P)) P = std::move(Q);
    return true;
}

// ---------------------------------------------------------------------------
// k_rows_mfma plan
// ---------------------------------------------------------------------------
bool build_mfma_plan(int m, int n, const int *rp, const int *ci, MfmaPlan &P, std::string *err, const TileCaps &caps)
{
    P = MfmaPlan();
    TileCaps c = caps;
    c.ncap = 1 << 30;  // no LDS entry cap: A goes to registers block by block
    TileAnalysis T;
    analyse_tiles(m, n, rp, ci, T, c);
    std::vector<int> pos((size_t)std::max(n, 1), -1), seen((size_t)std::max(n, 1), -1);
    for (size_t t = 0; t < T.meta.size(); ++t) {
        const TileMeta &tm = T.meta[t];
        std::vector<int> rows;
        for (int k = 0; k < tm.nrows; ++k) {
            const int r = T.trows[tm.roff + k];
            bool dup = tm.direct != 0;
            for (int j = rp[r]; j < rp[r + 1] && !dup; ++j) {
                if (seen[ci[j]] == r) dup = true;
                seen[ci[j]] = r;
            }
            (dup ? P.direct : rows).push_back(r);
        }
        if (rows.empty()) continue;
        // union in first-use order of the kept rows
        std::vector<int> uc;
        for (int r : rows)
            for (int j = rp[r]; j < rp[r + 1]; ++j)
                if (pos[ci[j]] < 0) {
                    pos[ci[j]] = (int)uc.size();
                    uc.push_back(ci[j]);
                }
        const int nu = (int)uc.size();
        if (nu > WS_UCAP) {  // (cannot happen with WS caps; keep the invariant)
            for (int u : uc) pos[u] = -1;
            if (err) *err = "mfma plan: tile union over the cap";
            return false;
        }
        std::vector<int> rec(MF_RWORDS, 0);
        for (int k = 0; k < 64; ++k) rec[k] = k < (int)rows.size() ? rows[k] : -1;
        const int nsteps = (nu + 3) / 4;
        for (int g = 0; g < MF_GROUPS; ++g) {
            rec[64 + 2 * g] = (int)P.blocks;
            int cnt = 0;
            // dense 16 x nu slice of this group: per k-step, the 64 A slots
            std::vector<int> slot((size_t)nsteps * 64, -1);
            for (int i = 0; i < 16; ++i) {
                const int k = 16 * g + i;
                if (k >= (int)rows.size()) break;
                const int r = rows[k];
                for (int j = rp[r]; j < rp[r + 1]; ++j) {
                    const int u = pos[ci[j]];
                    slot[(size_t)(u / 4) * 64 + (u % 4) * 16 + i] = j;  // lane = row + 16 * (k within step)
                    ++P.tiled_nnz;
                }
            }
            for (int st = 0; st < nsteps; ++st) {
                bool any = false;
                for (int l = 0; l < 64 && !any; ++l) any = slot[(size_t)st * 64 + l] >= 0;
                if (!any) continue;
                P.bstep.push_back(st);
                P.tsrc.insert(P.tsrc.end(), slot.begin() + (size_t)st * 64, slot.begin() + (size_t)(st + 1) * 64);
                ++P.blocks;
                ++cnt;
            }
            rec[64 + 2 * g + 1] = cnt;
        }
        rec[64 + 2 * MF_GROUPS] = nu;
        P.rec.insert(P.rec.end(), rec.begin(), rec.end());
        for (int q = 0; q < WS_UCAP; ++q) P.ucols.push_back(q < nu ? uc[q] : 0);
        for (int u : uc) pos[u] = -1;
        P.union_rows += nu;
        ++P.ntiles;
    }
    std::sort(P.direct.begin(), P.direct.end());
    if ((int64_t)P.tsrc.size() > 0x7fffffff) {
        if (err) *err = "mfma plan: too many blocks";
        return false;
    }
    return true;
}

bool build_spmv_chunks(int m, int n, const int *rp, const int *ci, int cap, int maxrows, SpmvChunkPlan &P,
                       std::string *err, bool allow_wide)
{
    auto fail = [&](const char *what, long long a) {
        if (err) {
            char b[160];
            std::snprintf(b, sizeof b, "spmv chunk plan: %s (%lld)", what, a);
            *err = b;
        }
        return false;
    };
    if (cap <= 0 || cap > 65535 || maxrows <= 0 || maxrows > cap) return fail("bad caps", cap);
    P = SpmvChunkPlan();
    P.cap = cap;
    P.maxrows = maxrows;
    for (int r = 0; r < m; ++r) {
        if (rp[r + 1] - rp[r] > cap) return fail("row longer than a chunk", r);
        if (rp[r + 1] > rp[r]) {
            int lo = n, hi = -1;
            for (int j = rp[r]; j < rp[r + 1]; ++j) lo = std::min(lo, ci[j]), hi = std::max(hi, ci[j]);
            if (hi - lo > 65535) P.wide = true;
        }
    }
    if (P.wide && !allow_wide) return fail("row columns span more than 16 bits", 0);
    // greedy packing in row order: a chunk ends when the next row would pass
    // the entry cap, the row cap or (narrow layout) the 16-bit column span
    std::vector<int> first;
    std::vector<int> base;
    int r = 0;
    while (r < m) {
        const int r0 = r;
        int lo = n, hi = -1, cnt = 0;
        while (r < m && r - r0 < maxrows) {
            const int len = rp[r + 1] - rp[r];
            int rlo = lo, rhi = hi;
            if (!P.wide)
                for (int j = rp[r]; j < rp[r + 1]; ++j) rlo = std::min(rlo, ci[j]), rhi = std::max(rhi, ci[j]);
            if (len > 0 && rhi - rlo > 65535) break;  // (narrow only; never the chunk's first row)
            if (cnt + len > cap) break;
            lo = rlo, hi = rhi, cnt += len, ++r;
        }
        first.push_back(r0);
        base.push_back(hi >= 0 ? lo : 0);
    }
    first.push_back(m);
    const int nc = (int)base.size();
    P.nchunks = nc;
    P.hdr.assign((size_t)nc * 4, 0);
    P.rs.assign((size_t)nc * (maxrows + 1), 0);
    if (P.wide)
        P.col.assign((size_t)nc * cap, 0);
    else
        P.off.assign((size_t)nc * cap, 0);
    P.tsrc.assign((size_t)nc * cap, -1);
    for (int c = 0; c < nc; ++c) {
        const int r0 = first[c], nr = first[c + 1] - r0;
        int e = 0;
        for (int t = 0; t < nr; ++t) {
            P.rs[(size_t)c * (maxrows + 1) + t] = (uint16_t)e;
            for (int j = rp[r0 + t]; j < rp[r0 + t + 1]; ++j, ++e) {
                if (P.wide)
                    P.col[(size_t)c * cap + e] = ci[j];
                else
                    P.off[(size_t)c * cap + e] = (uint16_t)(ci[j] - base[c]);
                P.tsrc[(size_t)c * cap + e] = j;
            }
        }
        for (int t = nr; t <= maxrows; ++t) P.rs[(size_t)c * (maxrows + 1) + t] = (uint16_t)e;
        int *h = &P.hdr[(size_t)c * 4];
        h[0] = r0, h[1] = nr, h[2] = base[c], h[3] = e;
        P.entries += e;
    }
    // replay the kernel's reads: every row once, in order, each entry's value
    // index and column as CSR has them
    int next = 0;
    for (int c = 0; c < nc; ++c) {
        const int *h = &P.hdr[(size_t)c * 4];
        if (h[0] != next || h[1] < 0 || h[1] > maxrows || h[3] > cap) return fail("chunk header", c);
        const uint16_t *s = &P.rs[(size_t)c * (maxrows + 1)];
        for (int t = 0; t < h[1]; ++t) {
            const int r = h[0] + t;
            if (s[t + 1] - s[t] != rp[r + 1] - rp[r]) return fail("row length", r);
            for (int k = s[t]; k < s[t + 1]; ++k) {
                const size_t slot = (size_t)c * cap + k;
                const int j = rp[r] + (k - s[t]);
                const int col = P.wide ? P.col[slot] : h[2] + P.off[slot];
                if (P.tsrc[slot] != j || col != ci[j]) return fail("entry", j);
            }
        }
        if (s[h[1]] != h[3]) return fail("chunk entry count", c);
        for (int k = h[3]; k < cap; ++k) {
            const size_t slot = (size_t)c * cap + k;
            if (P.tsrc[slot] != -1 || (P.wide ? P.col[slot] : P.off[slot]) != 0) return fail("pad", c);
        }
        next = h[0] + h[1];
    }
    if (next != m || P.entries != (m ? (int64_t)rp[m] - rp[0] : 0)) return fail("rows not covered", next);
    return true;
}

}  // namespace smfv

// ---------------------------------------------------------------------------
// (r5) k_rows_wsn plan: narrow-team tiles for a 4- / 8-column window
// ---------------------------------------------------------------------------
namespace smfv {

namespace {
// Replays k_rows_wsn's reads for every tile: each row's entries must come out
// as its CSR non-zeros in order, then pads (zero image row, value -0.0).
bool verify_wsn_plan(int m, int n, const int *rp, const int *ci, const WsnPlan &P, std::string *err)
{
    auto fail = [&](const std::string &msg) {
        if (err) *err = "wsn plan: " + msg;
        return false;
    };
    const WsnGeom G = P.geom;
    const int R = G.rows(), TW = G.tw(), LWD = G.lwords();
    std::vector<char> seen((size_t)std::max(m, 1), 0);
    for (int r : P.direct) {
        if (r < 0 || r >= m || seen[r]) return fail("direct row out of range or repeated");
        seen[r] = 1;
    }
    if ((int64_t)P.loff.size() != P.entries + WS_SLACK || (int64_t)P.tsrc.size() != P.ventries + WS_SLACK)
        return fail("entry arrays");
    for (int t = 0; t < P.ntiles; ++t) {
        const int *g = &P.grec[(size_t)t * WSN_GWORDS];
        const int *l = &P.lrec[(size_t)t * LWD];
        const int noff = g[WSN_G_NOFF], tn = g[WSN_G_TN], nu = g[WSN_G_NU], voff = g[WSN_G_VOFF], tnv = g[WSN_G_TNV];
        for (int q = 0; q < 16; ++q)
            if (g[WSN_G_NOFF + q] != noff || g[WSN_G_TN + q] != tn || g[WSN_G_NU + q] != nu ||
                g[WSN_G_VOFF + q] != voff || g[WSN_G_TNV + q] != tnv)
                return fail("record header not replicated");
        if (noff % 8 || tn % 8 || tn <= 0 || tn > G.ncap || nu < 0 || nu > G.ucap || voff % 8 || tnv != tn ||
            (int64_t)noff + tn > P.entries || (int64_t)voff + tnv > P.ventries)
            return fail("tile header out of range");
        for (int u = 0; u < 1024; ++u)
            if (g[u] < 0 || g[u] >= std::max(n, 1) || (u >= nu && g[u] != 0)) return fail("union id out of range");
        for (int w = 0; w < 8; ++w) {
            const int lb = l[R + 2 * w], vb = l[R + 2 * w + 1];
            // the kernel takes n_b (teams of more than b batches) from a ballot
            // and places team k at c_b + k: the running teams must be a prefix
            std::vector<int> nb_at, cum(1, 0);
            for (int k = 0, prev = 255; k < TW; ++k) {
                const int word = l[w * TW + k];
                const int nbk = word == -1 ? 0 : (int)((unsigned)word >> 24);
                if (nbk > prev) return fail("wave rows not in decreasing batch order");
                prev = nbk;
                if ((int)nb_at.size() < nbk) nb_at.resize((size_t)nbk, 0);
                for (int b = 0; b < nbk; ++b) ++nb_at[(size_t)b];
            }
            for (int c : nb_at) cum.push_back(cum.back() + c);
            for (int k = 0; k < TW; ++k) {
                const int word = l[w * TW + k];
                if (word == -1) continue;
                const int r = word & 0xFFFFFF, nbat = (int)((unsigned)word >> 24);
                if (r < 0 || r >= m || seen[r]) return fail("tile row out of range or repeated");
                seen[r] = 1;
                const int rl = rp[r + 1] - rp[r];
                if (nbat != std::max(1, (rl + WSN_B - 1) / WSN_B)) return fail("row batches");
                for (int b = 0; b < nbat; ++b)
                    for (int e = 0; e < WSN_B; ++e) {
                        const int el = WSN_B * b + e;
                        const int64_t le = (int64_t)noff + WSN_B * (int64_t)(lb + cum[(size_t)b] + k) + e;
                        const int64_t ve =
                            (int64_t)voff +
                            2 * (int64_t)(vb + 2 * cum[(size_t)b] + (e / 2) * nb_at[(size_t)b] + k) + e % 2;
                        if (le < noff || le >= noff + tn || ve < voff || ve >= voff + tnv)
                            return fail("segment leaves its tile");
                        if (el < rl) {
                            const int j = rp[r] + el, u = P.loff[(size_t)le];
                            if (P.tsrc[(size_t)ve] != j || u >= nu || g[u] != ci[j])
                                return fail("row entry is not its CSR non-zero");
                        } else if (P.tsrc[(size_t)ve] != -1 || P.loff[(size_t)le] != G.ucap) {
                            return fail("pad entry does not read the zero row");
                        }
                    }
            }
        }
    }
    for (int r = 0; r < m; ++r)
        if (!seen[r]) return fail("row " + std::to_string(r) + " in no tile");
    return true;
}
}  // namespace

namespace {
// (r6) Image slots of a tile's union rows, coloured for the
// LDS banks of k_rows_wsn's X reads.  A team reads its entry's image row
// (XROW = 32 / 64 B: 8 / 16 of the 64 banks) with one ds_read_b128, whose 64
// lanes are serviced in 4 lane groups of 16 ({0-3,12-15,20-27},
// {4-11,16-19,28-31}, the same + 32): 8 teams of 2 lanes (KW = 4) or 4 of 4
// (KW = 8) per group.  Image row s sits in bank group s mod C (C = 256 /
// XROW = 8 / 4), so two teams of one lane group that read different rows of
// one colour in the same instruction conflict (each extra distinct address
// on a bank costs an LDS cycle: a group's cycles = its most-loaded colour).
// The plan is free to put any union row in any image slot, so this colours
// the union rows: the lane groups of every (wave, batch, entry) instruction
// are collected (teams still running in that batch; pads read the zero row,
// colour ucap mod C, all at one address), then each union row -- most-read
// first -- takes the colour that meets the fewest rows already placed in its
// groups, with at most ceil(nu / C) + 1 rows per colour; two refinement
// passes move single rows.  Colour c's i-th row gets slot c + C i; the image
// then has S >= nu rows (holes stage X row 0, unread).  `cycles` models the
// LDS cycles of the tile's X reads (one per non-empty lane group, plus its
// conflicts); `plain` the same for first-use slots (slot = union position).
struct WsnSlots {
    std::vector<int> slot;  // union position -> image row
    int S = 0;              // image rows staged
    int64_t groups = 0, cycles = 0, plain = 0;
};

inline int b128_lane_group(int l)
{
    const int h = l & 31;
    const bool a = h < 4 || (h >= 12 && h < 16) || (h >= 20 && h < 28);
    return (l >> 5) * 2 + (a ? 0 : 1);
}

WsnSlots colour_wsn_slots(const WsnGeom &G, const int *rp, const int *ci, const std::vector<int> &Rw,
                          const std::vector<int> &pos, int nu, bool colour, bool model_only_if_colour = true)
{
    WsnSlots W;
    if (!colour && model_only_if_colour) {  // first-use slots, no model (the fast path of the fraction search)
        W.slot.resize((size_t)nu);
        for (int u = 0; u < nu; ++u) W.slot[(size_t)u] = u;
        W.S = nu;
        return W;
    }
    const int TW = G.tw(), TL = G.tl(), C = 256 / G.xrow(), ZC = G.ucap % C;
    const int PAD = nu;  // the zero row, as a member id
    auto nbat = [&](int r) { return std::max(1, (rp[r + 1] - rp[r] + WSN_B - 1) / WSN_B); };
    // every running team's entry as (group key, member), bucketed by key
    // (counting sort: keys are dense), then de-duplicated inside each group
    // (one address reads once: broadcast)
    const int maxb = Rw.empty() ? 1 : nbat(Rw[0]) + 1;
    const int nkeys = 8 * maxb * WSN_B * 4;
    std::vector<int> kk, km;
    kk.reserve(4096), km.reserve(4096);
    for (int q = 0; q < 8 && (size_t)q * TW < Rw.size(); ++q) {
        const int nt_q = (int)std::min<size_t>(TW, Rw.size() - (size_t)q * TW);
        for (int k = 0; k < nt_q; ++k) {
            const int r = Rw[(size_t)(q * TW + k)], rl = rp[r + 1] - rp[r], lg = b128_lane_group(k * TL);
            for (int b = 0; b < nbat(r); ++b)
                for (int e = 0; e < WSN_B; ++e) {
                    const int el = WSN_B * b + e;
                    kk.push_back(((q * maxb + b) * WSN_B + e) * 4 + lg);
                    km.push_back(el < rl ? pos[ci[rp[r] + el]] : PAD);
                }
        }
    }
    std::vector<int> kstart((size_t)nkeys + 1, 0);
    for (int key : kk) ++kstart[(size_t)key + 1];
    for (int i = 0; i < nkeys; ++i) kstart[(size_t)i + 1] += kstart[(size_t)i];
    std::vector<int> memv(kk.size());
    {
        std::vector<int> at(kstart.begin(), kstart.end() - 1);
        for (size_t i = 0; i < kk.size(); ++i) memv[(size_t)at[(size_t)kk[i]]++] = km[i];
    }
    // groups: the non-empty keys, members sorted and unique (PAD = nu last)
    std::vector<int> gstart, mem;
    mem.reserve(memv.size());
    for (int key = 0; key < nkeys; ++key) {
        const int a = kstart[(size_t)key], b = kstart[(size_t)key + 1];
        if (a == b) continue;
        std::sort(memv.begin() + a, memv.begin() + b);
        gstart.push_back((int)mem.size());
        for (int i = a; i < b; ++i)
            if (i == a || memv[(size_t)i] != memv[(size_t)i - 1]) mem.push_back(memv[(size_t)i]);
    }
    const int ng = (int)gstart.size();
    gstart.push_back((int)mem.size());
    W.groups = ng;
    std::vector<int> deg((size_t)nu + 1, 0), gof((size_t)mem.size());
    for (int g = 0; g < ng; ++g)
        for (int i = gstart[g]; i < gstart[g + 1]; ++i) {
            gof[(size_t)i] = g;
            ++deg[(size_t)mem[(size_t)i]];
        }
    std::vector<int> cptr((size_t)nu + 2, 0), cg((size_t)mem.size());
    for (int u = 0; u <= nu; ++u) cptr[(size_t)u + 1] = cptr[(size_t)u] + deg[(size_t)u];
    {
        std::vector<int> fill(cptr.begin(), cptr.end() - 1);
        for (size_t i = 0; i < mem.size(); ++i) cg[(size_t)fill[(size_t)mem[i]]++] = gof[i];
    }
    auto model = [&](const std::vector<int> &col) {  // LDS cycles: per group its most-loaded colour
        int64_t cyc = 0;
        std::vector<int> cnt((size_t)C);
        for (int g = 0; g < ng; ++g) {
            std::fill(cnt.begin(), cnt.end(), 0);
            int mx = 0;
            for (int i = gstart[g]; i < gstart[g + 1]; ++i) {
                const int u = mem[(size_t)i];
                mx = std::max(mx, ++cnt[(size_t)(u == PAD ? ZC : col[(size_t)u])]);
            }
            cyc += mx;
        }
        return cyc;
    };
    std::vector<int> plain((size_t)nu);
    for (int u = 0; u < nu; ++u) plain[(size_t)u] = u % C;
    W.plain = model(plain);
    auto first_use = [&]() {
        W.slot.resize((size_t)nu);
        for (int u = 0; u < nu; ++u) W.slot[(size_t)u] = u;
        W.S = nu;
        W.cycles = W.plain;
        return W;
    };
    if (!colour || nu == 0) return first_use();
    // capacity per colour: slots c + C i below the zero row (ucap)
    const int want = (nu + C - 1) / C + 1;
    std::vector<int> cap((size_t)C), used((size_t)C, 0);
    for (int c = 0; c < C; ++c) cap[(size_t)c] = std::min(want, (G.ucap - c + C - 1) / C);
    std::vector<int> cnt((size_t)ng * C, 0), col((size_t)nu, -1);
    for (int g = 0; g < ng; ++g)
        if (mem[(size_t)gstart[g + 1] - 1] == PAD)
            cnt[(size_t)g * C + ZC] = 1;  // (PAD sorts last in its group)
    std::vector<int> order((size_t)nu);
    for (int u = 0; u < nu; ++u) order[(size_t)u] = u;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return deg[(size_t)a] > deg[(size_t)b]; });
    auto place = [&](int u) {
        int cost[8] = {};
        for (int i = cptr[(size_t)u]; i < cptr[(size_t)u + 1]; ++i) {
            const int *cc = &cnt[(size_t)cg[(size_t)i] * C];
            for (int c = 0; c < C; ++c) cost[c] += cc[c];
        }
        int best = -1;
        for (int c = 0; c < C; ++c) {
            if (used[(size_t)c] >= cap[(size_t)c]) continue;
            if (best < 0 || cost[c] < cost[best] || (cost[c] == cost[best] && used[(size_t)c] < used[(size_t)best]))
                best = c;
        }
        if (best < 0) return false;
        col[(size_t)u] = best;
        ++used[(size_t)best];
        for (int i = cptr[(size_t)u]; i < cptr[(size_t)u + 1]; ++i) ++cnt[(size_t)cg[(size_t)i] * C + best];
        return true;
    };
    for (int u : order)
        if (!place(u)) return first_use();
    for (int pass = 0; pass < 2; ++pass)
        for (int u : order) {
            const int c0 = col[(size_t)u];
            --used[(size_t)c0];
            for (int i = cptr[(size_t)u]; i < cptr[(size_t)u + 1]; ++i) --cnt[(size_t)cg[(size_t)i] * C + c0];
            place(u);  // (its own colour has room again: always placed)
        }
    const int64_t cyc = model(col);
    if (cyc >= W.plain) return first_use();  // never worse than first-use slots
    W.cycles = cyc;
    W.slot.assign((size_t)nu, 0);
    std::vector<int> next((size_t)C, 0);
    W.S = 0;
    for (int u = 0; u < nu; ++u) {
        const int c = col[(size_t)u];
        W.slot[(size_t)u] = c + C * next[(size_t)c]++;
        W.S = std::max(W.S, W.slot[(size_t)u] + 1);
    }
    return W;
}

bool build_wsn_plan_at(int m, int n, const int *rp, const int *ci, int kw, WsnPlan &P, std::string *err,
                       const TileCaps &caps_in, int frac_num, int frac_den)
{
    P = WsnPlan();
    if (kw != 4 && kw != 8) {
        if (err) *err = "wsn plan: window must be 4 or 8 columns";
        return false;
    }
    const WsnGeom G = wsn_geom(kw);
    P.geom = G;
    const int TW = G.tw(), R = G.rows(), LWD = G.lwords();
    TileCaps caps = caps_in;
    caps.ucap = G.ucap;
    caps.maxrows = R;
    caps.pad = WSN_B;
    // the analysis counts each row padded to WSN_B entries, the layout's own
    // figure for the trimmed batches but for its 16-byte round-up (hence the
    // 8 entries of room); the layout checks the real figure (splitting a tile
    // that still overflows, e.g. one holding empty rows, which own a batch)
    caps.ncap = G.ncap * frac_num / frac_den - 8;
    // SMFV_PLAN_TIMING=1: the phases' host times on stderr (diagnostic)
    static const bool timing = std::getenv("SMFV_PLAN_TIMING") != nullptr;
    auto tick = [t = std::chrono::steady_clock::now()](const char *what) mutable {
        const auto now = std::chrono::steady_clock::now();
        if (timing)
            std::fprintf(stderr, "[smfv wsn plan] %s %.1f ms\n", what,
                         std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    };
    TileAnalysis T;
    analyse_tiles(m, n, rp, ci, T, caps);
    tick("analyse_tiles");

    auto nbat = [&](int r) { return std::max(1, (rp[r + 1] - rp[r] + WSN_B - 1) / WSN_B); };
    auto by_length = [&](std::vector<int> &rows) {
        std::sort(rows.begin(), rows.end(), [&](int a, int b) {
            const int la = rp[a + 1] - rp[a], lb = rp[b + 1] - rp[b];
            return la != lb ? la > lb : a < b;
        });
    };
    auto layout = [&](const std::vector<int> &rows) {  // entries with pads, trimmed per batch (16-byte multiple)
        int64_t e = 0;
        for (int r : rows) e += (int64_t)nbat(r) * WSN_B;
        return (e + 7) & ~(int64_t)7;
    };
    std::vector<std::vector<int>> tiles, stack;
    const int np = (int)T.part_tile.size() - 1;
    std::vector<int> first_tile((size_t)np + 1, 0);
    for (size_t t = 0, part = 0; t < T.meta.size(); ++t) {
        while ((int)part < np && (int)t >= T.part_tile[part + 1]) first_tile[++part] = (int)tiles.size();
        const TileMeta &tm = T.meta[t];
        std::vector<int> rows(T.grow.begin() + tm.roff, T.grow.begin() + tm.roff + tm.nrows);
        if (tm.direct) {
            P.direct.insert(P.direct.end(), rows.begin(), rows.end());
            continue;
        }
        by_length(rows);
        stack.assign(1, rows);
        while (!stack.empty()) {
            std::vector<int> Rw = std::move(stack.back());
            stack.pop_back();
            if (layout(Rw) <= G.ncap && nbat(Rw[0]) <= 255) {
                tiles.push_back(std::move(Rw));
            } else if (Rw.size() == 1) {
                P.direct.push_back(Rw[0]);
            } else {
                const size_t h = Rw.size() / 2;
                stack.emplace_back(Rw.begin() + h, Rw.end());
                stack.emplace_back(Rw.begin(), Rw.begin() + h);
            }
        }
    }
    for (int x = 1; x <= np; ++x)
        if (x == np || T.part_tile[x] >= (int)T.meta.size()) first_tile[x] = std::max(first_tile[x], (int)tiles.size());
    const int64_t N = (int64_t)tiles.size();
    for (int x = 0; x <= 8; ++x) P.xcd[x] = np == 8 ? first_tile[x] : (int)(N * x / 8);
    if (np == 8 && N > 0) {  // no XCD runs a round more than the tile count needs (as build_ws_plan)
        const int64_t nbk = std::max(1, caps.xcd_blocks);
        const int64_t cap = nbk * ((N + 8 * nbk - 1) / (8 * nbk));
        for (int x = 1; x < 8; ++x)
            P.xcd[x] = (int)std::max<int64_t>(std::min<int64_t>(P.xcd[x], P.xcd[x - 1] + cap),
                                              std::max<int64_t>(N - cap * (8 - x), P.xcd[x - 1]));
    }
    const int nt = (int)N;
    tick("tiles split");
    std::vector<int64_t> toff((size_t)nt + 1, 0);
    for (int t = 0; t < nt; ++t) toff[(size_t)t + 1] = toff[(size_t)t] + layout(tiles[(size_t)t]);
    P.ntiles = nt;
    P.entries = P.ventries = toff[(size_t)nt];
    if (P.entries + WS_SLACK > 0x7fffffff) {
        if (err) *err = "wsn plan: too many tile entries for int32 offsets";
        return false;
    }
    P.loff.assign((size_t)(P.entries + WS_SLACK), (uint16_t)G.ucap);
    P.tsrc.assign((size_t)(P.ventries + WS_SLACK), -1);
    P.grec.assign((size_t)nt * WSN_GWORDS, 0);
    P.lrec.assign((size_t)nt * LWD, 0);
    std::vector<int> pos((size_t)std::max(n, 1), -1), ucols;
    for (int t = 0; t < nt; ++t) {
        const std::vector<int> &Rw = tiles[(size_t)t];
        const int64_t noff = toff[(size_t)t];
        ucols.clear();
        for (int r : Rw)
            for (int j = rp[r]; j < rp[r + 1]; ++j)
                if (pos[ci[j]] < 0) {
                    pos[ci[j]] = (int)ucols.size();
                    ucols.push_back(ci[j]);
                }
        const int nu = (int)ucols.size();
        int *g = &P.grec[(size_t)t * WSN_GWORDS];
        int *l = &P.lrec[(size_t)t * LWD];
        // (r6) union rows in bank-coloured image slots (holes: X row 0, unread)
        const WsnSlots SL = colour_wsn_slots(G, rp, ci, Rw, pos, nu, caps.wsn_colour, !caps.wsn_model);
        for (int u = 0; u < nu; ++u) g[SL.slot[(size_t)u]] = ucols[(size_t)u];
        P.x_groups += SL.groups;
        P.x_cycles += SL.cycles;
        P.x_cycles_plain += SL.plain;
        P.staged_rows += SL.S;
        for (int s = 0; s < R; ++s) l[s] = -1;
        // wave group q (TW consecutive rows of the sorted list) -> wave w;
        // groups q and 7 - q share a SIMD (waves w and w + 4)
        // (r5) per batch only the wave's teams still running (smfv_plan.h)
        int64_t chunk = 0;  // offset chunks so far (WSN_B entries each)
        int lbase[8] = {}, vbase[8] = {};
        for (int w = 0; w < 8; ++w) {
            const int q = w < 4 ? w : 11 - w;  // the wave's group
            lbase[w] = (int)chunk;
            vbase[w] = (int)(WSN_B / 2 * chunk);
            for (int k = 0; k < TW && (size_t)(q * TW + k) < Rw.size(); ++k) chunk += nbat(Rw[(size_t)(q * TW + k)]);
        }
        std::vector<int> nb_at, cum;
        for (int q = 0; q < 8 && (size_t)q * TW < Rw.size(); ++q) {
            const int w = q < 4 ? q : 11 - q;
            const int nt_q = (int)std::min<size_t>(TW, Rw.size() - (size_t)q * TW);
            const int NB = nbat(Rw[(size_t)q * TW]);
            nb_at.assign((size_t)NB, 0);
            cum.assign((size_t)NB + 1, 0);
            for (int k = 0; k < nt_q; ++k)
                for (int b = 0; b < nbat(Rw[(size_t)(q * TW + k)]); ++b) ++nb_at[(size_t)b];
            for (int b = 0; b < NB; ++b) cum[(size_t)b + 1] = cum[(size_t)b] + nb_at[(size_t)b];
            for (int k = 0; k < nt_q; ++k) {
                const int r = Rw[(size_t)(q * TW + k)];
                l[w * TW + k] = r | (nbat(r) << 24);
                for (int j = rp[r]; j < rp[r + 1]; ++j) {
                    const int el = j - rp[r], b = el / WSN_B, e = el % WSN_B;
                    P.loff[(size_t)(noff + WSN_B * (int64_t)(lbase[w] + cum[(size_t)b] + k) + e)] =
                        (uint16_t)SL.slot[(size_t)pos[ci[j]]];
                    P.tsrc[(size_t)(noff +
                                    2 * (int64_t)(vbase[w] + 2 * cum[(size_t)b] + (e / 2) * nb_at[(size_t)b] + k) +
                                    e % 2)] = j;
                }
                P.tiled_nnz += rp[r + 1] - rp[r];
            }
        }
        for (int w = 0; w < 8; ++w) {
            l[R + 2 * w] = lbase[w];
            l[R + 2 * w + 1] = vbase[w];
        }
        for (int q = 0; q < 16; ++q) {
            g[WSN_G_NOFF + q] = (int)noff;
            g[WSN_G_TN + q] = (int)(toff[(size_t)t + 1] - noff);
            g[WSN_G_NU + q] = SL.S;
            g[WSN_G_VOFF + q] = (int)noff;
            g[WSN_G_TNV + q] = (int)(toff[(size_t)t + 1] - noff);
        }
        for (int c : ucols) pos[c] = -1;
        P.union_rows += nu;
    }
    std::sort(P.direct.begin(), P.direct.end());
    tick("layout");
    const bool ok = verify_wsn_plan(m, n, rp, ci, P, err);
    tick("verify");
    return ok;
}
}  // namespace

// The analysis aims at a fraction of the entry cap (it counts each row
// padded to 4, as the layout's trimmed batches do; a tile that still
// overflows is split in halves).  The kernel's time follows the rounds of
// units on its busiest blocks (32 per XCD), so six fractions (3/4 .. 1) are
// built and the plan with the fewest rounds is kept, then the fewest tiles
// (r5, cop20k stand-ins: 705 / 968 stencil, 762 / 1,184 irregular tiles at
// K = 4 / 8: 3 / 4 / 3 / 5 rounds; ColumnWise rank panels 4-10 % faster
// than the previous 819 / 1,084 / 870 / 1,286, profiles/r05/wsn/README.md).
bool build_wsn_plan(int m, int n, const int *rp, const int *ci, int kw, WsnPlan &P, std::string *err,
                    const TileCaps &caps)
{
    static constexpr int fr[6][2] = {{3, 4}, {13, 16}, {7, 8}, {9, 10}, {15, 16}, {1, 1}};
    const int nbk = std::max(1, caps.xcd_blocks);
    auto rounds = [&](const WsnPlan &W) {  // units on the busiest blocks
        int r = 0;
        for (int x = 0; x < 8; ++x) r = std::max(r, (W.xcd[x + 1] - W.xcd[x] + nbk - 1) / nbk);
        return r;
    };
    bool any = false;
    // (r6) the fractions are compared on first-use slots (the choice does not
    // depend on the slot order); the winner alone is rebuilt with coloured
    // slots (A/B: SMFV_WSN_FIRST_USE_SLOTS keeps first-use slots)
    TileCaps cs = caps;
    const bool colour = caps.wsn_colour && !std::getenv("SMFV_WSN_FIRST_USE_SLOTS");
    cs.wsn_colour = false;
    int best = -1;
    for (int i = 0; i < 6; ++i) {
        WsnPlan Q;
        std::string e;
        if (!build_wsn_plan_at(m, n, rp, ci, kw, Q, &e, cs, fr[i][0], fr[i][1])) {
            if (err && !any) *err = e;
            continue;
        }
        const bool better = !any || rounds(Q) < rounds(P) ||
                            (rounds(Q) == rounds(P) &&
                             (Q.ntiles < P.ntiles || (Q.ntiles == P.ntiles && Q.union_rows < P.union_rows)));
        if (better) P = std::move(Q), best = i;
        any = true;
    }
    if (any && (colour || caps.wsn_model)) {
        cs.wsn_colour = colour;
        WsnPlan Q;
        std::string e;
        if (build_wsn_plan_at(m, n, rp, ci, kw, Q, &e, cs, fr[best][0], fr[best][1])) P = std::move(Q);
    }
    return any;
}

}  // namespace smfv
