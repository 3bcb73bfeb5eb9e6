// cs_plan_lab.cpp -- LAB ONLY (compiled into libsmfv_lab.so): the
// column-streamed tile plan of k_rows_cs (see cs_plan_lab.h).
#include "lab/cs_plan_lab.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>

namespace smfv {

// ---------------------------------------------------------------------------
// k_rows_cs plan (column-streamed tiles)
// ---------------------------------------------------------------------------
namespace {

// Replays k_rows_cs's reads of every chunk: each row's entries, chunk after
// chunk and step after step, must come out as its CSR non-zeros in order
// (value source and X row), everything else as pads on the zero row; each
// row's last real entry lies in the chunk tlast names.
bool verify_cs_plan(int m, int n, const int *rp, const int *ci, const CsPlan &P, std::string *err)
{
    auto fail = [&](const std::string &msg) {
        if (err) *err = "cs plan: " + msg;
        return false;
    };
    if ((int)P.tfirst.size() != P.ntiles || (int)P.trow.size() != P.ntiles * CS_ROWS ||
        P.tlast.size() != P.trow.size() || (int64_t)P.crec.size() != (int64_t)P.nchunks * CS_CWORDS)
        return fail("array sizes");
    if (P.xcd[0] != 0 || P.xcd[8] != P.ntiles) return fail("XCD ranges do not cover the tiles");
    for (int x = 0; x < 8; ++x)
        if (P.xcd[x] > P.xcd[x + 1]) return fail("XCD ranges out of order");
    std::vector<char> seen((size_t)std::max(m, 1), 0);
    for (int t = 0; t < P.ntiles; ++t)
        for (int s = 0; s < CS_ROWS; ++s) {
            const int r = P.trow[(size_t)t * CS_ROWS + s];
            if (r == -1) continue;
            if (r < 0 || r >= m || seen[r]) return fail("tile row out of range or repeated");
            seen[r] = 1;
        }
    for (int r = 0; r < m; ++r)
        if (!seen[r]) return fail("row " + std::to_string(r) + " in no tile");
    auto check_tile = [&](int t) -> const char * {
        const int c0 = P.tfirst[(size_t)t];
        const int *R0 = &P.crec[(size_t)c0 * CS_CWORDS];
        const int nch = R0[256 + CS_C_NCH];
        if (nch < 1 || c0 + nch > P.nchunks || (t + 1 < P.ntiles && P.tfirst[(size_t)t + 1] != c0 + nch))
            return "tile chunk range";
        int x = 0;
        while (x < 7 && t >= P.xcd[x + 1]) ++x;
        const int tn = t + CS_BLOCKS_PER_XCD;
        const int next = tn < P.xcd[x + 1] ? P.tfirst[(size_t)tn] : -1;
        int cur[CS_ROWS], seenlast[CS_ROWS];
        for (int s = 0; s < CS_ROWS; ++s) {
            const int r = P.trow[(size_t)t * CS_ROWS + s];
            cur[s] = r >= 0 ? rp[r] : 0;
            seenlast[s] = 0;
        }
        for (int c = 0; c < nch; ++c) {
            const int *R = &P.crec[(size_t)(c0 + c) * CS_CWORDS];
            for (int f = 0; f < 8; ++f)
                for (int q = 1; q < 16; ++q)
                    if (R[256 + 8 * q + f] != R[256 + f]) return "record field not replicated";
            const int nx = R[256 + CS_C_NX], vb = R[256 + CS_C_VB], nvp = R[256 + CS_C_NVP];
            const int ab = R[256 + CS_C_AB], nap = R[256 + CS_C_NAP];
            if (R[256 + CS_C_C] != c || R[256 + CS_C_NCH] != nch || R[256 + CS_C_NEXT] != next)
                return "record chunk fields";
            if (nx < 0 || nx > CS_XCAP || vb % 16 || ab % 128 || nvp < 0 || nvp * 1024 > CS_MV || nap < 1 ||
                nap * 1024 > CS_MA || (int64_t)vb + 128 * (int64_t)nvp > (int64_t)P.tsrc.size() ||
                (int64_t)ab + 1024 * (int64_t)nap > (int64_t)P.aux.size())
                return "chunk header out of range";
            int ids[256];
            for (int u = 0; u < 256; ++u) {
                const int piece = u / 4, w = piece % 8, i = piece / 8, q = u % 4;
                ids[u] = R[32 * w + 8 * q + i];
                if (ids[u] < 0 || ids[u] >= n) return "X row id out of range";
            }
            const int *H = reinterpret_cast<const int *>(&P.aux[(size_t)ab]);
            if (H[CS_H_C] != c || H[CS_H_NCH] != nch || H[CS_H_TILE] != t) return "aux header chunk fields";
            for (int w = 0; w < CS_WAVES; ++w) {
                const int S = H[4 * w], vo = H[4 * w + 1], lo = H[4 * w + 2];
                if (S < 0 || S % 2 || vo < 0 || vo % 64 || (int64_t)(vo + 32 * S) * 8 > 1024LL * nvp ||
                    lo < CS_HDR || lo % 64 || lo + 32 * S > 1024 * nap)
                    return "wave region out of range";
                for (int p = 0; p < CS_RPW; ++p) {
                    const int slot = w * CS_RPW + p, r = P.trow[(size_t)t * CS_ROWS + slot];
                    for (int s = 0; s < S; ++s) {
                        const int src = P.tsrc[(size_t)vb + vo + 64 * (s / 2) + 2 * p + s % 2];
                        const int o = P.aux[(size_t)ab + lo + 64 * (s / 2) + 2 * p + s % 2];
                        if (r >= 0 && cur[slot] < rp[r + 1] && src == cur[slot]) {
                            if (o >= nx || ids[o] != ci[src]) return "row entry does not read its X row";
                            ++cur[slot];
                            seenlast[slot] = c;
                        } else if (src != -1 || o != CS_XCAP) {
                            return "entry out of CSR order, or a pad off the zero row";
                        }
                    }
                }
            }
        }
        for (int s = 0; s < CS_ROWS; ++s) {
            const int r = P.trow[(size_t)t * CS_ROWS + s];
            if (r >= 0 && cur[s] != rp[r + 1]) return "row not complete";
            if (r >= 0 && P.tlast[(size_t)t * CS_ROWS + s] != seenlast[s]) return "last chunk of a row";
        }
        return nullptr;
    };
    const int nt = P.ntiles;
    const int nth = std::max(1, std::min({8, (nt + 15) / 16, (int)std::max(1u, std::thread::hardware_concurrency()),
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

// One tile's chunks: records (without the NEXT field), value sources and
// aux bytes relative to the tile's own start.
struct CsTile {
    std::vector<int> rec, tsrc;
    std::vector<uint8_t> aux;
    int slot_row[CS_ROWS], slot_last[CS_ROWS];
    int nch = 0;
    int64_t nx = 0;
    int simd_steps = 0;  // sum over the chunks of the busiest SIMD's steps (waves w, w + 4)
};

bool cs_emit_tile(const std::vector<int> &rows_in, int t, const int *rp, const int *ci, std::vector<int> &pos,
                  CsTile &T, std::string &why)
{
    T.rec.clear();
    T.tsrc.clear();
    T.aux.clear();
    T.nch = 0;
    T.nx = 0;
    T.simd_steps = 0;
    // rows by first column (rows with similar column ranges share a wave:
    // fewer pads per step), dealt to the waves in contiguous runs
    std::vector<int> rows = rows_in;
    auto key = [&](int r) { return rp[r + 1] > rp[r] ? ci[rp[r]] : INT32_MAX; };
    std::sort(rows.begin(), rows.end(), [&](int a, int b) {
        const int ka = key(a), kb = key(b);
        return ka != kb ? ka < kb : a < b;
    });
    const int nr = (int)rows.size(), per = (nr + CS_WAVES - 1) / CS_WAVES;
    for (int s = 0; s < CS_ROWS; ++s) T.slot_row[s] = -1, T.slot_last[s] = 0;
    std::vector<int> slots;  // slot of the k-th row
    // contiguous runs: wave w takes sorted rows [w per, (w + 1) per), so the
    // waves sharing a SIMD (w, w + 4) hold rows far apart in column order
    // (measured against round robin and adjacent pairs: fewest SIMD steps)
    for (int k = 0; k < nr; ++k) {
        const int s = (k / per) * CS_RPW + k % per;
        T.slot_row[s] = rows[(size_t)k];
        slots.push_back(s);
    }
    // the union, ascending
    std::vector<int> uc;
    for (int r : rows)
        for (int j = rp[r]; j < rp[r + 1]; ++j)
            if (pos[ci[j]] < 0) pos[ci[j]] = 0, uc.push_back(ci[j]);
    std::sort(uc.begin(), uc.end());
    for (int u = 0; u < (int)uc.size(); ++u) pos[uc[(size_t)u]] = u;
    const int nu = (int)uc.size();
    // entries per union column: the slots holding it (with multiplicity)
    std::vector<int> bstart((size_t)nu + 1, 0), bslot;
    for (int k = 0; k < nr; ++k)
        for (int j = rp[rows[(size_t)k]]; j < rp[rows[(size_t)k] + 1]; ++j) ++bstart[(size_t)pos[ci[j]] + 1];
    for (int u = 0; u < nu; ++u) bstart[(size_t)u + 1] += bstart[(size_t)u];
    bslot.resize((size_t)bstart[(size_t)nu]);
    {
        std::vector<int> fill(bstart.begin(), bstart.end() - 1);
        for (int k = 0; k < nr; ++k)
            for (int j = rp[rows[(size_t)k]]; j < rp[rows[(size_t)k] + 1]; ++j)
                bslot[(size_t)fill[(size_t)pos[ci[j]]]++] = slots[(size_t)k];
    }
    for (int c : uc) pos[c] = -1;
    // chunks: union columns in order while the X rows, values and offsets fit
    int cnt[CS_ROWS] = {}, S[CS_WAVES] = {};
    auto fits = [&](const int *Sw, int nx) {
        int64_t v = 0, a = CS_HDR;
        for (int w = 0; w < CS_WAVES; ++w) v += 512LL * ((Sw[w] + 1) / 2), a += 64LL * ((Sw[w] + 1) / 2);
        return nx <= CS_XCAP && v <= CS_MV && a <= CS_MA;
    };
    int cur[CS_ROWS];
    for (int s = 0; s < CS_ROWS; ++s) cur[s] = T.slot_row[s] >= 0 ? rp[T.slot_row[s]] : 0;
    auto emit_chunk = [&](int u0, int u1) {
        const int c = T.nch++;
        const int nx = u1 - u0;
        for (int w = 0; w < CS_WAVES; ++w) S[w] = (S[w] + 1) & ~1;  // whole step pairs
        // values region (16-double aligned) and aux region (128-B aligned) of this chunk
        const int vb = (int)T.tsrc.size(), ab = (int)T.aux.size();
        int vo[CS_WAVES], lo[CS_WAVES], vtot = 0, atot = CS_HDR;
        for (int w = 0; w < CS_WAVES; ++w) {
            vo[w] = vtot;
            lo[w] = atot;
            vtot += 32 * S[w];
            atot += 32 * S[w];
        }
        const int vlen = (vtot + 15) & ~15, alen = (atot + 127) & ~127;
        T.tsrc.resize((size_t)vb + vlen, -1);
        T.aux.resize((size_t)ab + alen, 0);
        int *H = reinterpret_cast<int *>(&T.aux[(size_t)ab]);
        for (int w = 0; w < CS_WAVES; ++w) H[4 * w] = S[w], H[4 * w + 1] = vo[w], H[4 * w + 2] = lo[w];
        H[CS_H_C] = c;
        H[CS_H_TILE] = t;  // CS_H_NCH is set once the tile's chunks are known
        for (int w = 0; w < CS_WAVES; ++w)
            for (int p = 0; p < CS_RPW; ++p) {
                const int slot = w * CS_RPW + p, r = T.slot_row[slot];
                for (int s = 0; s < S[w]; ++s) {
                    int src = -1, o = CS_XCAP;
                    if (r >= 0 && cur[slot] < rp[r + 1]) {
                        const int j = cur[slot];
                        const int u = (int)(std::lower_bound(uc.begin(), uc.end(), ci[j]) - uc.begin());
                        if (u >= u0 && u < u1) src = j, o = u - u0, ++cur[slot], T.slot_last[slot] = c;
                    }
                    T.tsrc[(size_t)vb + vo[w] + 64 * (s / 2) + 2 * p + s % 2] = src;
                    T.aux[(size_t)ab + lo[w] + 64 * (s / 2) + 2 * p + s % 2] = (uint8_t)o;
                }
            }
        std::vector<int> R((size_t)CS_CWORDS, 0);
        for (int u = 0; u < nx; ++u) {
            const int piece = u / 4, w = piece % 8, i = piece / 8, q = u % 4;
            R[(size_t)(32 * w + 8 * q + i)] = uc[(size_t)(u0 + u)];
        }
        const int f[7] = {nx, vb, (vlen * 8 + 1023) / 1024, ab, (alen + 1023) / 1024, c, 0};
        for (int k = 0; k < 7; ++k)
            for (int q = 0; q < 16; ++q) R[(size_t)(256 + 8 * q + k)] = f[k];
        T.rec.insert(T.rec.end(), R.begin(), R.end());
        T.nx += nx;
        int most = 0;
        for (int q = 0; q < CS_WAVES / 2; ++q) most = std::max(most, S[q] + S[q + CS_WAVES / 2]);
        T.simd_steps += most;
    };
    // chunk cuts by dynamic programming over the sorted union: a chunk
    // [a, b) is feasible when its X rows and its (even-rounded) steps fit the
    // LDS slots; it costs the steps of its busiest SIMD (waves w and w + 4
    // share one) plus a per-chunk overhead; the cuts minimise the tile's sum
    constexpr int lambda = 8;  // per-chunk overhead in steps (4 and 16: no better on the cop20k stand-ins)
    auto cost_of = [&](const int *Sw) {
        int most = 0;
        for (int q = 0; q < CS_WAVES / 2; ++q)
            most = std::max(most, ((Sw[q] + 1) & ~1) + ((Sw[q + CS_WAVES / 2] + 1) & ~1));
        return most + lambda;
    };
    const int INF = 1 << 30;
    std::vector<int> best((size_t)nu + 1, INF), from((size_t)nu + 1, -1), touched;
    best[0] = 0;
    for (int a = 0; a < nu; ++a) {
        if (best[(size_t)a] == INF) continue;
        for (int s : touched) cnt[s] = 0;
        touched.clear();
        std::fill(S, S + CS_WAVES, 0);
        for (int b = a + 1; b <= nu; ++b) {
            for (int e = bstart[(size_t)b - 1]; e < bstart[(size_t)b]; ++e) {
                const int s = bslot[(size_t)e];
                if (cnt[s]++ == 0) touched.push_back(s);
                S[s / CS_RPW] = std::max(S[s / CS_RPW], cnt[s]);
            }
            if (!fits(S, b - a)) break;
            const int c = best[(size_t)a] + cost_of(S);
            if (c < best[(size_t)b]) best[(size_t)b] = c, from[(size_t)b] = a;
        }
    }
    for (int s : touched) cnt[s] = 0;
    if (nu > 0 && best[(size_t)nu] == INF) {
        why = "one X row's entries overflow a chunk";
        return false;
    }
    std::vector<int> cuts;
    for (int b = nu; b > 0; b = from[(size_t)b]) cuts.push_back(b);
    std::reverse(cuts.begin(), cuts.end());
    int u0 = 0;
    for (size_t k = 0; k + 1 < cuts.size() || (k < cuts.size() && cuts[k] < nu); ++k) {
        const int u1 = cuts[k];
        std::fill(S, S + CS_WAVES, 0);
        for (int e = bstart[(size_t)u0]; e < bstart[(size_t)u1]; ++e) {
            const int s = bslot[(size_t)e];
            S[s / CS_RPW] = std::max(S[s / CS_RPW], ++cnt[s]);
        }
        for (int e = bstart[(size_t)u0]; e < bstart[(size_t)u1]; ++e) cnt[bslot[(size_t)e]] = 0;
        emit_chunk(u0, u1);
        u0 = u1;
    }
    std::fill(S, S + CS_WAVES, 0);
    for (int e = bstart[(size_t)u0]; e < bstart[(size_t)nu]; ++e) {
        const int s = bslot[(size_t)e];
        S[s / CS_RPW] = std::max(S[s / CS_RPW], ++cnt[s]);
    }
    emit_chunk(u0, nu);  // (a tile without non-zeros gets one empty chunk: its rows store zeros)
    for (int c = 0; c < T.nch; ++c) {
        const int ab = T.rec[(size_t)c * CS_CWORDS + 256 + CS_C_AB];
        reinterpret_cast<int *>(&T.aux[(size_t)ab])[CS_H_NCH] = T.nch;
        for (int q = 0; q < 16; ++q) T.rec[(size_t)c * CS_CWORDS + 256 + 8 * q + CS_C_NCH] = T.nch;
    }
    return true;
}

}  // namespace

bool build_cs_plan(int m, int n, const int *rp, const int *ci, CsPlan &P, std::string *err, const TileCaps &caps_in)
{
    static const bool timing = std::getenv("SMFV_PLAN_TIMING") != nullptr;
    auto tick = [t = std::chrono::steady_clock::now()](const char *what) mutable {
        const auto now = std::chrono::steady_clock::now();
        if (timing)
            std::fprintf(stderr, "[smfv cs plan] %s %.1f ms\n", what,
                         std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    };
    P = CsPlan();
    auto fail = [&](const std::string &msg) {
        if (err) *err = "cs plan: " + msg;
        return false;
    };
    for (int r = 0; r < m; ++r)
        for (int j = rp[r] + 1; j < rp[r + 1]; ++j)
            if (ci[j] < ci[j - 1]) return fail("row " + std::to_string(r) + " is not column-sorted");
    // tile size: every XCD part in at most CS_BLOCKS_PER_XCD x tpb tiles
    TileCaps caps = caps_in;
    int most = m;
    if (caps.part_start.size() >= 2) {
        most = 0;
        for (size_t x = 0; x + 1 < caps.part_start.size(); ++x)
            most = std::max(most, caps.part_start[x + 1] - caps.part_start[x]);
    } else {
        most = (m + 7) / 8;
    }
    const int64_t per_block = ((int64_t)most + CS_BLOCKS_PER_XCD - 1) / CS_BLOCKS_PER_XCD;
    const int64_t tpb = std::max<int64_t>(1, (per_block + CS_ROWS - 1) / CS_ROWS);
    int rows = (int)std::max<int64_t>(1, (per_block + tpb - 1) / tpb);
    if (caps.cs_rows > 0) rows = std::min(caps.cs_rows, CS_ROWS);
    caps.maxrows = rows;
    caps.ucap = 1 << 30;
    caps.ncap = 1 << 30;
    caps.pad = 1;
    // tiles: the clustered row analysis at this tile size
    std::vector<std::vector<int>> tl;
    std::vector<int> part_tile;
    {
        TileAnalysis A;
        analyse_tiles(m, n, rp, ci, A, caps);
        for (const TileMeta &tm : A.meta) tl.emplace_back(A.grow.begin() + tm.roff, A.grow.begin() + tm.roff + tm.nrows);
        part_tile = A.part_tile;
    }
    tick("tiles");
    const int nt = (int)tl.size();
    const int np = (int)part_tile.size() - 1;
    P.ntiles = nt;
    for (int x = 0; x <= 8; ++x)
        P.xcd[x] = np == 8 ? part_tile[(size_t)x] : (int)((int64_t)nt * x / 8);
    P.xcd[8] = nt;
    // tiles emitted in parallel, then concatenated in order
    std::vector<CsTile> out((size_t)nt);
    std::vector<std::string> why((size_t)std::max(nt, 1));
    {
        const int nth = std::max(1, std::min({8, (nt + 15) / 16, (int)std::max(1u, std::thread::hardware_concurrency()),
                                              analysis_threads > 0 ? analysis_threads : 8}));
        std::vector<char> bad((size_t)nth, 0);
        auto work = [&](int w) {
            std::vector<int> pos((size_t)std::max(n, 1), -1);
            for (int t = (int)((int64_t)nt * w / nth); t < (int)((int64_t)nt * (w + 1) / nth) && !bad[(size_t)w]; ++t) {
                if (!cs_emit_tile(tl[(size_t)t], t, rp, ci, pos, out[(size_t)t], why[(size_t)t]))
                    bad[(size_t)w] = 1;
            }
        };
        std::vector<std::thread> pool;
        for (int w = 1; w < nth; ++w) pool.emplace_back(work, w);
        work(0);
        for (auto &x : pool) x.join();
        for (int t = 0; t < nt; ++t)
            if (!why[(size_t)t].empty()) return fail(why[(size_t)t]);
    }
    tick("emit");
    int64_t nv = 0, na = 0, nc = 0;
    for (const CsTile &T : out) nv += (int64_t)T.tsrc.size(), na += (int64_t)T.aux.size(), nc += T.nch;
    if (nv + 128 > 0x7fffffff / 8 || na + 1024 > 0x7fffffff) return fail("snapshot or aux past the 32-bit offsets");
    P.nchunks = (int)nc;
    P.tfirst.resize((size_t)nt);
    P.trow.resize((size_t)nt * CS_ROWS);
    P.tlast.resize((size_t)nt * CS_ROWS);
    P.crec.reserve((size_t)nc * CS_CWORDS);
    P.tsrc.reserve((size_t)nv + 128);
    P.aux.reserve((size_t)na + 1024);
    for (int t = 0; t < nt; ++t) {
        CsTile &T = out[(size_t)t];
        const int c0 = (int)(P.crec.size() / CS_CWORDS), vb = (int)P.tsrc.size(), ab = (int)P.aux.size();
        P.tfirst[(size_t)t] = c0;
        for (int s = 0; s < CS_ROWS; ++s) {
            P.trow[(size_t)t * CS_ROWS + s] = T.slot_row[s];
            P.tlast[(size_t)t * CS_ROWS + s] = T.slot_last[s];
        }
        for (int c = 0; c < T.nch; ++c)
            for (int q = 0; q < 16; ++q) {
                T.rec[(size_t)c * CS_CWORDS + 256 + 8 * q + CS_C_VB] += vb;
                T.rec[(size_t)c * CS_CWORDS + 256 + 8 * q + CS_C_AB] += ab;
            }
        P.crec.insert(P.crec.end(), T.rec.begin(), T.rec.end());
        P.tsrc.insert(P.tsrc.end(), T.tsrc.begin(), T.tsrc.end());
        P.aux.insert(P.aux.end(), T.aux.begin(), T.aux.end());
        P.union_rows += T.nx;
        P.tsimd.push_back(T.simd_steps);
        std::vector<int>().swap(T.rec);
        std::vector<int>().swap(T.tsrc);
        std::vector<uint8_t>().swap(T.aux);
    }
    // NEXT: the first chunk of the tile the same block runs after this one
    for (int x = 0; x < 8; ++x)
        for (int t = P.xcd[x]; t < P.xcd[x + 1]; ++t) {
            const int tn = t + CS_BLOCKS_PER_XCD;
            const int next = tn < P.xcd[x + 1] ? P.tfirst[(size_t)tn] : -1;
            const int c1 = t + 1 < nt ? P.tfirst[(size_t)t + 1] : P.nchunks;
            for (int c = P.tfirst[(size_t)t]; c < c1; ++c)
                for (int q = 0; q < 16; ++q) P.crec[(size_t)c * CS_CWORDS + 256 + 8 * q + CS_C_NEXT] = next;
        }
    P.tsrc.resize(P.tsrc.size() + 128, -1);  // DMA slack
    P.aux.resize(P.aux.size() + 1024, 0);
    P.entries = (int64_t)P.tsrc.size();
    for (int r = 0; r < m; ++r) P.tiled_nnz += rp[r + 1] - rp[r];
    tick("concatenate");
    const bool ok = verify_cs_plan(m, n, rp, ci, P, err);
    tick("verify");
    return ok;
}

}  // namespace smfv
