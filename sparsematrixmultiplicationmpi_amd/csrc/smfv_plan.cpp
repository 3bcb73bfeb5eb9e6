// smfv_plan.cpp -- row-tile analysis of a CSR pattern (host, O(nnz)).
//
// The LDS-tiled row kernel processes a tile of consecutive rows in one
// workgroup: the distinct X rows the tile touches are staged into LDS once
// and every non-zero of the tile reads its X row from LDS.  This pass
// decides the tiles (greedy: grow while the column union fits TILE_UCAP and
// the tile has at most TILE_MAXROWS rows) and re-expresses every column
// index as a 16-bit position in its tile's union list.  Computation order is
// untouched: each row is still summed over its non-zeros in CSR order.
#include "smfv_plan.h"

#include <algorithm>

namespace smfv {

void analyse_tiles(int m, int n, const int *rp, const int *ci, TileAnalysis &A)
{
    A.tile_rows.clear();
    A.tile_uoff.clear();
    A.tile_direct.clear();
    A.ucols.clear();
    A.lidx.assign((size_t)(m > 0 ? rp[m] : 0), 0);
    A.union_rows = 0;
    // stamp[c] == tile id  <=> column c already in the current tile's union;
    // a negative stamp marks "seen while testing a row" (never a tile id)
    std::vector<int> stamp((size_t)std::max(n, 1), -1), pos((size_t)std::max(n, 1), 0);
    int tile = 0;
    int i = 0;
    while (i < m) {
        const int r0 = i;
        const size_t ubase = A.ucols.size();
        int ucount = 0;
        int64_t tnnz = 0;
        A.tile_rows.push_back(r0);
        A.tile_uoff.push_back((int)ubase);
        while (i < m && i - r0 < TILE_MAXROWS) {
            // distinct columns of row i not yet in the tile
            const int probe = -2 - tile;
            int fresh = 0;
            for (int j = rp[i]; j < rp[i + 1]; ++j) {
                const int c = ci[j];
                if (stamp[c] != tile && stamp[c] != probe) {
                    stamp[c] = probe;
                    ++fresh;
                }
            }
            const int64_t rlen = rp[i + 1] - rp[i];
            if ((ucount + fresh > TILE_UCAP || tnnz + rlen > TILE_NCAP) && i > r0) break;
            tnnz += rlen;
            for (int j = rp[i]; j < rp[i + 1]; ++j) {
                const int c = ci[j];
                if (stamp[c] != tile) {
                    stamp[c] = tile;
                    pos[c] = ucount++;
                    A.ucols.push_back(c);
                }
                A.lidx[j] = (uint16_t)std::min(pos[c], 0xFFFF);
            }
            ++i;
            if (ucount > TILE_UCAP || tnnz > TILE_NCAP) break;  // one row over a cap
        }
        if (ucount > TILE_UCAP || tnnz > TILE_NCAP) {
            A.ucols.resize(ubase);  // processed with direct X gathers
            A.tile_direct.push_back(1);
        } else {
            A.tile_direct.push_back(0);
            A.union_rows += ucount;
        }
        ++tile;
    }
    A.tile_rows.push_back(m);
    A.tile_uoff.push_back((int)A.ucols.size());
}

}  // namespace smfv
