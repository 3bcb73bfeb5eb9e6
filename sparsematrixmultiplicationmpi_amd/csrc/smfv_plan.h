// smfv_plan.h -- internal: row-tile analysis of a CSR pattern for the
// LDS-tiled row kernel (X-row reuse inside a tile of consecutive rows).
#pragma once

#include <cstdint>
#include <vector>

namespace smfv {

// Column-panel width the tiled kernel stages per X row (32 doubles = 256 B,
// a 16-lane team reads one row with one ds_read_b128 per lane).
constexpr int TILE_KP = 32;
// Union capacity: distinct X rows of one tile held in LDS (128 x 256 B = 32 KiB).
constexpr int TILE_UCAP = 128;
// Rows per tile: one 8-lane team per row in a 256-lane block.
constexpr int TILE_MAXROWS = 32;
// Non-zeros per tile staged in LDS (16-bit local column + f64 value).
constexpr int TILE_NCAP = 1024;

struct TileAnalysis {
    std::vector<int> tile_rows;    // T + 1 row boundaries (tiles are contiguous rows)
    std::vector<int> tile_uoff;    // T + 1 offsets into ucols; a tile whose union
                                   // exceeds TILE_UCAP gets an empty range and is
                                   // processed with direct gathers (tile_direct)
    std::vector<uint8_t> tile_direct;
    std::vector<int> ucols;        // distinct columns of each tile, first-use order
    std::vector<uint16_t> lidx;    // per non-zero: position of its column in its tile's ucols
    int64_t union_rows = 0;        // sum of tile unions (X rows staged per panel)
};

// Greedy tiling of consecutive rows: grow a tile while its column union
// stays <= TILE_UCAP, its non-zeros <= TILE_NCAP and it has <= TILE_MAXROWS
// rows.  A single row over either cap becomes a one-row "direct" tile.
void analyse_tiles(int m, int n, const int *row_ptr, const int *col_idx, TileAnalysis &out);

}  // namespace smfv
