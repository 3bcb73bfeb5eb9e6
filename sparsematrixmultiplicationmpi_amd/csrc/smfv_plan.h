// smfv_plan.h -- internal: clustered row-tile analysis of a CSR pattern for
// the LDS-tiled row kernel (X-row re-use inside a tile of rows).
#pragma once

#include <cstdint>
#include <vector>

namespace smfv {

// Column-panel width the tiled kernel stages per X row (32 doubles = 256 B).
constexpr int TILE_KP = 32;
// Union capacity: distinct X rows of one tile held in LDS (128 x 256 B = 32 KiB).
constexpr int TILE_UCAP = 128;
// Rows per tile: one 8-lane team per row in a 256-lane block.
constexpr int TILE_MAXROWS = 32;
// Non-zeros per tile staged in LDS (16-bit local column + f64 value).
constexpr int TILE_NCAP = 1024;

// Per-tile record (32 bytes), read with one scalar load by the kernel.
struct TileMeta {
    int32_t noff;   // start of the tile's non-zeros in tvals / tlidx (multiple of 8)
    int32_t tn;     // length of the tile's segment (rows padded to multiples of 8)
    int32_t uoff;   // start of the tile's union in ucols
    int32_t nu;     // distinct X rows (0 for a direct tile)
    int32_t roff;   // start of the tile's rows in trows / rbeg
    int32_t nrows;  // rows in the tile
    int32_t direct; // 1: one row over a cap, gathered straight from X
    int32_t pad;
};

// Fixed-size tile record for the pipelined kernel: 256 int32 words = 1 KiB,
// one word per lane of a 256-lane block, so a whole record is one coalesced
// load.  Layout: [0..7] TileMeta, [8..39] rows, [40..71] packed row info,
// [72..199] union column ids, id u at 72 + (u % 16) * 8 + u / 16 (each
// staging thread's 8 ids are contiguous).
constexpr int TREC_WORDS = 256;
constexpr int TREC_ROWS = 8, TREC_INFO = 40, TREC_UCOLS = 72;
static_assert(TREC_UCOLS + TILE_UCAP <= TREC_WORDS, "tile record too small");
static_assert(TILE_UCAP == 128 && TREC_UCOLS % 4 == 0, "record union layout: 16 x 8, 16-B aligned");
static_assert(TREC_INFO - TREC_ROWS >= TILE_MAXROWS, "tile record rows");

struct TileAnalysis {
    std::vector<TileMeta> meta;
    std::vector<int> trows;        // rows of each tile (any order of the matrix rows)
    std::vector<int> rbeg;         // per tile row: tile-local start | (length << 16)
    std::vector<int> ucols;        // distinct columns of each tile, first-use order
    std::vector<int> tsrc;         // per tile-ordered non-zero: its index in the CSR arrays
    std::vector<uint16_t> tlidx;   // per tile-ordered non-zero: position in its tile's ucols
    int64_t union_rows = 0;        // sum of tile unions (X rows staged per panel)
    int64_t tiled_nnz = 0;         // non-zeros in non-direct tiles
    int64_t padded_nnz = 0;        // length of tvals / tlidx / tsrc
};

// Clustered tiling: seed a tile at the first unassigned row, then repeatedly
// add the candidate row (a column index of a row already in the tile, i.e. a
// graph neighbour for square patterns) that adds the fewest new columns to
// the tile's union, while union <= TILE_UCAP, non-zeros <= TILE_NCAP and
// rows <= TILE_MAXROWS.  A row over a cap alone becomes a one-row "direct"
// tile.  Every row lands in exactly one tile; the per-row non-zero order is
// the CSR order, so results are unchanged.
void analyse_tiles(int m, int n, const int *row_ptr, const int *col_idx, TileAnalysis &out);

// Pack the analysis into 1 KiB records (TREC_WORDS per tile).
std::vector<int> pack_tile_records(const TileAnalysis &A);

}  // namespace smfv
