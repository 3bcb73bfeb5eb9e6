// smfv_plan.h -- internal: clustered row-tile analysis of a CSR pattern and
// the plan of the LDS-tiled row kernel k_rows_ws (X-row re-use inside a tile).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace smfv {

// Column-panel width the tiled kernel stages per X row (32 doubles = 256 B).
constexpr int TILE_KP = 32;

// ---------------------------------------------------------------------------
// Plan of the warp-specialised tiled kernel k_rows_ws (one 1024-lane block
// per CU: 8 compute waves = 64 eight-lane teams, 8 loader waves).
// A tile holds <= WS_ROWS rows and <= WS_UCAP distinct X rows; its LDS X
// image has WS_UCAP + 1 rows of 256 B, row WS_UCAP stays zero and is what
// pads read.  The caps are sized so that two X images and two meta slots
// (values, offsets, record) fill the CU's 160 KiB, and so that the tiles of
// the cop20k_A surrogate number <= 8 per CU (1,980 tiles: every block runs
// 8, where 2,081 tiles of the former 255 / 1,536 caps made some run 9).
// Rows are sorted by decreasing length and dealt in quads (4 teams of one
// lane group, similar lengths), two quads (8 consecutive rows) per compute
// wave, and the waves sharing a SIMD (w, w + 4) take a long and a short
// octet; a quad's entries are interleaved (the 8 u8 image rows of batch b of
// team k in the 8-byte chunk base + 4b + k, value pair c of team k in the
// 16-byte chunk base + 4c + k) so one meta read of a lane group touches four
// bank groups; a quad's value range ends after the last pair its rows sum.
// ---------------------------------------------------------------------------
constexpr int WS_UCAP = 239;     // union rows per tile
constexpr int WS_NCAP = 2048;    // LDS entries per tile (u8 image row + f64 value); (r5) 1792 -> 2048
constexpr int WS_ROWS = 64;      // rows per tile
constexpr int WS_LOADERS = 8;    // loader waves; each stages 8 x 1 KiB of X
constexpr int WS_ZOFF = WS_UCAP * 256;  // byte offset of the zero row
// global record (per tile, int32): [0, 256) union ids in loader-lane order
// (loader wave w, lane quarter q, its i-th piece -> union id 4 * (w + 8i) + q
// at word 32w + 8q + i), then noff / tn / nu (the tile's offsets: first entry,
// entries; its union rows) and voff / tnv (its values: first entry, entries),
// each replicated 16x so any lane reads its copy with no broadcast
constexpr int WS_GWORDS = 352, WS_G_NOFF = 256, WS_G_TN = 272, WS_G_NU = 288, WS_G_VOFF = 304, WS_G_TNV = 320;
// LDS record (per tile, 256 int32 = 1 KiB in global memory): with R rows per
// tile, [0, R) row per team slot (-1 none), [R, 2R) L chunk base | (padded
// length << 16), [2R, 3R) V chunk base; team slot = team-in-wave * (compute
// waves) + wave; (r5) [3R, 4R) the team's second row | its length (rounded
// up to even, <= 62) << 24 | (live values) its odd-length flag << 30, or -1:
// the team sums it after the first, from the batch after the first row's
// last (TileCaps::pairs)
constexpr int WS_LWORDS = 256;
constexpr int WS_SLACK = 2048;   // entries past the end (DMA over-read of the last tile)

// (r4) Geometry of a k_rows_ws launch.  cw compute waves of 8 eight-lane
// teams (rows per tile = 8 cw), lw loader waves of ppw one-KiB X pieces each
// (ucap + 1 <= 4 lw ppw), entry cap ncap, xcd_blocks blocks per XCD.
//   WS_GEOM1: one 1024-lane block per CU (8 + 8 waves), 64-row tiles, 158 KiB
//             of LDS.
//   WS_GEOM2: two 512-lane blocks per CU (4 + 4 waves), 32-row tiles, 80 KiB
//             of LDS each: two independent two-slot pipelines per CU.
//             Measured slower on whole matrices (2.6x the units;
//             profiles/r04/ab_geom); the automatic choice for small plans
//             (< 1.5 geometry-1 tiles per CU: smfv::plan_create).
//   WS_GEOM3: one 768-lane block per CU (8 compute + 4 loader waves of 16
//             pieces), 64-row tiles: 3 waves per SIMD, so a wave may hold up
//             to 168 VGPRs and the compute waves run a deeper read-ahead.
struct WsGeom {
    int id, cw, lw, ppw, ucap, ncap, xcd_blocks;
    int ncap1;  // (r5) entry cap of a plan of one row per team (row-pair plans take ncap)
    constexpr int rows() const { return 8 * cw; }
    constexpr int threads() const { return 64 * (cw + lw); }
    // global record word of loader wave w, lane quarter q, piece i (union id 4 (w + lw i) + q)
    constexpr int gword(int w, int q, int i) const { return 4 * ppw * w + ppw * q + i; }
};
constexpr WsGeom WS_GEOM1{1, 8, 8, 8, WS_UCAP, WS_NCAP, 32, 1792};
constexpr WsGeom WS_GEOM2{2, 4, 4, 8, 125, 896, 64, 896};
constexpr WsGeom WS_GEOM3{3, 8, 4, 16, WS_UCAP, WS_NCAP, 32, 1792};
constexpr WsGeom ws_geom(int id) { return id == 2 ? WS_GEOM2 : id == 3 ? WS_GEOM3 : WS_GEOM1; }

// Per-tile summary of the clustered analysis.
struct TileMeta {
    int32_t noff;   // start of the tile's non-zeros in tsrc / tlidx (multiple of 8)
    int32_t tn;     // length of the tile's segment (rows padded to multiples of 8)
    int32_t uoff;   // start of the tile's union in ucols
    int32_t nu;     // distinct X rows (0 for a direct tile)
    int32_t roff;   // start of the tile's rows in trows / rbeg
    int32_t nrows;  // rows in the tile
    int32_t direct; // 1: one row over a cap
    int32_t pad;
};

struct TileAnalysis {
    std::vector<TileMeta> meta;
    std::vector<int> trows;        // rows of each tile (any order of the matrix rows)
    std::vector<int> grow;         // the same rows in the order the tile grew (same offsets as trows)
    std::vector<int> rbeg;         // per tile row: tile-local start | (length << 16)
    std::vector<int> ucols;        // distinct columns of each tile, first-use order
    std::vector<int> tsrc;         // per tile-ordered non-zero: its index in the CSR arrays
    std::vector<uint16_t> tlidx;   // per tile-ordered non-zero: position in its tile's ucols
    int64_t union_rows = 0;        // sum of tile unions (X rows staged per panel)
    int64_t tiled_nnz = 0;         // non-zeros in non-direct tiles
    int64_t padded_nnz = 0;        // length of tsrc / tlidx
    std::vector<int> part_tile;    // parts + 1 entries: first tile of each part, then the tile count
};

// Clustered tiling: seed a tile at the first unassigned row (or, with
// caps.frontier, at the oldest unassigned neighbour of the tiles built so
// far: tiles then grow as a wavefront through the pattern's graph, so
// consecutive tiles -- which run together on one XCD -- are neighbours
// whatever the row numbering), then repeatedly
// add the candidate row (a column index of a row already in the tile, i.e. a
// graph neighbour for square patterns) that adds the fewest new columns to
// the tile's union (ties: more in-tile neighbours, more non-zeros), while
// union <= ucap, padded non-zeros <= ncap and rows <= maxrows.  A row over a
// cap alone becomes a one-row "direct" tile.  Every row lands in exactly one
// tile; the per-row non-zero order is the CSR order, so results are unchanged.
struct TileCaps {
    int ucap = WS_UCAP;            // distinct X rows
    int ncap = WS_NCAP - 192;      // padded non-zeros (room for the quads' interleave padding)
    int maxrows = WS_ROWS;         // rows
    int pad = 8;                   // row segments padded to a multiple of this (power of 2)
    int max_tiles = 0;             // > 0: stop after this many tiles (re-use estimate on a sample)
    bool frontier = false;         // seed each tile at the oldest unassigned neighbour of earlier tiles
    int split_ends = 0;            // build_ws_plan: > 0 = blocks per XCD whose first and last tile are halves
    int col_base = 0;              // row block of a square pattern: column c is the block's row c - col_base
    // row sets tiled one after the other, a tile taking rows of one set only
    // (part x = part_rows[part_start[x] .. part_start[x + 1]), seeds scanned in
    // that order); empty: one part, all rows in order.  build_ws_plan with 8
    // parts runs part x on XCD x (range_parts / bfs_parts below)
    std::vector<int> part_rows, part_start;
    int xcd_blocks = 32;           // k_rows_ws blocks per XCD (MI355X: 256 CUs / 8 XCDs)
    WsGeom geom = WS_GEOM1;        // build_ws_plan: the kernel geometry (ucap / ncap / maxrows follow it)
    bool live = false;             // build_ws_plan: live values (WsPlan::vidx) instead of a snapshot (tsrc)
    // (r5) build_ws_plan: row pairs -- tiles of up to 2 x geom.rows() rows,
    // a team summing two short rows one after the other (plans of < 2^24
    // rows), entry cap geom.ncap -- 0 never (one row per team, entry cap
    // geom.ncap1), 1 always, 2 whichever plan runs fewer rounds of tiles per
    // block (ties: one row per team)
    int pairs = 0;
    // (r5) analyse_tiles: a tile of n > team_rows rows (team_rows 0: no
    // limit) pairs its 2 (n - team_rows) shortest rows, the i-th longest with
    // the i-th shortest; a row joins only if no pair then outlasts the tile's
    // longest row by more than pair_slack batches and no second row has more than pair_len
    // non-zeros (rounded down to whole batches)
    int team_rows = 0;
    int pair_len = 56;
    int pair_slack = 1;            // batches a pair may run past the longest row
    // (r6) build_wsn_plan: union rows in bank-coloured image slots
    // (colour_wsn_slots, smfv_plan.cpp); false: first-use order
    bool wsn_colour = true;
    bool wsn_model = false;        // (r6) also model the X reads' LDS cycles (WsnPlan::x_*; smfv_wsn_plan_analyse)
};
// Independent parts are analysed on up to 8 threads; analysis_threads > 0
// caps that for analyses run on the calling thread (smfv_set_analysis_threads).
void analyse_tiles(int m, int n, const int *row_ptr, const int *col_idx, TileAnalysis &out,
                   const TileCaps &caps = TileCaps());
extern thread_local int analysis_threads;

struct WsPlan {
    WsGeom geom = WS_GEOM1;
    int ntiles = 0;
    std::vector<int> grec;         // WS_GWORDS per tile
    std::vector<int> lrec;         // WS_LWORDS per tile
    std::vector<uint8_t> loff;     // per offset entry: its X row in the LDS image (union position; WS_UCAP: pad)
    std::vector<int> tsrc;         // per value entry: CSR index of its value (-1: pad); empty when live
    // (r5) live values (TileCaps::live): the kernel's loaders DMA each value
    // pair straight from the caller's CSR values -- pair c of a row is
    // values[rp[r] + 2c], values[rp[r] + 2c + 1] (8-byte aligned: LDS-DMA
    // takes it) -- so no snapshot and no bind pass.  vidx[t * vstride + s]:
    // the (block-local) CSR index of value slot s's first entry in tile t
    // (slots no row sums: 0).  A row of odd length L reads one value past
    // its end (the next row's first, or past the block: the kernel's buffer
    // descriptor returns 0 there); bit 30 of its V base word flags it, and
    // its team writes -0.0 over that half in LDS before summing
    bool live = false;
    int vstride = 0;               // value slots per tile in vidx (ncap / 2)
    std::vector<int> vidx;
    std::vector<int> direct;       // rows over a cap alone, gathered straight from X
    int64_t union_rows = 0;        // X rows staged per 32-column panel
    int64_t tiled_nnz = 0;         // non-zeros in tiles (not direct)
    int64_t entries = 0;           // used length of loff (the vector carries WS_SLACK more)
    int64_t ventries = 0;          // used length of tsrc (the vector carries WS_SLACK more): a quad's
                                   // last batch stores only the value pairs its rows use
    int xcd[9] = {};               // XCD x runs tiles [xcd[x], xcd[x + 1])
    int64_t paired = 0;            // (r5) second rows of teams (TileCaps::pairs)
    int64_t split = 0;             // analysed tiles whose layout had to be split
};

// Tiles from analyse_tiles (WS caps), each packed into the interleaved
// layout; a tile whose layout overflows WS_NCAP is split in two (by sorted
// row order) until it fits; a single row that cannot fit becomes direct.
// caps.split_ends = nb (the kernel's blocks per XCD; opt-in, measured
// slower: one more unit per block costs more than the halved ends save): in each XCD's tile
// range the first nb tiles are cut in two halves (by growth order); the
// first halves become the blocks' first units and the second halves their
// last units, so the unoverlapped staging of a block's first tile and the
// unoverlapped compute of its last one are half as long.
// Every matrix row lands in exactly one tile or in `direct`; per-row order
// is CSR order.  The result is verified by replaying the kernel's reads;
// returns false (with *err) if an invariant fails.
bool build_ws_plan(int m, int n, const int *row_ptr, const int *col_idx, WsPlan &out, std::string *err,
                   const TileCaps &caps = TileCaps());

// Partitions of a block's rows into `parts` sets of equal non-zero count for
// TileCaps::part_rows / part_start: row ranges, or shares of the rows'
// breadth-first order from row 0 (col_base as TileCaps::col_base).
void range_parts(int m, const int *row_ptr, int parts, std::vector<int> &rows, std::vector<int> &start);
void bfs_parts(int m, const int *row_ptr, const int *col_idx, int col_base, int parts, std::vector<int> &rows,
               std::vector<int> &start);
// X rows the parts read, summed over the parts, over the block's distinct X
// rows.  Each XCD has its own L2, so with part x on XCD x this is the
// compulsory X traffic over X's size (1.0 = no X row read twice).  On the
// cop20k_A surrogate: ranges 1.30, breadth-first shares 1.51, one wavefront
// of frontier tiles cut in 8: 1.69.
double parts_footprint(int m, int n, const int *row_ptr, const int *col_idx, const std::vector<int> &rows,
                       const std::vector<int> &start);

// ---------------------------------------------------------------------------
// (r5) Plan of the narrow-team tiled kernel k_rows_wsn: a 4- or 8-column
// window (a ColumnWise rank's K/p panel, SC/...ColumnWise.cpp:25-48).  A
// team is KW/2 lanes (one double2 column pair each), so a wave holds
// TW = 128/KW rows and a tile 8 TW rows (256 at KW = 4, 128 at KW = 8): 4x /
// 2x the rows of a k_rows_ws tile, so a rank runs 2-4 units per CU instead
// of 8.  The X image rows are the window only (32 / 64 B), up to WSN_UCAP
// of them, addressed by u16 image offsets.  Per tile, rows sorted by
// decreasing length are dealt TW at a time to the 8 compute waves (wave
// groups g and 7 - g share a SIMD); a wave's rows run in lockstep batches of
// WSN_B = 4 entries, its teams' batches interleaved and trimmed to the teams
// still running: with n_b the wave's teams of more than b batches (a prefix,
// rows being sorted) and c_b = n_0 + ... + n_{b-1}, the offsets of batch b of
// team k sit in the 8-byte chunk base + c_b + k (4 u16) and value pair q of
// that batch in the 16-byte chunk vbase + 2 c_b + q n_b + k, so one wave read
// per lane touches n_b consecutive chunks and a wave's rows cost their own
// batches, not its longest row's (the kernel counts n_b with a ballot).  A
// row's entries past its length in its last batch are pads: the zero image
// row and value -0.0 (summed: +-0 changes nothing).
// ---------------------------------------------------------------------------
constexpr int WSN_LW = 8;        // loader waves (8 compute + 8 loader = 1024 lanes)
constexpr int WSN_B = 4;         // (r5) entries per batch (was 8: rows padded to 4, not 8 -- 21 % fewer entries)
constexpr int WSN_GWORDS = 1024 + 96;  // global record: union ids [0, 1024), then 6 x 16 header words
constexpr int WSN_G_NOFF = 1024, WSN_G_TN = 1040, WSN_G_NU = 1056, WSN_G_VOFF = 1072, WSN_G_TNV = 1088;
struct WsnGeom {
    int kw;     // window columns (4 or 8)
    int ucap;   // union rows (the image holds ucap + 1: the last is zero)
    int ncap;   // padded entries per tile
    constexpr int tl() const { return kw / 2; }        // lanes per team
    constexpr int tw() const { return 128 / kw; }      // teams (rows) per wave
    constexpr int rows() const { return 8 * tw(); }    // rows per tile
    constexpr int xrow() const { return 8 * kw; }      // image row bytes
    constexpr int lwords() const { return rows() + 16; }  // LDS record: rows | nbat << 24, then per wave lbase, vbase
};
constexpr WsnGeom WSN_K4{4, 1023, 4096};
constexpr WsnGeom WSN_K8{8, 639, 3072};
constexpr WsnGeom wsn_geom(int kw) { return kw == 4 ? WSN_K4 : WSN_K8; }

struct WsnPlan {
    WsnGeom geom = WSN_K4;
    int ntiles = 0;
    std::vector<int> grec;         // WSN_GWORDS per tile
    std::vector<int> lrec;         // geom.lwords() per tile
    std::vector<uint16_t> loff;    // per entry: image row (ucap: pad, the zero row)
    std::vector<int> tsrc;         // per value entry: CSR index (-1: pad)
    std::vector<int> direct;       // rows over a cap alone
    int64_t union_rows = 0, tiled_nnz = 0, entries = 0, ventries = 0;
    int xcd[9] = {};
    // (r6) image rows staged (union rows + the colouring's holes), and the
    // modelled LDS cycles of the X reads: lane groups (= cycles without any
    // bank conflict), with the plan's slots, with first-use slots
    int64_t staged_rows = 0, x_groups = 0, x_cycles = 0, x_cycles_plain = 0;
};
// Tiles from analyse_tiles (caps.ucap / ncap / maxrows follow the geometry;
// caps.part_* as for build_ws_plan), each laid out per wave; a tile whose
// layout overflows ncap is split in two until it fits, a single row that
// cannot fit becomes direct.  Verified by replaying the kernel's reads.
bool build_wsn_plan(int m, int n, const int *row_ptr, const int *col_idx, int kw, WsnPlan &out, std::string *err,
                    const TileCaps &caps);

// ---------------------------------------------------------------------------
// Plan of the opt-in MFMA tile kernel k_rows_mfma (SMFV_PLAN_MFMA; within
// tolerance, not bit-identical).  Same clustered tiles (WS caps); each tile's
// rows in groups of 16 (one wave each); per group the 16 x union part of A is
// cut into k-steps of 4 union columns and every non-zero 16 x 4 block is
// stored dense in the A-operand lane order of v_mfma_f64_16x16x4f64 (lane l:
// row l & 15, union column 4s + (l >> 4)), zeros as pads.  Rows with a
// repeated column (the dense block would have to sum them) or over a cap go
// to the direct list (k_rows_list, CSR order).
// ---------------------------------------------------------------------------
constexpr int MF_GROUPS = 4;                       // 16-row groups per tile (64 rows)
constexpr int MF_RWORDS = 64 + 2 * MF_GROUPS + 4;  // record: rows[64], (blk_off, blk_cnt) per group, nu, pad

struct MfmaPlan {
    int ntiles = 0;
    std::vector<int> rec;      // MF_RWORDS per tile (rows: -1 none)
    std::vector<int> ucols;    // WS_UCAP per tile: union ids (0 past nu)
    std::vector<int> bstep;    // per block: its k-step
    std::vector<int> tsrc;     // 64 per block: CSR index of the A value (-1: zero)
    std::vector<int> direct;   // rows gathered directly
    int64_t blocks = 0, tiled_nnz = 0, union_rows = 0;
};
bool build_mfma_plan(int m, int n, const int *row_ptr, const int *col_idx, MfmaPlan &out, std::string *err,
                     const TileCaps &caps = TileCaps());

// K = 1 chunk plan (k_spmv_chunks, the SpMV of BASELINE config 1 on the GPU).
// Consecutive rows are packed into chunks of at most `cap` non-zeros and
// `maxrows` rows; chunk c's entries sit at slots [c * cap, c * cap + count)
// in CSR order, so a block streams its chunk from an address it knows at
// launch (no row_ptr round trip first) and sums each row in CSR order from
// LDS (bit-identical to SC/SparseMatrixFatVectorMultiply.cpp:17-27 at K = 1).
// Each entry carries its column as a 16-bit offset from the chunk's lowest
// column (10 bytes per entry with the values snapshot, against CSR's 12);
// a pattern with a row whose columns span more than 65,535 takes the wide
// layout instead (32-bit columns, 12 bytes per entry, still streamed from
// fixed addresses).
struct SpmvChunkPlan {
    int nchunks = 0, cap = 0, maxrows = 0;
    bool wide = false;           // 32-bit columns in `col` (else 16-bit offsets in `off`)
    std::vector<int> hdr;        // 4 per chunk: first row, rows, base column (0 if wide), entries
    std::vector<uint16_t> rs;    // maxrows + 1 per chunk: row starts in the chunk (entry `rows` = entries)
    std::vector<uint16_t> off;   // cap per chunk: column - base column (pads 0); narrow layout
    std::vector<int> col;        // cap per chunk: column (pads 0); wide layout
    std::vector<int> tsrc;       // cap per chunk: CSR index of the entry's value (-1: pad)
    int64_t entries = 0;         // non-zeros placed (= nnz of the block)
};
// false (with *err saying why) when the pattern does not fit the layout: a
// row longer than cap (or, with allow_wide false, a row whose columns span
// more than 65,535).  The plan is verified by replaying the kernel's reads
// before it is returned.
bool build_spmv_chunks(int m, int n, const int *row_ptr, const int *col_idx, int cap, int maxrows,
                       SpmvChunkPlan &out, std::string *err, bool allow_wide = true);

}  // namespace smfv
