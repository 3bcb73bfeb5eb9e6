// cs_plan_lab.h -- LAB ONLY (libsmfv_lab.so, -DSMFV_LAB): the plan of the
// column-streamed tile kernel k_rows_cs, measured 3.4x slower than k_rows_ws
// and moved out of the product in round 4 (DESIGN.md section 4.5 keeps the
// A/B evidence).  libsmfv.so has none of it.
#pragma once

#include "smfv_plan.h"

namespace smfv {

// ---------------------------------------------------------------------------
// Plan of the column-streamed tiled kernel k_rows_cs (one 1024-lane block per
// CU: 8 compute waves of 32 two-lane rows, 8 loader waves).  A tile holds up
// to CS_ROWS rows (about m / 512: two tiles per CU), far more X rows than one
// LDS image takes, so its union -- sorted by column -- is streamed through
// LDS in CHUNKS of <= CS_XCAP X rows.  Each row accumulates all of its 32
// panel columns in registers over the tile's chunks; a row's entries falling
// in chunk c are a contiguous run of its CSR row (CSR rows are column-sorted,
// the chunks are column ranges), so chunk by chunk the row is summed in CSR
// order: bit-identical.  Per chunk and compute wave w, step s gives each of
// the wave's 32 rows one entry (value, u8 X-image row; rows with fewer
// entries take pads: value -0.0 on the zero image row CS_XCAP).  Layout:
// values  [w][s / 2][row 0..31][s % 2] f64 (one 16-byte read per two steps);
// offsets [w][s / 2][row 0..31][s % 2] u8 (one 2-byte read per two steps),
// after a 256-byte header (per wave: steps -- even --, value start, offset
// start; then chunk index, chunks, tile).
// ---------------------------------------------------------------------------
constexpr int CS_WAVES = 8, CS_RPW = 32, CS_ROWS = CS_WAVES * CS_RPW;
constexpr int CS_XCAP = 191;           // X rows per chunk; image row CS_XCAP stays zero
constexpr int CS_MV = 24 * 1024;       // LDS bytes of a chunk's values
constexpr int CS_MA = 4 * 1024;        // LDS bytes of a chunk's header + offsets
constexpr int CS_HDR = 256;            // header bytes at the start of a chunk's aux
constexpr int CS_H_C = 32, CS_H_NCH = 33, CS_H_TILE = 34;  // header words after the 8 wave quads
constexpr int CS_BLOCKS_PER_XCD = 32;  // the kernel's grid: 8 x 32 blocks, tile t + 32 follows t on a block
// chunk record (int32): [0, 256) X-row ids in loader-lane order (loader wave
// w, lane quarter q, piece i -> union index 4 (w + 8 i) + q at word
// 32 w + 8 q + i), then 8 fields replicated 16x (field f of copy q at word
// 256 + 8 q + f: a loader lane reads its copy with two 16-byte loads)
constexpr int CS_CWORDS = 256 + 16 * 8;
constexpr int CS_C_NX = 0, CS_C_VB = 1, CS_C_NVP = 2, CS_C_AB = 3, CS_C_NAP = 4, CS_C_C = 5, CS_C_NCH = 6,
              CS_C_NEXT = 7;  // NEXT: first chunk of tile t + 32 in the same XCD range, -1 none

struct CsPlan {
    int ntiles = 0, nchunks = 0;
    std::vector<int> crec;        // CS_CWORDS per chunk
    std::vector<int> trow;        // CS_ROWS per tile: block-local row of slot w * 32 + p (-1 none)
    std::vector<int> tlast;       // CS_ROWS per tile: the tile chunk holding the slot's last entry
    std::vector<int> tfirst;      // per tile: its first chunk (the chunks of a tile are consecutive)
    std::vector<int> tsrc;        // values snapshot sources (CSR index, -1 pad), + slack
    std::vector<uint8_t> aux;     // per chunk: header + offsets, + slack
    int xcd[9] = {};              // XCD x runs tiles [xcd[x], xcd[x + 1])
    int64_t union_rows = 0;       // X rows staged per panel (sum of the chunks' nx)
    int64_t tiled_nnz = 0, entries = 0;  // non-zeros, value slots incl. pads
    std::vector<int> tsimd;       // per tile: sum over its chunks of the busiest SIMD's steps (diagnostic)
};
// false (with *err) for patterns it does not take: a row whose columns are
// not sorted, a chunk over a cap with a single X row, offsets past 4 GiB.
bool build_cs_plan(int m, int n, const int *row_ptr, const int *col_idx, CsPlan &out, std::string *err,
                   const TileCaps &caps);

}  // namespace smfv
