// Per-rank tile geometry: the owned sub-grid plus a deep halo ring.
//
// Reference storage: a (w_l+2) x (h_l+2) byte slab with a 1-cell ghost ring
// and a row-pointer table (src/game_mpi.c:192-197, 268-273); CUDA uses a flat
// (W+2)(H+2) byte buffer in int arithmetic (src/game_cuda.cu:153-191, quirk
// Q10).  Here a tile is pitched, 64-bit indexed, and carries Dv halo rows and
// hw*32 halo cells on each side so that Dv generations can run between two
// halo exchanges ("deep halo" / temporal blocking).
//
// Padded coordinates: rows [0, R), cells [0, Wc).  Owned rows are
// [Dv, Dv + H), owned cells are [32*hw, 32*hw + W).  A "word" is a column of
// 32 cells: in the Bits layout it is one uint32, in the U8 layout 32 bytes.
#pragma once

#include "gol/common.hpp"

namespace gol {

struct TileGeom {
  Layout layout = Layout::Bits;
  int64_t H = 0, W = 0;  // owned rows, owned cells
  int Dv = 0;            // halo rows per side
  int hw = 0;            // halo width per side, in 32-cell words
  int64_t pitch = 0;     // bytes per padded row

  static TileGeom make(Layout layout, int64_t H, int64_t W, int Dv, int hw) {
    TileGeom g;
    g.layout = layout;
    g.H = H;
    g.W = W;
    g.Dv = Dv;
    g.hw = hw;
    GOL_REQUIRE(H > 0 && W > 0 && Dv >= 0 && hw >= 0, "bad tile geometry");
    if (layout == Layout::Bits) GOL_REQUIRE(W % 32 == 0, "bit layout needs width % 32 == 0");
    int64_t row_bytes = layout == Layout::Bits ? 4 * g.Wp() : 32 * g.Wp();
    g.pitch = round_up(row_bytes, 256);
    return g;
  }

  int64_t R() const { return H + 2 * int64_t(Dv); }
  int64_t Wc() const { return W + 64 * int64_t(hw); }   // padded cells per row
  int64_t Wp() const { return ceil_div(Wc(), 32); }     // padded words per row
  int64_t row0() const { return Dv; }
  int64_t cell0() const { return 32 * int64_t(hw); }
  int64_t bytes() const { return R() * pitch; }
  // Byte offset of (row, cell) for word-aligned cells (Bits) or any cell (U8).
  int64_t offset(int64_t row, int64_t cell) const {
    return row * pitch + (layout == Layout::Bits ? 4 * (cell / 32) : cell);
  }
  // Bytes that hold `cells` consecutive cells starting at a word boundary.
  int64_t span_bytes(int64_t cells) const {
    return layout == Layout::Bits ? 4 * ceil_div(cells, 32) : cells;
  }
};

// One temporal block: T generations evaluated in a single pass over the tile.
// Output rows are [row_lo, row_hi) (padded coordinates); the input must hold
// valid cells on [row_lo - T, row_hi + T).  The per-generation "changed" flags
// changed[t - flags_base] are set for t in (gen_base, gen_base + T] whenever
// any owned cell of a valid row differs from the previous generation.
struct BlockArgs {
  const void* in = nullptr;
  void* out = nullptr;
  TileGeom g;
  int64_t row_lo = 0, row_hi = 0;
  int T = 1;
  int64_t gen_base = 0;
  uint32_t* changed = nullptr;
  int64_t flags_base = 0;
  // Graph-replayable flag addressing: when gen_dev is set, the flags of
  // generation gen_base + 1 + L are changed[*gen_dev + gen_rel + L] (device
  // value read at run time), so a captured epoch can be replayed at any
  // generation; gen_base / flags_base are then ignored for addressing.
  const int64_t* gen_dev = nullptr;
  int64_t gen_rel = 0;
  // The backend may run a kernel that stores generation t+1's cell x-1 at
  // column x (one-sided window, no cross-lane ops): the stored frame then
  // drifts right by T cells, which run_block reports.  Only valid when the
  // tile is the whole torus width (the drift is a relabeling of columns).
  bool allow_drift = false;
  // The tile is the whole torus (one rank): a backend that wraps row reads
  // too (Backend::wraps_rows) reads rows modulo the owned rows, so the engine
  // neither fills nor exchanges halo rows.
  bool wrap_rows = false;
  // The tile is the whole torus width (Px == 1, W % 32 == 0): a backend may
  // wrap column reads within the owned words instead of reading halo columns,
  // which it then neither reads nor writes.
  bool full_width = false;
  // The backend may link this launch to the previous one (run both at once,
  // ordered by per-group completion words): Backend::KernelChoice::link, on
  // a single-rank ring tile whose epochs move no data between launches.
  bool link = false;
  // The tile is a row ring (Backend::row_ring_halo) and the block covers its
  // owned rows: rows outside them are the torus wrapped around, which a
  // linked launch's dependency waits must follow (life_group_impl.hpp).
  bool ring = false;
  // Boundary trigger (Backend::trigger_stream): the groups of this launch
  // whose output rows meet [trigger_rows[0], trigger_rows[1]) or
  // [trigger_rows[2], trigger_rows[3]) count themselves done on a device
  // counter once their rows are written, so a stream can start sending those
  // rows before the rest of the launch has finished.
  bool trigger = false;
  int64_t trigger_rows[4] = {0, 0, 0, 0};
  // Earlier blocks of a trigger epoch: the groups meeting trigger_rows (the
  // light cone of the boundary rows the epoch will send) run at top issue
  // priority, nothing counted - so the boundary region leads the interior.
  bool hot = false;
};

}  // namespace gol
