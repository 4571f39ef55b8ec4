// Launch interfaces of the hand-written CDNA4 kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include "gol/tile.hpp"

namespace gol {
namespace hipk {

struct LifeBlockParams {
  const uint8_t* in;
  uint8_t* out;
  int64_t pitch;
  int64_t row_lo, row_hi;
  int Wp;          // padded words per row
  int ncolw;       // column waves (62 output words each)
  int nseg;        // row segments
  int seg_rows;    // output rows per segment
  int own_w0, own_w1;
  uint32_t last_mask;
  uint32_t* changed;  // changed[L] <-> generation gen_base + 1 + L
};

struct LifeTuning {
  int target_waves = 4096;  // waves per launch to aim for (256 CUs x 16)
  int min_seg_rows = 64;    // lower bound on rows per wave segment
};

void launch_life_block(const BlockArgs& a, const LifeTuning& tune, hipStream_t stream);

// Tile utility kernels (tile_ops.hip).
void launch_fill_cols(uint8_t* buf, const TileGeom& g, hipStream_t s);
void launch_fill_rows(uint8_t* buf, const TileGeom& g, hipStream_t s);
void launch_alive(const uint8_t* buf, const TileGeom& g, uint32_t* any_flag,
                  unsigned long long* count, hipStream_t s);
// Owned rows [r0, r0+n) from a device staging array of 0/1-or-ASCII bytes.
void launch_load_rows(uint8_t* buf, const TileGeom& g, const uint8_t* stage, int64_t ld,
                      int64_t r0, int64_t n, hipStream_t s);
void launch_store_rows(const uint8_t* buf, const TileGeom& g, uint8_t* stage, int64_t ld,
                       int64_t r0, int64_t n, bool ascii, hipStream_t s);
void launch_init_random(uint8_t* buf, const TileGeom& g, uint64_t seed, uint32_t thresh24,
                        int64_t grow0, int64_t gcol0, hipStream_t s);

}  // namespace hipk
}  // namespace gol
