// life_block dispatcher: validates the launch and picks the compiled kernel
// variant (layout x words-per-lane x cross-lane primitive).  The kernel
// itself is in life_block_impl.hpp / life_group_impl.hpp (schedules in
// life_block_launch.hpp).
#include "life_kernels.hpp"

#include <string>

#include "gol/common.hpp"

namespace gol {
namespace hipk {

namespace {

const char* xlane_name(int x) { return x == kXlaneAuto ? "auto(add|dpp)" : x == kXlaneAdd ? "add" : "dpp"; }

}  // namespace

std::string life_block_variant(Layout layout, const LifeTuning& tune) {
  if (layout == Layout::U8 && tune.u8_lds)
    return tune.lds_T > 1 ? "u8 lds-tiled T=" + std::to_string(tune.lds_T) + (tune.lds_pack && tune.lds_T >= 8 ? " packed" : "")
                          : std::string("u8 lds-tiled single-step");
  const bool grouped = tune.group != 0;
  return std::string(layout == Layout::Bits ? "bits" : "u8") + " wpl=1 " + xlane_name(tune.xlane) +
         (grouped ? (tune.group < 0 ? std::string(" group=auto") : " group=" + std::to_string(tune.group)) : "") +
         (grouped && tune.chain == 1 ? " chain" : grouped && tune.chain < 0 ? " chain=tuned" : "");
}

int life_block_max_T(Layout layout, const LifeTuning& tune) {
  if (layout == Layout::U8 && tune.u8_lds) return tune.lds_T;
  // Register budget for 2 waves/SIMD (<= 256 VGPRs): T <= 16 (one word per lane).
  return 16;
}

int launch_life_block(const BlockArgs& a, const LifeTuning& tune, hipStream_t stream) {
  const TileGeom& g = a.g;
  GOL_REQUIRE(a.row_lo - a.T >= 0 && a.row_hi + a.T <= g.R() && a.row_lo < a.row_hi,
              "life_block: row range outside the tile");
  GOL_REQUIRE(g.Wp() < (int64_t(1) << 30), "life_block: row too wide");
  // Row stores go through a buffer descriptor per row (num_records = pitch)
  // and drop non-owned lanes at offset 2^30 (life_block_impl.hpp Writer).
  GOL_REQUIRE(g.pitch < (int64_t(1) << 30), "life_block: row pitch must be < 1 GiB");
  GOL_REQUIRE(g.Wp() >= 1, "life_block: tile narrower than one lane's word");
  GOL_REQUIRE(g.pitch >= (g.layout == Layout::Bits ? 4 : 32) * g.Wp(), "life_block: pitch too small");
  LifeBlockParams p{};
  p.in = static_cast<const uint8_t*>(a.in);
  p.out = static_cast<uint8_t*>(a.out);
  p.pitch = g.pitch;
  p.row_lo = a.row_lo;
  p.row_hi = a.row_hi;
  p.Wp = int(g.Wp());
  p.own_w0 = int(g.cell0() / 32);
  p.own_w1 = int(ceil_div(g.cell0() + g.W, 32));
  const int64_t tail = (g.cell0() + g.W) % 32;
  p.last_mask = tail ? (0xFFFFFFFFu >> (32 - tail)) : 0xFFFFFFFFu;
  if (a.gen_dev) {
    p.changed = a.changed;  // resolved on the device: changed + *gen_dev + gen_rel
    p.gen_dev = a.changed ? a.gen_dev : nullptr;
    p.gen_rel = a.gen_rel;
  } else {
    p.changed = a.changed ? a.changed + (a.gen_base + 1 - a.flags_base) : nullptr;
  }
  p.wg_trace = tune.wg_trace;
  p.err = tune.err;
  p.chain_spin_log2 = tune.chain_spin_log2;
  p.wrap_w = a.full_width && tune.wrap && g.W % 32 == 0 ? int(g.W / 32) : 0;
  p.fold = 1;
  p.fold_lanes = 64;
  p.link_ring_rows = a.ring && a.row_lo == g.Dv && a.row_hi == g.Dv + g.H ? g.H : 0;
  p.fault_delay = tune.fault_delay;
  const int64_t rows = a.row_hi - a.row_lo;
  int x = tune.xlane == kXlaneAdd || tune.xlane == kXlaneAuto ? tune.xlane : kXlaneDpp;
  if (g.layout == Layout::U8 && tune.u8_lds && (a.T == 1 || a.T == 2 || a.T == 4 || a.T == 8 || a.T == 16 || a.T == 32)) {
    // Packed tiles need 32-cell aligned rows (pitch) and owned cells.
    const bool pack = a.T >= 8 && (tune.lds_pack || a.T > 8) && g.pitch % 32 == 0 && g.cell0() % 32 == 0;
    GOL_REQUIRE(a.T <= 8 || pack, "life_block: LDS-tiled byte passes deeper than 8 need the packed tile");
    if (pack) return launch_life_lds_bits(a, tune.wrap, tune.lds_xcd, tune.lds_waves, tune.cus, stream);
    if (a.T == 1)
      launch_life_step_lds(a, tune.lds_rows, tune.wrap, stream);
    else
      launch_life_lds_multi(a, tune.wrap, stream);
    return 0;
  }
  // The adder window drifts the storage frame by T cells (see kXlaneAdd); the
  // engine allows that only for whole-width tiles of 32-cell words, and the
  // left halo must hold the 2T cells its one-sided light cone consumes (wrap
  // mode reads the wrapped owned words instead).
  if (x == kXlaneAuto) x = kXlaneAdd;  // the engine decided through allow_drift
  // The one-sided window also consumes 2T cells of its wave's single halo
  // word per pass, so passes deeper than 16 (the byte layout's T = 24 / 32)
  // run the DPP window.
  if (x == kXlaneAdd && !(a.allow_drift && a.T <= 16 && (p.wrap_w > 0 || 32 * g.hw >= 2 * a.T))) x = kXlaneDpp;
  if (x == kXlaneAdd) {
    (g.layout == Layout::U8 ? launch_u8_w1_add : launch_bits_w1_add)(p, rows, a.T, tune, stream);
    return a.T;
  }
  (g.layout == Layout::U8 ? launch_u8_w1_dpp : launch_bits_w1_dpp)(p, rows, a.T, tune, stream);
  return 0;
}

}  // namespace hipk
}  // namespace gol
