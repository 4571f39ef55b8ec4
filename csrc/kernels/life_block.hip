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

int words_per_lane(Layout layout, const LifeTuning& tune) {
  return layout == Layout::Bits ? (tune.wpl_bits >= 2 ? 2 : 1) : 1;
}

}  // namespace

namespace {

// Cross-lane primitive actually compiled for (layout, words per lane).
int xlane_of(Layout layout, int w, const LifeTuning& tune) {
  if ((tune.xlane == kXlaneAdd || tune.xlane == kXlaneAuto) && w == 1) return tune.xlane;
  if (tune.xlane == kXlaneCarry) return kXlaneCarry;
  if (tune.xlane == kXlaneBpermute && layout == Layout::Bits && w == 1) return kXlaneBpermute;
  return kXlaneDpp;
}

const char* xlane_name(int x) {
  return x == kXlaneAuto ? "auto(add|dpp)" : x == kXlaneAdd ? "add" : x == kXlaneCarry ? "carry"
         : x == kXlaneBpermute ? "bpermute" : "dpp";
}

}  // namespace

std::string life_block_variant(Layout layout, const LifeTuning& tune) {
  const int w = words_per_lane(layout, tune);
  if (layout == Layout::U8 && tune.u8_lds)
    return tune.lds_T > 1 ? "u8 lds-tiled T=" + std::to_string(tune.lds_T) + (tune.lds_pack && tune.lds_T >= 8 ? " packed" : "")
                          : std::string("u8 lds-tiled single-step");
  const bool grouped = tune.group != 0 && tune.split == 0 && !tune.skew;
  return std::string(layout == Layout::Bits ? "bits" : "u8") + " wpl=" + std::to_string(w) + " " +
         xlane_name(xlane_of(layout, w, tune)) + (tune.skew ? " skew" : "") +
         (tune.split > 0 ? " split" : tune.split < 0 ? " split=auto" : "") +
         (grouped ? (tune.group < 0 ? std::string(" group=auto") : " group=" + std::to_string(tune.group)) : "") +
         (grouped && tune.short_seg == 1 ? " short=auto" : grouped && tune.short_seg == 2 ? " short=forced" : "") +
         (grouped && tune.pipe == 1 ? " pipe=auto" : grouped && tune.pipe == 2 ? " pipe=forced" : "") +
         (grouped && tune.chain == 1    ? " chain"
          : grouped && tune.chain == 2 ? " chain=probe"
          : grouped && tune.chain < 0  ? " chain=tuned"
                                       : "");
}

int life_block_max_T(Layout layout, const LifeTuning& tune) {
  if (layout == Layout::U8 && tune.u8_lds) return tune.lds_T;
  // Register budget for 2 waves/SIMD (<= 256 VGPRs): T * words-per-lane <= 16.
  return words_per_lane(layout, tune) >= 2 ? 8 : 16;
}

int launch_life_block(const BlockArgs& a, const LifeTuning& tune, hipStream_t stream) {
  const TileGeom& g = a.g;
  GOL_REQUIRE(a.row_lo - a.T >= 0 && a.row_hi + a.T + a.dual_offset <= g.R() && a.row_lo < a.row_hi &&
                  a.dual_offset >= 0 && (a.dual_offset == 0 || a.dual_offset >= a.row_hi - a.row_lo),
              "life_block: row range outside the tile");
  GOL_REQUIRE(g.Wp() < (int64_t(1) << 30), "life_block: row too wide");
  // Row stores go through a buffer descriptor per row (num_records = pitch)
  // and drop non-owned lanes at offset 2^30 (life_block_impl.hpp Writer).
  GOL_REQUIRE(g.pitch < (int64_t(1) << 30), "life_block: row pitch must be < 1 GiB");
  const int w = words_per_lane(g.layout, tune);
  GOL_REQUIRE(g.Wp() >= w, "life_block: tile narrower than one lane's words");
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
  p.chain_acquire = tune.chain_acquire ? 1 : 0;
  p.row_alt = a.dual_offset;
  p.prio_boost = a.prio_boost ? 1 : 0;
  p.wrap_w = a.full_width && tune.wrap && g.W % 32 == 0 ? int(g.W / 32) : 0;
  p.fold = 1;
  p.fold_lanes = 64;
  p.link_ring_rows = a.ring && a.row_lo == g.Dv && a.row_hi == g.Dv + g.H ? g.H : 0;
  p.fault_delay = tune.fault_delay;
  const int64_t rows = a.row_hi - a.row_lo;
  int x = xlane_of(g.layout, w, tune);
  if (g.layout == Layout::U8 && tune.u8_lds && (a.T == 1 || a.T == 2 || a.T == 4 || a.T == 8 || a.T == 16 || a.T == 32)) {
    BlockArgs b = a;
    b.dual_offset = 0;
    // Packed tiles need 32-cell aligned rows (pitch) and owned cells.
    const bool pack = a.T >= 8 && (tune.lds_pack || a.T > 8) && g.pitch % 32 == 0 && g.cell0() % 32 == 0;
    GOL_REQUIRE(a.T <= 8 || pack, "life_block: LDS-tiled byte passes deeper than 8 need the packed tile");
    int drift = 0;
    for (int half = 0; half < (a.dual_offset ? 2 : 1); ++half) {
      if (a.T == 1)
        launch_life_step_lds(b, tune.lds_rows, tune.wrap, stream);
      else if (pack)
        drift = launch_life_lds_bits(b, tune.wrap, tune.lds_xcd, tune.lds_waves, tune.cus, stream);
      else
        launch_life_lds_multi(b, tune.wrap, stream);
      b.row_lo += a.dual_offset;
      b.row_hi += a.dual_offset;
    }
    return drift;
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
  // The pipelined T = 48 byte pass is compiled for the DPP window only.
  if (g.layout == Layout::U8 && a.T > 32) x = kXlaneDpp;
  if (x == kXlaneAdd) {
    (g.layout == Layout::U8 ? launch_u8_w1_add : launch_bits_w1_add)(p, rows, a.T, tune, stream);
    return a.T;
  }
#ifdef GOL_EXPERIMENTAL
  if (g.layout == Layout::U8) {
    (x == kXlaneCarry ? launch_u8_w1_carry : launch_u8_w1_dpp)(p, rows, a.T, tune, stream);
  } else if (w == 2) {
    (x == kXlaneCarry ? launch_bits_w2_carry : launch_bits_w2_dpp)(p, rows, a.T, tune, stream);
  } else {
    (x == kXlaneCarry ? launch_bits_w1_carry
                      : x == kXlaneBpermute ? launch_bits_w1_bperm : launch_bits_w1_dpp)(p, rows, a.T, tune, stream);
  }
#else
  // Default build: the DPP and adder windows, one word per lane (the
  // bpermute / carry-chain windows and two words per lane measured slower
  // and are compiled only with GOL_EXPERIMENTAL; HipBackend refuses them).
  GOL_REQUIRE(w == 1 && x == kXlaneDpp, "life_block: variant '" + life_block_variant(g.layout, tune) +
                                            "' needs an experimental build (GOL_EXPERIMENTAL=1)");
  (g.layout == Layout::U8 ? launch_u8_w1_dpp : launch_bits_w1_dpp)(p, rows, a.T, tune, stream);
#endif
  return 0;
}

bool life_flow_has_T(int T) { return kExperimentalBuild && (T == 8 || T == 12 || T == 16); }

int launch_life_flow(const FlowArgs& a, const LifeTuning& tune, FlowState& st, hipStream_t stream) {
#ifndef GOL_EXPERIMENTAL
  (void)a, (void)tune, (void)st, (void)stream;
  return -1;  // flow kernels are compiled into experimental builds only
#else
  const TileGeom& g = a.g;
  if (g.layout != Layout::Bits || words_per_lane(g.layout, tune) != 1 || a.nblk < 1 || !life_flow_has_T(a.T) ||
      !tune.chain_mem)
    return -1;
  const int64_t rows_min = (a.row_hi - a.row_lo) - 2 * int64_t(a.nblk - 1) * a.shrink;
  GOL_REQUIRE(a.shrink >= 0 && a.row_lo - a.T >= 0 && a.row_hi + a.T <= g.R() && rows_min > 0 &&
                  (a.shrink == 0 || a.shrink == a.T) && (!a.ring || (a.shrink == 0 && a.row_lo == g.Dv &&
                                                                      a.row_hi == g.Dv + g.H)),
              "life_flow: row ranges outside the tile");
  GOL_REQUIRE(g.Wp() < (int64_t(1) << 30) && g.pitch < (int64_t(1) << 30) && g.pitch >= 4 * g.Wp() &&
                  g.R() < (int64_t(1) << 30),
              "life_flow: row geometry");
  FlowParams f{};
  LifeBlockParams& p = f.p;
  p.pitch = g.pitch;
  p.row_lo = a.row_lo;
  p.row_hi = a.row_hi;
  p.Wp = int(g.Wp());
  p.own_w0 = int(g.cell0() / 32);
  p.own_w1 = int(ceil_div(g.cell0() + g.W, 32));
  const int64_t tail = (g.cell0() + g.W) % 32;
  p.last_mask = tail ? (0xFFFFFFFFu >> (32 - tail)) : 0xFFFFFFFFu;
  p.err = tune.err;
  p.fault_delay = tune.fault_delay;
  p.wrap_w = a.full_width && tune.wrap && g.W % 32 == 0 ? int(g.W / 32) : 0;
  // A ring's blocks read rows across the torus seam: its halo rows must be the
  // aliases, and every read of a block stays inside [row_lo - T, row_hi + T).
  f.buf[0] = static_cast<uint8_t*>(a.buf[0]);
  f.buf[1] = static_cast<uint8_t*>(a.buf[1]);
  f.changed0 = a.changed ? a.changed + (a.gen_base + 1 - a.flags_base) : nullptr;
  f.rows0 = a.row_hi - a.row_lo;
  f.ring_rows = a.ring ? g.H : 0;
  f.shrink = a.shrink;
  f.nblk = a.nblk;
  f.spin_log2 = tune.flow_spin_log2;
  f.trace = st.trace;
  // Window: the adder window (drifting frame) where the engine allows a
  // drift and the one-sided light cone of the whole run fits the left halo.
  int x = xlane_of(g.layout, 1, tune);
  if (x == kXlaneAuto) x = kXlaneAdd;
  if (x == kXlaneAdd &&
      !(a.allow_drift && (p.wrap_w > 0 || 32 * int64_t(g.hw) >= 2 * int64_t(a.T) * a.nblk)))
    x = kXlaneDpp;
  if (x != kXlaneAdd && x != kXlaneDpp) return -1;
  constexpr int kWaveOut = 63;  // both windows: 64 lanes, halo lane(s) excluded below
  const int wave_out = x == kXlaneAdd ? kWaveOut : 62;
  p.ncolw = int(ceil_div(p.wrap_w ? p.wrap_w : p.Wp, wave_out));
  p.fold = 1;
  p.fold_lanes = 64;
  if (p.wrap_w && tune.fold && p.ncolw >= 2 && (f.rows0 + 2) * p.pitch < (int64_t(1) << 30)) {
    const int lanes = p.wrap_w - (p.ncolw - 1) * wave_out + (x == kXlaneAdd ? 1 : 2);
    const int fo = std::min(4, 64 / lanes);
    if (fo >= 2) {
      p.fold = fo;
      p.fold_lanes = lanes;
    }
  }
  // Tickets and completion words (monotonic; FlowParams).
  f.counter = tune.chain_mem(9, 256);
  const int max_items = int(ceil_div(int64_t(p.ncolw) * rows_min, int64_t(2 * a.T)));  // any plan's item bound
  f.done = tune.chain_mem(8, size_t(std::max(1, max_items)) * 4);
  if (st.counter != f.counter) {  // (re)allocated and zeroed
    st.counter = f.counter;
    st.ticket = 0;
  }
  f.base = st.ticket;
  f.seq0 = st.seq + 1;
  std::string desc;
  int64_t tickets = 0;
  int items = 0;
  const bool ok = (x == kXlaneAdd ? launch_flow_bits_add : launch_flow_bits_dpp)(f, rows_min, a.T, tune, stream, &desc,
                                                                                  &tickets, &items);
  if (!ok) return -1;
  st.ticket += uint32_t(tickets);  // every item, plus one ticket past the last per workgroup
  st.items = items;
  st.seq += uint32_t(a.nblk);
  ++st.launches;
  st.blocks += a.nblk;
  st.last = (x == kXlaneAdd ? "adder " : "dpp ") + desc;
  return x == kXlaneAdd ? a.T * a.nblk : 0;
#endif  // GOL_EXPERIMENTAL
}

}  // namespace hipk
}  // namespace gol
