// Host-side launch of one compiled life_block variant (one translation unit
// per layout x words-per-lane x cross-lane primitive, life_block_*.hip):
// chooses the schedule of a temporal block and its launch shape.
//   grouped  life_group_kernel (life_group_impl.hpp): default for T >= 4 when
//            the rows allow M segments of 2T rows per group (GOL_GROUP);
//            linked (two launches in flight) or chained where that pays
//   classic  life_block_kernel: T < 4, short tiles, GOL_GROUP=0
// Schedules measured slower and removed in round 6 (docs/HISTORY.md): short
// segments, level-pipelined wave pairs (bit layout, and the byte layout's
// T = 48 pass, no faster than T = 32), split and skewed schedules.
#pragma once

#include "life_group_impl.hpp"

namespace gol {
namespace hipk {
namespace lb {

// Split schedule pays off when the classic schedule's redundant boundary
// triangles (about T^2 level-rows per segment boundary) are a large share of
// a segment's S*T level-rows.
constexpr int kSplitMaxRowsPerT = 8;

// Linked launch of the grouped kernel (LifeBlockParams::link_*): returns
// false (nothing launched) when the launch cannot be planned that way.  The
// first launch of a chain goes on stream[0] (the caller's `s`); a launch that
// reads the previous one's output and fits beside it goes on the other
// stream, after an event recorded just before the previous launch (so it
// starts no earlier than that one), and waits for its input rows group by
// group.
template <int T, class IO, int M = 8>
bool launch_linked(const LifeBlockParams& p0, int64_t out_rows, int simds, const LifeTuning& tune, hipStream_t s) {
  using LIO = Sc1IO<IO>;
  LinkState& L = *tune.link;
  if (s != L.stream[0]) return false;
  LifeBlockParams q = p0;  // keeps launch_T's folded last strip (q.fold): a folded block publishes
                           // the completion words of all its groups
  if (plan_group_memo<T, M>(q, out_rows, simds, group_waves_per_simd<T, LIO, M>(), tune.target_waves, IO::XL) <= 0)
    return false;
  const int64_t blocks = q.fold > 1 ? int64_t(q.ncolw - 1) * q.nseg + ceil_div(int64_t(q.nseg), int64_t(q.fold))
                                    : int64_t(q.ncolw) * q.nseg;
  static const int per_cu = occupancy_blocks(life_group_kernel<T, LIO, M>, 64 * M);
  const int64_t cap = int64_t(std::max(1, tune.cus)) * per_cu;
  // Two such launches never fit beside each other: the plain kernel (no
  // write-through stores, no completion words) serves the whole chain.
  if (2 * blocks > cap) {
    link_join(L);
    L.prev_valid = false;
    return false;
  }
  // Both launches fit at once: each one's share of the CUs (its workgroups
  // over how many of them fit, whatever resource binds) sums to at most 1,
  // which bounds every resource's use, also when the two launches are
  // different kernels (a T = 16 block of 8-wave groups, then a T = 8 block of
  // 4-wave groups).
  const double share = double(blocks) / double(cap);
  const bool link = L.prev_valid && L.prev_out == q.in && L.prev.ncolw == q.ncolw && L.prev.wrap_w == q.wrap_w &&
                    L.prev.pitch == q.pitch && L.prev.link_ring_rows == q.link_ring_rows &&
                    L.prev_share + share <= 1.0;
  // Completion words of this launch: the third buffer back, so neither the
  // previous launch's words (read by this one) nor the ones before it (read by
  // the previous launch, which may still run) are overwritten.
  const size_t need = size_t(q.ncolw) * size_t(q.nseg);  // one word per group
  if (L.flag_words < need) {
    if (!tune.chain_mem) return false;
    for (int i = 0; i < 3; ++i) L.flags[i] = tune.chain_mem(2 + i, need * 4);
    L.flag_words = need;
    L.prev_valid = false;
    if (link) return false;  // the buffers moved under the previous launch: start a new chain
  }
  if (++L.seq == 0) L.seq = 1;
  // Boundary trigger: count the groups meeting the trigger rows (the kernel
  // adds one per such group when it publishes).
  L.bnd_n = 0;
  q.bnd_count = nullptr;
  for (int& g : q.bnd_g) g = 0;
  if (L.bnd_req) {
    const int n = trigger_groups(q, L.bnd_r, q.bnd_g);
    if (L.bnd_count_req && L.bnd_count) {
      L.bnd_n = int64_t(n) * q.ncolw;
      q.bnd_count = L.bnd_count;
    }
  }
  L.bnd_req = false;
  q.link_flag = L.flags[L.seq % 3];
  q.link_seq = L.seq;
  hipStream_t st = L.stream[0];
  int which = 0;
  if (link) {
    which = 1 - L.cur;
    st = L.stream[which];
    q.link_prev_flag = L.prev.link_flag;
    q.link_prev_seq = L.prev.link_seq;
    q.link_prev_row_lo = L.prev.row_lo;
    q.link_prev_nseg = L.prev.nseg;
    q.link_prev_seg_rows = L.prev.seg_rows;
    q.link_prev_seg_rem = L.prev.seg_rem;
    // Only the chain's second launch waits for the first one's start (an
    // event): the first follows whatever the stream held before it (fills,
    // an exchange), which may take long, and a linked group's wait is
    // bounded.  Every later launch waits on one too: without them the early
    // consumers' spinning waves took the producer's slots (8192^2 1.81-1.85
    // vs 1.61 ms per 1000 generations, profiles/r04/linked_events_ab.jsonl),
    // although an event wait between two streams costs ~10 us of device time.
    // Its stream also orders it after the launch two back, whose completion
    // words (flags[seq % 3]) it overwrites.  After an armed boundary trigger
    // the stream's wait kernel already implies that start (LinkState::started).
    if (!L.started) (void)hipStreamWaitEvent(st, L.before[L.cur], 0);
    ++L.linked;
  } else {
    link_join(L);
    L.chain = 0;
  }
  (void)hipEventRecord(L.before[which], st);
  ++L.chain;
  hipLaunchKernelGGL((life_group_kernel<T, LIO, M>), dim3(unsigned(blocks)), dim3(64 * M), 0, st, q);
  L.started = false;
  L.cur = which;
  L.prev = q;
  L.prev_out = q.out;
  L.prev_blocks = blocks;
  L.prev_share = share;
  L.prev_valid = true;
  return true;
}

template <int T, class IO>
void launch_T(LifeBlockParams p, int64_t out_rows, const LifeTuning& tune, hipStream_t s) {
  constexpr int kWaveOut = wave_out_words<IO::XL, IO::W>();
  // Wrap mode (p.wrap_w > 0) covers the owned words only (lane_cols).
  p.ncolw = int(ceil_div(p.wrap_w ? p.wrap_w : p.Wp, kWaveOut));
  // Folded last strip (grouped kernel): 32768 cells are 16 strips of 63
  // words + 16 words; the last strip's 17 lanes fit three times in a wave,
  // so it costs a third of a strip instead of a whole one.  Lane offsets of
  // a folded wave span its groups' rows in one descriptor (< 2^30 bytes).
  p.fold = 1;
  p.fold_lanes = 64;
  if (p.wrap_w && IO::W == 1 && tune.fold && p.ncolw >= 2 &&
      (out_rows + 2) * p.pitch < (int64_t(1) << 30)) {
    const int lanes = p.wrap_w - (p.ncolw - 1) * kWaveOut + (IO::XL == kXlaneAdd ? 1 : 2);
    const int f = std::min(4, 64 / lanes);
    if (f >= 2) {
      p.fold = f;
      p.fold_lanes = lanes;
    }
  }
  const int simds = 4 * std::max(1, tune.cus);
  // Linked launches (GOL_LINK): this launch starts while the previous one
  // still runs, on the other stream, when both fit on the GPU at once (small
  // tiles, whose launches alone hold 2 waves per SIMD).  Any other launch
  // first joins the two streams.
  if (tune.link) {
    if constexpr (IO::kBits && IO::W == 1 && (T == 8 || T == 12 || T == 16) &&
                  (IO::XL == kXlaneDpp || IO::XL == kXlaneAdd)) {
      if (tune.group != 0) {
        // Blocks of T <= 8 link 4-wave groups where the unlinked path would
        // group 4 waves (tune group_small).
        if constexpr (T <= 8) {
          if (tune.group_small == 4) {
            if (launch_linked<T, IO, 4>(p, out_rows, simds, tune, s)) return;
          } else if (launch_linked<T, IO>(p, out_rows, simds, tune, s)) {
            return;
          }
        } else if (launch_linked<T, IO>(p, out_rows, simds, tune, s)) {
          return;
        }
      }
    }
    link_join(*tune.link);
  }
  if constexpr (T >= 4) {
    // Bit-layout blocks of T <= 8 (small tiles, HipBackend::choose_kernel)
    // group 4 waves by default: 8192^2 at T = 8 1.99 vs 2.06 ms per 1000
    // generations with 8-wave groups (profiles/r04/small_grid_ab.jsonl).
    const int group = (IO::kBits && T <= 8) ? tune.group_small : tune.group;
    if (group != 0) {
      // M = 4 or 8 waves per workgroup; auto (-1) takes the cheapest of
      // M = 4, M = 8 and the classic plan under the makespan model (classic
      // charged its redundant triangle, T-1 rows, at the triangles' ILP).
      LifeBlockParams g4 = p, g8 = p;
      const double c4 = (group == 4 || group < 0)
                            ? plan_group_memo<T, 4>(g4, out_rows, simds, group_waves_per_simd<T, IO, 4>(),
                                                    tune.target_waves, IO::XL)
                            : -1.0;
      const double c8 = (group == 8 || group < 0)
                            ? plan_group_memo<T, 8>(g8, out_rows, simds, group_waves_per_simd<T, IO, 8>(),
                                                    tune.target_waves, IO::XL)
                            : -1.0;
      double cc = -1.0;
      if (group < 0) {
        LifeBlockParams q = p;
        plan(q, T, out_rows, simds, waves_per_simd<T, IO>(), tune.min_seg_rows, tune.target_waves, 1.2 * (T - 1),
             &cc, IO::XL);
      }
      const auto better = [](double a, double b) { return a > 0 && (b < 0 || a <= b); };
      // Chained groups (GOL_CHAIN): every group boundary shared through
      // global memory, so no wave carries a redundant triangle but the
      // strip's last.  Stream launches only (the flags count launches, so a
      // replayed graph would see its own stale flags).
      if (tune.chain && tune.chain_ok && tune.chain_mem && tune.chain_seq) {
        LifeBlockParams ch = p;
        ch.fold = 1;
        ch.fold_lanes = 64;
        const bool m4 = group == 4;  // 4-wave groups: every 4th boundary chained
        const double cch =
            m4 ? plan_chain<T, 4>(ch, out_rows, simds, group_waves_per_simd<T, IO, 4>(), tune.target_waves, IO::XL)
               : plan_chain<T, 8>(ch, out_rows, simds, group_waves_per_simd<T, IO, 8>(), tune.target_waves, IO::XL);
        // tune.chain is set per launch by the backend (HipBackend's launch-
        // shape autotuning, or GOL_CHAIN=1 forced): +2 % on the 8-GPU rank
        // tile, -1 to -3 % on larger tiles and -12 % on 8192^2, where the
        // folded last strip it gives up is worth more; choosing it by the
        // makespan model measured slower than either (profiles/r02/chain/).
        if (cch > 0) {
          constexpr int64_t kSlot = int64_t(T - 1) * 2 * IO::W * 64;
          const int64_t slots = int64_t(ch.ncolw) * ch.nseg;
          ch.chain_flag = tune.chain_mem(0, size_t(slots) * 4);
          ch.chain_buf = tune.chain_mem(1, size_t(slots * kSlot) * 4);
          if (++*tune.chain_seq == 0) *tune.chain_seq = 1;  // 0 = never written
          ch.chain_seq = *tune.chain_seq;
          return m4 ? launch_group<T, IO, 4>(ch, s) : launch_group<T, IO, 8>(ch, s);
        }
      }
      if (better(c4, c8) && better(c4, cc)) return launch_group<T, IO, 4>(g4, s);
      if (better(c8, cc)) return launch_group<T, IO, 8>(g8, s);
    }
  }
  plan(p, T, out_rows, simds, waves_per_simd<T, IO>(), tune.min_seg_rows, tune.target_waves, -1, nullptr, IO::XL);
  const int waves = p.ncolw * p.nseg;
  const dim3 grid(unsigned(ceil_div(waves, 4))), block(256);
  hipLaunchKernelGGL((life_block_kernel<T, IO>), grid, block, 0, s, p);
}

// Deep byte-layout passes (T = 24, 32): instantiated in translation units of
// their own (life_block_u8_w1_*_t24 / _t32.hip, `extern template` in the
// variant TU), so the build compiles them in parallel.
template <int T, class IO>
void launch_deep(const LifeBlockParams& p, int64_t out_rows, const LifeTuning& tune, hipStream_t s) {
  launch_T<T, IO>(p, out_rows, tune, s);
}
#define GOL_U8_DEEP(KW, T_, XL_)                                                                   \
  namespace gol {                                                                                  \
  namespace hipk {                                                                                 \
  namespace lb {                                                                                   \
  KW template void launch_deep<T_, U8IO<1, XL_>>(const LifeBlockParams&, int64_t, const LifeTuning&, \
                                                 hipStream_t);                                     \
  }                                                                                                \
  }                                                                                                \
  }

// Host entry point of one compiled variant (instantiated once per
// translation unit, life_block_*.hip).
template <class IO>
void launch_variant(const LifeBlockParams& p, int64_t out_rows, int T, const LifeTuning& tune, hipStream_t s) {
  switch (T) {
    case 1: launch_T<1, IO>(p, out_rows, tune, s); break;
    case 2: launch_T<2, IO>(p, out_rows, tune, s); break;
    case 4: launch_T<4, IO>(p, out_rows, tune, s); break;
    case 8: launch_T<8, IO>(p, out_rows, tune, s); break;
    case 12: launch_T<12, IO>(p, out_rows, tune, s); break;
    case 16: launch_T<16, IO>(p, out_rows, tune, s); break;
    case 24:  // byte layout only: fewer byte-grid passes per generation
      // (the adder window never runs T > 16: launch_life_block switches it to DPP)
      if constexpr (!IO::kBits && IO::XL != kXlaneAdd) {
        launch_deep<24, IO>(p, out_rows, tune, s);
        break;
      }
      [[fallthrough]];
    case 32:
      if constexpr (!IO::kBits && IO::XL != kXlaneAdd) {
        if (T == 32) {
          launch_deep<32, IO>(p, out_rows, tune, s);
          break;
        }
      }
      [[fallthrough]];
    default: fail("life_block: unsupported temporal block size " + std::to_string(T));
  }
}

}  // namespace lb
}  // namespace hipk
}  // namespace gol
