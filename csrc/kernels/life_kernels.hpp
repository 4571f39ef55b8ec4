// Launch interfaces of the hand-written CDNA4 kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <functional>
#include <string>

#include "gol/tile.hpp"

namespace gol {
namespace hipk {

struct LifeBlockParams {
  const uint8_t* in;
  uint8_t* out;
  int64_t pitch;
  int64_t row_lo, row_hi;
  int Wp;          // padded words per row
  int ncolw;       // column waves (64*W-2 output words each)
  int nseg;        // row segments
  int seg_rows;    // output rows per segment (balanced: first seg_rem get +1)
  int seg_rem;
  int own_w0, own_w1;
  uint32_t last_mask;
  uint32_t* changed;  // changed[L] <-> generation gen_base + 1 + L (after resolving gen_dev)
  const int64_t* gen_dev;  // if set: changed += *gen_dev + gen_rel at run time (graph replay)
  int64_t gen_rel;
  // Grouped schedule (life_group_kernel): nseg = groups per column strip,
  // seg_rows/seg_rem = balanced OUTPUT rows per group, grp_q = output rows of
  // every wave of a group but the last.
  int grp_q;
  // Diagnostics (GOL_WG_TRACE): if set, every wave of the grouped kernel
  // writes {block<<8 | wave, XCC_ID<<32 | HW_ID, start, end} (s_memrealtime,
  // 100 MHz) at wg_trace[4 * (block * M + wave)], below kWgTraceWaves waves.
  uint64_t* wg_trace;
  // Device-visible error word (host-mapped, Backend::check_device_errors):
  // a kernel that has to give up (life_short_kernel's bounded LDS hand-off
  // wait) sets it instead of continuing silently with invalid rows.
  uint32_t* err;
  // Chained-group spin bound, log2 of polls (GOL_CHAIN_SPIN, default 16).
  int chain_spin_log2;
  // Wrap mode (BlockArgs::full_width): owned words per row, 0 = halo mode
  // (life_block_impl.hpp lane_cols).
  int wrap_w;
  // Folded last strip (life_group_kernel, wrap mode): `fold` groups per
  // block in sub-strips of fold_lanes lanes; 1 = no folding.
  int fold;
  int fold_lanes;
  // Chained groups (life_group_kernel, LifeTuning::chain; null chain_buf =
  // off): the last wave of group g ends like an inner wave, with the inverted
  // triangle fed by group g + 1's wave 0 through global memory, so no group
  // boundary keeps a redundant triangle.  Per (strip, group) slot: wave 0's
  // saved boundary rows in chain_buf, and chain_flag = chain_seq once they are
  // written.  Every group is M x grp_q rows but a strip's last one, which ends
  // at chain_end.
  uint32_t* chain_buf;
  uint32_t* chain_flag;
  uint32_t chain_seq;
  int64_t chain_end;
  // Linked launches (LifeTuning::link, life_group_kernel<..., LINK = true>):
  // this launch may run while the previous grouped launch, whose output is
  // its input, still runs.  Group (kcol, grp) first waits until every group
  // of that launch whose output rows it reads (its strip and the two beside
  // it) has published link_prev_flag[strip * link_prev_nseg + group] ==
  // link_prev_seq, and after its last store publishes link_flag[kcol * nseg
  // + grp] = link_seq.  Payload stores and input loads are sc1 (the no-
  // acquire valid form of cdna_hip_programming.md Guideline 16).
  uint32_t* link_flag;             // null: not a linked launch
  uint32_t link_seq;
  const uint32_t* link_prev_flag;  // null: nothing to wait for
  uint32_t link_prev_seq;
  int64_t link_prev_row_lo;
  int link_prev_nseg, link_prev_seg_rows, link_prev_seg_rem;
  // > 0: both launches cover the owned rows of a row ring of this many rows;
  // the rows a group reads beyond them wrap around the torus (link_wait).
  int64_t link_ring_rows;
  // Boundary trigger (BlockArgs::trigger / hot; linked launches only): the
  // groups grp in [bnd_g[0], bnd_g[1]) or [bnd_g[2], bnd_g[3]) - those whose
  // output rows meet the trigger rows, trigger_groups() - run at top issue
  // priority, and with bnd_count set each adds 1 to *bnd_count after its
  // link_flag store (a one-wave kernel on another stream waits on it,
  // launch_wait_counter).  Group indices, not rows, so the kernel's test is
  // a few scalar compares (row bounds in 64 bits cost the linked kernels
  // SGPR spills).
  unsigned long long* bnd_count;
  int bnd_g[4];
  // Fault injection (GOL_FAULT_DELAY_SPINS, tests): producers at the torus
  // seam - a linked launch's first and last groups - sleep this many s_sleep 127
  // rounds (~3.4 us each) before publishing, so a missing dependency wait
  // reads stale rows deterministically instead of by chance.
  int fault_delay;
};

constexpr int64_t kWgTraceWaves = int64_t(1) << 20;

// Cross-lane primitive that moves the edge words between lanes.
//   kXlaneAdd: no cross-lane data op at all.  The horizontal window is
//   one-sided (cells x-2, x-1, x): both shifts are add-with-carry
//   (v_add_co / v_addc_co) whose per-lane carry masks move one lane up on the
//   SALU (s_lshl_b64).  Each generation then stores cell x-1 at bit x, so the
//   tile's storage frame drifts one cell to the right per generation; the
//   engine tracks the drift and rotates it out before any read-out
//   (Engine::normalize).  Measured (ubench_dpp_mix.hip, git e36884f): any DPP,
//   v_alignbit or v_cmp in a v_bitop3 stream drops the SIMD from ~2.4 to
//   ~4.5 cycles per instruction; add-with-carry ops do not.
//   kXlaneAuto (default): the adder window where the engine allows a drift
//   (HipBackend::choose_kernel: whole-width tiles that fill four waves per
//   SIMD at T = 12), the DPP window everywhere else.
enum Xlane : int { kXlaneAuto = -1, kXlaneDpp = 0, kXlaneAdd = 3 };

// Backend-owned state of linked launches (GOL_LINK; LifeBlockParams::link_*):
// consecutive grouped launches of an epoch alternate between two streams and
// overlap, ordered by per-group completion words instead of the stream.
struct LinkState {
  hipStream_t stream[2] = {nullptr, nullptr};  // [0] = the backend's compute stream
  hipEvent_t before[2] = {nullptr, nullptr};   // recorded on stream[i] just before its last launch
  int cur = 0;                                  // stream of the last launch
  bool prev_valid = false;                      // the last launch may be linked to
  const void* prev_out = nullptr;               // its output buffer
  int64_t prev_blocks = 0;                      // its workgroups
  double prev_share = 0.0;                      // its workgroups / how many of them fit on the CUs
  LifeBlockParams prev{};                       // its plan and completion words
  uint32_t* flags[3] = {nullptr, nullptr, nullptr};  // completion words, rotating per launch
  size_t flag_words = 0;
  uint32_t seq = 0;
  int64_t linked = 0;                           // launches that ran linked (diagnostics)
  int chain = 0;  // launches in the current chain
  // The stream of the next launch already follows the last launch's start
  // (Backend::trigger_stream: its wait kernel returns only once that
  // launch's boundary groups are done), so a linked next launch needs no
  // cross-stream event wait (~10 us of device time on the epoch boundary).
  bool started = false;
  // Boundary trigger of the next launch (BlockArgs::trigger): requested
  // rows, the counter, and how many increments the launch will make
  // (launch_linked sets it; 0: the launch could not carry the trigger).
  bool bnd_req = false;
  bool bnd_count_req = false;  // count (the trigger launch) or priority only (BlockArgs::hot)
  int64_t bnd_r[4] = {0, 0, 0, 0};
  unsigned long long* bnd_count = nullptr;
  int64_t bnd_n = 0;
};

// The groups of a grouped plan whose output rows meet the trigger rows
// [r[0], r[1]) and [r[2], r[3]): index ranges [g[0], g[1]) and [g[2], g[3])
// (each contiguous: groups are ordered by row); returns how many groups meet
// either, per column strip (a folded strip publishes each of its groups once,
// so a counting launch makes ncolw times this many increments).
inline int trigger_groups(const LifeBlockParams& q, const int64_t* r, int* g) {
  int n = 0;
  g[0] = g[1] = g[2] = g[3] = 0;
  for (int s = 0; s < q.nseg; ++s) {
    const int64_t e = q.row_lo + int64_t(s) * q.seg_rows + std::min(s, q.seg_rem) + q.seg_rows + (s < q.seg_rem ? 1 : 0);
    const int64_t b = e - q.seg_rows - (s < q.seg_rem ? 1 : 0);
    bool any = false;
    for (int k = 0; k < 2; ++k)
      if (b < r[2 * k + 1] && e > r[2 * k]) {
        if (g[2 * k + 1] == 0) g[2 * k] = s;
        g[2 * k + 1] = s + 1;
        any = true;
      }
    n += any ? 1 : 0;
  }
  return n;
}

// Everything enqueued on stream[1] precedes what comes next on stream[0];
// the next launch starts a new chain.
inline void link_join(LinkState& L) {
  L.started = false;
  if (L.cur != 0) {
    (void)hipEventRecord(L.before[1], L.stream[1]);
    (void)hipStreamWaitEvent(L.stream[0], L.before[1], 0);
    L.cur = 0;
  }
  L.prev_valid = false;
}

struct LifeTuning {
  int cus = 256;            // compute units of the device
  int target_waves = 0;     // waves per launch round (0 = occupancy x CUs x 4 SIMDs)
  int min_seg_rows = 16;    // lower bound on rows per wave segment
  int xlane = kXlaneAuto;   // cross-lane primitive
  bool u8_lds = false;      // byte layout: single-step LDS-tiled kernel (T = 1)
  int lds_rows = 32;        // rows per LDS tile (32 or 64)
  int lds_T = 8;            // generations per launch of the LDS-tiled byte kernel (1, 2, 4, 8; 16, 32 packed)
  bool lds_pack = true;     // LDS-tiled byte kernel evaluates on bit words packed in LDS (T >= 8)
  bool lds_xcd = false;     // packed LDS tiles: XCD-aware workgroup order (column-major runs per XCD)
  int lds_waves = 0;        // packed LDS tiles: waves per workgroup (8, 16; 0 = by grid size)
  int group = 8;            // grouped schedule, waves per workgroup sharing boundaries: 4, 8, -1 auto, 0 off
  int group_small = 4;      // the same for bit-layout blocks of T <= 8 (GOL_GROUP_SMALL; GOL_GROUP sets both)
  bool wrap = true;         // wrap mode on whole-width tiles (BlockArgs::full_width, lane_cols)
  bool fold = true;         // folded last strip in wrap mode (life_group_kernel)
  int chain = 0;            // chained groups (LifeBlockParams::chain_buf): 0 off, 1 on, 2 timing probe
  bool chain_ok = false;    // this launch may use the chain memory (the backend's own stream, not captured)
  uint32_t* chain_seq = nullptr;  // host launch counter of the chain flags
  // Device memory of at least n bytes that persists across launches, stream-
  // ordered like `scratch`: which = 0 the chain flags (zeroed when allocated),
  // 1 the chain slots.
  std::function<uint32_t*(int which, size_t n)> chain_mem;
  LinkState* link = nullptr;     // linked launches on (null: every launch on the given stream)
  uint64_t* wg_trace = nullptr;  // per-wave placement/timing record of the next launch (LifeBlockParams)
  uint32_t* err = nullptr;       // LifeBlockParams::err (4 words: code, then a give-up's diagnostics)
  int chain_spin_log2 = 16;      // LifeBlockParams::chain_spin_log2
  int fault_delay = 0;  // LifeBlockParams::fault_delay (GOL_FAULT_DELAY_SPINS)
};

// Returns the storage-frame drift of the launch in cells (T for the adder
// window, 0 otherwise; BlockArgs::allow_drift).
int launch_life_block(const BlockArgs& a, const LifeTuning& tune, hipStream_t stream);
// Description of the kernel variant the tuning selects for a layout.
std::string life_block_variant(Layout layout, const LifeTuning& tune);
// Largest T that keeps 2 waves/SIMD for the variant's words-per-lane.
int life_block_max_T(Layout layout, const LifeTuning& tune);

// Compiled variants (one translation unit each): the DPP and adder windows,
// bit and byte layouts, one 32-cell word per lane.
#define GOL_LIFE_VARIANT(name) \
  void name(const LifeBlockParams& p, int64_t out_rows, int T, const LifeTuning& tune, hipStream_t s)
GOL_LIFE_VARIANT(launch_bits_w1_dpp);
GOL_LIFE_VARIANT(launch_u8_w1_dpp);
GOL_LIFE_VARIANT(launch_bits_w1_add);
GOL_LIFE_VARIANT(launch_u8_w1_add);

// Single-generation LDS-tiled byte-layout kernel (life_step_lds.hip).
void launch_life_step_lds(const BlockArgs& a, int lds_rows, bool wrap, hipStream_t stream);
// The same with T = 2, 4 or 8 generations per launch through two LDS row
// buffers (life_step_lds.hip life_lds_multi_kernel).
void launch_life_lds_multi(const BlockArgs& a, bool wrap, hipStream_t stream);
// The same tile packed to bit words in LDS (T = 8, 16 or 32 generations per
// launch, bit-sliced rule; life_step_lds.hip life_lds_bits_kernel).  Returns
// the drift of the stored frame (T with the adder window, which it runs
// where BlockArgs::allow_drift and the tile wraps its columns; else 0).
int launch_life_lds_bits(const BlockArgs& a, bool wrap, bool xcd_order, int waves, int cus, hipStream_t stream);

// Tile utility kernels (tile_ops.hip).
void launch_fill_cols(uint8_t* buf, const TileGeom& g, hipStream_t s);
// Column halos of padded rows [r0, r0 + nrows) only.
void launch_fill_cols_rows(uint8_t* buf, const TileGeom& g, int64_t r0, int64_t nrows, hipStream_t s);
void launch_fill_rows(uint8_t* buf, const TileGeom& g, hipStream_t s);
// Fused cols+rows periodic fill (bit layout); false if the geometry needs the two-launch path.
bool launch_fill_all(uint8_t* buf, const TileGeom& g, hipStream_t s);
void launch_alive(const uint8_t* buf, const TileGeom& g, uint32_t* any_flag,
                  unsigned long long* count, hipStream_t s);
// Owned rows [r0, r0+n) from a device staging array of 0/1-or-ASCII bytes.
void launch_load_rows(uint8_t* buf, const TileGeom& g, const uint8_t* stage, int64_t ld,
                      int64_t r0, int64_t n, hipStream_t s);
void launch_store_rows(const uint8_t* buf, const TileGeom& g, uint8_t* stage, int64_t ld,
                       int64_t r0, int64_t n, bool ascii, hipStream_t s);
void launch_i64(int64_t* p, int64_t v, bool add, hipStream_t s);
// Holds stream s until *counter >= target (one sleeping wave; error word 7
// after ~4 s): the boundary trigger's wait (Backend::trigger_stream).
void launch_wait_counter(const unsigned long long* counter, unsigned long long target, uint32_t* err, hipStream_t s);
void launch_init_random(uint8_t* buf, const TileGeom& g, uint64_t seed, uint32_t thresh24,
                        int64_t grow0, int64_t gcol0, hipStream_t s);
// Owned rows of `src` rotated left by `shift` cells (0 < shift < W) into
// `dst`: dst cell x = src cell (x + shift) mod W.  Undoes the adder window's
// storage drift.
void launch_rotate_cols(const uint8_t* src, uint8_t* dst, const TileGeom& g, int64_t shift, hipStream_t s);
// Owned rows [i0, i0 + nrows) of the owned cells, byte cells <-> bit words
// (the two geometries hold the same owned tile; halos and pitch may differ).
void launch_convert_rows(const uint8_t* src, const TileGeom& gs, uint8_t* dst, const TileGeom& gd, int64_t i0,
                         int64_t nrows, hipStream_t s);

}  // namespace hipk
}  // namespace gol
