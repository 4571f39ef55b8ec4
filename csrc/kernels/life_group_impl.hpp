// Grouped temporal-blocking schedule (default for T >= 4): the classic
// life_block sweep of life_block_impl.hpp with the per-segment redundancy
// removed inside a workgroup.
//
// The classic schedule starts every wave segment T rows above its output and
// recomputes the triangle of level rows that the segment above also computes:
// T(T-1) level-rows per boundary, 240 at T = 16, against 16 x 34 useful
// level-rows per wave on the 8-GPU per-rank tile (32768 x 4096).  A split
// schedule (the triangle in a second kernel) measured slower and was removed.
// Here a workgroup of M waves owns M consecutive
// segments of one column strip and shares its M-1 internal boundaries through
// LDS:
//   * wave m reads input rows from in0 = G0 + m q - T (G0 = first output row
//     of the group).  Wave m >= 1 thus starts exactly at its boundary
//     b_m = in0 (a trapezoid: its level-L rows begin at b_m + L) and saves,
//     during its 2T prologue steps, its level-L rows b_m + L and b_m + L + 1
//     (L = 1..T-1) in LDS;
//   * after one workgroup barrier, every wave but the last finishes with the
//     inverted triangle below its lower boundary b = in0 + q: 2T more steps
//     (epilogue_tri) in which level e/2 is fed the lower wave's saved row
//     instead of computing it, writing the level-T rows [b - T, b + T);
//   * wave 0 starts and wave M-1 ends like classic waves, so only one boundary
//     in M (the group boundaries) keeps the redundant triangle.
// Inside a group every level row is computed exactly once.  Waves 0..M-2
// produce q output rows each; the last wave, which also pays the redundant
// triangle (about T-1 rows' worth), produces the rest of the group.
//
// The reference has no counterpart: its CUDA evolve (src/game_cuda.cu:128-148)
// is one generation per launch, one thread per cell.
#pragma once

#include <cstdlib>

#include "life_block_impl.hpp"

// Epilogue steps per scheduling region (sched_barrier between regions); 1
// keeps the T = 16 kernel at 123 VGPRs (4 waves/SIMD), 2-4 let hipcc overlap
// neighbouring steps at 130 VGPRs (3 waves/SIMD).
#ifndef GOL_EPI_SCHED
#define GOL_EPI_SCHED 1
#endif

namespace gol {
namespace hipk {
namespace lb {

// LDS slot of one boundary: [L-1][j][word i][lane] (lane-contiguous: a wave's
// access is 64 consecutive dwords, conflict-free).  Slot m holds wave m's
// top rows; wave 0 writes slot 0, which nobody reads (a branch around the
// stores splits the prologue into ~30 blocks and doubled the registers;
// chained groups reuse it after the prologue barrier, chain_fetch).
template <int T, int W>
struct LdsSaver {
  uint32_t* slot;
  int lane;
  __device__ __forceinline__ void operator()(int L, int j, const Vec<W>& v) const {
#pragma unroll
    for (int i = 0; i < W; ++i) slot[(((L - 1) * 2 + j) * W + i) * 64 + lane] = v.w[i];
  }
};

// The grouped kernel's saver: LdsSaver, and with chained groups
// (LifeBlockParams::chain_buf) wave 0 also stores its rows to the group's
// global slot through `pub`, whose num_records is 0 for every
// other wave, so their copies are dropped by the range check without a branch
// in the unrolled prologue.  sc1 (kCpolSc1): written through to the
// device-coherent level (the reading group may run on another XCD, behind
// another L2).
template <int T, int W>
struct ChainSaver {
  uint32_t* slot;
  int lane;
  BufRsrc pub;
  __device__ __forceinline__ void operator()(int L, int j, const Vec<W>& v) const {
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const int idx = (((L - 1) * 2 + j) * W + i) * 64 + lane;
      slot[idx] = v.w[i];
      __builtin_amdgcn_raw_buffer_store_b32(v.w[i], pub, idx * 4, 0, kCpolSc1);
    }
  }
};

// Chained groups: the last wave of a group (not the strip's last) waits until
// the group below has published its wave 0 rows (flag == chain_seq) and
// copies them into LDS slot 0, which nobody reads once the prologue barrier
// has passed.  Deadlock-free: chained strips are launched bottom group first
// (life_group_kernel's block order), so the group waited on was dispatched
// earlier, and its wave 0 publishes right after its prologue, before it waits
// on anything.  Bounded (~0.1 s): giving up raises the launch's error word
// (Backend::check_device_errors) instead of hanging the GPU.
//
// Memory model (cdna_hip_programming.md §6 Guideline 16, recipe R1): the
// producer stores every payload word sc1 (ChainSaver: write-through to the
// device-coherent level, so no release fence is needed), the one storing wave
// drains them (s_waitcnt vmcnt(0)) and only then one of its lanes stores the
// flag with an agent-scope atomic; the consumer wave polls that one word
// relaxed at agent scope and, after the match, performs an agent-scope
// acquire (L1 invalidate + wait) before reading the payload with sc1 buffer
// loads to registers.  That is the formal release/acquire pair (the sc1
// loads alone match the guide's "valid forms" table row for one signalling
// lane per storing workgroup, which was measured only at one workgroup per
// CU, so the acquire stays).  (An LDS-DMA copy, global_load_lds, would not
// qualify either way: it is not a load to registers.)
template <int T, int W>
__device__ __forceinline__ void chain_fetch(const LifeBlockParams& p, int64_t slot_below, int64_t flag_below,
                                            uint32_t* lds_slot, int lane) {
  constexpr int kRows = (T - 1) * 2 * W;
  bool arrived = false;
  uint32_t seen = 0;
  const int spins = 1 << p.chain_spin_log2;
  for (int spin = 0; spin < spins; ++spin) {  // each poll is an L2-bypassing load (~1-2 us)
    seen = __hip_atomic_load(p.chain_flag + flag_below, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen == p.chain_seq) {
      arrived = true;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  if (!arrived && p.err && lane == 0) {  // diagnostics first, then the code the host checks
    __hip_atomic_store(p.err + 1, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.err + 2, p.chain_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.err + 3, uint32_t(flag_below), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // The formal pair of the producer's write-through stores: an agent-scope
  // acquire drops this CU's L1 lines, and the wait holds the loads below
  // until the invalidate has completed (MI355X_MICROARCH.md, visibility).
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const BufRsrc src = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(p.chain_buf + slot_below), short(0),
                                                        kRows * 64 * 4, kBufFlags);
  // Eight rows in flight per batch (8 VGPRs), sc1 loads to registers, then LDS.
  constexpr int kBatch = 8;
#pragma unroll 1
  for (int r0 = 0; r0 < kRows; r0 += kBatch) {
    uint32_t v[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j)
      v[j] = r0 + j < kRows ? __builtin_amdgcn_raw_buffer_load_b32(src, ((r0 + j) * 64 + lane) * 4, 0, kCpolSc1) : 0u;
#pragma unroll
    for (int j = 0; j < kBatch; ++j)
      if (r0 + j < kRows) lds_slot[(r0 + j) * 64 + lane] = v[j];
  }
}

// Linked launches (LifeBlockParams::link_prev_flag): wave 0 of a group
// waits, one flag per lane, until every group of the previous launch whose
// output rows [r0, r1) this group reads has published, in its own strip and
// the strips beside it (modulo the strip count in wrap mode, clipped in halo
// mode).  The previous launch's groups were all dispatched before or beside
// this one (the backend links two launches only when both fit on the GPU at
// once), so the wait ends; bounded (~0.1 s) like chain_fetch, it raises the
// error word 3 instead of hanging.
//   On a row ring (link_ring_rows > 0) the rows beyond the owned ones are the
// torus wrapped around: the top group reads the last rows and the bottom
// group the first ones, so the groups are counted around the torus (an
// unwrapped index, group + nseg per turn) and taken modulo nseg.
__device__ __forceinline__ void link_wait(const LifeBlockParams& p, int kcol, int64_t r0, int64_t r1, int lane) {
  const int q1 = p.link_prev_seg_rows + 1;
  const int64_t big = int64_t(p.link_prev_seg_rem) * q1;
  const int nseg = p.link_prev_nseg;
  const int64_t ring = p.link_ring_rows;
  const auto grp_of = [&](int64_t r) -> int64_t {
    int64_t x = r - p.link_prev_row_lo;
    int64_t turns = 0;
    if (ring > 0) {
      turns = x >= 0 ? x / ring : -((-x + ring - 1) / ring);
      x -= turns * ring;
    } else {
      x = max<int64_t>(0, x);
    }
    const int64_t g = x < big ? x / q1 : p.link_prev_seg_rem + (x - big) / max(1, p.link_prev_seg_rows);
    return turns * nseg + min<int64_t>(g, nseg - 1);
  };
  const int64_t g0 = grp_of(r0);
  const int ng = int(min<int64_t>(grp_of(r1 - 1) - g0 + 1, int64_t(nseg)));
  const int nflags = 3 * ng;
  for (int base = 0; base < nflags; base += 64) {
    const int f = base + lane;
    int k = kcol + f / ng - 1;
    if (p.wrap_w > 0) k = (k + p.ncolw) % p.ncolw;
    const bool mine = f < nflags && k >= 0 && k < p.ncolw;
    int g = int((g0 + f % ng) % nseg);
    if (g < 0) g += nseg;
    const uint32_t* w = p.link_prev_flag + (int64_t(mine ? k : 0) * nseg + (mine ? g : 0));
    bool done = !mine;
    for (int spin = 0; spin < (1 << 16); ++spin) {
      if (!done) done = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.link_prev_seq;
      if (__all(done)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (!__all(done) && p.err && lane == 0) __hip_atomic_store(p.err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // No load of the previous launch's rows may move above the wait.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef GOL_PRIO_BUCKETS
#define GOL_PRIO_BUCKETS 4
#endif

// Level bodies of epilogue steps 0..E-1 (step e advances levels e/2..T-1).
template <int T>
__host__ __device__ constexpr int epi_work_before(int E) {
  int w = 0;
  for (int e = 0; e < E; ++e) w += T - e / 2;
  return w;
}
template <int T>
__device__ __forceinline__ int epi_work(int nfull) {
  return nfull >= 2 * T ? epi_work_before<T>(2 * T) : nfull * T;  // the last wave's plain steps
}

// Progress-ordered issue priority (GOL_PRIO_BUCKETS): the SIMD arbiter
// favours the oldest of equal-priority waves, so co-resident waves with
// equal work otherwise finish in a staircase and the last one runs alone
// (15-20 % of a launch, scripts/wg_trace.py).  A wave drops one priority
// level per 1/GOL_PRIO_BUCKETS of its post-barrier work, so waves that are behind
// catch up.  Compiled out when off.
struct Prio {
  static constexpr int kLevels = GOL_PRIO_BUCKETS > 4 ? 4 : GOL_PRIO_BUCKETS;
  int quarter;   // post-barrier work / levels, in level bodies
  int done0 = 0;
  int next = 0;  // work at which the priority drops next
  int cur = kLevels - 1;
  bool boost = false;  // stay at priority 3 (hot groups of a trigger epoch)
  __device__ __forceinline__ Prio(int wtot, bool boost_)
      : quarter(max(1, wtot / max(kLevels, 1))), next(max(1, wtot / max(kLevels, 1))), boost(boost_) {
    if (boost) {
      __builtin_amdgcn_s_setprio(3);
      return;
    }
#if GOL_PRIO_BUCKETS
    if (cur == 3) __builtin_amdgcn_s_setprio(3);
    else if (cur == 2) __builtin_amdgcn_s_setprio(2);
    else if (cur == 1) __builtin_amdgcn_s_setprio(1);
#endif
  }
  __device__ __forceinline__ void at(int done) {
#if GOL_PRIO_BUCKETS
    if (!boost && cur > 0 && done >= next) {  // wave-uniform; one scalar compare per step
      next += quarter;
      --cur;
      if (cur == 2) __builtin_amdgcn_s_setprio(2);
      else if (cur == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#else
    (void)done;
#endif
  }
  __device__ __forceinline__ void reset() {
#if GOL_PRIO_BUCKETS
    __builtin_amdgcn_s_setprio(0);
#endif
  }
};

// Epilogue step E (0..2T-1) at sweep step k = kmain + E, window slot S: level
// L0 = E/2 receives its row in0 + k - L0 = b + L0 + (E & 1), which is the
// input row for L0 = 0 and the lower wave's saved row otherwise; levels
// L0..T-1 advance and the level-T row b + E - T is written.
// The last wave of a group shares steps E < nfull (plain input steps: the
// 0-2 steps of its classic end that do not fill a 3-step loop iteration) and
// stops there.  One code path for both kinds of wave: a separate remainder
// branch beside the epilogue made hipcc allocate 199 instead of 123 VGPRs.
template <int T, class IO, int E, int S>
__device__ __forceinline__ void epilogue_tri(Levels<T, IO::W>& st, RowReader<IO>& rd, const uint32_t* below,
                                             int lane, const Writer<IO>& wr, int k, int nfull, Prio& prio) {
  if constexpr (E < 2 * T) {
    if (E >= nfull) return;  // wave-uniform
    prio.at(prio.done0 + epi_work_before<T>(E));
    constexpr int W = IO::W;
    constexpr int L0 = E / 2;
    Vec<W> cur;
    if constexpr (L0 == 0) {
      cur = rd.template take<S>(k);
    } else {
#pragma unroll
      for (int i = 0; i < W; ++i) cur.w[i] = below[(((L0 - 1) * 2 + (E & 1)) * W + i) * 64 + lane];
    }
    wr.row(k - T, levels_full<T, IO, S, L0, T>(st, cur));
    // Keep the scheduler inside one step: interleaving the whole epilogue
    // (272 level bodies at T = 16) blows the register budget.
    if constexpr (E % GOL_EPI_SCHED == GOL_EPI_SCHED - 1) __builtin_amdgcn_sched_barrier(0);
    epilogue_tri<T, IO, E + 1, (S + 1) % 3>(st, rd, below, lane, wr, k + 1, nfull, prio);
  }
}

#ifndef GOL_GROUP_T16_WAVES
#define GOL_GROUP_T16_WAVES 2
#endif
// The adder window's T = 16 grouped kernel lands at ~156 VGPRs (3 waves/SIMD)
// unconstrained; its level body is 17% cheaper at 4 waves/SIMD than at 3
// (ubench_body.hip, git e36884f), so it is held to 128 VGPRs.
#ifndef GOL_GROUP_T16_ADD_WAVES
#define GOL_GROUP_T16_ADD_WAVES 4
#endif

// Occupancy floor of the grouped kernel (a register cap, not a target: the
// allocator lands at 123 VGPRs = 4 waves/SIMD for bits T = 16 and at 183 for
// the byte layout).  Without a cap, an early version with a separate
// remainder branch took ~400 registers (VGPR + AGPR, one wave per SIMD).
#ifndef GOL_GROUP_T12_ADD_WAVES
#define GOL_GROUP_T12_ADD_WAVES 3
#endif
template <int T, class IO>
constexpr int group_min_waves() {
  if constexpr (IO::W >= 2) return T >= 12 ? 2 : T >= 8 ? 3 : 4;
  if constexpr (IO::XL == kXlaneAdd) return T >= 16 ? GOL_GROUP_T16_ADD_WAVES : T >= 12 ? GOL_GROUP_T12_ADD_WAVES : 4;
  return T >= 16 ? GOL_GROUP_T16_WAVES : T >= 12 ? 3 : 4;
}

// One record per wave (LifeBlockParams::wg_trace): where it ran (HW_ID:
// wave, SIMD, CU, SE fields; XCC_ID) and when it started and ended.
__device__ __forceinline__ void wg_trace_record(uint64_t* tr, int M, int m, int lane, uint64_t t_start) {
  const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
  const int64_t idx = int64_t(blockIdx.x) * M + m;
  if (lane != 0 || idx >= kWgTraceWaves) return;
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID, 32 bits
  const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID, 16 bits
  tr[4 * idx + 0] = (uint64_t(blockIdx.x) << 8) | uint64_t(m) | (uint64_t(1) << 63);
  tr[4 * idx + 1] = (uint64_t(xcc) << 32) | hw;
  tr[4 * idx + 2] = t_start;
  tr[4 * idx + 3] = t_end;
}

template <int T, class IO, int M>
__global__ __launch_bounds__(64 * M) __attribute__((amdgpu_waves_per_eu(group_min_waves<T, IO>())))
void life_group_kernel(const LifeBlockParams p) {
  constexpr int W = IO::W;
  constexpr int kSlot = (T - 1) * 2 * W * 64;  // dwords per boundary
  __shared__ uint32_t saved[M * kSlot];
  const int lane = threadIdx.x & 63;
  const int m = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t t_start = p.wg_trace ? __builtin_amdgcn_s_memrealtime() : 0;
  const int blk = blockIdx.x;
  // Folded last strip (wrap mode): one block runs p.fold groups of the
  // narrow last strip side by side in lane sub-strips.  Every sub-strip then
  // takes the largest group size (a smaller group starts one row early and
  // recomputes its upper neighbour's last row, identically), so the wave's
  // control flow is the same for all of them; lanes carry their group's row
  // offset in their read / store offsets.
  const bool chain = p.chain_buf != nullptr;  // fold == 1 (launch_T)
  int kcol, grp, nsub = 1, sub_lanes = 64;
  if (p.fold > 1 && blk >= (p.ncolw - 1) * p.nseg) {
    kcol = p.ncolw - 1;
    grp = (blk - kcol * p.nseg) * p.fold;
    nsub = p.fold;
    sub_lanes = p.fold_lanes;
  } else {
    kcol = blk / p.nseg;
    grp = blk - kcol * p.nseg;
    if (chain) grp = p.nseg - 1 - grp;  // bottom group first: see chain_fetch
  }
  const auto group_end = [&](int g) {
    return p.row_lo + int64_t(g) * p.seg_rows + min(g, p.seg_rem) + p.seg_rows + (g < p.seg_rem ? 1 : 0);
  };
  // Boundary trigger: the groups whose rows the exchange waits for run at
  // top issue priority throughout, so their count completes ahead of the
  // interior groups sharing their SIMDs (wave-uniform).  Linked kernels
  // only: a runtime flag in the others stopped the compiler from splitting
  // the main loop per priority level (+15 SALU per step, 32768^2 +3 %).
  const auto trig = [&](int g0, int g1) {  // groups [g0, g1) meet the trigger rows
    return (g0 < p.bnd_g[1] && g1 > p.bnd_g[0]) || (g0 < p.bnd_g[3] && g1 > p.bnd_g[2]);
  };
  const bool hot = IO::kLinked && trig(grp, grp + nsub);
  if (hot) __builtin_amdgcn_s_setprio(3);
  // Chained strips: wave wi = grp M + m starts at row_lo + wi q + 3 min(wi, x),
  // the first x = seg_rem waves taking q + 3 rows; the strip's last wave ends
  // at chain_end.
  const int wi = grp * M + m;
  const int64_t G1 = chain ? p.chain_end : group_end(grp);
  const int64_t G0 = G1 - p.seg_rows - (nsub > 1 ? (p.seg_rem > 0 ? 1 : 0) : (grp < p.seg_rem ? 1 : 0));
  const int64_t in0 = chain ? p.row_lo + int64_t(wi) * p.grp_q + 3 * min(wi, p.seg_rem) - T
                            : G0 + int64_t(m) * p.grp_q - T;
  const bool chain_down = chain && m == M - 1 && grp < p.nseg - 1;  // fed by the group below
  const bool last = m == M - 1 && !chain_down;
  constexpr int kPro = 2 * T;
  // Steps of the 3-step main loop end at kmain: q for waves 0..M-2 ((q - 2T)
  // % 3 == 0 by plan); the last wave's classic end (level-T rows up to
  // G1 - 1) takes kend steps, of which the last (kend - 2T) % 3 run as the
  // epilogue's plain input steps.
  const int kend = int(G1 + T - in0);
  const int kmain = last ? kend - (kend - kPro) % 3 : p.grp_q + (chain && wi < p.seg_rem ? 3 : 0);
  const int nfull = last ? (kend - kPro) % 3 : 2 * T;

  const LaneCols<IO> lc = lane_cols<IO>(p, kcol, lane, sub_lanes, nsub);
  const int64_t pitch = p.pitch;
  int64_t dl = 0;  // rows between this lane's group and the wave's (folded strips)
  Writer<IO> wr;
  if (nsub > 1) {
    dl = group_end(min(grp + min(lc.sub, nsub - 1), p.nseg - 1)) - G1;
    wr.roff = int(dl * pitch);
    wr.nrec = int((group_end(min(grp + nsub - 1, p.nseg - 1)) - G1 + 1) * pitch);
  }
  RowReader<IO> rd;
  uint32_t fmask[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
    rd.ok[i] = lc.ok[i];
    wr.own[i] = lc.own[i];
    fmask[i] = lc.fmask[i];
  }

  Levels<T, W> st;
#pragma unroll
  for (int L = 0; L < T; ++L) {
#pragma unroll
    for (int i = 0; i < W; ++i) {
#pragma unroll
      for (int s = 0; s < 3; ++s) st.h0[L][s].w[i] = st.h1[L][s].w[i] = st.cc[L][s].w[i] = 0u;
      st.acc[L].w[i] = 0u;
    }
  }

  if constexpr (IO::kLinked) {  // wait for the previous launch's rows this group reads
    // (a folded block: the rows of all its groups)
    const int64_t Gend = nsub > 1 ? group_end(min(grp + nsub - 1, p.nseg - 1)) : G1;
    if (p.link_prev_flag && m == 0) link_wait(p, kcol, G0 - T, Gend + T, lane);
    __syncthreads();
  }
  rd.base = p.in + in0 * pitch;  // input row of step k: in0 + k
  rd.pitch = pitch;
  rd.kmax = last ? kend - 1 : kmain + 1;
#pragma unroll
  for (int i = 0; i < W; ++i) rd.off[i] = lc.off[i] + int(dl * (pitch / IO::kWordBytes));
  rd.init();
  wr.out = p.out + in0 * pitch;  // level-T row of step k: in0 + k - T
  wr.pitch = pitch;
  wr.col = lc.store_col;

  const int64_t chain_at = int64_t(kcol) * p.nseg + grp;  // this group's chain slot / flag
  const bool publish = chain && m == 0 && grp > 0;
  const ChainSaver<T, W> saver{saved + m * kSlot, lane,
                             __builtin_amdgcn_make_buffer_rsrc(chain ? p.chain_buf + chain_at * kSlot : nullptr,
                                                               short(0), publish ? kSlot * 4 : 0, kBufFlags)};
  // A publishing wave runs its prologue at top priority and publishes before
  // the barrier: its store round trip then overlaps the other waves'
  // prologues, and the group above finds the rows ready when its last wave
  // reaches the epilogue (on small tiles that wave has no main loop between).
  if (publish) __builtin_amdgcn_s_setprio(3);
  prologue_tri<T, IO, 0>(st, rd, saver, NoBottom{});
  if (publish) {  // wave-uniform: the rows are written through, then the flag
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0) __hip_atomic_store(p.chain_flag + chain_at, p.chain_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!hot) __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();  // every wave's boundary rows are in LDS

  int k = kPro;
  constexpr int S0 = kPro % 3, S1 = (S0 + 1) % 3, S2 = (S0 + 2) % 3;
  // Post-barrier work in level bodies: main loop + epilogue triangle.
  Prio prio((kmain - kPro) * T + epi_work<T>(nfull), hot);
  for (; k + 3 <= kmain; k += 3) {
    prio.at((k - kPro) * T);
    wr.row(k - T, levels_full<T, IO, S0, 0, T>(st, rd.template take<S0>(k)));
    wr.row(k + 1 - T, levels_full<T, IO, S1, 0, T>(st, rd.template take<S1>(k + 1)));
    wr.row(k + 2 - T, levels_full<T, IO, S2, 0, T>(st, rd.template take<S2>(k + 2)));
  }

  prio.done0 = (kmain - kPro) * T;
  if (chain_down) chain_fetch<T, W>(p, (chain_at + 1) * kSlot, chain_at + 1, saved, lane);
  epilogue_tri<T, IO, 0, S0>(st, rd, saved + (chain_down ? 0 : m + 1) * kSlot, lane, wr, k, nfull,
                             prio);  // k == kmain
  prio.reset();

  if (p.changed) {
    uint32_t mask = 0;
#pragma unroll
    for (int L = 0; L < T; ++L) {
      uint32_t any = 0;
#pragma unroll
      for (int i = 0; i < W; ++i) any |= st.acc[L].w[i] & fmask[i];
      mask |= (__ballot(any != 0u) != 0ull ? 1u : 0u) << L;
    }
    uint32_t* ch = p.gen_dev ? p.changed + (*p.gen_dev + p.gen_rel) : p.changed;
    if (lane < T && ((mask >> lane) & 1u)) ch[lane] = 1u;
  }
  if constexpr (IO::kLinked) {  // every wave's rows are written through, then one flag
    __builtin_amdgcn_s_waitcnt(0);
    if (p.fault_delay && (grp == 0 || grp + nsub >= p.nseg))  // tests: the seam's producers publish late
      for (int i = 0; i < p.fault_delay; ++i) __builtin_amdgcn_s_sleep(127);
    __syncthreads();
    // One word per group: a folded block publishes each of its groups.
    if (p.link_flag && m == 0 && lane < nsub && grp + lane < p.nseg) {
      __hip_atomic_store(p.link_flag + (int64_t(kcol) * p.nseg + grp + lane), p.link_seq, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      // Boundary trigger: the rows were written through (sc1) and drained
      // above; a wave of another stream polls the counter (launch_wait_counter).
      if (p.bnd_count && trig(grp + lane, grp + lane + 1))
        __hip_atomic_fetch_add(p.bnd_count, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (p.wg_trace) wg_trace_record(p.wg_trace, M, m, lane, t_start);
}

// Plan: groups per strip (p.nseg), balanced group sizes (p.seg_rows,
// p.seg_rem) and the per-wave row count q (p.grp_q) with q >= 2T and
// (q - 2T) % 3 == 0, so that every non-last wave's main loop ends on the
// window slot its epilogue starts with.  The score is plan()'s makespan
// model: rounds x (longest wave + overhead) x resident waves x issue factor,
// in rows of T level bodies.  Returns the cost, or -1 when the rows are too
// few for M segments of 2T rows.
template <int T, int M>
double plan_group(LifeBlockParams& p, int64_t out_rows, int simds, int occ, int target_waves, int xl = kXlaneDpp) {
  // A folded last strip (p.fold groups per block) costs 1/fold of a strip.
  const auto strip_groups = [&](int64_t n) {
    return p.fold > 1 ? int64_t(p.ncolw - 1) * n + ceil_div(n, int64_t(p.fold)) : int64_t(p.ncolw) * n;
  };
  constexpr double kOverhead = 0.4 * T;  // the two triangles (4T steps) run at lower ILP
  const int64_t max_n = out_rows / (int64_t(M - 1) * 2 * T + 1);
  int64_t best_n = 0;
  int best_q = 0;
  double best = 1e300;
  for (int64_t n = 1; n <= max_n; ++n) {
    const int64_t lo = out_rows / n, hi = lo + (out_rows % n ? 1 : 0);
    // q near the balance point (Lg + T - 1) / M, on the right residue.
    const int64_t ideal = std::max<int64_t>(2 * T, (hi + T - 1) / M);
    int q = 0;
    double span = 1e300;
    for (int64_t c = ideal - 3; c <= ideal + 3; ++c) {
      if (c < 2 * T || (c - 2 * T) % 3 != 0 || lo - int64_t(M - 1) * c < 0) continue;
      const double s = std::max<double>(double(c), double(hi - int64_t(M - 1) * c) + (T - 1));
      if (s < span) {
        span = s;
        q = int(c);
      }
    }
    if (q == 0) continue;
    const int64_t waves = strip_groups(n) * M;
    const int64_t k = ceil_div(waves, int64_t(simds));
    const int64_t rounds = ceil_div(k, int64_t(occ));
    const int64_t kk = std::min<int64_t>(k, occ);
    double cost = double(rounds) * (span + kOverhead) * double(kk) * issue_factor(xl, kk);
    if (target_waves > 0)
      cost = 1.0 + double(std::llabs(waves - int64_t(target_waves)));
    else if (rounds > 4)
      break;  // more groups only add rounds from here on
    if (cost < best * 0.999) {
      best = cost;
      best_n = n;
      best_q = q;
    }
  }
  if (best_n == 0) return -1.0;
  p.nseg = int(best_n);
  p.seg_rows = int(out_rows / best_n);
  p.seg_rem = int(out_rows % best_n);
  p.grp_q = best_q;
  return best;
}

// plan_group behind a one-entry memo per thread and instantiation:
// consecutive blocks of a tile plan the same launch, and the host path of a
// block is what bounds the smallest tiles (8192^2: ~11 us of host time per
// linked launch against ~13 us on the device, profiles/r05/host_probe.txt).
template <int T, int M>
double plan_group_memo(LifeBlockParams& p, int64_t out_rows, int simds, int occ, int target_waves, int xl) {
  struct Memo {
    int64_t rows = -1;
    int simds = 0, occ = 0, target = 0, xl = 0, fold = 0, ncolw = 0;
    double cost = -1.0;
    int nseg = 0, seg_rows = 0, seg_rem = 0, grp_q = 0;
  };
  thread_local Memo m;
  if (m.rows == out_rows && m.simds == simds && m.occ == occ && m.target == target_waves && m.xl == xl &&
      m.fold == p.fold && m.ncolw == p.ncolw) {
    if (m.cost > 0) {
      p.nseg = m.nseg;
      p.seg_rows = m.seg_rows;
      p.seg_rem = m.seg_rem;
      p.grp_q = m.grp_q;
    }
    return m.cost;
  }
  const double c = plan_group<T, M>(p, out_rows, simds, occ, target_waves, xl);
  m = Memo{out_rows, simds, occ, target_waves, xl, p.fold, p.ncolw, c, p.nseg, p.seg_rows, p.seg_rem, p.grp_q};
  return c;
}

// Plan of a chained launch (LifeBlockParams::chain_buf): n groups per strip,
// waves of q or q + 3 rows (q >= 2T, (q - 2T) % 3 == 0; the first x take
// q + 3) except the strip's last wave, which takes the remaining
// r = out_rows - (n M - 1) q - 3x >= 0 rows with the classic end (span
// r + T - 1).  No group boundary keeps a redundant triangle and no wave but
// one per strip carries one.  Same makespan model as plan_group.  Returns
// the cost, or -1 when no plan fits.
template <int T, int M>
double plan_chain(LifeBlockParams& p, int64_t out_rows, int simds, int occ, int target_waves, int xl) {
  constexpr double kOverhead = 0.4 * T;
  const int64_t max_n = out_rows / (int64_t(M) * 2 * T);
  int64_t best_n = 0, best_x = 0;
  int best_q = 0;
  double best = 1e300;
  for (int64_t n = 1; n <= max_n; ++n) {
    const int64_t nw = n * M;
    const int64_t ideal = std::max<int64_t>(2 * T, (out_rows + T - 1) / nw);
    int q = 0;
    int64_t qx = 0;
    double span = 1e300;
    for (int64_t c = ideal - 6; c <= ideal + 3; ++c) {
      if (c < 2 * T || (c - 2 * T) % 3 != 0) continue;
      const int64_t rest = out_rows - (nw - 1) * c;  // the +3s and the last wave
      if (rest < 0) continue;
      const int64_t want_r = std::max<int64_t>(0, c + 4 - T);  // last wave's span ~ c + 3
      const int64_t x = std::min<int64_t>(nw - 1, std::max<int64_t>(0, (rest - want_r) / 3));
      const int64_t r = rest - 3 * x;
      const double sp = std::max<double>(double(c + (x > 0 ? 3 : 0)), double(r + T - 1));
      if (sp < span) {
        span = sp;
        q = int(c);
        qx = x;
      }
    }
    if (q == 0) continue;
    const int64_t waves = int64_t(p.ncolw) * nw;
    const int64_t k = ceil_div(waves, int64_t(simds));
    const int64_t rounds = ceil_div(k, int64_t(occ));
    const int64_t kk = std::min<int64_t>(k, occ);
    double cost = double(rounds) * (span + kOverhead) * double(kk) * issue_factor(xl, kk);
    if (target_waves > 0)
      cost = 1.0 + double(std::llabs(waves - int64_t(target_waves)));
    else if (rounds > 4)
      break;
    if (cost < best * 0.999) {
      best = cost;
      best_n = n;
      best_q = q;
      best_x = qx;
    }
  }
  if (best_n == 0) return -1.0;
  p.nseg = int(best_n);
  p.grp_q = best_q;
  p.seg_rows = 0;
  p.seg_rem = int(best_x);  // waves with q + 3 rows
  p.chain_end = p.row_lo + out_rows;
  return best;
}

template <class K>
int occupancy_blocks(K kernel, int threads) {
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kernel, threads, 0) != hipSuccess || blocks <= 0)
    blocks = 1;
  return blocks;
}

// Resident waves per SIMD of the grouped kernel (a workgroup of M waves
// spreads over the CU's 4 SIMDs).
template <int T, class IO, int M>
int group_waves_per_simd() {
  static const int cached = std::max(1, occupancy_blocks(life_group_kernel<T, IO, M>, 64 * M) * M / 4);
  return cached;
}

template <int T, class IO, int M>
void launch_group(const LifeBlockParams& p, hipStream_t s) {
  const int64_t blocks = p.fold > 1 ? int64_t(p.ncolw - 1) * p.nseg + ceil_div(int64_t(p.nseg), int64_t(p.fold))
                                    : int64_t(p.ncolw) * p.nseg;
  hipLaunchKernelGGL((life_group_kernel<T, IO, M>), dim3(unsigned(blocks)), dim3(64 * M), 0, s, p);
}

}  // namespace lb
}  // namespace hipk
}  // namespace gol
