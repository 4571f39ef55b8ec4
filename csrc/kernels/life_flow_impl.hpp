// Persistent dataflow launch: a run of temporal blocks in ONE kernel.
//
// Every other schedule here launches one kernel per temporal block of T
// generations.  Each launch ramps up, runs, and drains: its last waves run
// alone while the next launch cannot start (the stream orders them), so a
// small tile spends a large share of every launch below full occupancy
// (8-GPU rank tile 32768 x 4096: 1.39 measured of 1.99 possible waves per
// SIMD, profiles/r04/occupancy.md).  Linked launches (life_group_impl.hpp
// link_wait) overlap two launches; this kernel removes the launch boundary:
//
//   * Work items are the grouped schedule's workgroups: (block j, column
//     strip, group of M wave segments).  A fixed grid of persistent
//     workgroups (the device's occupancy) takes tickets from one atomic
//     counter, in item order: block-major, then row position, every strip of
//     a position before the next (FlowOrder).  On a row ring (whole torus,
//     every block over the owned rows) block j starts at row position j, so
//     the items an item waits on sit about one block back in ticket order.
//   * Item (j, strip, g) reads block j-1's rows [G0 - T, G1 + T) in its own
//     strip and the strip on each side (the horizontal light cone), and
//     overwrites rows [G0, G1) that exactly those items of block j-1 read.
//     So it waits for their completion words - RAW and WAR in one wait -
//     and publishes its own when its rows are written.  Rows wrap around the
//     torus on a ring; the groups of block j-1 come from its own partition
//     (trapezoid blocks shrink by T rows per side).
//   * Deadlock-free by ticket order alone: an item waits only on items with
//     smaller tickets, which were taken by running workgroups.  No co-
//     residency or launch-size assumption (unlike linked launches), so other
//     kernels on the GPU (RCCL, other ranks' processes) only slow it down.
//   * Hand-off (cdna_hip_programming.md §6 Guideline 16, R1, the "every load
//     sc1" valid form): row stores are written through (sc1), every wave
//     drains its stores, the workgroup meets at a barrier and one lane
//     stores the completion word with an agent-scope atomic; the waiting wave
//     polls relaxed at agent scope, the workgroup meets at a barrier, and
//     every row load of the item is an sc1 load to registers (Sc1IO).
//   * Tickets and completion words are monotonic across launches (a launch
//     takes exactly items + grid tickets; block j publishes seq0 + j and a
//     wait compares with a signed difference), so nothing is cleared between
//     launches.  Waits are bounded; giving up raises the error word 6.
//
// Reference counterpart: the per-generation launch sequence of
// src/game_cuda.cu:213-276 (five kernels and four device syncs per
// generation) and the per-rank evolve loop of src/game_mpi.c:385-422.
#pragma once

#include "life_group_impl.hpp"

namespace gol {
namespace hipk {
namespace lb {

// Block j's plan: buffers, first output row and balanced group sizes (the
// group count and every other field are the launch's).
__device__ __forceinline__ void flow_block(const FlowParams& f, int j, LifeBlockParams& p) {
  // Selects, not an index: a runtime index into the argument's array would
  // copy it to scratch.
  p.in = (j & 1) ? f.buf[1] : f.buf[0];
  p.out = (j & 1) ? f.buf[0] : f.buf[1];
  const int rows = int(f.rows0) - 2 * j * f.shrink;  // 32-bit: tiles hold < 2^31 rows (launch_life_flow)
  p.row_lo = f.p.row_lo + int64_t(j) * f.shrink;
  p.seg_rows = rows / f.p.nseg;
  p.seg_rem = rows - p.seg_rows * f.p.nseg;
}

// Output rows [G0, G1) of group g of a block plan (balanced: the first
// seg_rem groups have one row more).
__device__ __forceinline__ int64_t flow_group_end(const LifeBlockParams& p, int g) {
  return p.row_lo + int64_t(g) * p.seg_rows + min(g, p.seg_rem) + p.seg_rows + (g < p.seg_rem ? 1 : 0);
}

// One item: the grouped kernel's workgroup body (life_group_kernel without
// chained groups, dual ranges or linking), on the block plan p.  nsub > 1:
// the folded last strip, groups grp .. grp + nsub - 1 side by side in lane
// sub-strips.  Returns the wave's changed-level mask (bit L: generation L+1
// of the block changed an owned cell of its rows).
template <int T, class IO, int M>
__device__ __forceinline__ uint32_t flow_item(const LifeBlockParams& p, int kcol, int grp, int nsub, int sub_lanes,
                                              uint32_t* saved, int lane, int m) {
  constexpr int W = IO::W;
  constexpr int kSlot = (T - 1) * 2 * W * 64;
  const int64_t G1 = flow_group_end(p, grp);
  const int64_t G0 = G1 - p.seg_rows - (nsub > 1 ? (p.seg_rem > 0 ? 1 : 0) : (grp < p.seg_rem ? 1 : 0));
  const int64_t in0 = G0 + int64_t(m) * p.grp_q - T;
  const bool last = m == M - 1;
  constexpr int kPro = 2 * T;
  const int kend = int(G1 + T - in0);
  const int kmain = last ? kend - (kend - kPro) % 3 : p.grp_q;
  const int nfull = last ? (kend - kPro) % 3 : 2 * T;

  const LaneCols<IO> lc = lane_cols<IO>(p, kcol, lane, sub_lanes, nsub);
  const int64_t pitch = p.pitch;
  int64_t dl = 0;  // rows between this lane's group and the wave's (folded strip)
  Writer<IO> wr;
  if (nsub > 1) {
    dl = flow_group_end(p, min(grp + min(lc.sub, nsub - 1), p.nseg - 1)) - G1;
    wr.roff = int(dl * pitch);
    wr.nrec = int((flow_group_end(p, min(grp + nsub - 1, p.nseg - 1)) - G1 + 1) * pitch);
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
      st.pipe[L].w[i] = st.acc[L].w[i] = 0u;
    }
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

  prologue_tri<T, IO, 0>(st, rd, LdsSaver<T, W>{saved + m * kSlot, lane}, NoBottom{});
  __syncthreads();  // every wave's boundary rows are in LDS

  int k = kPro;
  constexpr int S0 = kPro % 3, S1 = (S0 + 1) % 3, S2 = (S0 + 2) % 3;
  Prio prio((kmain - kPro) * T + epi_work<T>(nfull), false);
  for (; k + 3 <= kmain; k += 3) {
    prio.at((k - kPro) * T);
    wr.row(k - T, levels_full<T, IO, S0, 0, T>(st, rd.template take<S0>(k)));
    wr.row(k + 1 - T, levels_full<T, IO, S1, 0, T>(st, rd.template take<S1>(k + 1)));
    wr.row(k + 2 - T, levels_full<T, IO, S2, 0, T>(st, rd.template take<S2>(k + 2)));
  }
  prio.done0 = (kmain - kPro) * T;
  epilogue_tri<T, IO, 0, S0>(st, rd, saved + (m + 1) * kSlot, lane, wr, k, nfull, prio);  // k == kmain
  prio.reset();

  uint32_t mask = 0;
#pragma unroll
  for (int L = 0; L < T; ++L) {
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) any |= st.acc[L].w[i] & fmask[i];
    mask |= (__ballot(any != 0u) != 0ull ? 1u : 0u) << L;
  }
  return mask;
}

// Rows [r0, r1) of block j - 1's output: wait (one wave, one word per lane)
// until every item of block j - 1 that wrote them or read them - its groups
// over those rows, in `strip` and the strips beside it - has published.
// Returns false when the bounded wait gave up (the error word is then set).
__device__ __forceinline__ bool flow_wait(const FlowParams& f, const FlowOrder& ord, int j, int strip, int64_t r0,
                                          int64_t r1, int lane) {
  if (j == 0) return true;
  LifeBlockParams q = f.p;
  flow_block(f, j - 1, q);
  const int rows = int(f.rows0) - 2 * (j - 1) * f.shrink;
  const int q1 = q.seg_rows + 1;
  const int big = q.seg_rem * q1;
  const int nseg = q.nseg;
  // Group of row r (r within T rows of the block's range), unwrapped on a
  // ring: group index + nseg per turn around the torus.
  const auto gu = [&](int64_t r) -> int {
    int x = int(r - q.row_lo);
    int turns = 0;
    if (f.ring_rows > 0) {
      if (x < 0) {
        x += rows;
        turns = -1;
      } else if (x >= rows) {
        x -= rows;
        turns = 1;
      }
    } else {
      x = min(max(x, 0), rows - 1);
    }
    const int g = x < big ? x / q1 : q.seg_rem + (x - big) / max(1, q.seg_rows);
    return turns * nseg + min(g, nseg - 1);
  };
  const int ga = gu(r0);
  const int ng = min(gu(r1 - 1) - ga + 1, nseg);
  const int nstrip = q.ncolw;
  const int nflags = 3 * ng;
  const uint32_t want = f.seq0 + uint32_t(j - 1);
  bool ok = true;
  for (int b = 0; b < nflags; b += 64) {
    const int x = b + lane;
    int ks = strip + x / ng - 1;
    if (q.wrap_w > 0) ks = (ks + nstrip) % nstrip;
    const bool mine = x < nflags && ks >= 0 && ks < nstrip;
    int g = (ga + x % ng) % nseg;
    if (g < 0) g += nseg;
    const int slot = mine ? ord.slot(ks, g) : 0;
    bool done = !mine;
    const int spins = 1 << f.spin_log2;
    for (int spin = 0; spin < spins; ++spin) {
      if (!done)
        done = int(__hip_atomic_load(f.done + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) >= 0;
      if (__all(done)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (!__all(done)) ok = false;
  }
  // No row load may move above the wait (every one of them is an sc1 load).
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok;
}

// Register cap: four waves per SIMD (<= 128 VGPRs) for the adder window up
// to T = 12, where it reaches its issue rate (issue_factor), and for T <= 8;
// the grouped kernel's floor otherwise (the DPP window issues at its rate
// from two waves per SIMD).
template <int T, class IO>
constexpr int flow_min_waves() {
  return (T <= 8 || (T <= 12 && IO::XL == kXlaneAdd)) ? 4 : group_min_waves<T, IO>();
}

template <int T, class IO, int M>
__global__ __launch_bounds__(64 * M) __attribute__((amdgpu_waves_per_eu(flow_min_waves<T, IO>())))
void life_flow_kernel(const FlowParams f) {
  constexpr int kSlot = (T - 1) * 2 * IO::W * 64;
  __shared__ uint32_t saved[M * kSlot];
  __shared__ uint32_t item_sh;
  const int lane = threadIdx.x & 63;
  const int m = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const FlowOrder ord{f.p.nseg, f.nn, f.p.fold};
  const uint32_t total = uint32_t(f.nblk) * uint32_t(f.items);
  // Wave 0 takes the tickets, one ahead: the next ticket's atomic round trip
  // overlaps the current item.
  uint32_t next = 0;
  if (m == 0) next = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(f.counter, 1u) : 0u);
  bool waits = true;  // false once a wait of this workgroup gave up (no second bounded wait)
  uint64_t t_deq = 0, t_ready = 0;  // GOL_FLOW_TRACE
  for (;;) {
    if (m == 0) {
      if (f.trace) t_deq = __builtin_amdgcn_s_memrealtime();
      const uint32_t i = next - f.base;
      if (i < total) {
        next = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(f.counter, 1u) : 0u);
        const int j = int(i / uint32_t(f.items));
        int s = int(i - uint32_t(j) * uint32_t(f.items));
        if (f.rotate) s = (s + ord.start(j % ord.nseg)) % f.items;
        int r = 0;
        const int pos = ord.pos_of(s, &r);
        LifeBlockParams q = f.p;
        flow_block(f, j, q);
        const bool fold_item = r >= ord.nn;
        const int g0 = fold_item ? (pos / ord.fold) * ord.fold : pos;
        const int g1 = fold_item ? min(g0 + ord.fold, ord.nseg) - 1 : pos;
        // Rows the item writes: its groups (a folded sub-strip of a smaller
        // group starts one row early); it reads T more on each side.
        const int64_t e1 = flow_group_end(q, g1);
        const int64_t b0 = flow_group_end(q, g0) - q.seg_rows - (fold_item ? (q.seg_rem > 0 ? 1 : 0) : (g0 < q.seg_rem ? 1 : 0));
        if (waits && !flow_wait(f, ord, j, fold_item ? ord.nn : r, b0 - T, e1 + T, lane)) {
          waits = false;
          if (f.p.err && lane == 0) __hip_atomic_store(f.p.err, 6u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      if (lane == 0) item_sh = i;
      if (f.trace) t_ready = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const uint32_t i = __builtin_amdgcn_readfirstlane(item_sh);
    if (i >= total) break;  // workgroup-uniform
    const int j = int(i / uint32_t(f.items));
    int s = int(i - uint32_t(j) * uint32_t(f.items));
    if (f.rotate) s = (s + ord.start(j % ord.nseg)) % f.items;
    int r = 0;
    const int pos = ord.pos_of(s, &r);
    LifeBlockParams p = f.p;
    flow_block(f, j, p);
    p.changed = f.changed0 ? f.changed0 + int64_t(j) * T : nullptr;
    const bool fold_item = r >= ord.nn;
    const int kcol = fold_item ? ord.nn : r;
    const int grp = fold_item ? (pos / ord.fold) * ord.fold : pos;
    // One inlined body for both kinds of item (a second copy for the folded
    // strip doubled the kernel's code).
    const uint32_t mask = flow_item<T, IO, M>(p, kcol, grp, fold_item ? p.fold : 1, fold_item ? p.fold_lanes : 64,
                                              saved, lane, m);
    if (p.changed && lane < T && ((mask >> lane) & 1u)) p.changed[lane] = 1u;
    // Every wave's rows are written through, then one completion word.
    __builtin_amdgcn_s_waitcnt(0);
    if (f.p.fault_delay && (pos == 0 || pos == ord.nseg - 1 || fold_item))  // tests: late producers at the seam
      for (int d = 0; d < f.p.fault_delay; ++d) __builtin_amdgcn_s_sleep(127);
    __syncthreads();
    if (m == 0 && lane == 0) {
      __hip_atomic_store(f.done + s, f.seq0 + uint32_t(j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (f.trace) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
        uint64_t* r = f.trace + 4 * int64_t(i);
        r[0] = uint64_t(blockIdx.x) | (uint64_t(xcc & 0xFF) << 32) | (uint64_t(hw) << 40);
        r[1] = t_deq;
        r[2] = t_ready;
        r[3] = __builtin_amdgcn_s_memrealtime();
      }
    }
  }
}

// issue_factor between whole resident-wave counts.
inline double issue_factor_at(int xl, double k) {
  const int lo = std::max(1, std::min(4, int(k)));
  const int hi = std::min(4, lo + 1);
  const double t = std::min(1.0, std::max(0.0, k - lo));
  return issue_factor(xl, lo) * (1 - t) + issue_factor(xl, hi) * t;
}

// Plan of a flow launch: groups per strip (f.p.nseg) and the per-wave rows q
// (f.p.grp_q) for the smallest block (rows_min rows; larger trapezoid blocks
// give their extra rows to each group's last wave).  Score: the dataflow
// makespan of one block, (items x M waves x (span + overhead) level rows)
// spread over the SIMDs at the issue rate of the resident waves per SIMD the
// launch can keep busy - at most the device's occupancy, and at most about
// one block of items (an item waits for the block before it).  Returns the
// score, or -1 when no plan fits.
template <int T, int M>
double plan_flow(FlowParams& f, int64_t rows_min, int simds, int occ_waves, int nseg_req, int xl) {
  LifeBlockParams& p = f.p;
  const int64_t max_n = rows_min / (int64_t(M - 1) * 2 * T + 1);
  const int strips_eff = p.fold > 1 ? p.ncolw - 1 : p.ncolw;
  double best = 1e300;
  int64_t best_n = 0;
  int best_q = 0;
  for (int64_t n = 1; n <= max_n; ++n) {
    if (nseg_req > 0 && n != nseg_req) continue;
    const int64_t lo = rows_min / n, hi = lo + (rows_min % n ? 1 : 0);
    const int64_t ideal = std::max<int64_t>(2 * T, (hi + T - 1) / M);
    int q = 0;
    double span = 1e300;
    for (int64_t c = ideal - 3; c <= ideal + 3; ++c) {
      if (c < 2 * T || (c - 2 * T) % 3 != 0 || lo - int64_t(M - 1) * c < 0) continue;
      const double sp = std::max<double>(double(c), double(hi - int64_t(M - 1) * c) + (T - 1));
      if (sp < span) {
        span = sp;
        q = int(c);
      }
    }
    if (q == 0) continue;
    const FlowOrder ord{int(n), strips_eff, p.fold};
    const int64_t items = ord.items();
    // Items that can run at once: an item waits for the item of the block
    // before it up to three row positions ahead in ticket order (its own
    // position + 1, the folded strip's item up to fold - 1 more), so about one
    // block less those, with a margin for uneven item times.
    const double inflight = std::max<double>(1.0, double(items) - (2.0 + p.fold) * strips_eff);
    const double k = std::min<double>(double(occ_waves), inflight * M / (1.25 * simds));
    const double ovh = 0.4 * T + 4.0;  // triangles at lower ILP; ticket, wait and barriers per item
    const double cost = double(items) * M * (span + ovh) * issue_factor_at(xl, k) / (simds * std::min(1.0, k));
    if (cost < best * 0.999) {
      best = cost;
      best_n = n;
      best_q = q;
    }
  }
  if (best_n == 0) return -1.0;
  p.nseg = int(best_n);
  p.grp_q = best_q;
  return best;
}

// Host side of one compiled (T, window, M): plan (go = false: score only,
// *cost), or plan and launch (*tickets: counter tickets the launch takes,
// *desc).
template <int T, class IO, int M>
bool launch_flow_TM(FlowParams f, int64_t rows_min, const LifeTuning& tune, hipStream_t s, bool go, double* cost,
                    std::string* desc, int64_t* tickets, int* items) {
  using LIO = Sc1IO<IO>;
  const auto kern = life_flow_kernel<T, LIO, M>;
  static const int per_cu = occupancy_blocks(kern, 64 * M);
  const int simds = 4 * std::max(1, tune.cus);
  const double c = plan_flow<T, M>(f, rows_min, simds, std::max(1, per_cu * M / 4), tune.flow_nseg, IO::XL);
  if (c < 0) return false;
  *cost = c;
  if (!go) return true;
  const FlowOrder ord{f.p.nseg, f.p.fold > 1 ? f.p.ncolw - 1 : f.p.ncolw, f.p.fold};
  f.items = ord.items();
  f.nn = ord.nn;
  f.rotate = f.ring_rows > 0 && f.p.nseg > 1;
  // Block 0's balanced groups (the kernel recomputes every block's).
  f.p.seg_rows = int(f.rows0 / f.p.nseg);
  f.p.seg_rem = int(f.rows0 % f.p.nseg);
  const int64_t total = int64_t(f.nblk) * f.items;
  const int64_t g = std::min<int64_t>(total, int64_t(per_cu) * std::max(1, tune.cus));
  GOL_REQUIRE(total + g < (int64_t(1) << 30), "life_flow: too many items in one launch");
  hipLaunchKernelGGL(kern, dim3(unsigned(g)), dim3(64 * M), 0, s, f);
  *tickets = total + g;  // every item, plus the ticket past the last that ends each workgroup
  *items = f.items;
  if (desc)
    *desc = "flow T=" + std::to_string(T) + " M=" + std::to_string(M) + " groups/strip=" + std::to_string(f.p.nseg) +
            " q=" + std::to_string(f.p.grp_q) + " items/block=" + std::to_string(f.items) +
            " blocks=" + std::to_string(f.nblk) + " grid=" + std::to_string(g) + " (" + std::to_string(per_cu) +
            "/CU)";
  return true;
}

// One window's flow kernels at T: M = 4 and 8 waves per item scored by the
// planner (tune.flow_m forces one), the cheaper one launched.
template <int T, class IO>
bool launch_flow_T(const FlowParams& f, int64_t rows_min, const LifeTuning& tune, hipStream_t s, std::string* desc,
                   int64_t* tickets, int* items) {
  double c4 = -1, c8 = -1;
  const bool ok4 = tune.flow_m != 8 && launch_flow_TM<T, IO, 4>(f, rows_min, tune, s, false, &c4, desc, tickets, items);
  const bool ok8 = tune.flow_m != 4 && launch_flow_TM<T, IO, 8>(f, rows_min, tune, s, false, &c8, desc, tickets, items);
  if (!ok4 && !ok8) return false;
  double c = 0;
  if (ok4 && (!ok8 || c4 < c8)) return launch_flow_TM<T, IO, 4>(f, rows_min, tune, s, true, &c, desc, tickets, items);
  return launch_flow_TM<T, IO, 8>(f, rows_min, tune, s, true, &c, desc, tickets, items);
}

}  // namespace lb
}  // namespace hipk
}  // namespace gol
