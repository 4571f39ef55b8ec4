// Level-pipelined grouped schedule: the grouped kernel of
// life_group_impl.hpp with every wave's T levels split over two waves.
//
// A CDNA4 SIMD issues a wave's VALU instructions no faster than about one per
// 5 cycles, while the SIMD as a whole takes one per ~2.45 cycles from 4
// waves (ubench_body.hip, git e36884f: a level body costs 96 / 51 / 49 / 42
// cycles per SIMD at 1 / 2 / 3 / 4 resident waves).  The grouped kernel's
// wave count is fixed by q >= 2T rows per wave, so the 8-GPU per-rank tile
// (32768 x 4096) runs at 2-3 waves per SIMD.  Here wave pair m of a workgroup
// owns the segment wave m of the grouped kernel owns, and
//   * stage A (levels 0..T1-1) reads the input rows from global memory and
//     hands its level-T1 rows to stage B through an LDS ring of kPipeRing
//     rows (a produced / consumed counter per pair, workgroup-scope release
//     and acquire);
//   * stage B (levels T1..T1+T2-1) is a grouped wave of T2 levels whose input
//     stream is that ring, starting at row in0 + T1, and writes the output.
// Both stages keep the grouped kernel's boundary sharing: each saves its
// top-boundary level rows in LDS before the workgroup barrier, stage A also
// its first two level-T1 rows (the lower boundary rows stage B of the pair
// above needs, as local level 0).  Every level row of the group is computed
// exactly once, as in the grouped kernel, so the change flags are the same.
// A pair is two waves with half the registers each: twice the waves per
// SIMD for the same rows, at the cost of one LDS row write + read per row.
//
// Alignment: the 3-step main loops need (q - kPro) % 3 == 0 for both stages;
// stage B's prologue is 2 T2 steps, stage A runs 2 T + T1 % 3 steps before
// the barrier (its prologue, the rows stage B's prologue consumes, and up to
// two more), so q = 2 T2 (mod 3) serves both.
//
// Measured on the 8-GPU tile (32768 x 4096, per 1000 generations;
// profiles/r02/pipe/): 8 + 8 adder levels 2.51 ms against 3.07 for the
// T = 16 adder grouped kernel (register-bound at 2 waves/SIMD) and 2.35 for
// the default DPP T = 16 grouped kernel; 6 + 6 2.69 ms.  A timing probe with
// the ring waits removed (wrong results) ran 2.26 ms: the hand-off and the
// pipeline fill / drain cost about 10%, and a pair's extra per-row work the
// rest of what the doubled occupancy gains.  On 32768^2 the pairs are slower
// than the grouped kernel (13.6 vs 11.6 ms).  Opt-in: GOL_PIPE=1 model,
// 2 forced.
//
// The reference has no counterpart (src/game_cuda.cu:128-148 is one
// generation per launch).
#pragma once

#include "life_group_impl.hpp"

namespace gol {
namespace hipk {
namespace lb {

#ifndef GOL_PIPE_BATCH
#define GOL_PIPE_BATCH 3  // ring rows per counter update (1 measured the same)
#endif
constexpr int kPipeRing = 12;  // level-T1 rows in flight per pair
constexpr int kPipeSpin = 1 << 22;  // bounded wait (~0.1 s), then LifeBlockParams::err

// Bounded wait until *ctr satisfies ok(value); returns the last value read.
// Giving up raises the launch's error word (Backend::check_device_errors):
// a wrong result is reported instead of a hung GPU.
template <class Ok>
__device__ __forceinline__ int pipe_wait(const uint32_t* ctr, int seen, const Ok& ok, uint32_t* err, bool& dead) {
  for (int spin = 0; !ok(seen); ++spin) {
    if (spin == kPipeSpin) {
      if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      dead = true;
      break;
    }
    if (spin) __builtin_amdgcn_s_sleep(1);
    seen = __builtin_amdgcn_readfirstlane(
        int(__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)));
  }
  return seen;
}

// One pair's ring: rows[slot][word][lane], prod / cons counters.
template <int W>
struct PipeRing {
  uint32_t* rows;
  uint32_t* prod;
  uint32_t* cons;
  uint32_t* err;
  int lane;
  int seen = 0;       // last counter value read by this wave
  bool dead = false;  // a wait gave up: stop waiting (the error word is raised)

  // Stage A: ring row j (level-T1 row in0 + T1 + j).
  __device__ __forceinline__ void put(int j, const Vec<W>& v) {
    if (!dead) seen = pipe_wait(cons, seen, [j](int c) { return j - c < kPipeRing; }, err, dead);
    uint32_t* r = rows + (j % kPipeRing) * W * 64;
#pragma unroll
    for (int i = 0; i < W; ++i) r[i * 64 + lane] = v.w[i];
    if (j % GOL_PIPE_BATCH == GOL_PIPE_BATCH - 1) publish(prod, j + 1);
  }
  // Counter update (every GOL_PIPE_BATCH rows, and at the ends of the
  // pre-barrier phase and of the sweep: flush()).
  __device__ __forceinline__ void publish(uint32_t* ctr, int v) const {
    if (lane == 0) __hip_atomic_store(ctr, uint32_t(v), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ __forceinline__ void flush_prod(int n) const { publish(prod, n); }
  __device__ __forceinline__ void flush_cons(int n) const { publish(cons, n); }
  // Stage B: ring row j (RowReader interface: the window slot is implied).
  template <int S>
  __device__ __forceinline__ Vec<W> take(int j) {
    if (!dead) seen = pipe_wait(prod, seen, [j](int c) { return c > j; }, err, dead);
    const uint32_t* r = rows + (j % kPipeRing) * W * 64;
    Vec<W> v;
#pragma unroll
    for (int i = 0; i < W; ++i) v.w[i] = r[i * 64 + lane];
    if (j % GOL_PIPE_BATCH == GOL_PIPE_BATCH - 1) publish(cons, j + 1);
    return v;
  }
};

template <int W>
__device__ __forceinline__ Vec<W> lds_row(const uint32_t* slot, int idx, int lane) {
  Vec<W> v;
#pragma unroll
  for (int i = 0; i < W; ++i) v.w[i] = slot[(idx * W + i) * 64 + lane];
  return v;
}

// Stage A steps K..KEND-1 after its prologue (all T1 levels valid): ring row
// K - 2 T1; the first two are also the level-T1 boundary rows of this pair.
template <int T1, class IO, int K, int KEND, class RD>
__device__ __forceinline__ void pipe_a_straight(Levels<T1, IO::W>& st, RD& rd, PipeRing<IO::W>& ring,
                                                const LdsSaver<T1, IO::W>& save) {
  if constexpr (K < KEND) {
    constexpr int S = K % 3;
    const Vec<IO::W> out = levels_full<T1, IO, S, 0, T1>(st, rd.template take<S>(K));
    if constexpr (K - 2 * T1 < 2) save(T1, K - 2 * T1, out);
    ring.put(K - 2 * T1, out);
    pipe_a_straight<T1, IO, K + 1, KEND>(st, rd, ring, save);
  }
}

// Stage A epilogue (grouped kernel's epilogue_tri with a ring sink): step E
// feeds level E/2 the input row (E < 2) or the lower pair's saved row.
template <int T1, class IO, int E, int S, class RD>
__device__ __forceinline__ void pipe_a_epilogue(Levels<T1, IO::W>& st, RD& rd, const uint32_t* below, int lane,
                                                PipeRing<IO::W>& ring, int k, int nfull) {
  if constexpr (E < 2 * T1) {
    if (E >= nfull) return;  // wave-uniform
    constexpr int L0 = E / 2;
    Vec<IO::W> cur;
    if constexpr (L0 == 0)
      cur = rd.template take<S>(k);
    else
      cur = lds_row<IO::W>(below, (L0 - 1) * 2 + (E & 1), lane);
    ring.put(k - 2 * T1, levels_full<T1, IO, S, L0, T1>(st, cur));
    __builtin_amdgcn_sched_barrier(0);
    pipe_a_epilogue<T1, IO, E + 1, (S + 1) % 3>(st, rd, below, lane, ring, k + 1, nfull);
  }
}

// Stage B epilogue: local level 0 comes from the ring (last pair's plain
// steps) or the lower pair's stage-A level-T1 rows, higher levels from the
// lower pair's stage-B rows.
template <int T1, int T2, class IO, int E, int S>
__device__ __forceinline__ void pipe_b_epilogue(Levels<T2, IO::W>& st, PipeRing<IO::W>& ring,
                                                const uint32_t* below_a, const uint32_t* below_b, int lane,
                                                const Writer<IO>& wr, int j, int nfull, bool last) {
  if constexpr (E < 2 * T2) {
    if (E >= nfull) return;  // wave-uniform
    constexpr int L0 = E / 2;
    Vec<IO::W> cur;
    if constexpr (L0 == 0) {
      if (last)
        cur = ring.template take<S>(j);
      else
        cur = lds_row<IO::W>(below_a, (T1 - 1) * 2 + (E & 1), lane);
    } else {
      cur = lds_row<IO::W>(below_b, (L0 - 1) * 2 + (E & 1), lane);
    }
    wr.row(j - T2, levels_full<T2, IO, S, L0, T2>(st, cur));
    __builtin_amdgcn_sched_barrier(0);
    pipe_b_epilogue<T1, T2, IO, E + 1, (S + 1) % 3>(st, ring, below_a, below_b, lane, wr, j + 1, nfull, last);
  }
}

template <int T, int W>
__device__ __forceinline__ void zero_levels(Levels<T, W>& st) {
#pragma unroll
  for (int L = 0; L < T; ++L)
#pragma unroll
    for (int i = 0; i < W; ++i) {
#pragma unroll
      for (int s = 0; s < 3; ++s) st.h0[L][s].w[i] = st.h1[L][s].w[i] = st.cc[L][s].w[i] = 0u;
      st.acc[L].w[i] = 0u;
    }
}

// Change flags of levels [0, T) of this stage -> generations gbase + 1 + L.
template <int T, int W>
__device__ __forceinline__ void pipe_flags(const LifeBlockParams& p, const Levels<T, W>& st, const uint32_t (&fmask)[W],
                                           int lane, int gbase) {
  if (!p.changed) return;
  uint32_t mask = 0;
#pragma unroll
  for (int L = 0; L < T; ++L) {
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) any |= st.acc[L].w[i] & fmask[i];
    mask |= (__ballot(any != 0u) != 0ull ? 1u : 0u) << L;
  }
  uint32_t* ch = (p.gen_dev ? p.changed + (*p.gen_dev + p.gen_rel) : p.changed) + gbase;
  if (lane < T && ((mask >> lane) & 1u)) ch[lane] = 1u;
}

template <int T1, int T2, int M>
struct PipeGeom {
  static constexpr int T = T1 + T2;
  static constexpr int kProA = 2 * T + T1 % 3;  // stage A steps before the barrier
  static constexpr int kProB = 2 * T2;
};

template <int T1, int T2, class IO, int M>
__global__ __launch_bounds__(128 * M) void life_pipe_kernel(const LifeBlockParams p) {
  static_assert(T1 >= 2 && T2 >= 2, "both stages need a prologue triangle");
  constexpr int W = IO::W;
  constexpr int T = T1 + T2;
  constexpr int kProA = PipeGeom<T1, T2, M>::kProA, kProB = PipeGeom<T1, T2, M>::kProB;
  constexpr int kSlotA = T1 * 2 * W * 64;        // levels 1..T1, rows b + L, b + L + 1
  constexpr int kSlotB = (T2 - 1) * 2 * W * 64;  // local levels 1..T2-1
  constexpr int kRing = kPipeRing * W * 64;
  __shared__ uint32_t lds[M * (kSlotA + kSlotB + kRing) + 2 * M];
  uint32_t* const slot_a = lds;
  uint32_t* const slot_b = slot_a + M * kSlotA;
  uint32_t* const rings = slot_b + M * kSlotB;
  uint32_t* const ctrs = rings + M * kRing;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Stage A = waves 0..M-1, B = waves M..2M-1: waves go to the CU's SIMDs
  // round-robin, so every SIMD runs both stages and an idle stage's issue
  // slots go to the other.  Pairs of adjacent waves put all A waves on SIMDs
  // 0/2 and all B waves on 1/3: 14% slower on the tile.
  const int m = w % M;
  const bool stage_b = w >= M;
  if (threadIdx.x < 2 * M) ctrs[threadIdx.x] = 0u;
  __syncthreads();

  const int blk = blockIdx.x;
  const int kcol = blk / p.nseg;
  const int grp = blk - kcol * p.nseg;
  const int64_t G0 = p.row_lo + int64_t(grp) * p.seg_rows + min(grp, p.seg_rem);
  const int64_t G1 = G0 + p.seg_rows + (grp < p.seg_rem ? 1 : 0);
  const int64_t in0 = G0 + int64_t(m) * p.grp_q - T;
  const bool last = m == M - 1;
  const int kendA = int(G1 + T - in0);

  const LaneCols<IO> lc = lane_cols<IO>(p, kcol, lane);
  const int col = lc.store_col;
  const int64_t pitch = p.pitch;
  uint32_t fmask[W];
  Writer<IO> wr;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    wr.own[i] = lc.own[i];
    fmask[i] = lc.fmask[i];
  }
  PipeRing<W> ring{rings + m * kRing, ctrs + 2 * m, ctrs + 2 * m + 1, p.err, lane};

  if (!stage_b) {
    const int kmain = last ? kendA - (kendA - kProA) % 3 : p.grp_q;
    const int nfull = last ? (kendA - kProA) % 3 : 2 * T1;
    RowReader<IO> rd;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      rd.ok[i] = lc.ok[i];
      rd.off[i] = lc.off[i];
    }
    rd.base = p.in + in0 * pitch;  // input row of step k: in0 + k
    rd.pitch = pitch;
    rd.kmax = last ? kendA - 1 : kmain + 1;
    rd.init();
    Levels<T1, W> st;
    zero_levels(st);
    const LdsSaver<T1, W> saver{slot_a + m * kSlotA, lane};
    prologue_tri<T1, IO, 0>(st, rd, saver, NoBottom{});
    pipe_a_straight<T1, IO, 2 * T1, kProA>(st, rd, ring, saver);
    ring.flush_prod(kProA - 2 * T1);  // everything stage B's prologue reads
    __syncthreads();  // boundary rows of both stages are in LDS
    constexpr int S0 = kProA % 3, S1 = (S0 + 1) % 3, S2 = (S0 + 2) % 3;
    int k = kProA;
    for (; k + 3 <= kmain; k += 3) {
      ring.put(k - 2 * T1, levels_full<T1, IO, S0, 0, T1>(st, rd.template take<S0>(k)));
      ring.put(k + 1 - 2 * T1, levels_full<T1, IO, S1, 0, T1>(st, rd.template take<S1>(k + 1)));
      ring.put(k + 2 - 2 * T1, levels_full<T1, IO, S2, 0, T1>(st, rd.template take<S2>(k + 2)));
    }
    pipe_a_epilogue<T1, IO, 0, S0>(st, rd, slot_a + (m + 1) * kSlotA, lane, ring, k, nfull);
    ring.flush_prod(k + nfull - 2 * T1);
    pipe_flags(p, st, fmask, lane, 0);
  } else {
    const int kendB = kendA - 2 * T1;
    const int kmain = last ? kendB - (kendB - kProB) % 3 : p.grp_q;
    const int nfull = last ? (kendB - kProB) % 3 : 2 * T2;
    const int64_t in0b = in0 + T1;  // level-T1 row of ring row j: in0b + j
    wr.out = p.out + in0b * pitch;  // level-T row of step j: in0b + j - T2
    wr.pitch = pitch;
    wr.col = col;
    Levels<T2, W> st;
    zero_levels(st);
    const LdsSaver<T2, W> saver{slot_b + m * kSlotB, lane};
    prologue_tri<T2, IO, 0>(st, ring, saver, NoBottom{});
    ring.flush_cons(kProB);
    __syncthreads();
    constexpr int S0 = kProB % 3, S1 = (S0 + 1) % 3, S2 = (S0 + 2) % 3;
    int j = kProB;
    for (; j + 3 <= kmain; j += 3) {
      wr.row(j - T2, levels_full<T2, IO, S0, 0, T2>(st, ring.template take<S0>(j)));
      wr.row(j + 1 - T2, levels_full<T2, IO, S1, 0, T2>(st, ring.template take<S1>(j + 1)));
      wr.row(j + 2 - T2, levels_full<T2, IO, S2, 0, T2>(st, ring.template take<S2>(j + 2)));
    }
    pipe_b_epilogue<T1, T2, IO, 0, S0>(st, ring, slot_a + (m + 1) * kSlotA, slot_b + (m + 1) * kSlotB, lane, wr, j,
                                       nfull, last);
    pipe_flags(p, st, fmask, lane, T1);
  }
}

// Plan (plan_group's model): q >= kProA on the residue q = 2 T2 (mod 3), the
// last pair at least T1 % 3 rows past its prologue; cost in rows of T level
// bodies, each wave doing T1 (or T2) of them plus the ring hand-off.
template <int T1, int T2, int M>
double plan_pipe(LifeBlockParams& p, int64_t out_rows, int simds, int occ, int target_waves, int xl) {
  using G = PipeGeom<T1, T2, M>;
  constexpr int T = G::T;
  constexpr int XA = T1 % 3;
  constexpr double kOverhead = 0.4 * T;
  // Ring hand-off (LDS write + read + counters) and the pipeline fill and
  // drain (stage B idles for stage A's 2 T1 prologue steps, A for B's last
  // rows): 10-25% measured on the 8-GPU tile.
  constexpr double kRingCost = 1.2;
  const int64_t max_n = out_rows / (int64_t(M - 1) * G::kProA + XA + 1);
  int64_t best_n = 0;
  int best_q = 0;
  double best = 1e300;
  for (int64_t n = 1; n <= max_n; ++n) {
    const int64_t lo = out_rows / n, hi = lo + (out_rows % n ? 1 : 0);
    const int64_t ideal = std::max<int64_t>(G::kProA, (hi + T - 1) / M);
    int q = 0;
    double span = 1e300;
    for (int64_t c = ideal - 3; c <= ideal + 3; ++c) {
      if (c < G::kProA || (c - G::kProA) % 3 != 0 || lo - int64_t(M - 1) * c < XA) continue;
      const double s = std::max<double>(double(c), double(hi - int64_t(M - 1) * c) + (T - 1));
      if (s < span) {
        span = s;
        q = int(c);
      }
    }
    if (q == 0) continue;
    const int64_t waves = int64_t(p.ncolw) * n * 2 * M;
    const int64_t k = ceil_div(waves, int64_t(simds));
    const int64_t rounds = ceil_div(k, int64_t(occ));
    const int64_t kk = std::min<int64_t>(k, occ);
    double cost = double(rounds) * (span + kOverhead) * double(kk) * issue_factor(xl, kk) * 0.5 * kRingCost;
    if (target_waves > 0)
      cost = 1.0 + double(std::llabs(waves - int64_t(target_waves)));
    else if (rounds > 4)
      break;
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

template <int T1, int T2, class IO, int M>
int pipe_waves_per_simd() {
  static const int cached = std::max(1, occupancy_blocks(life_pipe_kernel<T1, T2, IO, M>, 128 * M) * 2 * M / 4);
  return cached;
}

template <int T1, int T2, class IO, int M>
void launch_pipe(const LifeBlockParams& p, hipStream_t s) {
  hipLaunchKernelGGL((life_pipe_kernel<T1, T2, IO, M>), dim3(unsigned(int64_t(p.ncolw) * p.nseg)), dim3(128 * M), 0,
                     s, p);
}

}  // namespace lb
}  // namespace hipk
}  // namespace gol
