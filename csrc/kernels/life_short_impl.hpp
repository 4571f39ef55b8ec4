// Short-segment grouped schedule ("parallelogram"): the grouped kernel of
// life_group_impl.hpp for segments shorter than its 2T-step prologue.
//
// On the 8-GPU per-rank tile (32768 x 4096) a launch that gives every SIMD 4
// waves leaves each wave q ~ 17-20 output rows.  The grouped kernel needs
// q >= 2T (its prologue and epilogue triangles must not overlap), so it runs
// that tile with 2 waves per SIMD.  Here a wave's whole sweep is unrolled at
// compile time for a fixed Q.  With in0 the wave's first input row and
// b = in0 + Q its lower boundary, level L (0 = input) receives one row per
// step k for k in [2L, Q + 2L + 2):
//   * k < Q + 2L: computed this step by level L-1 (L = 0: the input row);
//   * k = Q + 2L, Q + 2L + 1: the lower wave's level-L rows b + L, b + L + 1,
//     saved in LDS during its own first steps (waited for on an LDS flag);
// and evaluates level L+1 from its 3-row window at steps k in [2L + 2, Q + 2L + 2).
// The level-T rows of steps [2T, Q + 2T) are the wave's Q output rows.  The
// levels coming online (trapezoid top) and the levels retiring (inverted
// triangle bottom) overlap in the same unrolled step sequence.
//
// As in the grouped kernel, M waves of a workgroup own consecutive segments
// of one column strip; wave m saves its level-L rows in0 + L, in0 + L + 1 for
// wave m - 1.  The last wave has no lower neighbour in the group and ends like
// a classic segment (runtime length, life_block_kernel's loop); it also pays
// the group boundary's redundant triangle, so it gets about T - 1 fewer rows.
//
// Measured (profiles/sweep_short_segments.jsonl, 32768 x 4096): exact, but
// 2.76 us/gen at 4 waves/SIMD against 2.44 for the grouped kernel at 2: the
// unrolled sweep is ~50 KB of straight-line code per Q, fetched once per wave,
// and its level chains are short.  Opt-in (GOL_SHORT=1 model, 2 forced).
#pragma once

#include "life_group_impl.hpp"

namespace gol {
namespace hipk {
namespace lb {

// Boundary rows plus a per-level ready flag (LDS).  The flag is set after the
// level's second row; LDS stores of one wave complete in order, and the
// workgroup-scope release / acquire keeps the compiler from reordering them.
template <int T, int W>
struct LdsFlagSaver {
  uint32_t* slot;
  uint32_t* ready;  // ready[L] of this wave's slot
  int lane;
  __device__ __forceinline__ void operator()(int L, int j, const Vec<W>& v) const {
#pragma unroll
    for (int i = 0; i < W; ++i) slot[(((L - 1) * 2 + j) * W + i) * 64 + lane] = v.w[i];
    if (j == 1) __hip_atomic_store(ready + L, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
};

template <int T, int W>
struct Below {
  const uint32_t* slot;
  uint32_t* ready;
  int lane;
  uint32_t* err;
  template <int L, int J>
  __device__ __forceinline__ Vec<W> row() const {
    if constexpr (J == 0) {
      // The lower wave saves level L at its steps 2L, 2L + 1; this wave needs
      // it at step Q + 2L.  Waves of a workgroup are co-resident and the lower
      // wave never waits on this one, so the spin ends.
      // Bounded (~0.1 s) instead of a hung GPU; giving up raises the launch's
      // error word, which the host turns into an error at its next poll
      // (Backend::check_device_errors), so the invalid rows never go unnoticed.
      bool arrived = false;
      for (int spin = 0; spin < (1 << 22); ++spin) {
        if (__hip_atomic_load(ready + L, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) {
          arrived = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!arrived && err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    Vec<W> v;
#pragma unroll
    for (int i = 0; i < W; ++i) v.w[i] = slot[(((L - 1) * 2 + J) * W + i) * 64 + lane];
    return v;
  }
};

template <int A, int B>
constexpr int cmin() {
  return A < B ? A : B;
}

// Levels L..LHI of step K (slot S): L < K/2 evaluates the next level, L = K/2
// (a level coming online) only fills its window and saves its row.  Returns
// the level-T row when level T-1 evaluated this step.
template <int T, class IO, int K, int S, int L, int LHI, class Save>
__device__ __forceinline__ void para_levels(Levels<T, IO::W>& st, const Vec<IO::W>& cur, const Save& save,
                                            const Writer<IO>& wr, int64_t out_row) {
  if constexpr (L <= LHI) {
    if constexpr (2 * L + 2 <= K) {
      const Vec<IO::W> nxt = level_full<T, IO, S, L>(st, cur);
      if constexpr (L + 1 == T)
        wr.row(out_row, nxt);
      else
        para_levels<T, IO, K, S, L + 1, LHI, Save>(st, nxt, save, wr, out_row);
    } else {
      // K = 2L or 2L + 1: the level's first two rows (trapezoid top).
      if constexpr (L >= 1) save(L, K - 2 * L, cur);
      level_store<T, IO, S, L>(st, cur);
    }
  }
}

template <int T, class IO, int Q, int K, class Save>
__device__ __forceinline__ void para_steps(Levels<T, IO::W>& st, RowReader<IO>& rd, const Save& save,
                                           const Below<T, IO::W>& below, const Writer<IO>& wr) {
  if constexpr (K < Q + 2 * T) {
    constexpr int S = K % 3;
    constexpr int LLO = K >= Q ? (K - Q) / 2 : 0;  // lowest level that receives a row
    constexpr int LHI = cmin<T - 1, K / 2>();       // highest
    Vec<IO::W> cur;
    if constexpr (LLO == 0)
      cur = rd.template take<S>(K);
    else
      cur = below.template row<LLO, (K - Q) & 1>();
    para_levels<T, IO, K, S, LLO, LHI, Save>(st, cur, save, wr, K - T);
    para_steps<T, IO, Q, K + 1, Save>(st, rd, save, below, wr);
  }
}

// 4 waves/SIMD is the point of this kernel: pin the register budget (<= 128).
template <int T, class IO, int M, int Q>
__global__ __launch_bounds__(64 * M) __attribute__((amdgpu_waves_per_eu(4)))
void life_short_kernel(const LifeBlockParams p) {
  constexpr int W = IO::W;
  constexpr int kSlot = (T - 1) * 2 * W * 64;
  __shared__ uint32_t saved[M * kSlot];
  __shared__ uint32_t ready[M * T];
  const int lane = threadIdx.x & 63;
  const int m = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < M * T; i += 64 * M) ready[i] = 0u;
  __syncthreads();

  const int kcol = blockIdx.x / p.nseg;
  const int grp = blockIdx.x - kcol * p.nseg;
  const int64_t G0 = p.row_lo + int64_t(grp) * p.seg_rows + min(grp, p.seg_rem);
  const int64_t G1 = G0 + p.seg_rows + (grp < p.seg_rem ? 1 : 0);
  const int64_t in0 = G0 + int64_t(m) * Q - T;
  const bool last = m == M - 1;
  const int kend = int(G1 + T - in0);  // last wave: level-T rows up to G1 - 1

  const LaneCols<IO> lc = lane_cols<IO>(p, kcol, lane);
  const int col = lc.store_col;
  const int64_t pitch = p.pitch;
  RowReader<IO> rd;
  Writer<IO> wr;
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
  rd.base = p.in + in0 * pitch;
  rd.pitch = pitch;
  rd.kmax = last ? kend - 1 : Q + 1;
#pragma unroll
  for (int i = 0; i < W; ++i) rd.off[i] = lc.off[i];
  rd.init();
  wr.out = p.out + in0 * pitch;  // level-T row of step k: in0 + k - T
  wr.pitch = pitch;
  wr.col = col;
  const LdsFlagSaver<T, W> saver{saved + m * kSlot, ready + m * T, lane};

  if (!last) {
    const Below<T, W> below{saved + (m + 1) * kSlot, ready + (m + 1) * T, lane, p.err};
    para_steps<T, IO, Q, 0>(st, rd, saver, below, wr);
  } else {
    prologue_tri<T, IO, 0>(st, rd, saver, NoBottom{});
    constexpr int kPro = 2 * T;
    constexpr int S0 = kPro % 3, S1 = (S0 + 1) % 3, S2 = (S0 + 2) % 3;
    int k = kPro;
    for (; k + 3 <= kend; k += 3) {
      wr.row(k - T, levels_full<T, IO, S0, 0, T>(st, rd.template take<S0>(k)));
      wr.row(k + 1 - T, levels_full<T, IO, S1, 0, T>(st, rd.template take<S1>(k + 1)));
      wr.row(k + 2 - T, levels_full<T, IO, S2, 0, T>(st, rd.template take<S2>(k + 2)));
    }
    if (k < kend) {
      wr.row(k - T, levels_full<T, IO, S0, 0, T>(st, rd.template take<S0>(k)));
      if (k + 1 < kend) wr.row(k + 1 - T, levels_full<T, IO, S1, 0, T>(st, rd.template take<S1>(k + 1)));
    }
  }

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
}

// Segment lengths compiled (q < 2T; longer segments use the grouped kernel):
// T = 16 DPP window and T = 12 adder window.
constexpr int kShortQ[] = {16, 18, 20, 22, 24, 26, 28, 30};

// Plan over groups per strip and the compiled Q: non-last waves Q rows, the
// last wave Lg - (M-1)Q >= 0 rows plus the redundant triangle (~T-1 rows).
// Same makespan model as plan_group.  Returns the cost (p.grp_q = Q) or -1.
template <int T, int M>
double plan_short(LifeBlockParams& p, int64_t out_rows, int simds, int occ, int target_waves, int xl = kXlaneDpp) {
  constexpr double kOverhead = 0.4 * T;
  double best = 1e300;
  int64_t best_n = 0;
  int best_q = 0;
  for (int Q : kShortQ) {
    if (Q >= 2 * T) continue;
    // Balanced: Lg ~ M Q - (T - 1); n groups of Lg rows.
    const int64_t lg_ideal = int64_t(M) * Q - (T - 1);
    if (lg_ideal <= 0) continue;
    for (int64_t n = std::max<int64_t>(1, out_rows / lg_ideal - 1); n <= out_rows / lg_ideal + 1; ++n) {
      const int64_t lo = out_rows / n, hi = lo + (out_rows % n ? 1 : 0);
      if (lo - int64_t(M - 1) * Q < 0) continue;
      const double span = std::max<double>(Q, double(hi - int64_t(M - 1) * Q) + (T - 1));
      const int64_t waves = int64_t(p.ncolw) * n * M;
      const int64_t k = ceil_div(waves, int64_t(simds));
      const int64_t rounds = ceil_div(k, int64_t(occ));
      const int64_t kk = std::min<int64_t>(k, occ);
      double cost = double(rounds) * (span + kOverhead) * double(kk) * issue_factor(xl, kk);
      if (target_waves > 0) cost = 1.0 + double(std::llabs(waves - int64_t(target_waves)));
      if (cost < best * 0.999) {
        best = cost;
        best_n = n;
        best_q = Q;
      }
    }
  }
  if (best_n == 0) return -1.0;
  p.nseg = int(best_n);
  p.seg_rows = int(out_rows / best_n);
  p.seg_rem = int(out_rows % best_n);
  p.grp_q = best_q;
  return best;
}

template <int T, class IO, int M>
int short_waves_per_simd() {
  static const int cached = std::max(1, occupancy_blocks(life_short_kernel<T, IO, M, kShortQ[0]>, 64 * M) * M / 4);
  return cached;
}

template <int T, class IO, int M, int I = 0>
void launch_short(const LifeBlockParams& p, hipStream_t s) {
  if constexpr (I < int(sizeof(kShortQ) / sizeof(kShortQ[0]))) {
    if (p.grp_q == kShortQ[I]) {
      hipLaunchKernelGGL((life_short_kernel<T, IO, M, kShortQ[I]>), dim3(unsigned(int64_t(p.ncolw) * p.nseg)),
                         dim3(64 * M), 0, s, p);
      return;
    }
    launch_short<T, IO, M, I + 1>(p, s);
  } else {
    fail("life_short: segment length " + std::to_string(p.grp_q) + " not compiled");
  }
}

}  // namespace lb
}  // namespace hipk
}  // namespace gol
