// life_block: T generations of B3/S23 in one pass over a tile, on MI355X.
//
// What the reference does per generation (src/game_cuda.cu:213-276): five
// kernel launches (halo_rows, halo_cols, evolve, compare, empty), one thread
// per cell in 32x32 blocks, nine byte loads per cell from global memory, four
// device-wide synchronisations and one or two 4-byte D2H copies.
//
// What this kernel does instead (CDNA4-first design):
//   * Cells are processed 32 at a time as bit planes: one lane owns a column
//     of 32-cell words; a wave64 owns 64 adjacent columns (62 produce output,
//     the two edge lanes are its halo).  The neighbour count is a bit-sliced
//     adder tree built from v_bitop3_b32 (any 3-input boolean function in ONE
//     VALU op on gfx950), v_alignbit_b32 (funnel shift) and DPP wave_shr /
//     wave_shl moves for the bits of the neighbouring lanes: 15 VALU ops per
//     32 cell-updates, flag tracking included.
//   * Temporal blocking in registers: the wave streams down its column strip
//     one row at a time and carries T generation levels, each with a 3-row
//     sliding window of horizontal partial sums.  Every input row is read
//     from HBM once per T generations and every output row written once, so
//     the kernel is VALU-bound, not HBM-bound (0.125 B/cell-update at T=16 vs
//     the 2 B/cell-update of a byte-per-cell single-step stencil).
//   * The per-generation "changed" flags that replace the reference's
//     compare/empty kernels (src/game_cuda.cu:76-126) are fused: one bitop3
//     per word per level, reduced with __ballot at the end of the wave.
//   * Two storage layouts share the compute core: Bits (1 bit per cell) and
//     U8 (1 byte per cell, packed to bits on load with v_dot4_u32_u8 and
//     unpacked on store with v_mul_u32_u24).
#include <hip/hip_runtime.h>

#include "gol/common.hpp"
#include "gol/tile.hpp"
#include "life_kernels.hpp"

namespace gol {
namespace hipk {

namespace {

constexpr int kWaveCols = 62;  // output words per wave (lanes 1..62)

__device__ __forceinline__ uint32_t from_left(uint32_t x) {
  // wave_shr:1 -> lane i receives lane i-1 (lane 0 receives 0)
  return __builtin_amdgcn_mov_dpp(x, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t from_right(uint32_t x) {
  // wave_shl:1 -> lane i receives lane i+1 (lane 63 receives 0)
  return __builtin_amdgcn_mov_dpp(x, 0x130, 0xF, 0xF, true);
}

template <unsigned TT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}

// Horizontal 3-sum (h1:h0) = left + centre + right of the 32 cells in `c`.
__device__ __forceinline__ void hsum(uint32_t c, uint32_t& h0, uint32_t& h1) {
  const uint32_t lw = from_left(c), rw = from_right(c);
  const uint32_t l = __builtin_amdgcn_alignbit(c, lw, 31);
  const uint32_t r = __builtin_amdgcn_alignbit(rw, c, 1);
  h0 = bop3<tt::XOR3>(l, c, r);
  h1 = bop3<tt::MAJ>(l, c, r);
}

// next = (S == 3) | (ctr & S == 4), S = 3x3 sum (see common.hpp rule_host).
__device__ __forceinline__ uint32_t rule(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1,
                                         uint32_t c0, uint32_t c1, uint32_t ctr) {
  const uint32_t x0 = bop3<tt::XOR3>(a0, b0, c0);
  const uint32_t x1 = bop3<tt::MAJ>(a0, b0, c0);
  const uint32_t y0 = bop3<tt::XOR3>(a1, b1, c1);
  const uint32_t y1 = bop3<tt::MAJ>(a1, b1, c1);
  const uint32_t s3 = bop3<tt::ANDN_XOR>(y1, x1, y0);
  const uint32_t s4 = bop3<tt::EQ_NE>(x1, y0, y1);
  return bop3<tt::SEL>(x0, s3, ctr & s4);
}

// ---- storage layouts -------------------------------------------------------
struct BitsIO {
  __device__ static __forceinline__ uint32_t load(const uint8_t* row, int col, bool ok) {
    const uint32_t w = reinterpret_cast<const uint32_t*>(row)[col];  // col is clamped in-bounds
    return ok ? w : 0u;
  }
  __device__ static __forceinline__ void store(uint8_t* row, int col, uint32_t w) {
    reinterpret_cast<uint32_t*>(row)[col] = w;
  }
};

struct U8IO {
  // 32 bytes (0/1 each) -> 32 bits.  x_k holds cells 4k..4k+3 in its bytes;
  // (x_{2j} | x_{2j+1} << 4) dotted with bytes (1,2,4,8) is the 8-bit pattern
  // of cells 8j..8j+7.
  __device__ static __forceinline__ uint32_t load(const uint8_t* row, int col, bool ok) {
    const uint4* p = reinterpret_cast<const uint4*>(row + 32 * col);
    const uint4 q0 = p[0];
    const uint4 q1 = p[1];
    constexpr uint32_t kW = 0x08040201u;
    const uint32_t b0 = __builtin_amdgcn_udot4(q0.x | (q0.y << 4), kW, 0u, false);
    const uint32_t b1 = __builtin_amdgcn_udot4(q0.z | (q0.w << 4), kW, 0u, false);
    const uint32_t b2 = __builtin_amdgcn_udot4(q1.x | (q1.y << 4), kW, 0u, false);
    const uint32_t b3 = __builtin_amdgcn_udot4(q1.z | (q1.w << 4), kW, 0u, false);
    const uint32_t w = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    return ok ? w : 0u;
  }
  // nibble n -> bytes (n&1, n>>1&1, n>>2&1, n>>3&1): n * 0x204081 puts bit i
  // at bit 8i (plus non-colliding cross terms), masked by 0x01010101.
  __device__ static __forceinline__ uint32_t spread(uint32_t w, int k) {
    return __umul24((w >> (4 * k)) & 0xFu, 0x204081u) & 0x01010101u;
  }
  __device__ static __forceinline__ void store(uint8_t* row, int col, uint32_t w) {
    uint4* p = reinterpret_cast<uint4*>(row + 32 * col);
    p[0] = make_uint4(spread(w, 0), spread(w, 1), spread(w, 2), spread(w, 3));
    p[1] = make_uint4(spread(w, 4), spread(w, 5), spread(w, 6), spread(w, 7));
  }
};

// Per-wave state.  Level L (0..T-1) keeps, for its last three rows (slot =
// row index mod 3), the horizontal sums h0/h1 and the cells themselves.
template <int T>
struct Levels {
  uint32_t h0[T][3], h1[T][3], cc[T][3];
  uint32_t acc[T];  // OR of (new ^ old) per produced level L+1
};

// One row step.  `cur` enters as the new level-0 row and leaves as the new
// level-T row.  MASKED: prologue steps where level L+1 is valid only when
// k >= 2(L+1) (k = step index within the segment).
template <int T, int S, bool MASKED>
__device__ __forceinline__ uint32_t row_step(Levels<T>& st, uint32_t cur, int k) {
  constexpr int s0 = S, s1 = (S + 1) % 3, s2 = (S + 2) % 3;
#pragma unroll
  for (int L = 0; L < T; ++L) {
    uint32_t h0, h1;
    hsum(cur, h0, h1);
    st.h0[L][s0] = h0;
    st.h1[L][s0] = h1;
    st.cc[L][s0] = cur;
    const uint32_t ctr = st.cc[L][s2];
    const uint32_t nxt = rule(st.h0[L][s1], st.h1[L][s1], st.h0[L][s2], st.h1[L][s2], h0, h1, ctr);
    if (MASKED) {
      const uint32_t m = (k >= 2 * (L + 1)) ? 0xFFFFFFFFu : 0u;
      st.acc[L] |= (nxt ^ ctr) & m;
    } else {
      st.acc[L] = bop3<tt::OR_XOR>(st.acc[L], nxt, ctr);
    }
    cur = nxt;
  }
  return cur;
}

template <int T, class IO>
__global__ __launch_bounds__(256) void life_block_kernel(const LifeBlockParams p) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= p.ncolw * p.nseg) return;  // wave-uniform
  const int kcol = gw / p.nseg;
  const int seg = gw - kcol * p.nseg;
  const int64_t o0 = p.row_lo + int64_t(seg) * p.seg_rows;
  const int64_t o1 = min(o0 + p.seg_rows, p.row_hi);
  if (o0 >= o1) return;  // wave-uniform

  const int col = kcol * kWaveCols - 1 + lane;
  const bool col_ok = col >= 0 && col < p.Wp;
  const int lcol = min(max(col, 0), p.Wp - 1);  // clamped load column (value discarded if !col_ok)
  const bool out_lane = col_ok && lane >= 1 && lane <= kWaveCols;
  uint32_t fmask = 0;
  if (out_lane && col >= p.own_w0 && col < p.own_w1)
    fmask = (col == p.own_w1 - 1) ? p.last_mask : 0xFFFFFFFFu;

  Levels<T> st;
#pragma unroll
  for (int L = 0; L < T; ++L) {
#pragma unroll
    for (int s = 0; s < 3; ++s) st.h0[L][s] = st.h1[L][s] = st.cc[L][s] = 0u;
    st.acc[L] = 0u;
  }

  const uint8_t* in = p.in + (o0 - T) * p.pitch;
  uint8_t* out = p.out + (o0 - T) * p.pitch;  // row of step k for level T is k - T
  const int64_t pitch = p.pitch;

  // Prologue: 2T steps, level L+1 becomes valid at step 2(L+1); no stores.
  int k = 0;
  constexpr int kPro = 2 * T;
  for (; k + 3 <= kPro; k += 3) {
    row_step<T, 0, true>(st, IO::load(in + (k + 0) * pitch, lcol, col_ok), k + 0);
    row_step<T, 1, true>(st, IO::load(in + (k + 1) * pitch, lcol, col_ok), k + 1);
    row_step<T, 2, true>(st, IO::load(in + (k + 2) * pitch, lcol, col_ok), k + 2);
  }
  if constexpr (kPro % 3 >= 1) {
    row_step<T, 0, true>(st, IO::load(in + (k + 0) * pitch, lcol, col_ok), k + 0);
  }
  if constexpr (kPro % 3 >= 2) {
    row_step<T, 1, true>(st, IO::load(in + (k + 1) * pitch, lcol, col_ok), k + 1);
  }
  k = kPro;

  // Steady state: every level valid; level T row (o0 + k - 2T) is stored.
  constexpr int S0 = kPro % 3, S1 = (S0 + 1) % 3, S2 = (S0 + 2) % 3;
  const int kend = kPro + int(o1 - o0);
  for (; k + 3 <= kend; k += 3) {
    uint32_t w0 = row_step<T, S0, false>(st, IO::load(in + (k + 0) * pitch, lcol, col_ok), 0);
    if (out_lane) IO::store(out + int64_t(k + 0 - T) * pitch, col, w0);
    uint32_t w1 = row_step<T, S1, false>(st, IO::load(in + (k + 1) * pitch, lcol, col_ok), 0);
    if (out_lane) IO::store(out + int64_t(k + 1 - T) * pitch, col, w1);
    uint32_t w2 = row_step<T, S2, false>(st, IO::load(in + (k + 2) * pitch, lcol, col_ok), 0);
    if (out_lane) IO::store(out + int64_t(k + 2 - T) * pitch, col, w2);
  }
  if (k < kend) {
    uint32_t w0 = row_step<T, S0, false>(st, IO::load(in + (k + 0) * pitch, lcol, col_ok), 0);
    if (out_lane) IO::store(out + int64_t(k + 0 - T) * pitch, col, w0);
    if (k + 1 < kend) {
      uint32_t w1 = row_step<T, S1, false>(st, IO::load(in + (k + 1) * pitch, lcol, col_ok), 0);
      if (out_lane) IO::store(out + int64_t(k + 1 - T) * pitch, col, w1);
    }
  }

  // Fused termination flags: one bit per generation level.
  if (p.changed) {
    uint32_t mask = 0;
#pragma unroll
    for (int L = 0; L < T; ++L) mask |= (__ballot((st.acc[L] & fmask) != 0u) != 0ull ? 1u : 0u) << L;
    if (lane < T && ((mask >> lane) & 1u)) p.changed[lane] = 1u;
  }
}

// Rows of each wave's segment: long enough to amortise the 2T-row prologue,
// short enough to give every SIMD several waves.
void plan(LifeBlockParams& p, int T, int64_t out_rows, int target_waves, int min_seg) {
  const int64_t want_segs = std::max<int64_t>(1, target_waves / std::max(1, p.ncolw));
  int64_t seg = ceil_div(out_rows, want_segs);
  seg = std::max<int64_t>(seg, std::max<int64_t>(min_seg, 4 * int64_t(T)));
  seg = std::min<int64_t>(seg, out_rows);
  p.seg_rows = int(seg);
  p.nseg = int(ceil_div(out_rows, seg));
}

template <int T>
void launch_T(const LifeBlockParams& p, Layout layout, hipStream_t s) {
  const int waves = p.ncolw * p.nseg;
  const dim3 grid(unsigned(ceil_div(waves, 4))), block(256);
  if (layout == Layout::Bits)
    hipLaunchKernelGGL((life_block_kernel<T, BitsIO>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((life_block_kernel<T, U8IO>), grid, block, 0, s, p);
}

}  // namespace

void launch_life_block(const BlockArgs& a, const LifeTuning& tune, hipStream_t stream) {
  const TileGeom& g = a.g;
  GOL_REQUIRE(a.row_lo - a.T >= 0 && a.row_hi + a.T <= g.R() && a.row_lo < a.row_hi,
              "life_block: row range outside the tile");
  GOL_REQUIRE(g.Wp() < (int64_t(1) << 30), "life_block: row too wide");
  LifeBlockParams p{};
  p.in = static_cast<const uint8_t*>(a.in);
  p.out = static_cast<uint8_t*>(a.out);
  p.pitch = g.pitch;
  p.row_lo = a.row_lo;
  p.row_hi = a.row_hi;
  p.Wp = int(g.Wp());
  p.ncolw = int(ceil_div(g.Wp(), kWaveCols));
  p.own_w0 = int(g.cell0() / 32);
  p.own_w1 = int(ceil_div(g.cell0() + g.W, 32));
  const int64_t tail = (g.cell0() + g.W) % 32;
  p.last_mask = tail ? (0xFFFFFFFFu >> (32 - tail)) : 0xFFFFFFFFu;
  p.changed = a.changed ? a.changed + (a.gen_base + 1 - a.flags_base) : nullptr;
  plan(p, a.T, a.row_hi - a.row_lo, tune.target_waves, tune.min_seg_rows);
  switch (a.T) {
    case 1: launch_T<1>(p, g.layout, stream); break;
    case 2: launch_T<2>(p, g.layout, stream); break;
    case 4: launch_T<4>(p, g.layout, stream); break;
    case 8: launch_T<8>(p, g.layout, stream); break;
    case 16: launch_T<16>(p, g.layout, stream); break;
    case 32: launch_T<32>(p, g.layout, stream); break;
    default: fail("life_block: unsupported temporal block size " + std::to_string(a.T));
  }
}

}  // namespace hipk
}  // namespace gol
