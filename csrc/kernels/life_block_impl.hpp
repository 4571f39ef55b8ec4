// life_block: T generations of B3/S23 in one pass over a tile, on MI355X.
//
// What the reference does per generation (src/game_cuda.cu:213-276): five
// kernel launches (halo_rows, halo_cols, evolve, compare, empty), one thread
// per cell in 32x32 blocks, nine byte loads per cell from global memory, four
// device-wide synchronisations and one or two 4-byte D2H copies.
//
// What this kernel does instead (CDNA4-first design):
//   * Cells are processed 32 at a time as bit planes: a lane owns W adjacent
//     32-cell words of a row (W = 1); a wave64 owns 64*W
//     adjacent words (its outermost word(s) are halo).  The neighbour count is
//     a bit-sliced adder tree built from v_bitop3_b32 (any 3-input boolean
//     function in ONE full-rate VALU op on gfx950).  The two bits that cross a
//     lane boundary come from one of two horizontal windows:
//       - the adder window (kXlaneAdd, the default wherever a tile fills four
//         waves per SIMD): one-sided cells x-2, x-1, x from add-with-carry
//         ops whose lane masks move on the SALU; the storage frame drifts one
//         cell per generation (adder_window);
//       - the symmetric DPP window (kXlaneDpp, smaller tiles): DPP wave
//         shifts and v_alignbit funnel shifts.
//     Per word and generation: 10 bitop3/AND + 4 carry ops (adder) or
//     2 DPP + 2 alignbit (DPP).  Issue classes measured per instruction form:
//     csrc/tools/ubench_vop3.hip (profiles/r04/ubench_vop3.txt).
//   * Temporal blocking in registers: the wave streams down its column strip
//     one row at a time and carries T generation levels, each with a 3-row
//     sliding window of horizontal partial sums.  Every input row is read
//     from HBM once per T generations and every output row written once
//     (0.03 B/cell-update at T=8 vs 2 B/cell-update for a byte-per-cell
//     single-step stencil).  Input rows are prefetched 3 row-steps ahead.
//   * The per-generation "changed" flags that replace the reference's
//     compare/empty kernels (src/game_cuda.cu:76-126) are fused: one bitop3
//     per word per level, reduced with __ballot at the end of the wave.
//   * Two storage layouts share the compute core: Bits (1 bit per cell) and
//     U8 (1 byte per cell, packed to bits on load with v_dot4_u32_u8 and
//     unpacked on store with v_mul_u32_u24).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>

#include "gol/common.hpp"
#include "gol/tile.hpp"
#include "life_kernels.hpp"

#ifndef GOL_T16_WAVES
#define GOL_T16_WAVES 1
#endif


namespace gol {
namespace hipk {

namespace lb {

template <unsigned TT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}

template <int W>
struct Vec {
  uint32_t w[W];
};

// Raw buffer descriptor (V#) for range-checked stores; flags = gfx950 data
// format word of the descriptor (cdna_hip_programming.md T8).
using BufRsrc = __amdgpu_buffer_rsrc_t;
using U32x4 = uint32_t __attribute__((ext_vector_type(4)));
constexpr int kBufFlags = 0x00020000;
// Cache policy aux bits of a buffer access: sc1 = device scope (written
// through to the device-coherent level; loads bypass this CU's L1).
constexpr int kCpolSc1 = 16;

// Words of the neighbouring lanes: lane i gets lane i-1's last word (left)
// and lane i+1's first word (right).  Edge lanes receive don't-care values;
// they only feed the wave's halo words.
template <int W>
__device__ __forceinline__ void neighbours(const Vec<W>& c, uint32_t& lw, uint32_t& rw) {
  lw = __builtin_amdgcn_mov_dpp(c.w[W - 1], 0x138, 0xF, 0xF, true);  // wave_shr:1
  rw = __builtin_amdgcn_mov_dpp(c.w[0], 0x130, 0xF, 0xF, true);      // wave_shl:1
}

// Words produced per wave, and which lane words are the wave's halo: the
// symmetric windows need one halo word per side; the one-sided adder window
// (kXlaneAdd) reads nothing to its right, so only lane 0 is a halo.  A pass
// deeper than 32 generations consumes more than one 32-cell word of its
// light cone per side: the T = 48 byte pass (U8IO<1, XL, 2>) keeps H = 2
// halo lanes per side (60 output words per wave).
template <int XL, int W, int H = 1>
constexpr int wave_out_words() {
  return XL == kXlaneAdd ? 64 * W - H : 64 * W - 2 * H;
}
template <int XL, int W, int H = 1>
__device__ __forceinline__ bool wave_halo(int lane, int i) {
  if constexpr (H == 1) {
    return (lane == 0 && i == 0) || (XL != kXlaneAdd && lane == 63 && i == W - 1);
  } else {
    static_assert(W == 1, "wide wave halos: one word per lane");
    return lane < H || (XL != kXlaneAdd && lane >= 64 - H);
  }
}

// Column map of one lane (all life_block kernels).
//   Halo mode (p.wrap_w == 0): the lane's words are padded-row words
//   kcol * kWaveOut - 1 + W * lane + i; the engine keeps the halo columns
//   valid (periodic fill or column exchange).
//   Wrap mode (p.wrap_w > 0: the tile is the whole torus width, Px == 1): the
//   lane's logical words lc = kcol * kWaveOut - 1 + W * lane + i are owned
//   words mod wrap_w, read at own_w0 + (lc mod wrap_w); halo columns are
//   neither read nor written, and the strips cover wrap_w words instead of
//   the padded width.
//   Folded strip (wrap mode, W == 1, life_group_kernel): the narrow last strip
//   of rem words is packed `nsub` times into one wave, as sub-strips of
//   sub_lanes = rem + halo lanes each; lane = sub * sub_lanes + j, and sub
//   runs the rows of another group (life_group_impl.hpp).
template <class IO>
struct LaneCols {
  static constexpr int W = IO::W;
  int store_col;  // Writer::col (padded word of the lane's word 0)
  int sub;        // sub-strip of a folded strip (0 otherwise)
  bool ok[W], own[W];
  int off[W];
  uint32_t fmask[W];
};

template <class IO>
__device__ __forceinline__ LaneCols<IO> lane_cols(const LifeBlockParams& p, int kcol, int lane, int sub_lanes = 64,
                                                  int nsub = 1) {
  constexpr int W = IO::W, XL = IO::XL, H = IO::kHalo;
  constexpr int kWaveOut = wave_out_words<XL, W, H>();
  LaneCols<IO> c;
  int j = lane;
  c.sub = 0;
  if (sub_lanes < 64) {
    c.sub = lane / sub_lanes;
    j = lane - c.sub * sub_lanes;
  }
  const int lc0 = kcol * kWaveOut - H + W * j;
  if (p.wrap_w == 0) {
    c.store_col = lc0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const int cc = lc0 + i;
      c.ok[i] = cc >= 0 && cc < p.Wp;
      c.own[i] = c.ok[i] && !wave_halo<XL, W, H>(lane, i);
      c.fmask[i] = (c.own[i] && cc >= p.own_w0 && cc < p.own_w1) ? (cc == p.own_w1 - 1 ? p.last_mask : ~0u) : 0u;
      c.off[i] = min(max(cc, 0), p.Wp - 1);
    }
    return c;
  }
  const int ww = p.wrap_w;
  c.store_col = p.own_w0 + lc0;
  const bool live = c.sub < nsub;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const int lc = lc0 + i;
    const bool halo =
        sub_lanes < 64 ? (j == 0 || (XL != kXlaneAdd && j == sub_lanes - 1)) : wave_halo<XL, W, H>(lane, i);
    c.ok[i] = true;
    c.own[i] = live && !halo && lc >= 0 && lc < ww;
    c.fmask[i] = c.own[i] ? (lc == ww - 1 ? p.last_mask : ~0u) : 0u;
    c.off[i] = p.own_w0 + ((lc % ww) + ww) % ww;
  }
  return c;
}

// One-sided window for the adder mode: l1 = cells x-1, l2 = cells x-2 at bit
// x.  v_add_co_u32 doubles a word (shift left by one) and leaves every lane's
// top bit in an SGPR-pair lane mask; s_lshl_b64 moves each mask bit one lane
// up; v_addc_co_u32 adds it back in as bit 0.  All VALU ops here issue at the
// full v_bitop3 rate (ubench_dpp_mix.hip, git e36884f), unlike DPP/v_alignbit.
#ifndef GOL_ADDER_NOP
#define GOL_ADDER_NOP 0
#endif
#ifndef GOL_ADDER_DPP
#define GOL_ADDER_DPP 0
#endif
#ifndef GOL_ADDER_FAKE
#define GOL_ADDER_FAKE 0
#endif
// Timing probes only (a linked launch needs both): Sc1IO's write-through
// row stores and its L1-bypassing row loads.
#ifndef GOL_SC1_LOADS
#define GOL_SC1_LOADS 1
#endif
#ifndef GOL_SC1_STORES
#define GOL_SC1_STORES 1
#endif
__device__ __forceinline__ void adder_window(uint32_t c, uint32_t& l1, uint32_t& l2) {
  // One block so the pair of lane masks never outlives the window (no SGPR
  // pressure across levels).  gfx950 wants a wait state between the last
  // carry-writing VALU op and a read of its VGPR result; the compiler pads
  // that hazard after the block itself (an s_nop 0 or an independent op), so
  // the block no longer ends in its own s_nop (GOL_ADDER_NOP=1 restores it):
  // one instruction less per level body, 32768^2 10.40-10.48 -> 10.35 ms per
  // 1000 generations (profiles/r03/adder_nop_ab.jsonl).
  uint32_t t1;
  uint64_t m1, m2;
  asm("v_add_co_u32_e64 %[t1], %[m1], %[c], %[c]\n\t"    // c << 1; carry = bit 31
      "s_lshl_b64 %[m1], %[m1], 1\n\t"                    // lane j <- lane j-1
      "v_add_co_u32_e64 %[l2], %[m2], %[t1], %[t1]\n\t"   // carry = bit 30
      "v_addc_co_u32_e64 %[l1], %[m1], %[t1], 0, %[m1]\n\t"
      "s_lshl_b64 %[m2], %[m2], 1\n\t"
      "v_addc_co_u32_e64 %[l2], %[m2], %[l1], %[l1], %[m2]"
#if GOL_ADDER_NOP
      "\n\ts_nop 0"
#endif
      : [l1] "=&v"(l1), [l2] "=&v"(l2), [t1] "=&v"(t1), [m1] "=&s"(m1), [m2] "=&s"(m2)
      : [c] "v"(c)
      : "scc");
}

// Horizontal 3-sums (h1:h0) = left + centre + right for every word, and the
// word of the cells the rule treats as centre (the input word itself, or for
// the one-sided adder window the word shifted by one cell, ctr = x-1).
template <int XL, int W>
__device__ __forceinline__ void hsum(const Vec<W>& c, Vec<W>& h0, Vec<W>& h1, Vec<W>& ctr) {
  if constexpr (XL == kXlaneAdd) {
    static_assert(W == 1, "adder window: one word per lane");
    {
      uint32_t l1, l2;
#if GOL_ADDER_FAKE
      // Timing probe only (WRONG cells): the window's shifts without the
      // cross-lane carries, to price them in the level-body microbenchmark.
      l1 = c.w[0] + c.w[0];
      l2 = l1 + l1;
#elif GOL_ADDER_DPP
      // Experiment: the same one-sided window from one DPP lane shift and
      // two funnel shifts (3 half-rate VALU ops instead of the 4 carry ops).
      const uint32_t lw = __builtin_amdgcn_mov_dpp(c.w[0], 0x138, 0xF, 0xF, true);  // wave_shr:1
      l1 = __builtin_amdgcn_alignbit(c.w[0], lw, 31);
      l2 = __builtin_amdgcn_alignbit(c.w[0], lw, 30);
#else
      adder_window(c.w[0], l1, l2);
#endif
      h0.w[0] = bop3<tt::XOR3>(l2, l1, c.w[0]);
      h1.w[0] = bop3<tt::MAJ>(l2, l1, c.w[0]);
      ctr.w[0] = l1;
    }
    return;
  }
  ctr = c;
  uint32_t lw, rw;
  neighbours(c, lw, rw);
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const uint32_t hi = i == W - 1 ? rw : c.w[i + 1];
    const uint32_t l = __builtin_amdgcn_alignbit(c.w[i], i == 0 ? lw : c.w[i - 1], 31);  // cell x-1
    const uint32_t r = __builtin_amdgcn_alignbit(hi, c.w[i], 1);            // cell x+1
    h0.w[i] = bop3<tt::XOR3>(l, c.w[i], r);
    h1.w[i] = bop3<tt::MAJ>(l, c.w[i], r);
  }
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
// load_raw() issues the global loads for one lane's W words of a row;
// convert() turns them into bit words.  Splitting the two lets the row reader
// keep three rows of loads in flight.
template <int W_, int XL_>
struct BitsIO {
  static constexpr int W = W_, XL = XL_;
  static constexpr int kHalo = 1;  // halo lanes per wave side
  static constexpr bool kLinked = false;  // Sc1IO
  static constexpr bool kBits = true;
  struct Raw {
    uint32_t w[W];
  };
  // off[i]: in-bounds (clamped) word index of the lane's word i.
  __device__ static __forceinline__ Raw load_raw(const uint8_t* row, const int (&off)[W]) {
    Raw r;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(row);
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = p[off[i]];
    return r;
  }
  __device__ static __forceinline__ Vec<W> convert(const Raw& r, const bool (&ok)[W]) {
    Vec<W> v;
#pragma unroll
    for (int i = 0; i < W; ++i) v.w[i] = ok[i] ? r.w[i] : 0u;
    return v;
  }
  __device__ static __forceinline__ void store(uint8_t* row, int col, int i, uint32_t w) {
    reinterpret_cast<uint32_t*>(row)[col + i] = w;
  }
  static constexpr int kWordBytes = 4;
  __device__ static __forceinline__ void store_buf(BufRsrc row, int voff, uint32_t w) {
    __builtin_amdgcn_raw_buffer_store_b32(w, row, voff, 0, 0);
  }
};

// Byte-layout cache policies (experiment knobs; aux bits of the buffer
// store: 2 = nt): the byte kernel streams the whole grid once per pass.
#ifndef GOL_U8_STORE_CPOL
#define GOL_U8_STORE_CPOL 0
#endif
#ifndef GOL_U8_LOAD_NT
#define GOL_U8_LOAD_NT 0
#endif

template <int W_, int XL_, int HALO_ = 1>
struct U8IO {
  static constexpr int W = W_, XL = XL_;
  static constexpr int kHalo = HALO_;  // halo lanes per wave side (2: passes deeper than 32)
  static constexpr bool kLinked = false;  // Sc1IO
  static constexpr bool kBits = false;
  struct Raw {
    uint4 q[2 * W];
  };
  __device__ static __forceinline__ Raw load_raw(const uint8_t* row, const int (&off)[W]) {
    Raw r;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const uint4* p = reinterpret_cast<const uint4*>(row + 32 * int64_t(off[i]));
#if GOL_U8_LOAD_NT
      const U32x4* v = reinterpret_cast<const U32x4*>(p);
      const U32x4 v0 = __builtin_nontemporal_load(v), v1 = __builtin_nontemporal_load(v + 1);
      r.q[2 * i] = make_uint4(v0.x, v0.y, v0.z, v0.w);
      r.q[2 * i + 1] = make_uint4(v1.x, v1.y, v1.z, v1.w);
#else
      r.q[2 * i] = p[0];
      r.q[2 * i + 1] = p[1];
#endif
    }
    return r;
  }
  // 32 bytes (0/1 each) -> 32 bits.  x_k holds cells 4k..4k+3 in its bytes;
  // (x_{2j} | x_{2j+1} << 4) dotted with bytes (1,2,4,8) is the 8-bit pattern
  // of cells 8j..8j+7.
  __device__ static __forceinline__ uint32_t pack(const uint4& a, const uint4& b) {
    constexpr uint32_t kW = 0x08040201u;
    const uint32_t b0 = __builtin_amdgcn_udot4(a.x | (a.y << 4), kW, 0u, false);
    const uint32_t b1 = __builtin_amdgcn_udot4(a.z | (a.w << 4), kW, 0u, false);
    const uint32_t b2 = __builtin_amdgcn_udot4(b.x | (b.y << 4), kW, 0u, false);
    const uint32_t b3 = __builtin_amdgcn_udot4(b.z | (b.w << 4), kW, 0u, false);
    return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  }
  __device__ static __forceinline__ Vec<W> convert(const Raw& r, const bool (&ok)[W]) {
    Vec<W> v;
#pragma unroll
    for (int i = 0; i < W; ++i) v.w[i] = ok[i] ? pack(r.q[2 * i], r.q[2 * i + 1]) : 0u;
    return v;
  }
  // nibble n -> bytes (n&1, n>>1&1, n>>2&1, n>>3&1): n * 0x204081 puts bit i
  // at bit 8i (plus non-colliding cross terms), masked by 0x01010101.
  __device__ static __forceinline__ uint32_t spread(uint32_t w, int k) {
    return __umul24((w >> (4 * k)) & 0xFu, 0x204081u) & 0x01010101u;
  }
  __device__ static __forceinline__ void store(uint8_t* row, int col, int i, uint32_t w) {
    uint4* p = reinterpret_cast<uint4*>(row + 32 * int64_t(col + i));
    p[0] = make_uint4(spread(w, 0), spread(w, 1), spread(w, 2), spread(w, 3));
    p[1] = make_uint4(spread(w, 4), spread(w, 5), spread(w, 6), spread(w, 7));
  }
  static constexpr int kWordBytes = 32;
  __device__ static __forceinline__ void store_buf(BufRsrc row, int voff, uint32_t w) {
    const U32x4 a = {spread(w, 0), spread(w, 1), spread(w, 2), spread(w, 3)};
    const U32x4 b = {spread(w, 4), spread(w, 5), spread(w, 6), spread(w, 7)};
    __builtin_amdgcn_raw_buffer_store_b128(a, row, voff, 0, GOL_U8_STORE_CPOL);
    __builtin_amdgcn_raw_buffer_store_b128(b, row, voff + 16, 0, GOL_U8_STORE_CPOL);
  }
};

// Storage layout of a linked launch (LifeBlockParams::link_flag): rows are
// handed between launches that run at the same time, so every row store is
// written through (sc1) and every row load is an sc1 load to registers, the
// form that needs no agent-scope acquire on the consumer
// (cdna_hip_programming.md §6 Guideline 16, "Valid forms").
template <class IO>
struct Sc1IO : IO {
  using Raw = typename IO::Raw;
  static constexpr int W = IO::W;
  static constexpr bool kLinked = true;
  __device__ static __forceinline__ Raw load_raw(const uint8_t* row, const int (&off)[W]) {
    static_assert(IO::kBits, "linked launches: bit layout");
    Raw r;
    const BufRsrc rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(row), short(0), 0x7FFFFFFF, kBufFlags);
#pragma unroll
    for (int i = 0; i < W; ++i)
      r.w[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, off[i] * 4, 0, GOL_SC1_LOADS ? kCpolSc1 : 0);
    return r;
  }
  __device__ static __forceinline__ void store_buf(BufRsrc row, int voff, uint32_t w) {
    __builtin_amdgcn_raw_buffer_store_b32(w, row, voff, 0, GOL_SC1_STORES ? kCpolSc1 : 0);
  }
};

// Row reader with a 3-deep register prefetch: the row for step k sits in
// slot k % 3 and is replaced by the load for step k + 3 when consumed.
// Rows in flight per wave: sets of 3 (the window's slots), the oldest set
// consumed first.  The adder window's waves (4 per SIMD, SALU round trips in
// every level body) hide a deeper prefetch: 32768^2 10.41 -> 10.13 ms with
// two sets (profiles/r05/prefetch6.jsonl); the DPP window's 2-wave tiles lose
// with it (the 8-GPU tile's ring +1 %).
#ifndef GOL_PREFETCH_SETS_ADD
#define GOL_PREFETCH_SETS_ADD 2
#endif
template <class IO>
constexpr int prefetch_sets() {
  return IO::XL == kXlaneAdd ? GOL_PREFETCH_SETS_ADD : 1;
}

// Row reader with a register prefetch of 3 N rows (N = prefetch_sets): the
// row for step k sits in slot k % 3 of the oldest set and, when consumed, the
// newer sets move down and the load for step k + 3 N fills the newest.
template <class IO>
struct RowReader {
  static constexpr int W = IO::W;
  static constexpr int N = prefetch_sets<IO>();
  typename IO::Raw buf[N][3];
  const uint8_t* base;
  int64_t pitch;
  int kmax;
  int off[W];  // clamped word index per lane word (values of !ok words are discarded)
  bool ok[W];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
      for (int s = 0; s < 3; ++s) buf[n][s] = IO::load_raw(base + int64_t(min(3 * n + s, kmax)) * pitch, off);
  }
  template <int S>
  __device__ __forceinline__ Vec<W> take(int k) {
    const typename IO::Raw r = buf[0][S];
#pragma unroll
    for (int n = 0; n + 1 < N; ++n) buf[n][S] = buf[n + 1][S];
    buf[N - 1][S] = IO::load_raw(base + int64_t(min(k + 3 * N, kmax)) * pitch, off);
    return IO::convert(r, ok);
  }
};

// Per-wave state.  Level L (0..T-1) keeps, for its last three rows (slot =
// row index mod 3), the horizontal sums h0/h1 and the cells themselves.
template <int T, int W>
struct Levels {
  Vec<W> h0[T][3], h1[T][3], cc[T][3];
  Vec<W> acc[T];  // per word: OR of (new ^ old) per produced level L+1
};

// Level L at a step in slot S: push the new level-L row `cur` into the
// window and produce the level-(L+1) row one row above it.
template <int T, class IO, int S, int L, int W = IO::W>
__device__ __forceinline__ Vec<W> level_full(Levels<T, W>& st, const Vec<W>& cur) {
  constexpr int s1 = (S + 1) % 3, s2 = (S + 2) % 3;
  Vec<W> h0, h1, nxt, c;
  hsum<IO::XL>(cur, h0, h1, c);
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const uint32_t ctr = st.cc[L][s2].w[i];
    nxt.w[i] = rule(st.h0[L][s1].w[i], st.h1[L][s1].w[i], st.h0[L][s2].w[i], st.h1[L][s2].w[i], h0.w[i],
                    h1.w[i], ctr);
    st.acc[L].w[i] = bop3<tt::OR_XOR>(st.acc[L].w[i], nxt.w[i], ctr);
    // Opaque def: in straight-line code (prologue / grouped epilogue) hipcc
    // otherwise reassociates the flag ORs of many steps into one late tree
    // and keeps every step's rows live for it (+75 VGPRs at T = 16).
    asm("" : "+v"(st.acc[L].w[i]));
  }
  st.h0[L][S] = h0;
  st.h1[L][S] = h1;
  st.cc[L][S] = c;
  return nxt;
}

// Window fill only (the level's output row would still be invalid).
template <int T, class IO, int S, int L, int W = IO::W>
__device__ __forceinline__ void level_store(Levels<T, W>& st, const Vec<W>& cur) {
  Vec<W> h0, h1, c;
  hsum<IO::XL>(cur, h0, h1, c);
  st.h0[L][S] = h0;
  st.h1[L][S] = h1;
  st.cc[L][S] = c;
}

template <int T, class IO, int S, int L, int LEND, int W = IO::W>
__device__ __forceinline__ Vec<W> levels_full(Levels<T, W>& st, const Vec<W>& cur) {
  if constexpr (L < LEND) {
    return levels_full<T, IO, S, L + 1, LEND>(st, level_full<T, IO, S, L>(st, cur));
  } else {
    return cur;
  }
}

// Triangular prologue, fully unrolled: at step K only levels 1..K/2 hold
// valid rows, so only those are evaluated; level K/2+1 just fills its
// window.
// RD: RowReader<IO>, or any source with take<S>(k).
template <int T, class IO, int K, class Save, class Bottom, class RD>
__device__ __forceinline__ void prologue_tri(Levels<T, IO::W>& st, RD& rd, const Save& save, const Bottom& bottom) {
  if constexpr (K < 2 * T) {
    constexpr int S = K % 3;
    constexpr int nfull = K / 2;
    const Vec<IO::W> cur = levels_full<T, IO, S, 0, nfull>(st, rd.template take<S>(K));
    // Level `nfull` rows in0 + nfull (K even) and in0 + nfull + 1 (K odd):
    // the grouped kernel shares them with the wave above (life_group_impl.hpp).
    if constexpr (nfull >= 1 && nfull < T) save(nfull, K - 2 * nfull, cur);
    if constexpr (nfull < T) level_store<T, IO, S, nfull>(st, cur);
    prologue_tri<T, IO, K + 1>(st, rd, save, bottom);
  }
}

struct NoSave {
  template <class V>
  __device__ __forceinline__ void operator()(int, int, const V&) const {}
};

struct NoBottom {
  template <int S, class St>
  __device__ __forceinline__ void at(const St&, int) const {}
};

// Output of one row: lanes store the words they own (not the wave halos).
// Branch-free: every lane issues a buffer store through a descriptor over the
// row (wave-uniform base, num_records = pitch), and lanes that own no word
// pass an offset past num_records, which the hardware range check drops.  A
// per-lane `if (own) store` puts an exec-masked block around every row store;
// in the grouped kernel's straight-line epilogue those 32 blocks drove hipcc
// to 400 registers.
// Folded strips (LaneCols::sub) store rows of several groups from one wave:
// lane rows sit `roff` bytes below the wave's row, and the descriptor spans
// `nrec` bytes (0: one row).
template <class IO>
struct Writer {
  static constexpr int W = IO::W;
  static constexpr int kDrop = 0x40000000;  // >= any row pitch: dropped
  uint8_t* out;
  int64_t pitch;
  int col;
  bool own[W];
  int roff = 0;
  int nrec = 0;
  __device__ __forceinline__ void row(int64_t r, const Vec<W>& v) const {
    const BufRsrc rs =
        __builtin_amdgcn_make_buffer_rsrc(out + r * pitch, short(0), nrec ? nrec : int(pitch), kBufFlags);
#pragma unroll
    for (int i = 0; i < W; ++i) IO::store_buf(rs, own[i] ? (col + i) * IO::kWordBytes + roff : kDrop, v.w[i]);
  }
};

// Optional occupancy target for the bit-layout T = 16 kernel (171 VGPRs
// unconstrained = 2 waves/SIMD).  Forcing 3 waves/SIMD (-DGOL_T16_WAVES=3,
// <= 168 VGPRs with small spills) measured 3-8% slower, so it is off.
template <int T, class IO>
constexpr int min_waves_per_eu() {
  return (T == 16 && IO::W == 1 && IO::kBits) ? GOL_T16_WAVES : 1;
}

// The classic schedule (life_block_launch.hpp): one wave per (column strip,
// row segment), its 2T-row prologue redundant with the wave above's rows.
template <int T, class IO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(min_waves_per_eu<T, IO>())))
void life_block_kernel(const LifeBlockParams p) {
  constexpr int W = IO::W;
  const int lane = threadIdx.x & 63;
  // readfirstlane: the wave index is uniform, so everything derived from it
  // (segment bounds, loop trip counts) lives in SGPRs with scalar branches.
  const int gw = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gw >= p.ncolw * p.nseg) return;  // wave-uniform
  const int kcol = gw / p.nseg;
  const int seg = gw - kcol * p.nseg;
  // Balanced segments: the first `seg_rem` segments get one extra row.
  const int64_t base = p.row_lo;
  const int64_t o0 = base + int64_t(seg) * p.seg_rows + min(seg, p.seg_rem);  // level-T output rows [o0, o1)
  const int64_t o1 = o0 + p.seg_rows + (seg < p.seg_rem ? 1 : 0);
  if (o0 >= o1) return;  // wave-uniform

  // Lane words (lane_cols): the wave's first and last words are halo words.
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
      st.acc[L].w[i] = 0u;
    }
  }

  constexpr int kPro = 2 * T;
  const int kend = kPro + int(o1 - o0);
  rd.base = p.in + (o0 - T) * pitch;  // input row of step k: o0 - T + k
  rd.pitch = pitch;
  rd.kmax = kend - 1;
#pragma unroll
  for (int i = 0; i < W; ++i) rd.off[i] = lc.off[i];
  rd.init();
  wr.out = p.out + (o0 - T) * pitch;  // level-T row of step k: o0 - 2T + k
  wr.pitch = pitch;
  wr.col = col;

  // Prologue: 2T steps, no stores.
  prologue_tri<T, IO, 0>(st, rd, NoSave{}, NoBottom{});
  int k = kPro;
  constexpr int S0 = kPro % 3, S1 = (S0 + 1) % 3, S2 = (S0 + 2) % 3;
  for (; k + 3 <= kend; k += 3) {
    wr.row(k - T, levels_full<T, IO, S0, 0, T>(st, rd.template take<S0>(k)));
    wr.row(k + 1 - T, levels_full<T, IO, S1, 0, T>(st, rd.template take<S1>(k + 1)));
    wr.row(k + 2 - T, levels_full<T, IO, S2, 0, T>(st, rd.template take<S2>(k + 2)));
  }
  if (k < kend) {
    wr.row(k - T, levels_full<T, IO, S0, 0, T>(st, rd.template take<S0>(k)));
    if (k + 1 < kend) wr.row(k + 1 - T, levels_full<T, IO, S1, 0, T>(st, rd.template take<S1>(k + 1)));
  }

  // Fused termination flags: one bit per generation level, counting only
  // owned cells (fmask excludes wave-halo words and the tail beyond W).
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


// Segment planning.  A wave owns a column strip and a balanced segment of
// output rows.  Its 2T-row prologue is redundant work (about T/2 rows' worth
// of level bodies), so segments want to be long; the launch wants every SIMD
// busy, and two resident waves per SIMD issue ~1.2x faster than one
// (ubench_level.hip, git e36884f: 97 vs 80 cycles per level body).  The
// planner scores each segment count by the makespan of the most loaded SIMD:
//     rounds * (seg_rows + T/2 + 2) * k * t(k),   k = resident waves/SIMD
// and keeps the cheapest.  (Filling 1122 waves into 1024 SIMDs would put two
// waves on a tenth of them and nearly double the kernel time; the model
// prefers 1020 or 2040 waves there.)
// Returns whether every segment has >= T rows; *cost_out (optional)
// receives the model's score of the chosen plan.
// Relative time per level body of a SIMD holding k resident waves (k = 1..4),
// per kernel family.  DPP/alignbit windows (ubench_level.hip, git e36884f):
// ~1.2x slower with one wave, flat from two.  The adder window issues two
// extra SALU shifts per body and only reaches its rate with four waves per
// SIMD (bench: 32768 x 16384 tile at T = 12, 2.5 / 3 / 4 waves per SIMD =
// 8.05 / 7.35 / 5.86 ms per 1000 generations), so its planner aims there.
inline double issue_factor(int xl, int64_t k) {
  static constexpr double kSym[] = {0, 1.2, 1.0, 0.97, 0.95};
  static constexpr double kAdd[] = {0, 2.0, 1.45, 1.25, 1.0};
  const int64_t i = std::min<int64_t>(std::max<int64_t>(k, 1), 4);
  return xl == kXlaneAdd ? kAdd[i] : kSym[i];
}

inline bool plan(LifeBlockParams& p, int T, int64_t out_rows, int simds, int occ, int min_seg,
                 int target_waves, double overhead_rows = -1, double* cost_out = nullptr, int xl = kXlaneDpp) {
  if (overhead_rows < 0) overhead_rows = 0.5 * T + 2;
  const int64_t smin = std::max<int64_t>({int64_t(min_seg), 2 * int64_t(T), 1});
  const int64_t max_nseg = std::max<int64_t>(1, out_rows / smin);
  int64_t best_n = 1;
  double best = 1e300;
  if (target_waves > 0) {
    best_n = std::min<int64_t>(max_nseg, std::max<int64_t>(1, target_waves / std::max(1, p.ncolw)));
  } else {
    for (int64_t n = 1; n <= max_nseg; ++n) {
      const int64_t waves = int64_t(p.ncolw) * n;
      const int64_t k = ceil_div(waves, int64_t(simds));
      const int64_t rounds = ceil_div(k, int64_t(occ));
      const int64_t kk = std::min<int64_t>(k, occ);
      const double seg = double(ceil_div(out_rows, n));
      const double cost = double(rounds) * (seg + overhead_rows) * double(kk) * issue_factor(xl, kk);
      if (cost < best * 0.999) {
        best = cost;
        best_n = n;
      }
    }
  }
  p.nseg = int(best_n);
  p.seg_rows = int(out_rows / best_n);
  p.seg_rem = int(out_rows % best_n);
  if (cost_out) *cost_out = target_waves > 0 ? 0.0 : best;
  return p.seg_rows >= T;
}

// Resident waves per SIMD (one 4-wave workgroup spreads over a CU's 4 SIMDs).
template <class K>
int occupancy_of(K kernel) {
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kernel, 256, 0) != hipSuccess || blocks <= 0)
    blocks = 1;
  return blocks;
}

template <int T, class IO>
int waves_per_simd() {
  static const int cached = occupancy_of(life_block_kernel<T, IO>);
  return cached;
}

}  // namespace lb
}  // namespace hipk
}  // namespace gol
