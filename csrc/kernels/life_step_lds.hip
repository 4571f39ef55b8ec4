// life_step_lds: one generation of B3/S23 on the byte-per-cell layout,
// staged through LDS - the direct MI355X counterpart of the reference's CUDA
// evolve kernel (src/game_cuda.cu:128-148: one thread per cell, 32x32
// blocks, nine 1-byte global loads per cell, no shared memory) with its
// compare/empty reductions (src/game_cuda.cu:76-126) fused in.
//
// Design (CDNA4):
//   * A 256-thread workgroup (4 x wave64) owns a 64-row x 1024-cell tile.
//     The tile plus a 1-row / 16-byte halo is loaded with 16-byte vector
//     loads into LDS (66 x 1056 B = 68 KiB, two workgroups per CU), so every
//     input byte is fetched from HBM once per generation.
//   * Thread (tx, ty) owns 16 consecutive cells (one uint4) of 16 rows and
//     slides a 3-row window down them: each LDS row is read once per thread
//     (one ds_read_b128; the neighbour words move between lanes with DPP).
//   * SWAR byte arithmetic: cells are 0/1 bytes, so horizontal 3-sums
//     (v_alignbyte funnel shifts + v_add3) and the 3x3 sum S <= 9 never carry
//     across bytes; "S == 3" / "S == 4" per byte come from
//     ((S ^ k) + 0x7f7f7f7f) & 0x80808080 (bytes of S ^ k are <= 15).
//   * The changed flag (next != current over owned cells) is reduced with
//     __ballot and one plain store per wave.
//   * Torus wrap in the loads (single rank, width % 32 == 0): staging
//     chunks and halo rows are read modulo the owned columns and rows, so the
//     tile has no halo columns, the engine runs one-generation epochs with no
//     periodic fill launches at all (each was ~5 us per epoch, a sixth of a
//     generation at 8192^2), and every generation is exactly one launch.
// The single-step kernel is HBM-bound (1 B read + 1 B write per
// cell-update, 2.6e12 cell-updates/s at 8192^2).  The same file holds the
// LDS-tiled family that GOL_U8_KERNEL=lds selects (with --u8-compute bytes):
//   * life_lds_multi_kernel: T = 2, 4, 8 generations per launch on the byte
//     tile in LDS (GOL_LDS_PACK=0);
//   * life_lds_bits_kernel (the default of that family, T = 32; 8 and 16
//     compiled): the byte tile is staged into LDS once, packed to bit words
//     there, stepped T generations with the bit-sliced rule, and unpacked on
//     the way out: 1.57e13 at 8192^2 (docs/PERFORMANCE.md).
// BASELINE config 2 (8192^2 byte-per-cell) runs faster on the default path,
// which is not LDS-tiled: the byte grid packed to bit words once per run and
// stepped by the register-blocked kernels (life_block_impl.hpp,
// Engine::epoch_via_bits), 4.0-4.2e13 - 2.6x this family.  These kernels stay
// as the reference-shaped LDS path and the byte layout's cross-check.
#include <type_traits>
#include <hip/hip_runtime.h>

#include "gol/common.hpp"
#include "life_block_impl.hpp"  // bit-sliced rule, byte <-> bit packing (U8IO)
#include "life_kernels.hpp"

namespace gol {
namespace hipk {
namespace {

constexpr int kTileW = 1024;           // cells per workgroup tile
constexpr int kHaloB = 16;             // bytes of column halo on each side
constexpr int kLdsStride = kTileW + 2 * kHaloB;  // 1056
constexpr int kChunksPerRow = kLdsStride / 16;   // 66

__device__ __forceinline__ uint32_t is_val(uint32_t s, uint32_t k) {
  // bit 7 of each byte set where the byte of s != k (bytes of s ^ k <= 15)
  return ((s ^ k) + 0x7F7F7F7Fu) & 0x80808080u;
}

__device__ __forceinline__ uint32_t rule_bytes(uint32_t s, uint32_t c) {
  const uint32_t ne3 = is_val(s, 0x03030303u), ne4 = is_val(s, 0x04040404u);
  // next = (S == 3) | (c & S == 4), computed in bit 7 of every byte
  const uint32_t hi = (~ne3 | (~ne4 & (c << 7))) & 0x80808080u;
  return hi >> 7;
}

// kTileH rows per workgroup tile (4 row groups of kTileH / 4): 64 rows use
// 68 KiB of LDS (2 workgroups per CU), 32 rows 35 KiB (4 per CU).
template <int kTileH>
__global__ __launch_bounds__(256) void life_step_lds_kernel(const uint8_t* __restrict__ in,
                                                            uint8_t* __restrict__ out, int64_t pitch,
                                                            int64_t row_lo, int64_t row_hi, int64_t Wc,
                                                            int64_t own_c0, int64_t own_c1,
                                                            uint32_t* changed, const int64_t* gen_dev,
                                                            int64_t wrap_w, int64_t wrap_h, int64_t row0) {
  constexpr int kLdsRows = kTileH + 2;
  constexpr int kRowsPerThread = kTileH / 4;
  __shared__ __attribute__((aligned(16))) uint8_t tile[kLdsRows * kLdsStride];
  const int64_t r0 = row_lo + int64_t(blockIdx.y) * kTileH;   // first output row
  const int64_t c0 = int64_t(blockIdx.x) * kTileW;            // first output cell
  const int tid = threadIdx.x;

  // Stage rows r0-1 .. r0+64 and cells c0-16 .. c0+1040 (16-byte chunks):
  // all loads of a thread are issued before the first LDS write.
  constexpr int kChunks = kLdsRows * kChunksPerRow;
  constexpr int kPerThread = (kChunks + 255) / 256;
  uint4 v[kPerThread];
  bool ok[kPerThread];
#pragma unroll
  for (int k = 0; k < kPerThread; ++k) {
    const int idx = tid + 256 * k;
    const int lr = idx / kChunksPerRow, ch = idx - lr * kChunksPerRow;
    const int64_t gr = r0 - 1 + lr;
    const int64_t gc = c0 - kHaloB + 16 * int64_t(ch);
    // Unconditional load from a clamped (or wrapped) address, zeroed
    // afterwards, so the loads are not serialised behind branches.
    int64_t grc = gr < row_hi + 1 ? gr : row_hi;
    int64_t gcc = gc < 0 ? 0 : (gc + 16 <= pitch ? gc : pitch - 16);
    // Wrap: a staged row or chunk is at most one halo row / chunk outside the
    // owned range, so one conditional add or subtract (no 64-bit modulo).
    if (wrap_h) grc = grc < row0 ? grc + wrap_h : grc >= row0 + wrap_h ? grc - wrap_h : grc;  // owned rows
    // 16-byte chunks (W % 16 == 0); chunks two widths out (narrow tiles) only
    // neighbour unstored cells: clamped into the row and zeroed.
    if (wrap_w) gcc = min(gc < 0 ? gc + wrap_w : gc >= wrap_w ? gc - wrap_w : gc, pitch - 16);
    ok[k] = idx < kChunks && gr < row_hi + 1 &&
            (wrap_w ? gc >= -wrap_w && gc < 2 * wrap_w : gc >= 0 && gc + 16 <= pitch);
    v[k] = *reinterpret_cast<const uint4*>(in + grc * pitch + gcc);
  }
#pragma unroll
  for (int k = 0; k < kPerThread; ++k)
    if (!ok[k]) v[k] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < kPerThread; ++k) {
    const int idx = tid + 256 * k;
    if (idx < kChunks) *reinterpret_cast<uint4*>(tile + idx * 16) = v[k];
  }
  __syncthreads();

  const int tx = tid & 63, ty = tid >> 6;
  const int64_t cell = c0 + 16 * int64_t(tx);
  const int lcol = kHaloB + 16 * tx;
  // Owned-cell byte masks for the changed flag.
  uint32_t own[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int64_t x = cell + 4 * k + b;
      if (x >= own_c0 && x < own_c1) m |= 0xFFu << (8 * b);
    }
    own[k] = m;
  }

  // Neighbour words come from the adjacent lanes (DPP wave shifts); only the
  // wave's edge lanes read them from LDS (strided b32 reads would conflict).
  const bool edge_l = tx == 0, edge_r = tx == 63;
  auto hrow = [&](int lr, uint32_t (&h)[4], uint32_t (&c)[4]) {
    const uint8_t* p = tile + lr * kLdsStride + lcol;
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    c[0] = w.x;
    c[1] = w.y;
    c[2] = w.z;
    c[3] = w.w;
    uint32_t lw = __builtin_amdgcn_mov_dpp(c[3], 0x138, 0xF, 0xF, true);  // wave_shr:1
    uint32_t rw = __builtin_amdgcn_mov_dpp(c[0], 0x130, 0xF, 0xF, true);  // wave_shl:1
    if (edge_l) lw = *reinterpret_cast<const uint32_t*>(p - 4);
    if (edge_r) rw = *reinterpret_cast<const uint32_t*>(p + 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t prev = k == 0 ? lw : c[k - 1];
      const uint32_t next = k == 3 ? rw : c[k + 1];
      const uint32_t l = __builtin_amdgcn_alignbyte(c[k], prev, 3);  // cell x-1
      const uint32_t r = __builtin_amdgcn_alignbyte(next, c[k], 1);  // cell x+1
      h[k] = l + c[k] + r;
    }
  };

  uint32_t ha[4], hb[4], hc[4], ca[4], cb[4], cc[4];
  const int lr0 = ty * kRowsPerThread;  // LDS row of (first output row - 1)
  hrow(lr0, ha, ca);
  hrow(lr0 + 1, hb, cb);
  uint32_t diff = 0;
  for (int i = 0; i < kRowsPerThread; ++i) {
    const int64_t row = r0 + ty * kRowsPerThread + i;
    if (row >= row_hi) break;
    hrow(lr0 + i + 2, hc, cc);
    uint32_t nx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      nx[k] = rule_bytes(ha[k] + hb[k] + hc[k], cb[k]);
      diff |= (nx[k] ^ cb[k]) & own[k];
    }
    if (cell < Wc) *reinterpret_cast<uint4*>(out + row * pitch + cell) = make_uint4(nx[0], nx[1], nx[2], nx[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ha[k] = hb[k];
      hb[k] = hc[k];
      ca[k] = cb[k];
      cb[k] = cc[k];
    }
  }
  // Idempotent plain store (an atomic per wave to one address serialises in L2).
  if (changed && __ballot(diff != 0u) != 0ull && (tid & 63) == 0) (gen_dev ? changed + *gen_dev : changed)[0] = 1u;
}

// ---- T generations per launch on an LDS-resident tile ----------------------
// The same SWAR byte rule on T generations of a tile staged once: a 512-thread
// workgroup (8 waves) stages 64 rows x 1024 bytes (the 64 - 2T output rows of
// its tile plus T halo rows per side; 992 owned cells plus one 16-byte halo
// chunk per side) into LDS, then evaluates generation g = 1..T in place on
// the rows [g, 64 - g) (the dependence cone shrinks one row and one cell per
// generation and side), the waves splitting the rows (each saves its
// neighbours' edge rows before a barrier, then sweeps down its own rows).  Lane l of a wave owns the 16
// cells of chunk l of a row (lanes 0 and 63 are the halo chunks, evaluated
// too so that T <= 16 generations stay exact inside); the neighbour words
// move between lanes with DPP.  The last generation goes to global memory.
// HBM traffic: the tile once in and once out per T generations (plus the
// 2T halo rows and 2 halo chunks), instead of per generation.
constexpr int kMultiRows = 64;                        // LDS rows per buffer
constexpr int kMultiOwn = 1024 - 2 * kHaloB;          // owned cells per tile (992)

template <int T>
__global__ __launch_bounds__(512) void life_lds_multi_kernel(const uint8_t* __restrict__ in,
                                                             uint8_t* __restrict__ out, int64_t pitch,
                                                             int64_t row_lo, int64_t row_hi, int64_t Wc,
                                                             int64_t own_c0, int64_t own_c1, uint32_t* changed,
                                                             const int64_t* gen_dev, int64_t wrap_w, int64_t wrap_h,
                                                             int64_t row0, int64_t c_first, int64_t c_end) {
  static_assert(T >= 1 && T <= 16, "one 16-byte halo chunk holds 16 generations of the light cone");
  constexpr int kTH = kMultiRows - 2 * T;  // output rows per tile
  constexpr int kRowB = 1024;              // LDS bytes per row: 64 chunks
  __shared__ __attribute__((aligned(16))) uint8_t buf[kMultiRows * kRowB];  // 64 KB: two workgroups per CU
  const int64_t r0 = row_lo + int64_t(blockIdx.y) * kTH;          // first output row
  const int64_t c0 = c_first - kHaloB + int64_t(blockIdx.x) * kMultiOwn;  // first staged cell
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

  // Stage rows r0 - T .. r0 + kTH + T - 1, cells c0 .. c0 + 1023 (16-byte chunks).
  constexpr int kPer = kMultiRows * 64 / 512;
  uint4 v[kPer];
  bool ok[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int idx = tid + 512 * k;
    const int lr = idx >> 6, ch = idx & 63;
    const int64_t gr = r0 - T + lr;
    const int64_t gc = c0 + 16 * int64_t(ch);
    int64_t grc = gr < row_hi + T ? gr : row_hi + T - 1;
    int64_t gcc = gc < 0 ? 0 : (gc + 16 <= pitch ? gc : pitch - 16);
    if (wrap_h) grc = row0 + (((grc - row0) % wrap_h) + wrap_h) % wrap_h;
    if (wrap_w) gcc = min(((gc % wrap_w) + wrap_w) % wrap_w, pitch - 16);
    ok[k] = gr < row_hi + T && (wrap_w ? true : gc >= 0 && gc + 16 <= pitch);
    v[k] = *reinterpret_cast<const uint4*>(in + grc * pitch + gcc);
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int idx = tid + 512 * k;
    *reinterpret_cast<uint4*>(buf + idx * 16) = ok[k] ? v[k] : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  // Owned-cell byte masks for the changed flags (lanes 1..62 of the tile's
  // owned columns, rows [T, T + kTH) of output rows < row_hi).
  const int64_t cell = c0 + 16 * int64_t(lane);
  uint32_t own[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int64_t x = cell + 4 * k + b;
      if (lane >= 1 && lane <= 62 && x >= own_c0 && x < own_c1) m |= 0xFFu << (8 * b);
    }
    own[k] = m;
  }
  uint32_t* flags = changed ? (gen_dev ? changed + *gen_dev : changed) : nullptr;

  // Horizontal 3-sums of one row chunk (16 cells per lane); the neighbour
  // words move between lanes with DPP (lanes 0 and 63 get 0: tile halo).
  auto hsum = [&](const uint4 x, uint32_t (&h)[4], uint32_t (&c)[4]) {
    c[0] = x.x;
    c[1] = x.y;
    c[2] = x.z;
    c[3] = x.w;
    const uint32_t lw = __builtin_amdgcn_mov_dpp(c[3], 0x138, 0xF, 0xF, true);  // wave_shr:1
    const uint32_t rw = __builtin_amdgcn_mov_dpp(c[0], 0x130, 0xF, 0xF, true);  // wave_shl:1
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t prev = k == 0 ? lw : c[k - 1];
      const uint32_t next = k == 3 ? rw : c[k + 1];
      h[k] = __builtin_amdgcn_alignbyte(c[k], prev, 3) + c[k] + __builtin_amdgcn_alignbyte(next, c[k], 1);
    }
  };

#pragma unroll 1
  for (int g = 1; g <= T; ++g) {
    // Rows [g, kMultiRows - g) split over the 8 waves, contiguous, updated in
    // place: each wave first saves the old rows just above and below its
    // range (its neighbours' edge rows), then a barrier, then it sweeps down.
    const int n = kMultiRows - 2 * g;
    const int lo = g + (n * w) / 8, hi = g + (n * (w + 1)) / 8;
    const uint4 up = *reinterpret_cast<const uint4*>(buf + (lo - 1) * kRowB + 16 * lane);
    const uint4 dn = *reinterpret_cast<const uint4*>(buf + hi * kRowB + 16 * lane);
    __syncthreads();
    uint32_t ha[4], hb[4], hc[4], ca[4], cb[4], cc[4];
    uint32_t diff = 0;
    if (lo < hi) {
      hsum(up, ha, ca);
      hsum(*reinterpret_cast<const uint4*>(buf + lo * kRowB + 16 * lane), hb, cb);
      for (int i = lo; i < hi; ++i) {
        hsum(i + 1 < hi ? *reinterpret_cast<const uint4*>(buf + (i + 1) * kRowB + 16 * lane) : dn, hc, cc);
        uint32_t nx[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) nx[k] = rule_bytes(ha[k] + hb[k] + hc[k], cb[k]);
        const int64_t row = r0 - T + i;
        const bool counted = i >= T && i < T + kTH && row < row_hi;
        if (counted) {
#pragma unroll
          for (int k = 0; k < 4; ++k) diff |= (nx[k] ^ cb[k]) & own[k];
        }
        if (g < T) {
          *reinterpret_cast<uint4*>(buf + i * kRowB + 16 * lane) = make_uint4(nx[0], nx[1], nx[2], nx[3]);
        } else if (counted && lane >= 1 && lane <= 62 && cell < c_end) {
          *reinterpret_cast<uint4*>(out + row * pitch + cell) = make_uint4(nx[0], nx[1], nx[2], nx[3]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          ha[k] = hb[k];
          hb[k] = hc[k];
          ca[k] = cb[k];
          cb[k] = cc[k];
        }
      }
    }
    if (flags && __ballot(diff != 0u) != 0ull && lane == 0) flags[g - 1] = 1u;  // idempotent plain store
    if (g < T) __syncthreads();
  }
}

// ---- T generations per launch on a bit-packed LDS tile ---------------------
// Byte-per-cell storage, bit-sliced evaluation: a 512-thread workgroup stages
// a 128-row x 2048-cell tile of bytes (64 words of 32 cells per row: 62
// owned words plus one halo word per side; T halo rows per side), packs each
// 32-byte run into a bit word (v_dot4, U8IO::pack) in LDS (32 KB), evaluates
// T generations in place with the bit-sliced rule (DPP neighbour words,
// 15 VALU ops per 32 cells instead of ~60 per 16 with bytes), the eight
// waves splitting the rows as in the byte kernel, and unpacks the last
// generation to bytes on the way out.  One halo word holds 32 generations of
// the symmetric light cone.
#ifndef GOL_LDS_BIT_ROWS
#define GOL_LDS_BIT_ROWS 160
#endif
// LDS rows: 160 (40 KB) still fits four workgroups in a CU's 160 KB and
// recomputes fewer light-cone rows per owned row than 128 (T = 32: 1.32x vs
// 1.48x); measured +1 % at 8192^2, +12 % at 32768^2, 192 rows (three per CU)
// slower (profiles/r03/lds_packed_rows_160.jsonl).
constexpr int kBitRows = GOL_LDS_BIT_ROWS;
// Words staged per thread per batch (NW waves per workgroup).
template <int NW>
constexpr int bit_stage_batch() {
  constexpr int words = kBitRows * 64 / (64 * NW);
  return words % 4 == 0 ? 4 : words % 2 == 0 ? 2 : 1;
}

// ADD: the adder window (life_block_impl.hpp kXlaneAdd: no DPP / v_alignbit
// in the level body, the stored frame drifts one cell right per generation;
// whole-width torus tiles only).  Its light cone is one-sided, 2 cells per
// generation on the left, so the tile keeps ceil(2T / 32) halo words on the
// left and none on the right.
template <int T, bool ADD, int NW>
__global__ __launch_bounds__(64 * NW) void life_lds_bits_kernel(const uint8_t* __restrict__ in,
                                                            uint8_t* __restrict__ out, int64_t pitch,
                                                            int64_t row_lo, int64_t row_hi, int64_t own_c0,
                                                            int64_t own_c1, uint32_t* changed,
                                                            const int64_t* gen_dev, int64_t wrap_w, int64_t wrap_h,
                                                            int64_t row0, int64_t c_first, int64_t c_end,
                                                            int ny, int xcd_order) {
  static_assert(T >= 1 && T <= 32, "at most 32 generations of the light cone per launch");
  constexpr int kTH = kBitRows - 2 * T;
  // Tile of this workgroup.  Workgroups go round-robin to the 8 XCDs (block
  // b to XCD b % 8), so with xcd_order (GOL_LDS_XCD=1) each XCD takes a contiguous run of
  // tiles in column-major order: vertically adjacent tiles, whose staged
  // rows overlap by 2T, read them through the same L2.  Otherwise row-major.
  const int nblk = int(gridDim.x), b = int(blockIdx.x);
  int bx, by;
  if (xcd_order) {
    const int q = nblk / 8, r = nblk % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    bx = L / ny;
    by = L % ny;
  } else {
    const int nx = nblk / ny;
    bx = b % nx;
    by = b / nx;
  }
  constexpr int kHL = ADD ? (2 * T + 31) / 32 : 1, kHR = ADD ? 0 : 1;  // halo words left / right
  constexpr int kOwn = 64 - kHL - kHR;                                   // owned words per tile row
  using IO = lb::U8IO<1, kXlaneDpp>;
  __shared__ uint32_t bits[kBitRows * 64];
  const int64_t r0 = row_lo + int64_t(by) * kTH;                          // first output row
  const int64_t c0 = c_first - 32 * kHL + int64_t(bx) * (32 * kOwn);    // first staged cell
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

  // Stage: word idx = tid + kThreads k (row idx / 64, word idx % 64), 32 bytes each.
  constexpr int kThreads = 64 * NW, kBitStageBatch = bit_stage_batch<NW>();
  static_assert(kBitRows * 64 % kThreads == 0, "whole staging passes");
  constexpr int kWords = kBitRows * 64 / kThreads;
#pragma unroll
  for (int k0 = 0; k0 < kWords; k0 += kBitStageBatch) {
    uint4 v[kBitStageBatch][2];
    bool ok[kBitStageBatch];
#pragma unroll
    for (int kk = 0; kk < kBitStageBatch; ++kk) {
      const int idx = tid + kThreads * (k0 + kk);
      const int lr = idx >> 6, wl = idx & 63;
      const int64_t gr = r0 - T + lr;
      const int64_t gc = c0 + 32 * int64_t(wl);
      int64_t grc = gr < row_hi + T ? gr : row_hi + T - 1;
      int64_t gcc = gc < 0 ? 0 : (gc + 32 <= pitch ? gc : pitch - 32);
      if (wrap_h) grc = row0 + (((grc - row0) % wrap_h) + wrap_h) % wrap_h;
      if (wrap_w) gcc = min(((gc % wrap_w) + wrap_w) % wrap_w, pitch - 32);
      ok[kk] = gr < row_hi + T && (wrap_w ? true : gc >= 0 && gc + 32 <= pitch);
      const uint4* q = reinterpret_cast<const uint4*>(in + grc * pitch + gcc);
      v[kk][0] = q[0];
      v[kk][1] = q[1];
    }
#pragma unroll
    for (int kk = 0; kk < kBitStageBatch; ++kk)
      bits[tid + kThreads * (k0 + kk)] = ok[kk] ? IO::pack(v[kk][0], v[kk][1]) : 0u;
  }
  __syncthreads();

  // Owned-cell bits of this lane's word (changed flags).
  const int64_t cell = c0 + 32 * int64_t(lane);
  const bool own_lane = lane >= kHL && lane < 64 - kHR;
  uint32_t own = 0;
  if (own_lane) {
    const int64_t a = max(own_c0, cell), b = min(own_c1, cell + 32);
    if (a < b) own = (b - a >= 32 ? 0xFFFFFFFFu : ((1u << (b - a)) - 1u)) << (a - cell);
  }
  uint32_t* flags = changed ? (gen_dev ? changed + *gen_dev : changed) : nullptr;

  // Horizontal 3-sums of a row word and the centre the rule uses: cells
  // x-1, x, x+1 (DPP neighbour words), or with ADD x-2, x-1, x (centre x-1).
  auto hsum = [&](uint32_t c, uint32_t& h0, uint32_t& h1, uint32_t& ctr) {
    if constexpr (ADD) {
      uint32_t l1, l2;
      lb::adder_window(c, l1, l2);
      h0 = lb::bop3<tt::XOR3>(l2, l1, c);
      h1 = lb::bop3<tt::MAJ>(l2, l1, c);
      ctr = l1;
    } else {
      const uint32_t lw = __builtin_amdgcn_mov_dpp(c, 0x138, 0xF, 0xF, true);  // wave_shr:1 (lane 0: 0)
      const uint32_t rw = __builtin_amdgcn_mov_dpp(c, 0x130, 0xF, 0xF, true);  // wave_shl:1 (lane 63: 0)
      const uint32_t l = __builtin_amdgcn_alignbit(c, lw, 31);
      const uint32_t r = __builtin_amdgcn_alignbit(rw, c, 1);
      h0 = lb::bop3<tt::XOR3>(l, c, r);
      h1 = lb::bop3<tt::MAJ>(l, c, r);
      ctr = c;
    }
  };

#pragma unroll 1
  for (int g = 1; g <= T; ++g) {
    const int n = kBitRows - 2 * g;
    const int lo = g + (n * w) / NW, hi = g + (n * (w + 1)) / NW;
    const uint32_t up = bits[(lo - 1) * 64 + lane];
    const uint32_t dn = bits[hi * 64 + lane];
    __syncthreads();
    uint32_t diff = 0;
    if (lo < hi) {
      uint32_t a0, a1, actr, b0, b1, bctr, c0w, c1w, cctr;
      hsum(up, a0, a1, actr);
      hsum(bits[lo * 64 + lane], b0, b1, bctr);
      for (int i = lo; i < hi; ++i) {
        const uint32_t cc = i + 1 < hi ? bits[(i + 1) * 64 + lane] : dn;
        hsum(cc, c0w, c1w, cctr);
        const uint32_t nx = lb::rule(a0, a1, b0, b1, c0w, c1w, bctr);
        const int64_t row = r0 - T + i;
        const bool counted = i >= T && i < T + kTH && row < row_hi;
        if (counted) diff |= (nx ^ bctr) & own;
        if (g < T) {
          bits[i * 64 + lane] = nx;
        } else if (counted && own_lane && cell < c_end) {
          uint4* o = reinterpret_cast<uint4*>(out + row * pitch + cell);
          o[0] = make_uint4(IO::spread(nx, 0), IO::spread(nx, 1), IO::spread(nx, 2), IO::spread(nx, 3));
          o[1] = make_uint4(IO::spread(nx, 4), IO::spread(nx, 5), IO::spread(nx, 6), IO::spread(nx, 7));
        }
        a0 = b0;
        a1 = b1;
        b0 = c0w;
        b1 = c1w;
        bctr = cctr;
      }
    }
    if (flags && __ballot(diff != 0u) != 0ull && lane == 0) flags[g - 1] = 1u;  // idempotent plain store
    if (g < T) __syncthreads();
  }
}

}  // namespace

int lds_multi_tile_rows(int T) { return kMultiRows - 2 * T; }

int launch_life_lds_bits(const BlockArgs& a, bool wrap, bool xcd_order, int waves, int cus, hipStream_t stream) {
  const TileGeom& g = a.g;
  GOL_REQUIRE(g.layout == Layout::U8, "life_lds_bits: byte layout only");
  GOL_REQUIRE(a.T == 8 || a.T == 16 || a.T == 32, "life_lds_bits: T = 8, 16 or 32");
  GOL_REQUIRE(a.row_lo >= a.T && a.row_hi + a.T <= g.R() && a.row_lo < a.row_hi,
              "life_lds_bits: row range outside the tile");
  GOL_REQUIRE(g.pitch % 32 == 0 && g.cell0() % 32 == 0, "life_lds_bits: 32-byte aligned rows and owned cells");
  const int64_t rows = a.row_hi - a.row_lo;
  uint32_t* changed = a.changed ? a.changed + (a.gen_dev ? a.gen_rel : a.gen_base + 1 - a.flags_base) : nullptr;
  const int64_t* gen_dev = a.changed ? a.gen_dev : nullptr;
  const int64_t wrap_w = wrap && a.full_width && g.hw == 0 && g.W % 32 == 0 ? g.W : 0;
  const int64_t wrap_h = wrap_w && a.wrap_rows ? g.H : 0;
  GOL_REQUIRE(!a.wrap_rows || wrap_h, "life_lds_bits: row wrap needs a whole-width tile without halo columns");
  GOL_REQUIRE(wrap_w || 32 * g.hw >= a.T, "life_lds_bits: a tile without column wrap needs T halo cells");
  // The DPP window: the packed tile's adder window (template ADD, a drifting
  // frame on whole-width torus rows) measured 5 % slower and is not launched.
  constexpr bool add = false;
  // Tiles as in launch_life_lds_multi: owned cells (wrap) or the padded row.
  const int64_t c_first = wrap_w ? g.cell0() : 0;
  const int64_t c_end = wrap_w ? g.cell0() + g.W : g.Wc();
  const int th = kBitRows - 2 * a.T;
  const int own_words = add ? 64 - (2 * a.T + 31) / 32 : 62;
  const int64_t nx = ceil_div(c_end - c_first, int64_t(32 * own_words)), ny = ceil_div(rows, int64_t(th));
  GOL_REQUIRE(nx * ny < (int64_t(1) << 31), "life_lds_bits: grid too large");
  const dim3 grid(unsigned(nx * ny));
  // 16 waves per workgroup when the grid fits the GPU in one round at 8
  // (small grids: 8192^2 +6 %), 8 otherwise (32768^2: 16 waves -19 %;
  // profiles/r03/lds_packed_waves_xcd.jsonl, lds_packed_waves_auto.jsonl).
  const int nw = waves == 8 || waves == 16 ? waves : (nx * ny <= int64_t(4) * cus ? 16 : 8);
  using K = void (*)(const uint8_t*, uint8_t*, int64_t, int64_t, int64_t, int64_t, int64_t, uint32_t*,
                     const int64_t*, int64_t, int64_t, int64_t, int64_t, int64_t, int, int);
  const auto pick = [&](auto nw_c) -> K {
    constexpr int NW = decltype(nw_c)::value;
    return a.T == 8 ? life_lds_bits_kernel<8, false, NW> : a.T == 16 ? life_lds_bits_kernel<16, false, NW>
                                                                     : life_lds_bits_kernel<32, false, NW>;
  };
  const K k = nw == 16 ? pick(std::integral_constant<int, 16>{}) : pick(std::integral_constant<int, 8>{});
  hipLaunchKernelGGL(k, grid, dim3(64 * nw), 0, stream, static_cast<const uint8_t*>(a.in), static_cast<uint8_t*>(a.out),
                     g.pitch, a.row_lo, a.row_hi, g.cell0(), g.cell0() + g.W, changed, gen_dev, wrap_w, wrap_h,
                     g.row0(), c_first, c_end, int(ny), xcd_order ? 1 : 0);
  return add ? a.T : 0;
}

void launch_life_lds_multi(const BlockArgs& a, bool wrap, hipStream_t stream) {
  const TileGeom& g = a.g;
  GOL_REQUIRE(g.layout == Layout::U8, "life_lds_multi: byte layout only");
  GOL_REQUIRE(a.T == 2 || a.T == 4 || a.T == 8, "life_lds_multi: T = 2, 4 or 8");
  GOL_REQUIRE(a.row_lo >= a.T && a.row_hi + a.T <= g.R() && a.row_lo < a.row_hi,
              "life_lds_multi: row range outside the tile");
  GOL_REQUIRE(g.pitch % 16 == 0 && g.cell0() % 16 == 0, "life_lds_multi: 16-byte aligned rows and owned cells");
  const int64_t rows = a.row_hi - a.row_lo;
  uint32_t* changed = a.changed ? a.changed + (a.gen_dev ? a.gen_rel : a.gen_base + 1 - a.flags_base) : nullptr;
  const int64_t* gen_dev = a.changed ? a.gen_dev : nullptr;
  const int64_t wrap_w = wrap && a.full_width && g.hw == 0 && g.W % 16 == 0 ? g.W : 0;
  const int64_t wrap_h = wrap_w && a.wrap_rows ? g.H : 0;
  GOL_REQUIRE(!a.wrap_rows || wrap_h, "life_lds_multi: row wrap needs a whole-width tile without halo columns");
  GOL_REQUIRE(wrap_w || 32 * g.hw >= 16, "life_lds_multi: a tile without halo columns needs column wrap");
  const int th = lds_multi_tile_rows(a.T);
  // Wrap: tiles cover the owned cells [cell0, cell0 + W), the chunk staged
  // left of the first one being the wrapped last chunk.  Halo mode: tiles
  // cover the whole padded row [0, Wc), halo columns included - a block's
  // output feeds the next block of the epoch, whose halo columns must be the
  // evolved ones (valid up to the light cone from the padded row's ends).
  const int64_t c_first = wrap_w ? g.cell0() : 0;
  const int64_t c_end = wrap_w ? g.cell0() + g.W : g.Wc();
  const dim3 grid(unsigned(ceil_div(c_end - c_first, int64_t(kMultiOwn))), unsigned(ceil_div(rows, int64_t(th))));
  auto k = a.T == 2 ? life_lds_multi_kernel<2> : a.T == 4 ? life_lds_multi_kernel<4> : life_lds_multi_kernel<8>;
  hipLaunchKernelGGL(k, grid, dim3(512), 0, stream, static_cast<const uint8_t*>(a.in), static_cast<uint8_t*>(a.out),
                     g.pitch, a.row_lo, a.row_hi, g.Wc(), g.cell0(), g.cell0() + g.W, changed, gen_dev, wrap_w, wrap_h,
                     g.row0(), c_first, c_end);
}

void launch_life_step_lds(const BlockArgs& a, int lds_rows, bool wrap, hipStream_t stream) {
  const TileGeom& g = a.g;
  GOL_REQUIRE(g.layout == Layout::U8, "life_step_lds: byte layout only");
  GOL_REQUIRE(a.T == 1, "life_step_lds: single-step kernel (T = 1)");
  GOL_REQUIRE(a.row_lo >= 1 && a.row_hi + 1 <= g.R() && a.row_lo < a.row_hi,
              "life_step_lds: row range outside the tile");
  GOL_REQUIRE(g.pitch % 16 == 0, "life_step_lds: pitch must be 16-byte aligned");
  const int64_t rows = a.row_hi - a.row_lo;
  uint32_t* changed = a.changed ? a.changed + (a.gen_dev ? a.gen_rel : a.gen_base + 1 - a.flags_base) : nullptr;
  const int64_t* gen_dev = a.changed ? a.gen_dev : nullptr;
  const int th = lds_rows == 32 ? 32 : 64;
  // Torus wrap: whole-width tile without halo columns (and, with wrap_rows,
  // the whole torus: owned rows read modulo H).
  const int64_t wrap_w = wrap && a.full_width && g.hw == 0 && g.W % 16 == 0 ? g.W : 0;
  const int64_t wrap_h = wrap_w && a.wrap_rows ? g.H : 0;
  GOL_REQUIRE(!a.wrap_rows || wrap_h, "life_step_lds: row wrap needs a whole-width tile without halo columns");
  GOL_REQUIRE(wrap_w || g.hw > 0, "life_step_lds: a tile without halo columns needs column wrap");
  GOL_REQUIRE(ceil_div(rows, int64_t(th)) < (int64_t(1) << 31), "life_step_lds: too many rows");
  const dim3 grid(unsigned(ceil_div(g.Wc(), int64_t(kTileW))), unsigned(ceil_div(rows, int64_t(th))));
  auto k = th == 32 ? life_step_lds_kernel<32> : life_step_lds_kernel<64>;
  hipLaunchKernelGGL(k, grid, dim3(256), 0, stream, static_cast<const uint8_t*>(a.in), static_cast<uint8_t*>(a.out),
                     g.pitch, a.row_lo, a.row_hi, g.Wc(), g.cell0(), g.cell0() + g.W, changed, gen_dev, wrap_w,
                     wrap_h, g.row0());
}

}  // namespace hipk
}  // namespace gol
