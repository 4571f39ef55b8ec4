// Resident epoch kernel: a whole halo epoch (T generations) of a per-rank
// tile in one launch, the tile held in the register file.
//
// Why: the grouped temporal-blocking kernel (life_group_impl.hpp) streams
// the tile through registers T <= 16 generations per launch and needs
// segments of at least 2T rows per wave.  The 8-GPU rank tile (32768 x 4096)
// then has too few segments for four waves per SIMD, the occupancy the adder
// window needs, and runs at ~55 % of the full-grid per-cell rate
// (docs/PERFORMANCE.md).  A 16 MiB bit tile is an eighth of the chip's
// register file, so instead of streaming it, keep it resident:
//
//   * one 1024-thread workgroup per CU (LDS > 80 KB forces it), 255 of them
//     for the 8-GPU tile: 17 column strips x 15 row bands;
//   * a workgroup owns one column strip (64 lanes: the left halo lane of the
//     one-sided adder window + up to 63 owned words) x one row band, plus k
//     halo rows above and below; its 16 waves stack down the band, RW rows
//     of one 32-bit word per lane each, in VGPRs (4 waves per SIMD);
//   * every generation each wave updates its RW rows in place (adder window:
//     15 full-rate VALU ops + 2 SALU shifts per row, no cross-lane data op)
//     after trading its first and last row with the waves above and below
//     through LDS (one barrier per generation);
//   * every k generations the workgroups trade what the light cone has
//     consumed: the k halo rows per side and the halo lane's word of every
//     owned row, through a global mirror of the tile (sc1 write-through
//     stores, s_waitcnt vmcnt(0), barrier, relaxed agent-scope flag; the
//     consumer polls its 8 neighbours' flags and reads with sc1 loads - the
//     no-acquire valid form of cdna_hip_programming.md §6 Guideline 16).
//     The adder window consumes 2 cells of the halo lane per generation, so
//     k <= 16; the halo rows erode one row per generation.
//
// Exactness: the rows a workgroup stores are its owned rows of the block's
// output range [row_lo, row_hi); the per-generation change flags cover the
// same rows and its owned words (one LDS slot per generation, flushed to the
// engine's flag array every 64 generations).  The storage frame drifts one
// cell right per generation like every adder-window kernel (kXlaneAdd).
//
// Deadlock freedom needs every workgroup co-resident: the grid is at most one
// workgroup per CU and each holds 96 KB of LDS, so no CU takes two; every
// wait is bounded and raises the device error word (4) instead of hanging.
//
// Reference: the per-generation MPI halo exchange + evolve of
// src/game_mpi.c:392-402 and the CUDA evolve of src/game_cuda.cu:128-148.
#pragma once

#include "life_block_impl.hpp"

namespace gol {
namespace hipk {
namespace lr {

using lb::bop3;
using lb::BufRsrc;
using lb::kBufFlags;
using lb::kCpolSc1;

constexpr int kM = kResidentWaves;          // waves per workgroup, stacked down the band
constexpr int kBndWords = 2 * kM * 2 * 64;   // [parity][wave][first/last row][lane]
constexpr int kFlagWords = 128;              // generation flags, a ring (slot = generation & 127)
constexpr int kCntWords = kM;                // GOL_RES_SYNC=1: per-wave generation counters
// One workgroup per CU: more than half of the CU's 160 KB LDS (a small RW
// alone would let the register file take two workgroups).
constexpr int kLdsWords = 96 * 1024 / 4;
constexpr int kOOR = int(0x80000000u);       // buffer offset past any record count: access dropped
// Per-region exchange record in a mirror (bytes): k <= 16 first rows, k last
// rows (64 words each), then one halo-lane word per register row.
constexpr int kRecB = 16 * 256;
constexpr int kRecC = 2 * 16 * 256;
constexpr int kRecBytes = kRecC + 4 * kM * 88;
static_assert(kRecBytes == kResidentRecBytes, "exchange record size");
static_assert(kBndWords + kFlagWords + kCntWords + 2 * kRecBytes / 4 <= kLdsWords, "LDS layout");

#ifndef GOL_RES_ROW_FENCE
#define GOL_RES_ROW_FENCE 2
#endif
constexpr int kRowFence = GOL_RES_ROW_FENCE;  // rows between scheduling barriers (0: none)
constexpr int kLoadBatch = 8;                 // refresh loads per batch (two batches in flight)
constexpr int kTwoBodyMaxRW = 48;             // larger RW: one masked generation body
// Edge-row hand-off between the waves of a band each generation:
//   0: one workgroup barrier per generation;
//   1: per-wave generation counters in LDS: a wave publishes its edge rows,
//      updates its interior rows, and only then waits for its two neighbours
//      (no workgroup barrier between refreshes).
#ifndef GOL_RES_SYNC
#define GOL_RES_SYNC 0
#endif

struct HS {
  uint32_t h0, h1, c;
};

// Horizontal 3-sum of a row word and its centre cell (adder window: cells
// x-2, x-1, x at bit x; the centre is x-1).
__device__ __forceinline__ HS hs(uint32_t x) {
  uint32_t l1, l2;
  lb::adder_window(x, l1, l2);
  return {bop3<tt::XOR3>(l2, l1, x), bop3<tt::MAJ>(l2, l1, x), l1};
}

// One generation of the wave's RW rows, in place; returns the OR of
// (new ^ old) over the rows [i_lo, i_hi) (all rows unless MASKED).
template <int RW, bool MASKED>
__device__ __forceinline__ uint32_t gen_rows(uint32_t (&s)[RW], uint32_t above, uint32_t below, int i_lo,
                                             int i_hi) {
  uint32_t acc = 0;
  HS prev = hs(above), cur = hs(s[0]);
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const HS nxt = hs(i + 1 < RW ? s[i + 1] : below);
    const uint32_t n = lb::rule(prev.h0, prev.h1, cur.h0, cur.h1, nxt.h0, nxt.h1, cur.c);
    if constexpr (MASKED) {
      const uint32_t x = (i >= i_lo && i < i_hi) ? cur.c : n;  // wave-uniform select
      acc = bop3<tt::OR_XOR>(acc, n, x);
    } else {
      acc = bop3<tt::OR_XOR>(acc, n, cur.c);
    }
    // Opaque def: otherwise the flag ORs of many rows are deferred into one
    // late tree that keeps every row's old centre word live.
    asm("" : "+v"(acc));
    s[i] = n;
    prev = cur;
    cur = nxt;
    // Rows in order: hoisting later rows' window sums would hold three VGPRs
    // per row (the scheduler has the whole 128-VGPR budget of four waves per
    // SIMD to fill); the four waves of a SIMD supply the overlap instead.
    if constexpr (kRowFence > 0)
      if ((i + 1) % kRowFence == 0) __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

// The same generation with the edge rows last (GOL_RES_SYNC=1): rows
// 1..RW-2 need no neighbour, so they run while the waves above and below
// finish publishing; edges() then returns (above, below).
template <int RW, bool MASKED, class Edges>
__device__ __forceinline__ uint32_t gen_rows_split(uint32_t (&s)[RW], int i_lo, int i_hi, const Edges& edges) {
  static_assert(RW >= 3, "split generation body: at least three rows per wave");
  uint32_t acc = 0;
  const auto flag = [&](int i, uint32_t n, uint32_t c) {
    if constexpr (MASKED) {
      const uint32_t x = (i >= i_lo && i < i_hi) ? c : n;
      acc = bop3<tt::OR_XOR>(acc, n, x);
    } else {
      acc = bop3<tt::OR_XOR>(acc, n, c);
    }
    asm("" : "+v"(acc));
  };
  const HS a0 = hs(s[0]), a1 = hs(s[1]);
  HS prev = a0, cur = a1;
#pragma unroll
  for (int i = 1; i < RW - 1; ++i) {
    const HS nxt = hs(s[i + 1]);
    const uint32_t n = lb::rule(prev.h0, prev.h1, cur.h0, cur.h1, nxt.h0, nxt.h1, cur.c);
    flag(i, n, cur.c);
    s[i] = n;
    prev = cur;
    cur = nxt;
    if constexpr (kRowFence > 0)
      if (i % kRowFence == 0) __builtin_amdgcn_sched_barrier(0);
  }
  uint32_t above, below;
  edges(above, below);
  const HS ha = hs(above), hb = hs(below);
  const uint32_t n0 = lb::rule(ha.h0, ha.h1, a0.h0, a0.h1, a1.h0, a1.h1, a0.c);
  flag(0, n0, a0.c);
  const uint32_t nl = lb::rule(prev.h0, prev.h1, cur.h0, cur.h1, hb.h0, hb.h1, cur.c);
  flag(RW - 1, nl, cur.c);
  s[0] = n0;
  s[RW - 1] = nl;
  return acc;
}

// Wave 0 copies the flags of generations [g0, g0 + n) (n <= 64) from the
// LDS ring to the engine's array and clears their slots.
__device__ __forceinline__ void flush_flags(uint32_t* lflag, uint32_t* changed, int g0, int n, int lane) {
  if (lane < n) {
    const int sl = (g0 + lane) & (kFlagWords - 1);
    if (lflag[sl]) changed[g0 + lane] = 1u;
    lflag[sl] = 0u;
  }
}

template <int RW>
__global__ __launch_bounds__(64 * kM) void life_resident_kernel(ResidentParams p) {
  __shared__ uint32_t lds[kLdsWords];
  uint32_t* const bnd = lds;
  uint32_t* const lflag = lds + kBndWords;
  const int lane = int(threadIdx.x & 63);
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));

  // XCD-aware region map: dispatch puts block b on XCD b % 8, so XCD x gets a
  // contiguous run of regions (strip-major: a strip's bands are neighbours).
  const int G = p.nreg, b = int(blockIdx.x);
  const int per = G >> 3, rem = G & 7, xcd = b & 7;
  const int j = xcd * per + min(xcd, rem) + (b >> 3);
  const int strip = j / p.nb, band = j - strip * p.nb;

  // Columns: lane 0 is the halo word left of the strip (the adder window
  // reads nothing to its right), lanes 1..own_cnt own words.
  const int own_cnt = min(p.sw, p.ww - strip * p.sw);
  const int lc = strip * p.sw - 1 + lane;
  const bool own = lane >= 1 && lane <= own_cnt;
  const bool last_own = lane == own_cnt;
  const int vw = 4 * (p.own_w0 + ((lc % p.ww) + p.ww) % p.ww);

  // Rows (extended coordinates, 0 = row_lo - T): the band owns [q0, q0 + cnt);
  // register row i of wave w holds row eb + i.
  const int q0 = band * p.band_rows + min(band, p.band_rem);
  const int cnt = p.band_rows + (band < p.band_rem ? 1 : 0);
  const int eb = q0 - p.k + w * RW;
  const int olo = max(q0, p.T), ohi = min(q0 + cnt, p.ext_rows - p.T);  // owned rows of the output range
  const int i_lo = min(max(olo - eb, 0), RW), i_hi = min(max(ohi - eb, 0), RW);
  const bool outw = i_lo < i_hi;
  const bool partial = outw && (i_lo > 0 || i_hi < RW);
  const int ip = int(p.pitch);
  const int64_t base = p.row0 * p.pitch;
  const int range = int(int64_t(p.ext_rows) * p.pitch);

  // Trace slot 0 (GOL_RES_TRACE): kernel start, state loaded, loop done, end.
  uint64_t* const tr0 = (p.trace && threadIdx.x == 0) ? p.trace + int64_t(j) * kResTraceRefreshes * 6 : nullptr;
  if (tr0) {
    tr0[0] = __builtin_amdgcn_s_memrealtime();
    tr0[4] = __builtin_amdgcn_s_memtime();
  }
  uint32_t s[RW];
  {
    const BufRsrc rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.in) + base, short(0), range, kBufFlags);
#pragma unroll
    for (int i = 0; i < RW; ++i) s[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, (eb + i) * ip + vw, 0, 0);
  }
  uint32_t* const cntw = lflag + kFlagWords;
  uint32_t* const recs = cntw + kCntWords;     // outgoing exchange record
  uint32_t* const stage = recs + kRecBytes / 4;  // incoming halo rows + halo-lane words
  if (threadIdx.x < kFlagWords + kCntWords) lflag[threadIdx.x] = 0u;
  __syncthreads();
  if (tr0) tr0[1] = __builtin_amdgcn_s_memrealtime();
  uint32_t* changed = p.changed;
  if (changed && p.gen_dev) changed += *p.gen_dev + p.gen_rel;
  const bool rec = changed != nullptr && outw;

  for (int t = 0; t < p.T; ++t) {
    if (t > 0 && t % p.k == 0 && p.probe) {  // timing probe: no exchange, but the flags still flush
      __syncthreads();
      if (w == 0 && changed) flush_flags(lflag, changed, t - p.k, p.k, lane);
      const int m = t / p.k;
      if (p.trace && m < kResTraceRefreshes && threadIdx.x == 0) {
        uint64_t* tr = p.trace + (int64_t(j) * kResTraceRefreshes + m) * 6;
        tr[0] = tr[1] = tr[2] = tr[3] = __builtin_amdgcn_s_memrealtime();
        tr[4] = tr[5] = __builtin_amdgcn_s_memtime();
      }
    }
    if (t > 0 && t % p.k == 0 && !p.probe) {
      // ---- refresh m: publish, signal, wait for the 8 neighbours, read ----
      const uint32_t m = uint32_t(t / p.k);
      // Opaque copies of the band geometry (see the generation step below).
      int r0 = __builtin_amdgcn_readfirstlane(w * RW), nc = __builtin_amdgcn_readfirstlane(cnt);
      int kk = __builtin_amdgcn_readfirstlane(p.k), qa = __builtin_amdgcn_readfirstlane(q0);
      int ne = __builtin_amdgcn_readfirstlane(p.ext_rows);
      asm volatile("" : "+s"(r0), "+s"(nc), "+s"(kk), "+s"(qa), "+s"(ne));
      // Exchange record of a region (words): its first k owned rows [0, 1024),
      // its last k owned rows [1024, 2048) (64 lanes each), and its last owned
      // lane's word of every band row [2048, 2048 + 16 RW).  Staged in LDS so
      // that the whole workgroup stores / loads it coalesced, all in flight.
      const BufRsrc mr = __builtin_amdgcn_make_buffer_rsrc(p.mirror[m & 1], short(0), p.nreg * kRecBytes, kBufFlags);
      uint64_t* const tr = (p.trace && m < kResTraceRefreshes && threadIdx.x == 0)
                               ? p.trace + (int64_t(j) * kResTraceRefreshes + m) * 6 : nullptr;
      if (tr) {
        tr[0] = __builtin_amdgcn_s_memrealtime();
        tr[4] = __builtin_amdgcn_s_memtime();
      }
      constexpr int kRecUsed = kRecC / 4 + kM * RW;  // words of the record this RW fills
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const int q = r0 + i - kk;  // owned-row index in the band
        if (q >= 0 && q < kk) recs[q * 64 + lane] = s[i];
        if (q >= nc - kk && q < nc && q >= 0) recs[kRecB / 4 + (q - (nc - kk)) * 64 + lane] = s[i];
        if (lane == own_cnt) recs[kRecC / 4 + r0 + i] = s[i];  // the right neighbour's halo lane
      }
      __syncthreads();
#pragma unroll
      for (int x0 = 0; x0 < kRecUsed; x0 += 64 * kM) {
        const int x = x0 + int(threadIdx.x);
        if (x0 + 64 * kM <= kRecUsed || x < kRecUsed)
          __builtin_amdgcn_raw_buffer_store_b32(recs[min(x, kRecUsed - 1)], mr, j * kRecBytes + 4 * x, 0, kCpolSc1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tr) tr[1] = __builtin_amdgcn_s_memrealtime();
      if (threadIdx.x == 0) __hip_atomic_store(p.flags + j, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0) {
        const int nn = lane < 4 ? lane : lane + 1;  // 3 x 3 neighbourhood without its centre
        const int nbd = band + nn / 3 - 1;
        const bool valid = lane < 8 && nbd >= 0 && nbd < p.nb;
        const int nst = (strip + nn % 3 - 1 + p.ns) % p.ns;
        const uint32_t* f = p.flags + (valid ? nst * p.nb + nbd : 0);
        bool done = !valid;
        const int spins = 1 << p.spin_log2;
        for (int it = 0; it < spins; ++it) {
          if (!done) done = int(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - m) >= 0;
          if (__all(done)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        if (!__all(done) && lane == 0 && p.err)
          __hip_atomic_store(p.err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (tr) tr[2] = __builtin_amdgcn_s_memrealtime();
      }
      __syncthreads();
      // Every wave has finished generations < t: wave 0 moves their flags out.
      if (w == 0 && changed) flush_flags(lflag, changed, t - p.k, p.k, lane);
      // The neighbours' records, staged the same way: halo rows above (the
      // band above's last k rows, lane 0 from the up-left region) and below
      // (the band below's first k rows, lane 0 from the down-left region),
      // then the left region's halo-lane words of every band row.
      {
        const int sl = strip > 0 ? strip - 1 : p.ns - 1;  // the strip to the left (torus)
        const int ocl = min(p.sw, p.ww - sl * p.sw);      // its last owned lane
        const int hup = band > 0 ? kk : 0, hdn = band < p.nb - 1 ? kk : 0;
        const int nrows = hup + hdn;
        const int used = 64 * nrows + kM * RW;
        uint32_t v[(kRecC / 4 + kM * 88 + 64 * kM - 1) / (64 * kM)];
#pragma unroll
        for (int u = 0; u < int(sizeof(v) / 4); ++u) {
          const int x = u * 64 * kM + int(threadIdx.x);
          int off = kOOR;
          if (x < 64 * nrows) {
            const int r = x >> 6, l = x & 63;
            const bool upr = r < hup;
            const int src = (l == 0 ? sl : strip) * p.nb + band + (upr ? -1 : 1);
            off = src * kRecBytes + 4 * ((upr ? kRecB / 4 + (r + kk - hup) * 64 : (r - hup) * 64) + (l == 0 ? ocl : l));
          } else if (x < used) {
            off = (sl * p.nb + band) * kRecBytes + kRecC + 4 * (x - 64 * nrows);
          }
          v[u] = __builtin_amdgcn_raw_buffer_load_b32(mr, off, 0, kCpolSc1);
        }
#pragma unroll
        for (int u = 0; u < int(sizeof(v) / 4); ++u) {
          const int x = u * 64 * kM + int(threadIdx.x);
          if (x < used) stage[x] = v[u];
        }
        __syncthreads();
        asm volatile("" : "+s"(r0), "+s"(nc), "+s"(kk), "+s"(qa), "+s"(ne));
#pragma unroll
        for (int i = 0; i < RW; ++i) {
          const int q = r0 + i - kk, e = qa + q;
          if (q < 0 && e >= 0) {
            s[i] = stage[(q + hup) * 64 + lane];
          } else if (q >= nc && e < ne) {
            s[i] = stage[(hup + q - nc) * 64 + lane];
          } else if (q >= 0 && q < nc) {
            const uint32_t c = stage[64 * nrows + r0 + i];
            s[i] = lane == 0 ? c : s[i];
          }
        }
      }
      if (tr) {
        tr[3] = __builtin_amdgcn_s_memrealtime();
        tr[5] = __builtin_amdgcn_s_memtime();
      }
    }
    // ---- one generation: trade edge rows with the waves above / below ----
    uint32_t* const slot = bnd + (t & 1) * (kM * 128);
    slot[w * 128 + lane] = s[0];
    slot[w * 128 + 64 + lane] = s[RW - 1];
    // Opaque copies: the per-row conditions are re-derived each generation
    // instead of being hoisted out of the loop as RW lane masks (SGPR spills).
    int lo = __builtin_amdgcn_readfirstlane(i_lo), hi = __builtin_amdgcn_readfirstlane(i_hi);
    asm volatile("" : "+s"(lo), "+s"(hi));
    uint32_t acc;
#if GOL_RES_SYNC == 1
    if (lane == 0) __hip_atomic_store(cntw + w, uint32_t(t + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    const auto edges = [&](uint32_t& above, uint32_t& below) {
      // Bounded wait for the neighbours' generation-t edge rows.
      const uint32_t want = uint32_t(t + 1);
      bool ok_up = w == 0, ok_dn = w == kM - 1;
      for (int it = 0; it < (1 << 22) && !(ok_up && ok_dn); ++it) {
        if (!ok_up) ok_up = __hip_atomic_load(cntw + w - 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= want;
        if (!ok_dn) ok_dn = __hip_atomic_load(cntw + w + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= want;
      }
      if (!(ok_up && ok_dn) && lane == 0 && p.err)
        __hip_atomic_store(p.err, 5u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t up = slot[max(w - 1, 0) * 128 + 64 + lane];
      const uint32_t dn = slot[min(w + 1, kM - 1) * 128 + lane];
      above = w > 0 ? up : 0u;
      below = w < kM - 1 ? dn : 0u;
    };
    if constexpr (RW > kTwoBodyMaxRW) {
      acc = gen_rows_split<RW, true>(s, lo, hi, edges);
    } else {
      acc = partial ? gen_rows_split<RW, true>(s, lo, hi, edges) : gen_rows_split<RW, false>(s, 0, RW, edges);
    }
#else
    __syncthreads();
    const uint32_t up = slot[max(w - 1, 0) * 128 + 64 + lane];
    const uint32_t dn = slot[min(w + 1, kM - 1) * 128 + lane];
    const uint32_t above = w > 0 ? up : 0u;
    const uint32_t below = w < kM - 1 ? dn : 0u;
    // Two bodies (masked for the few waves whose rows straddle the output
    // range) cost a second copy of the rows in registers; above 48 rows per
    // wave that would spill, so one masked body serves every wave there
    // (one more VALU op per row).
    if constexpr (RW > kTwoBodyMaxRW) {
      acc = gen_rows<RW, true>(s, above, below, lo, hi);
    } else {
      acc = partial ? gen_rows<RW, true>(s, above, below, lo, hi) : gen_rows<RW, false>(s, above, below, 0, RW);
    }
#endif
    if (rec) {
      const bool any = __ballot(own && acc != 0u) != 0;
      if (any && lane == 0) lflag[t & (kFlagWords - 1)] = 1u;
    }
  }
  __syncthreads();
  if (tr0) tr0[2] = __builtin_amdgcn_s_memrealtime();
  if (w == 0 && changed && p.T > 0) {
    const int g0 = ((p.T - 1) / p.k) * p.k;  // the generations since the last refresh
    flush_flags(lflag, changed, g0, p.T - g0, lane);
  }
  // Opaque copies again: offsets derived from eb before the loop would stay
  // live through it (RW VGPRs).
  int ef = __builtin_amdgcn_readfirstlane(eb), flo = __builtin_amdgcn_readfirstlane(i_lo);
  int fhi = __builtin_amdgcn_readfirstlane(i_hi), ipf = ip;
  asm volatile("" : "+s"(ef), "+s"(flo), "+s"(fhi), "+s"(ipf));
  const BufRsrc ro = __builtin_amdgcn_make_buffer_rsrc(p.out + base, short(0), range, kBufFlags);
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const bool ok = own && i >= flo && i < fhi;
    __builtin_amdgcn_raw_buffer_store_b32(s[i], ro, ok ? (ef + i) * ipf + vw : kOOR, 0, 0);
  }
  if (tr0) {
    tr0[3] = __builtin_amdgcn_s_memrealtime();
    tr0[5] = __builtin_amdgcn_s_memtime();
  }
}

// Every workgroup waits on its neighbours, so all of them must be resident at
// once: a cooperative launch, which the runtime refuses (instead of letting
// the waits time out) when the grid cannot be co-resident.  It does not fence
// off kernels of other streams or processes (RCCL's, another rank's), which is
// why the backend turns resident epochs off when ranks share the GPU and why
// they are experimental.
template <int RW>
void launch_resident(const ResidentParams& p, hipStream_t s) {
  static const int per_cu = [] {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, life_resident_kernel<RW>, 64 * kM, 0) != hipSuccess) b = 0;
    return b;
  }();
  GOL_REQUIRE(per_cu >= 1, "resident kernel: a workgroup does not fit a CU");
  ResidentParams arg = p;
  void* args[] = {&arg};
  const hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&life_resident_kernel<RW>),
                                                  dim3(unsigned(p.nreg)), dim3(64 * kM), args, 0, s);
  GOL_REQUIRE(e == hipSuccess, std::string("resident kernel: cooperative launch refused: ") + hipGetErrorString(e));
}

}  // namespace lr
}  // namespace hipk
}  // namespace gol

#define GOL_RESIDENT_RW(RW)                                                   \
  namespace gol {                                                             \
  namespace hipk {                                                            \
  namespace lr {                                                              \
  template void launch_resident<RW>(const ResidentParams&, hipStream_t);      \
  }                                                                           \
  }                                                                           \
  }
