// Tile utility kernels: periodic halo fill, alive reduction, host-format
// conversion and counter-based random init.
//
// Reference equivalents: halo_rows / halo_cols (src/game_cuda.cu:52-74, one
// 32-thread block per 32 cells, called every generation with a device sync)
// and the empty() reduction (src/game_cuda.cu:102-126: 32-int shared-memory
// tree + int atomicAdd, covering only ~3% of the grid for W > 64, quirks
// Q9/Q19).  Here the halo fill runs once per epoch of Dv generations, the
// reduction is a wave64 reduction with 64-bit counts over every owned cell,
// and all loops are grid-stride with 256-thread (4 x wave64) blocks.
#include <hip/hip_runtime.h>

#include "gol/backend.hpp"
#include "life_kernels.hpp"

namespace gol {
namespace hipk {
namespace {

constexpr int kBlock = 256;

inline unsigned grid_for(int64_t n, int64_t cap = 256 * 8 * 4) {
  return unsigned(std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, kBlock), cap)));
}

__device__ __forceinline__ int64_t pmod(int64_t x, int64_t m) {
  int64_t r = x % m;
  return r < 0 ? r + m : r;
}

__global__ void fill_cols_bits(uint32_t* buf, int64_t pitch_w, int64_t row0, int64_t H, int hw,
                               int64_t ow) {
  const int64_t nh = 2 * int64_t(hw);
  const int64_t n = H * nh;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / nh, j = t - i * nh;
    const int64_t c = j < hw ? j : ow + j;  // left halo words, then right ones
    uint32_t* row = buf + (row0 + i) * pitch_w;
    row[c] = row[hw + pmod(c - hw, ow)];
  }
}

__global__ void fill_cols_u8(uint8_t* buf, int64_t pitch, int64_t row0, int64_t H, int64_t c0,
                             int64_t W) {
  const int64_t nh = 2 * c0;
  const int64_t n = H * nh;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / nh, j = t - i * nh;
    const int64_t x = j < c0 ? j : W + j;  // [0,c0) then [c0+W, 2c0+W)
    uint8_t* row = buf + (row0 + i) * pitch;
    row[x] = row[c0 + pmod(x - c0, W)];
  }
}

__global__ void fill_rows_k(uint4* buf, int64_t pitch16, int64_t Dv, int64_t H) {
  const int64_t n = 2 * Dv * pitch16;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t hr = t / pitch16, x = t - hr * pitch16;
    const int64_t r = hr < Dv ? hr : H + hr;  // top halo rows, then bottom ones
    const int64_t src = Dv + pmod(r - Dv, H);
    buf[r * pitch16 + x] = buf[src * pitch16 + x];
  }
}

// Both periodic fills of a single-rank bit tile in one launch: the column
// halos of the owned rows, and the Dv halo rows on each side copied over the
// full pitch with the column wrap applied on the fly (so corners come out as
// after fill_cols_bits + fill_rows_k).  Every read is an owned word of an
// owned row, never a word this launch writes, so there is no ordering hazard.
// One launch per epoch instead of two (each ~4.6 us; rocprof_marker_bench).
__global__ void fill_all_bits(uint32_t* buf, int64_t pitch_w, int64_t Dv, int64_t H, int hw,
                              int64_t ow) {
  const int64_t nrow = 2 * Dv * pitch_w;  // halo rows, whole pitch
  const int64_t nh = 2 * int64_t(hw);
  const int64_t n = nrow + H * nh;       // + column halos of the owned rows
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n;
       t += int64_t(gridDim.x) * blockDim.x) {
    int64_t r, c, src_r;
    if (t < nrow) {
      const int64_t hr = t / pitch_w;
      c = t - hr * pitch_w;
      r = hr < Dv ? hr : H + hr;  // top halo rows, then bottom ones
      src_r = Dv + pmod(r - Dv, H);
    } else {
      const int64_t u = t - nrow, i = u / nh, j = u - i * nh;
      c = j < hw ? j : ow + j;  // left halo words, then right ones
      r = src_r = Dv + i;
    }
    const int64_t src_c = (c < hw || (c >= hw + ow && c < 2 * hw + ow)) ? hw + pmod(c - hw, ow) : c;
    buf[r * pitch_w + c] = buf[src_r * pitch_w + src_c];
  }
}

__global__ void alive_k(const uint8_t* buf, int64_t pitch, int64_t row0, int64_t H,
                        int64_t byte0, int64_t nbytes, uint32_t* any_flag,
                        unsigned long long* count) {
  // Owned span of each row: [byte0, byte0 + nbytes); 4-byte chunks, the last
  // one masked.  Bits layout: popcount of words; U8: bytes are 0/1, so the
  // popcount of a 4-byte chunk is its live-cell count.
  const int64_t chunks = ceil_div(nbytes, 4);
  const int64_t n = H * chunks;
  unsigned long long local = 0;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / chunks, j = t - i * chunks;
    const uint8_t* p = buf + (row0 + i) * pitch + byte0 + 4 * j;
    uint32_t v = *reinterpret_cast<const uint32_t*>(p);
    const int64_t rem = nbytes - 4 * j;
    if (rem < 4) v &= (1u << (8 * rem)) - 1u;
    local += __popc(v);
  }
  // wave64 reduction, one atomic per wave
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0 && local) {
    if (count) atomicAdd(count, local);
    if (any_flag) *any_flag = 1u;  // idempotent: no atomic needed
  }
}

__global__ void load_rows_bits(uint32_t* buf, int64_t pitch_w, int64_t first_row, int hw, int64_t ow,
                               const uint8_t* stage, int64_t ld, int64_t n) {
  const int64_t total = n * ow;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / ow, c = t - i * ow;
    const uint8_t* s = stage + i * ld + 32 * c;
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) w |= uint32_t(s[j] == 1 || s[j] == '1') << j;
    buf[(first_row + i) * pitch_w + hw + c] = w;
  }
}

__global__ void load_rows_u8(uint8_t* buf, int64_t pitch, int64_t first_row, int64_t c0, int64_t W,
                             const uint8_t* stage, int64_t ld, int64_t n) {
  const int64_t total = n * W;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / W, x = t - i * W;
    const uint8_t b = stage[i * ld + x];
    buf[(first_row + i) * pitch + c0 + x] = uint8_t(b == 1 || b == '1');
  }
}

__global__ void store_rows_k(const uint8_t* buf, int64_t pitch, int64_t first_row, int64_t c0,
                             int64_t W, bool bits, uint8_t* stage, int64_t ld, int64_t n,
                             uint8_t base) {
  const int64_t total = n * W;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / W, x = t - i * W;
    const uint8_t* row = buf + (first_row + i) * pitch;
    uint8_t v;
    if (bits) {
      const int64_t cell = c0 + x;
      v = uint8_t((reinterpret_cast<const uint32_t*>(row)[cell / 32] >> (cell % 32)) & 1u);
    } else {
      v = row[c0 + x] != 0;
    }
    stage[i * ld + x] = uint8_t(base + v);
  }
}

__global__ void init_random_bits(uint32_t* buf, int64_t pitch_w, int64_t row0, int hw, int64_t H,
                                 int64_t ow, uint64_t seed, uint32_t th, int64_t grow0,
                                 int64_t gcol0) {
  const int64_t total = H * ow;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / ow, c = t - i * ow;
    uint32_t w = 0;
    for (int j = 0; j < 32; ++j) w |= uint32_t(rng_cell(seed, grow0 + i, gcol0 + 32 * c + j, th)) << j;
    buf[(row0 + i) * pitch_w + hw + c] = w;
  }
}

__global__ void init_random_u8(uint8_t* buf, int64_t pitch, int64_t row0, int64_t c0, int64_t H,
                               int64_t W, uint64_t seed, uint32_t th, int64_t grow0, int64_t gcol0) {
  const int64_t total = H * W;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total;
       t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / W, x = t - i * W;
    buf[(row0 + i) * pitch + c0 + x] = uint8_t(rng_cell(seed, grow0 + i, gcol0 + x, th));
  }
}

__global__ void i64_k(int64_t* p, int64_t v, int add) { *p = add ? *p + v : v; }

// Stream wait on a device counter (the boundary trigger, Backend::
// trigger_stream): one wave whose lane 0 polls *counter >= target, sleeping
// s_sleep 127 (~3.4 us) between polls, so the wave that holds the stream
// costs the launches beside it almost no issue slots (ROCm's
// hipStreamWaitValue64 kernel polled hard enough to slow the linked launches
// around it by ~36 us per epoch, profiles/r06/).  Bounded (~4 s): it gives up
// with the error word's code 7 instead of holding the stream forever.
__global__ void wait_counter_k(const unsigned long long* counter, unsigned long long target, uint32_t* err) {
  if (threadIdx.x != 0) return;
  for (int spin = 0; spin < (1 << 20); ++spin) {
    if (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      return;
    }
    __builtin_amdgcn_s_sleep(127);
  }
  if (err) __hip_atomic_store(err, 7u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Undo the adder window's storage drift (life_kernels.hpp kXlaneAdd): owned
// word k of the output row is cells [32k, 32k+32) of the true frame, which
// the drifted input holds at cells [32k + s, 32k + s + 32) (mod W).
__global__ void rotate_cols_bits(const uint32_t* in, uint32_t* out, int64_t pitch_w, int64_t row0, int64_t H,
                                 int hw, int64_t ow, int64_t s) {
  const int64_t q0 = s / 32;
  const int sh = int(s % 32);
  const int64_t n = H * ow;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n; t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / ow, k = t - i * ow;
    const uint32_t* row = in + (row0 + i) * pitch_w + hw;
    int64_t q = k + q0;
    if (q >= ow) q -= ow;
    const uint32_t lo = row[q];
    const uint32_t hi = row[q + 1 == ow ? 0 : q + 1];
    out[(row0 + i) * pitch_w + hw + k] = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
  }
}

__global__ void rotate_cols_u8(const uint8_t* in, uint8_t* out, int64_t pitch, int64_t row0, int64_t H, int64_t c0,
                               int64_t W, int64_t s) {
  const int64_t n = H * W;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n; t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / W, x = t - i * W;
    int64_t y = x + s;
    if (y >= W) y -= W;
    out[(row0 + i) * pitch + c0 + x] = in[(row0 + i) * pitch + c0 + y];
  }
}

// Byte cells <-> bit words (one 32-cell word per thread, two 16-byte loads or
// stores).  Four cells at a time: the 0/1 bytes of a dword are gathered into
// its top nibble by one multiply (byte k lands on bit 24 + k), and a nibble is
// spread back over four bytes by the inverse multiply (disjoint shifts 0, 7,
// 14, 21, so no carries).
__device__ __forceinline__ uint32_t nibble_of(uint32_t v) {
  v = ((v & 0x7f7f7f7fu) + 0x7f7f7f7fu) | v;  // any nonzero byte -> top bit set
  return (((v >> 7) & 0x01010101u) * 0x01020408u) >> 24;
}
__device__ __forceinline__ uint32_t bytes_of(uint32_t n) { return ((n & 0xfu) * 0x00204081u) & 0x01010101u; }

// Owned cells only: `src`/`dst` point at owned row 0, owned word 0 of each
// geometry (the two may differ in halo rows, halo words and pitch).
__global__ void pack_rows_k(const uint8_t* u8, int64_t pitch, uint32_t* bits, int64_t pitch_w, int64_t nrows,
                            int64_t ow) {
  const int64_t n = nrows * ow;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n; t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / ow, k = t - i * ow;
    const uint4* src = reinterpret_cast<const uint4*>(u8 + i * pitch + 32 * k);
    const uint4 a = src[0], b = src[1];
    const uint32_t w = nibble_of(a.x) | nibble_of(a.y) << 4 | nibble_of(a.z) << 8 | nibble_of(a.w) << 12 |
                       nibble_of(b.x) << 16 | nibble_of(b.y) << 20 | nibble_of(b.z) << 24 | nibble_of(b.w) << 28;
    bits[i * pitch_w + k] = w;
  }
}

__global__ void unpack_rows_k(const uint32_t* bits, int64_t pitch_w, uint8_t* u8, int64_t pitch, int64_t nrows,
                              int64_t ow) {
  const int64_t n = nrows * ow;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < n; t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = t / ow, k = t - i * ow;
    const uint32_t w = bits[i * pitch_w + k];
    uint4* dst = reinterpret_cast<uint4*>(u8 + i * pitch + 32 * k);
    dst[0] = make_uint4(bytes_of(w), bytes_of(w >> 4), bytes_of(w >> 8), bytes_of(w >> 12));
    dst[1] = make_uint4(bytes_of(w >> 16), bytes_of(w >> 20), bytes_of(w >> 24), bytes_of(w >> 28));
  }
}

}  // namespace

void launch_convert_rows(const uint8_t* src, const TileGeom& gs, uint8_t* dst, const TileGeom& gd, int64_t i0,
                         int64_t nrows, hipStream_t s) {
  GOL_REQUIRE(gs.layout != gd.layout, "convert_rows: layouts must differ");
  GOL_REQUIRE(gs.H == gd.H && gs.W == gd.W && gs.W % 32 == 0, "convert_rows: geometries differ");
  GOL_REQUIRE(i0 >= 0 && nrows >= 0 && i0 + nrows <= gs.H, "convert_rows: rows out of range");
  GOL_REQUIRE(gs.cell0() % 32 == 0 && gd.cell0() % 32 == 0 && gs.pitch % 16 == 0 && gd.pitch % 16 == 0,
              "convert_rows: owned words must be 16-byte aligned");
  if (nrows == 0) return;
  const int64_t ow = gs.W / 32;
  const uint8_t* a = src + gs.offset(gs.row0() + i0, gs.cell0());
  uint8_t* b = dst + gd.offset(gd.row0() + i0, gd.cell0());
  if (gs.layout == Layout::U8)
    hipLaunchKernelGGL(pack_rows_k, dim3(grid_for(nrows * ow, 1 << 16)), dim3(kBlock), 0, s, a, gs.pitch,
                       reinterpret_cast<uint32_t*>(b), gd.pitch / 4, nrows, ow);
  else
    hipLaunchKernelGGL(unpack_rows_k, dim3(grid_for(nrows * ow, 1 << 16)), dim3(kBlock), 0, s,
                       reinterpret_cast<const uint32_t*>(a), gs.pitch / 4, b, gd.pitch, nrows, ow);
}

void launch_i64(int64_t* p, int64_t v, bool add, hipStream_t s) {
  hipLaunchKernelGGL(i64_k, dim3(1), dim3(1), 0, s, p, v, add ? 1 : 0);
}

void launch_wait_counter(const unsigned long long* counter, unsigned long long target, uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(wait_counter_k, dim3(1), dim3(64), 0, s, counter, target, err);
}

void launch_fill_cols(uint8_t* buf, const TileGeom& g, hipStream_t s) {
  launch_fill_cols_rows(buf, g, g.row0(), g.H, s);
}

void launch_fill_cols_rows(uint8_t* buf, const TileGeom& g, int64_t r0, int64_t nrows, hipStream_t s) {
  if (g.hw == 0 || nrows <= 0) return;
  if (g.layout == Layout::Bits) {
    const int64_t n = nrows * 2 * g.hw;
    hipLaunchKernelGGL(fill_cols_bits, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       reinterpret_cast<uint32_t*>(buf), g.pitch / 4, r0, nrows, g.hw, g.W / 32);
  } else {
    const int64_t n = nrows * 2 * g.cell0();
    hipLaunchKernelGGL(fill_cols_u8, dim3(grid_for(n)), dim3(kBlock), 0, s, buf, g.pitch, r0, nrows,
                       g.cell0(), g.W);
  }
}

void launch_fill_rows(uint8_t* buf, const TileGeom& g, hipStream_t s) {
  if (g.Dv == 0) return;
  const int64_t n = 2 * int64_t(g.Dv) * (g.pitch / 16);
  hipLaunchKernelGGL(fill_rows_k, dim3(grid_for(n)), dim3(kBlock), 0, s, reinterpret_cast<uint4*>(buf),
                     g.pitch / 16, int64_t(g.Dv), g.H);
}

bool launch_fill_all(uint8_t* buf, const TileGeom& g, hipStream_t s) {
  if (g.layout != Layout::Bits || g.hw == 0 || g.Dv == 0 || g.pitch % 4) return false;
  const int64_t pitch_w = g.pitch / 4;
  const int64_t n = 2 * int64_t(g.Dv) * pitch_w + g.H * 2 * g.hw;
  hipLaunchKernelGGL(fill_all_bits, dim3(grid_for(n)), dim3(kBlock), 0, s, reinterpret_cast<uint32_t*>(buf),
                     pitch_w, int64_t(g.Dv), g.H, g.hw, g.W / 32);
  return true;
}

void launch_alive(const uint8_t* buf, const TileGeom& g, uint32_t* any_flag,
                  unsigned long long* count, hipStream_t s) {
  const int64_t byte0 = g.offset(0, g.cell0());
  const int64_t nbytes = g.span_bytes(g.W);
  const int64_t n = g.H * ceil_div(nbytes, 4);
  hipLaunchKernelGGL(alive_k, dim3(grid_for(n)), dim3(kBlock), 0, s, buf, g.pitch, int64_t(g.row0()),
                     g.H, byte0, nbytes, any_flag, count);
}

void launch_load_rows(uint8_t* buf, const TileGeom& g, const uint8_t* stage, int64_t ld, int64_t r0,
                      int64_t n, hipStream_t s) {
  if (g.layout == Layout::Bits) {
    hipLaunchKernelGGL(load_rows_bits, dim3(grid_for(n * (g.W / 32))), dim3(kBlock), 0, s,
                       reinterpret_cast<uint32_t*>(buf), g.pitch / 4, g.row0() + r0, g.hw, g.W / 32,
                       stage, ld, n);
  } else {
    hipLaunchKernelGGL(load_rows_u8, dim3(grid_for(n * g.W)), dim3(kBlock), 0, s, buf, g.pitch,
                       g.row0() + r0, g.cell0(), g.W, stage, ld, n);
  }
}

void launch_store_rows(const uint8_t* buf, const TileGeom& g, uint8_t* stage, int64_t ld, int64_t r0,
                       int64_t n, bool ascii, hipStream_t s) {
  hipLaunchKernelGGL(store_rows_k, dim3(grid_for(n * g.W)), dim3(kBlock), 0, s, buf, g.pitch,
                     g.row0() + r0, g.cell0(), g.W, g.layout == Layout::Bits, stage, ld, n,
                     uint8_t(ascii ? '0' : 0));
}

void launch_init_random(uint8_t* buf, const TileGeom& g, uint64_t seed, uint32_t th, int64_t grow0,
                        int64_t gcol0, hipStream_t s) {
  if (g.layout == Layout::Bits) {
    hipLaunchKernelGGL(init_random_bits, dim3(grid_for(g.H * (g.W / 32))), dim3(kBlock), 0, s,
                       reinterpret_cast<uint32_t*>(buf), g.pitch / 4, int64_t(g.row0()), g.hw, g.H,
                       g.W / 32, seed, th, grow0, gcol0);
  } else {
    hipLaunchKernelGGL(init_random_u8, dim3(grid_for(g.H * g.W)), dim3(kBlock), 0, s, buf, g.pitch,
                       int64_t(g.row0()), g.cell0(), g.H, g.W, seed, th, grow0, gcol0);
  }
}

void launch_rotate_cols(const uint8_t* src, uint8_t* dst, const TileGeom& g, int64_t shift, hipStream_t s) {
  GOL_REQUIRE(src != dst, "rotate_cols: source and destination must differ");
  shift = ((shift % g.W) + g.W) % g.W;
  if (g.layout == Layout::Bits) {
    GOL_REQUIRE(g.W % 32 == 0, "rotate_cols: bit layout needs width % 32 == 0");
    hipLaunchKernelGGL(rotate_cols_bits, dim3(grid_for(g.H * (g.W / 32))), dim3(kBlock), 0, s,
                       reinterpret_cast<const uint32_t*>(src), reinterpret_cast<uint32_t*>(dst), g.pitch / 4,
                       int64_t(g.row0()), g.H, g.hw, g.W / 32, shift);
  } else {
    hipLaunchKernelGGL(rotate_cols_u8, dim3(grid_for(g.H * g.W)), dim3(kBlock), 0, s, src, dst, g.pitch,
                       int64_t(g.row0()), g.H, g.cell0(), g.W, shift);
  }
}

}  // namespace hipk
}  // namespace gol
