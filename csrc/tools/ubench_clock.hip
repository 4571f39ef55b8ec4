// Microbenchmark: shader clock under a sustained life-kernel-like VALU load.
// Every wave runs the level-body instruction mix (bitop3 adder tree, DPP wave
// shifts, alignbit funnels) for a fixed number of iterations and stamps
// s_memtime (shader clock) and s_memrealtime (constant 100 MHz) around the
// loop; clock = d(memtime) / d(memrealtime) * 100 MHz (MI355X_MICROARCH.md,
// DVFS check).  Reports the median over waves for 1, 2 and 4 waves per SIMD.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

template <unsigned TT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}

__device__ __forceinline__ uint32_t body(uint32_t cur, uint32_t& a0, uint32_t& a1, uint32_t& b0, uint32_t& b1,
                                         uint32_t& ctr, uint32_t& acc) {
  const uint32_t lw = __builtin_amdgcn_mov_dpp(cur, 0x138, 0xF, 0xF, true);
  const uint32_t rw = __builtin_amdgcn_mov_dpp(cur, 0x130, 0xF, 0xF, true);
  const uint32_t l = __builtin_amdgcn_alignbit(cur, lw, 31), r = __builtin_amdgcn_alignbit(rw, cur, 1);
  const uint32_t h0 = bop3<0x96>(l, cur, r), h1 = bop3<0xe8>(l, cur, r);
  const uint32_t x0 = bop3<0x96>(a0, b0, h0), x1 = bop3<0xe8>(a0, b0, h0);
  const uint32_t y0 = bop3<0x96>(a1, b1, h1), y1 = bop3<0xe8>(a1, b1, h1);
  const uint32_t s3 = bop3<0x06>(y1, x1, y0), s4 = bop3<0x42>(x1, y0, y1);
  const uint32_t nxt = bop3<0xca>(x0, s3, ctr & s4);
  acc = bop3<0xf6>(acc, nxt, ctr);
  a0 = b0; a1 = b1; b0 = h0; b1 = h1; ctr = cur;
  return nxt;
}

__global__ __launch_bounds__(256) void clock_k(unsigned long long* out, int iters, uint32_t seed) {
  constexpr int N = 8;
  uint32_t cur[N], a0[N], a1[N], b0[N], b1[N], ctr[N], acc[N];
#pragma unroll
  for (int c = 0; c < N; ++c) {
    cur[c] = seed * (threadIdx.x + 3 * c + 1);
    a0[c] = cur[c] * 3; a1[c] = cur[c] * 5; b0[c] = cur[c] * 7; b1[c] = cur[c] * 9; ctr[c] = cur[c] * 11; acc[c] = 0;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < N; ++c) cur[c] = body(cur[c], a0[c], a1[c], b0[c], b1[c], ctr[c], acc[c]);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < N; ++c) s ^= acc[c] ^ cur[c];
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) {
    out[2 * wave] = t1 - t0;
    out[2 * wave + 1] = (r1 - r0) | (uint64_t(s & 1) << 63);  // keep the loop alive
  }
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned long long* out;
  const int max_waves = cus * 4 * 4;
  CHK(hipMalloc(&out, size_t(max_waves) * 16));
  std::vector<unsigned long long> h(size_t(max_waves) * 2);
  for (int wps : {1, 2, 4}) {
    const int blocks = cus * wps;  // 256 threads = one wave per SIMD per block
    const int iters = 200000;
    hipLaunchKernelGGL(clock_k, dim3(blocks), dim3(256), 0, 0, out, 1000, 7u);  // warm
    CHK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(clock_k, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const int waves = blocks * 4;
    CHK(hipMemcpy(h.data(), out, size_t(waves) * 16, hipMemcpyDeviceToHost));
    std::vector<double> mhz;
    for (int w = 0; w < waves; ++w) {
      const double dt = double(h[2 * w]), dr = double(h[2 * w + 1] & ~(1ull << 63));
      if (dr > 0) mhz.push_back(dt / dr * 100.0);
    }
    std::sort(mhz.begin(), mhz.end());
    const double bodies = double(wps) * iters * 8;  // per SIMD
    std::printf("waves/SIMD=%d  kernel %.1f ms  clock median %.0f MHz (p10 %.0f, p90 %.0f)  "
                "%.1f ns/body/SIMD = %.1f cycles at the measured clock\n",
                wps, ms, mhz[mhz.size() / 2], mhz[mhz.size() / 10], mhz[mhz.size() * 9 / 10],
                ms * 1e6 / bodies, ms * 1e6 / bodies * mhz[mhz.size() / 2] / 1e3);
  }
  return 0;
}
