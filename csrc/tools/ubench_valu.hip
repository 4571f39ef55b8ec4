// Microbenchmark: throughput of the VALU instructions the life_block kernel
// is built from (v_bitop3_b32, v_alignbit_b32, DPP wave/row shifts), at 1-8
// waves per SIMD with 8 independent dependency chains per wave.
// Prints cycles per wave-instruction per SIMD (2.0 = full rate for wave64 on
// a SIMD32).  Build: hipcc --offload-arch=gfx950 -O3 ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

constexpr int kIters = 4096;
constexpr int kChains = 8;

template <int OP>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b) {
  if constexpr (OP == 0) return __builtin_amdgcn_bitop3_b32(a, b, a ^ 0x55u, 0x96);
  if constexpr (OP == 1) return __builtin_amdgcn_alignbit(a, b, 31);
  if constexpr (OP == 2) return __builtin_amdgcn_mov_dpp(a, 0x138, 0xF, 0xF, true) + b;  // wave_shr
  if constexpr (OP == 3) return __builtin_amdgcn_mov_dpp(a, 0x111, 0xF, 0xF, true) + b;  // row_shr:1
  if constexpr (OP == 4) return a + b;                                                  // v_add baseline
  if constexpr (OP == 5) return __builtin_amdgcn_mov_dpp(a, 0x130, 0xF, 0xF, true) + b;  // wave_shl
  return a;
}

template <int OP, bool DEP>
__global__ void bench(uint32_t* out, uint32_t seed) {
  uint32_t x[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) x[c] = seed * (threadIdx.x + c + 1);
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (DEP)
        x[0] = op<OP>(x[0], x[c]);
      else
        x[c] = op<OP>(x[c], x[(c + 1) % kChains]);
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP, bool DEP>
void run(const char* name, int cus, uint32_t* out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int wps : {1, 2, 4, 8}) {
    // one block = 4 waves (one per SIMD); wps blocks per CU
    const int blocks = cus * wps;
    hipLaunchKernelGGL((bench<OP, DEP>), dim3(blocks), dim3(256), 0, 0, out, 7u);
    CHK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((bench<OP, DEP>), dim3(blocks), dim3(256), 0, 0, out, 7u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    // instructions per SIMD: wps waves * iters * chains (the op may be 2 instrs for dpp+add)
    const double instr = double(wps) * kIters * kChains * 5;
    const double cyc = ms * 1e-3 * 2.4e9 / instr;
    std::printf("%-28s %-4s waves/SIMD=%d  %.2f cycles per op per SIMD (at 2.4GHz)\n", name,
                DEP ? "dep" : "ind", wps, cyc);
  }
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  CHK(hipMalloc(&out, size_t(cus) * 8 * 256 * 4));
  std::printf("device %s, %d CUs\n", p.gcnArchName, cus);
  run<4, false>("v_add_u32", cus, out);
  run<0, false>("v_bitop3_b32", cus, out);
  run<0, true>("v_bitop3_b32", cus, out);
  run<1, false>("v_alignbit_b32", cus, out);
  run<2, false>("dpp wave_shr + v_add", cus, out);
  run<5, false>("dpp wave_shl + v_add", cus, out);
  run<3, false>("dpp row_shr + v_add", cus, out);
  run<2, true>("dpp wave_shr + v_add", cus, out);
  CHK(hipFree(out));
  return 0;
}
