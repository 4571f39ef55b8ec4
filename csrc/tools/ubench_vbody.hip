// Level-body microbenchmark: the production row-word bodies (adder window and
// DPP window, life_block_impl.hpp level_full) against a column-word body.
//
// Column words ("vertical" bit layout): a 32-bit word holds 32 consecutive
// ROWS of one column, a lane owns C adjacent columns, and the sweep steps
// down 32 rows at a time.  Horizontal neighbours are then the lane's own
// registers (only the lane's two edge columns need a neighbour lane, four
// DPP moves per C columns and level), and the vertical shifts are add-with-
// carry chains inside the lane: rows y-1 at bit y = v_addc(w, w, carry of
// the word above), the carry coming from the previous step's same op, so no
// SALU lane-mask shift and no funnel shift is needed.  The window is one-
// sided (rows y-2, y-1, y; the frame drifts one row per generation, realigned
// once per block by the kernel), like the adder window but rotated.
//
// Per level and column: 2 v_addc (+2 v_add_co to regenerate the carries in
// the VGPR-state variant) + 2 v_bitop3 (vertical sum) + 7 (rule) + 1 (flag);
// plus 4 DPP per C columns.  The row-word adder window: 4 VALU + 2 SALU
// (window) + 2 + 7 + 1 + 1 (AND) per word.
//
// Every variant runs `steps` steps of T levels; cells per body = 32 (one word
// of one generation).  Occupancy is fixed by dynamic LDS (N waves per SIMD).
//   ubench_vbody [steps]   ->  cycles per body per SIMD, per variant and N
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../kernels/life_block_impl.hpp"

using namespace gol;
using namespace gol::hipk;
using namespace gol::hipk::lb;

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP %s at line %d\n", hipGetErrorString(e_), __LINE__);     \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint32_t xs(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  return x ^ (x << 5);
}

// Production row-word bodies: Levels<T, 1> with the real level_full.
template <int T, int XL>
__global__ __launch_bounds__(256) void k_row(uint32_t* out, int steps) {
  using IO = BitsIO<1, XL>;
  Levels<T, 1> st;
#pragma unroll
  for (int L = 0; L < T; ++L)
#pragma unroll
    for (int s = 0; s < 3; ++s) st.h0[L][s].w[0] = st.h1[L][s].w[0] = st.cc[L][s].w[0] = st.acc[L].w[0] = 0u;
  uint32_t seed = threadIdx.x * 2654435761u + blockIdx.x;
  uint32_t sink = 0;
  for (int k = 0; k + 3 <= steps; k += 3) {
    Vec<1> a{{seed = xs(seed)}};
    sink ^= levels_full<T, IO, 0, 0, T>(st, a).w[0];
    Vec<1> b{{seed = xs(seed)}};
    sink ^= levels_full<T, IO, 1, 0, T>(st, b).w[0];
    Vec<1> c{{seed = xs(seed)}};
    sink ^= levels_full<T, IO, 2, 0, T>(st, c).w[0];
  }
#pragma unroll
  for (int L = 0; L < T; ++L) sink ^= st.acc[L].w[0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
}

// (w << 1) | carry_in; returns the carry out (w's msb) through *co.
__device__ __forceinline__ uint32_t shl_cin(uint32_t w, uint64_t cin, uint64_t* co) {
  uint32_t r;
  uint64_t c;
  asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(c) : "v"(w), "s"(cin));
  *co = c;
  return r;
}
// Lane mask of the words' msbs (carry of w + w).
__device__ __forceinline__ uint64_t msb_mask(uint32_t w) {
  uint32_t t;
  uint64_t c;
  asm("v_add_co_u32_e64 %0, %1, %2, %2" : "=v"(t), "=s"(c) : "v"(w));
  (void)t;
  return c;
}

// Column words, VGPR state (previous cells and previous 1-row shift per level
// and column; carries regenerated each step).
template <int T, int C, bool SGPR_CARRY>
__global__ __launch_bounds__(256) void k_col(uint32_t* out, int steps) {
  uint32_t pc[T][C], ps[T][C], acc[T];
  uint64_t c1[T][C], c2[T][C];
#pragma unroll
  for (int L = 0; L < T; ++L) {
    acc[L] = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      pc[L][c] = ps[L][c] = 0;
      c1[L][c] = c2[L][c] = 0;
    }
  }
  uint32_t seed = threadIdx.x * 2654435761u + blockIdx.x;
  uint32_t sink = 0;
  for (int k = 0; k < steps; ++k) {
    uint32_t cur[C];
#pragma unroll
    for (int c = 0; c < C; ++c) cur[c] = seed = xs(seed);
#pragma unroll
    for (int L = 0; L < T; ++L) {
      uint32_t v0[C + 2], v1[C + 2], s1[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        uint64_t a1 = SGPR_CARRY ? c1[L][c] : msb_mask(pc[L][c]);
        uint64_t a2 = SGPR_CARRY ? c2[L][c] : msb_mask(ps[L][c]);
        uint64_t o1, o2;
        s1[c] = shl_cin(cur[c], a1, &o1);
        const uint32_t s2 = shl_cin(s1[c], a2, &o2);
        if (SGPR_CARRY) {
          c1[L][c] = o1;
          c2[L][c] = o2;
        } else {
          pc[L][c] = cur[c];
          ps[L][c] = s1[c];
        }
        v0[c + 1] = bop3<tt::XOR3>(cur[c], s1[c], s2);
        v1[c + 1] = bop3<tt::MAJ>(cur[c], s1[c], s2);
      }
      v0[0] = __builtin_amdgcn_mov_dpp(v0[C], 0x138, 0xF, 0xF, true);  // wave_shr:1 (left lane's last column)
      v1[0] = __builtin_amdgcn_mov_dpp(v1[C], 0x138, 0xF, 0xF, true);
      v0[C + 1] = __builtin_amdgcn_mov_dpp(v0[1], 0x130, 0xF, 0xF, true);  // wave_shl:1
      v1[C + 1] = __builtin_amdgcn_mov_dpp(v1[1], 0x130, 0xF, 0xF, true);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint32_t nx = rule(v0[c], v1[c], v0[c + 1], v1[c + 1], v0[c + 2], v1[c + 2], s1[c]);
        acc[L] = bop3<tt::OR_XOR>(acc[L], nx, s1[c]);
        asm("" : "+v"(acc[L]));
        cur[c] = nx;
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) sink ^= cur[c];
  }
#pragma unroll
  for (int L = 0; L < T; ++L) sink ^= acc[L];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
}

template <class K>
static double run(K kernel, int waves_per_simd, int steps, int cus, uint32_t* out, double bodies_per_wave_step) {
  const int blocks = cus * waves_per_simd;  // 4 waves per block: one per SIMD
  // Dynamic LDS caps the co-resident blocks per CU at waves_per_simd.
  const size_t lds = size_t(160 * 1024) / size_t(waves_per_simd) - 1024;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), lds, 0, out, steps / 8);
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), lds, 0, out, steps);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipGetLastError());
  const double ghz = 2.4;
  const double cycles = double(ms) * 1e-3 * ghz * 1e9;
  const double bodies_per_simd = double(waves_per_simd) * steps * bodies_per_wave_step;
  return cycles / bodies_per_simd;
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? std::atoi(argv[1]) : 3000;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_row<8, kXlaneAdd>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  uint32_t* out = nullptr;
  CHK(hipMalloc(&out, size_t(cus) * 4 * 256 * 4 * 64));
  const auto attr = [](const void* f) {
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  };
  std::printf("cycles per level body (32 cells x 1 generation) per SIMD, at 2.4 GHz\n");
  std::printf("%-34s %8s %8s %8s\n", "variant", "1 w/SIMD", "2 w/SIMD", "4 w/SIMD");
#define ROW(T, XL, name)                                                                      \
  do {                                                                                        \
    attr(reinterpret_cast<const void*>(&k_row<T, XL>));                                       \
    std::printf("%-34s", name);                                                               \
    for (int n : {1, 2, 4}) std::printf(" %8.2f", run(k_row<T, XL>, n, steps, cus, out, T)); \
    std::printf("\n");                                                                        \
  } while (0)
#define COL(T, C, SC, name)                                                                           \
  do {                                                                                                \
    attr(reinterpret_cast<const void*>(&k_col<T, C, SC>));                                            \
    std::printf("%-34s", name);                                                                       \
    for (int n : {1, 2, 4}) std::printf(" %8.2f", run(k_col<T, C, SC>, n, steps, cus, out, T * C)); \
    std::printf("\n");                                                                                \
  } while (0)
  if (argc > 2 && std::atoi(argv[2]) == 1) {  // occupancy sweep of the row-word bodies: 1-8 waves per SIMD
    std::printf("%-34s %8s %8s %8s %8s %8s\n", "variant", "1 w", "2 w", "4 w", "6 w", "8 w");
#define ROWN(T, XL, name)                                                                                \
  do {                                                                                                   \
    attr(reinterpret_cast<const void*>(&k_row<T, XL>));                                                  \
    std::printf("%-34s", name);                                                                          \
    for (int n : {1, 2, 4, 6, 8}) std::printf(" %8.2f", run(k_row<T, XL>, n, steps, cus, out, T));     \
    std::printf("\n");                                                                                   \
  } while (0)
    ROWN(4, kXlaneAdd, "row words, adder window, T=4");
    ROWN(8, kXlaneAdd, "row words, adder window, T=8");
    ROWN(12, kXlaneAdd, "row words, adder window, T=12");
    ROWN(8, kXlaneDpp, "row words, DPP window, T=8");
    CHK(hipFree(out));
    return 0;
  }
  ROW(8, kXlaneAdd, "row words, adder window, T=8");
  ROW(8, kXlaneDpp, "row words, DPP window, T=8");
  ROW(12, kXlaneAdd, "row words, adder window, T=12");
  ROW(16, kXlaneDpp, "row words, DPP window, T=16");
  COL(8, 2, false, "column words C=2, VGPR carries, T=8");
  COL(8, 4, false, "column words C=4, VGPR carries, T=8");
  COL(8, 8, false, "column words C=8, VGPR carries, T=8");
  COL(16, 4, false, "column words C=4, VGPR carries, T=16");
  COL(4, 2, true, "column words C=2, SGPR carries, T=4");
  COL(8, 2, true, "column words C=2, SGPR carries, T=8");
  COL(4, 4, true, "column words C=4, SGPR carries, T=4");
  CHK(hipFree(out));
  return 0;
}
