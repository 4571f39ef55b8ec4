// Microbenchmark: VALU issue cost vs. source-operand count and VGPR bank
// placement (bank = VGPR index mod 4) on gfx950, using fixed registers via
// inline asm.  8 independent instructions per unrolled group, 2-8 waves/SIMD.
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

constexpr int kIters = 2048;

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", \
             "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", \
             "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71"

// Each body = 8 instructions; destinations v64..v71, sources from v40..v63.
#define BODY_BITOP3_DISTINCT                                          \
  "v_bitop3_b32 v64, v41, v42, v43 bitop3:0x96\n"                     \
  "v_bitop3_b32 v65, v45, v46, v47 bitop3:0x96\n"                     \
  "v_bitop3_b32 v66, v49, v50, v51 bitop3:0x96\n"                     \
  "v_bitop3_b32 v67, v53, v54, v55 bitop3:0x96\n"                     \
  "v_bitop3_b32 v68, v57, v58, v59 bitop3:0x96\n"                     \
  "v_bitop3_b32 v69, v61, v62, v63 bitop3:0x96\n"                     \
  "v_bitop3_b32 v70, v41, v46, v51 bitop3:0x96\n"                     \
  "v_bitop3_b32 v71, v45, v50, v55 bitop3:0x96\n"
#define BODY_BITOP3_SAMEBANK                                          \
  "v_bitop3_b32 v64, v40, v44, v48 bitop3:0x96\n"                     \
  "v_bitop3_b32 v65, v41, v45, v49 bitop3:0x96\n"                     \
  "v_bitop3_b32 v66, v42, v46, v50 bitop3:0x96\n"                     \
  "v_bitop3_b32 v67, v43, v47, v51 bitop3:0x96\n"                     \
  "v_bitop3_b32 v68, v52, v56, v60 bitop3:0x96\n"                     \
  "v_bitop3_b32 v69, v53, v57, v61 bitop3:0x96\n"                     \
  "v_bitop3_b32 v70, v54, v58, v62 bitop3:0x96\n"                     \
  "v_bitop3_b32 v71, v55, v59, v63 bitop3:0x96\n"
#define BODY_XOR2                                                     \
  "v_xor_b32 v64, v41, v42\n"                                         \
  "v_xor_b32 v65, v45, v46\n"                                         \
  "v_xor_b32 v66, v49, v50\n"                                         \
  "v_xor_b32 v67, v53, v54\n"                                         \
  "v_xor_b32 v68, v57, v58\n"                                         \
  "v_xor_b32 v69, v61, v62\n"                                         \
  "v_xor_b32 v70, v41, v46\n"                                         \
  "v_xor_b32 v71, v45, v50\n"
#define BODY_XOR3_DISTINCT                                            \
  "v_or3_b32 v64, v41, v42, v43\n"                                   \
  "v_or3_b32 v65, v45, v46, v47\n"                                   \
  "v_or3_b32 v66, v49, v50, v51\n"                                   \
  "v_or3_b32 v67, v53, v54, v55\n"                                   \
  "v_or3_b32 v68, v57, v58, v59\n"                                   \
  "v_or3_b32 v69, v61, v62, v63\n"                                   \
  "v_or3_b32 v70, v41, v46, v51\n"                                   \
  "v_or3_b32 v71, v45, v50, v55\n"
#define BODY_ALIGNBIT                                                 \
  "v_alignbit_b32 v64, v41, v42, 31\n"                                \
  "v_alignbit_b32 v65, v45, v46, 31\n"                                \
  "v_alignbit_b32 v66, v49, v50, 31\n"                                \
  "v_alignbit_b32 v67, v53, v54, 31\n"                                \
  "v_alignbit_b32 v68, v57, v58, 31\n"                                \
  "v_alignbit_b32 v69, v61, v62, 31\n"                                \
  "v_alignbit_b32 v70, v41, v46, 31\n"                                \
  "v_alignbit_b32 v71, v45, v50, 31\n"
#define BODY_DPP                                                                      \
  "v_mov_b32_dpp v64, v41 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"       \
  "v_mov_b32_dpp v65, v45 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"       \
  "v_mov_b32_dpp v66, v49 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"       \
  "v_mov_b32_dpp v67, v53 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"       \
  "v_mov_b32_dpp v68, v57 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"       \
  "v_mov_b32_dpp v69, v61 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"       \
  "v_mov_b32_dpp v70, v42 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"       \
  "v_mov_b32_dpp v71, v46 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define BODY_MOV                                                      \
  "v_mov_b32 v64, v41\n"                                              \
  "v_mov_b32 v65, v45\n"                                              \
  "v_mov_b32 v66, v49\n"                                              \
  "v_mov_b32 v67, v53\n"                                              \
  "v_mov_b32 v68, v57\n"                                              \
  "v_mov_b32 v69, v61\n"                                              \
  "v_mov_b32 v70, v42\n"                                              \
  "v_mov_b32 v71, v46\n"

#define KERNEL(NAME, BODY)                                                     \
  __global__ void NAME(uint32_t* out) {                                        \
    for (int i = 0; i < kIters; ++i) {                                         \
      asm volatile(BODY BODY BODY BODY ::: CLOB);                              \
    }                                                                          \
    if (threadIdx.x == 1234567) out[0] = 1;                                    \
  }

KERNEL(k_bitop3_distinct, BODY_BITOP3_DISTINCT)
KERNEL(k_bitop3_samebank, BODY_BITOP3_SAMEBANK)
KERNEL(k_xor2, BODY_XOR2)
KERNEL(k_xor3, BODY_XOR3_DISTINCT)
KERNEL(k_alignbit, BODY_ALIGNBIT)
KERNEL(k_dpp, BODY_DPP)
KERNEL(k_mov, BODY_MOV)

typedef void (*KFn)(uint32_t*);

void run(const char* name, KFn fn, int cus, uint32_t* out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = cus * wps;
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, out);
    CHK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, out);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double instr = double(wps) * kIters * 32 * 5;  // per SIMD
    std::printf("%-20s waves/SIMD=%d  %.3f ns per instr per SIMD  (%.2f cyc @2.3GHz)\n", name, wps,
                ms * 1e6 / instr, ms * 1e6 / instr * 2.3);
  }
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  CHK(hipMalloc(&out, 64));
  run("v_mov", k_mov, cus, out);
  run("v_xor_b32 (2 vgpr)", k_xor2, cus, out);
  run("v_or3 (3 vgpr)", k_xor3, cus, out);
  run("bitop3 distinct", k_bitop3_distinct, cus, out);
  run("bitop3 same bank", k_bitop3_samebank, cus, out);
  run("alignbit", k_alignbit, cus, out);
  run("mov_dpp wave_sh", k_dpp, cus, out);
  return 0;
}
