// Microbenchmark: ways of bringing the neighbouring lanes' edge bits into a
// lane for the life_block "level body" (hsum + rule + flag).  Baseline is two
// DPP wave shifts + two v_alignbit; the variants try VOP2-fused DPP, the VCC
// carry trick (v_add_co/v_addc with the lane mask shifted on the SALU),
// DPP ops grouped back-to-back, and ds_bpermute.
// Prints cycles per level body per SIMD (wave64, 32 cells per lane).
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

template <unsigned TT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}

constexpr uint8_t A = 0xF0, B = 0xCC, C = 0xAA;
constexpr uint8_t XOR3 = A ^ B ^ C, MAJ = (A & B) | (A & C) | (B & C), ANDN_XOR = uint8_t(~A & (B ^ C)),
                  EQ_NE = uint8_t(~(A ^ B) & (A ^ C)), SEL = uint8_t((A & B) | (~A & C)),
                  OR_XOR = uint8_t(A | (B ^ C));

// l = cell x-1, r = cell x+1 for the lane's 32 cells.
template <int V>
__device__ __forceinline__ void lr(uint32_t c, uint32_t& l, uint32_t& r) {
  if constexpr (V == 0) {  // baseline: DPP mov + alignbit
    const uint32_t lw = __builtin_amdgcn_mov_dpp(c, 0x138, 0xF, 0xF, true);
    const uint32_t rw = __builtin_amdgcn_mov_dpp(c, 0x130, 0xF, 0xF, true);
    l = __builtin_amdgcn_alignbit(c, lw, 31);
    r = __builtin_amdgcn_alignbit(rw, c, 1);
  } else if constexpr (V == 1) {  // VOP2-fusable: shifted edge bit moved by DPP, OR'd in
    l = __builtin_amdgcn_mov_dpp(c >> 31, 0x138, 0xF, 0xF, true) | (c << 1);
    r = __builtin_amdgcn_mov_dpp(c << 31, 0x130, 0xF, 0xF, true) | (c >> 1);
  } else if constexpr (V == 2) {  // carry trick for l, DPP for r
    asm volatile(
        "v_add_co_u32 %0, vcc, %1, %1\n\t"
        "s_lshl_b64 vcc, vcc, 1\n\t"
        "v_addc_co_u32 %0, vcc, 0, %0, vcc"
        : "=&v"(l)
        : "v"(c)
        : "vcc");
    const uint32_t rw = __builtin_amdgcn_mov_dpp(c, 0x130, 0xF, 0xF, true);
    r = __builtin_amdgcn_alignbit(rw, c, 1);
  } else if constexpr (V == 3) {  // carry trick both ways (lsb mask via shl+add_co)
    uint32_t t;
    asm volatile(
        "v_add_co_u32 %0, vcc, %2, %2\n\t"
        "s_lshl_b64 vcc, vcc, 1\n\t"
        "v_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
        "v_lshlrev_b32 %1, 31, %2\n\t"
        "v_add_co_u32 %1, vcc, %1, %1\n\t"
        "s_lshr_b64 vcc, vcc, 1\n\t"
        "v_cndmask_b32 %1, 0, 1, vcc"
        : "=&v"(l), "=&v"(t)
        : "v"(c)
        : "vcc");
    r = __builtin_amdgcn_alignbit(t, c, 1);
  } else if constexpr (V == 4) {  // ds_bpermute
    const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const uint32_t lw = __builtin_amdgcn_ds_bpermute((lane - 1) * 4, c);
    const uint32_t rw = __builtin_amdgcn_ds_bpermute((lane + 1) * 4, c);
    l = __builtin_amdgcn_alignbit(c, lw, 31);
    r = __builtin_amdgcn_alignbit(rw, c, 1);
  } else if constexpr (V == 5) {  // no cross-lane at all (lower bound)
    l = __builtin_amdgcn_alignbit(c, c ^ 0x1234u, 31);
    r = __builtin_amdgcn_alignbit(c ^ 0x4321u, c, 1);
  } else if constexpr (V == 6) {  // VOP3 shift-or instead of alignbit, no cross-lane
    l = (c << 1) | ((c ^ 0x1234u) >> 31);
    r = (c >> 1) | ((c ^ 0x4321u) << 31);
  }
}

template <int V>
__device__ __forceinline__ uint32_t body(uint32_t cur, uint32_t& a0, uint32_t& a1, uint32_t& b0, uint32_t& b1,
                                         uint32_t& ctr, uint32_t& acc) {
  uint32_t l, r;
  lr<V>(cur, l, r);
  const uint32_t h0 = bop3<XOR3>(l, cur, r), h1 = bop3<MAJ>(l, cur, r);
  const uint32_t x0 = bop3<XOR3>(a0, b0, h0), x1 = bop3<MAJ>(a0, b0, h0);
  const uint32_t y0 = bop3<XOR3>(a1, b1, h1), y1 = bop3<MAJ>(a1, b1, h1);
  const uint32_t s3 = bop3<ANDN_XOR>(y1, x1, y0), s4 = bop3<EQ_NE>(x1, y0, y1);
  const uint32_t nxt = bop3<SEL>(x0, s3, ctr & s4);
  acc = bop3<OR_XOR>(acc, nxt, ctr);
  a0 = b0;
  a1 = b1;
  b0 = h0;
  b1 = h1;
  ctr = cur;
  return nxt;
}

// Grouped: the 2N DPP moves of all chains issued back-to-back in one block.
template <int N>
__device__ __forceinline__ void grouped_dpp(const uint32_t (&cur)[N], uint32_t (&lw)[N], uint32_t (&rw)[N]) {
#pragma unroll
  for (int c = 0; c < N; ++c) {
    lw[c] = __builtin_amdgcn_mov_dpp(cur[c], 0x138, 0xF, 0xF, true);
    rw[c] = __builtin_amdgcn_mov_dpp(cur[c], 0x130, 0xF, 0xF, true);
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int V, int N>
__global__ __launch_bounds__(256) void bench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t cur[N], a0[N], a1[N], b0[N], b1[N], ctr[N], acc[N];
#pragma unroll
  for (int c = 0; c < N; ++c) {
    cur[c] = seed * (threadIdx.x + 3 * c + 1);
    a0[c] = cur[c] * 3;
    a1[c] = cur[c] * 5;
    b0[c] = cur[c] * 7;
    b1[c] = cur[c] * 9;
    ctr[c] = cur[c] * 11;
    acc[c] = 0;
  }
  for (int i = 0; i < iters; ++i) {
    if constexpr (V == 7) {
      uint32_t lw[N], rw[N];
      grouped_dpp<N>(cur, lw, rw);
#pragma unroll
      for (int c = 0; c < N; ++c) {
        const uint32_t l = __builtin_amdgcn_alignbit(cur[c], lw[c], 31);
        const uint32_t r = __builtin_amdgcn_alignbit(rw[c], cur[c], 1);
        const uint32_t h0 = bop3<XOR3>(l, cur[c], r), h1 = bop3<MAJ>(l, cur[c], r);
        const uint32_t x0 = bop3<XOR3>(a0[c], b0[c], h0), x1 = bop3<MAJ>(a0[c], b0[c], h0);
        const uint32_t y0 = bop3<XOR3>(a1[c], b1[c], h1), y1 = bop3<MAJ>(a1[c], b1[c], h1);
        const uint32_t s3 = bop3<ANDN_XOR>(y1, x1, y0), s4 = bop3<EQ_NE>(x1, y0, y1);
        const uint32_t nxt = bop3<SEL>(x0, s3, ctr[c] & s4);
        acc[c] = bop3<OR_XOR>(acc[c], nxt, ctr[c]);
        a0[c] = b0[c];
        a1[c] = b1[c];
        b0[c] = h0;
        b1[c] = h1;
        ctr[c] = cur[c];
        cur[c] = nxt;
      }
    } else {
#pragma unroll
      for (int c = 0; c < N; ++c) cur[c] = body<V>(cur[c], a0[c], a1[c], b0[c], b1[c], ctr[c], acc[c]);
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < N; ++c) s ^= acc[c] ^ cur[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V, int N>
void run(const char* name, int cus, uint32_t* out, double ghz) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int iters = 1024;
  for (int wps : {1, 2, 4}) {
    const int blocks = cus * wps;
    hipLaunchKernelGGL((bench<V, N>), dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
    CHK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((bench<V, N>), dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double bodies = double(wps) * iters * N * 5;  // per SIMD
    std::printf("%-34s chains=%d waves/SIMD=%d  %6.1f cyc/body\n", name, N, wps, ms * 1e6 / bodies * ghz);
  }
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double ghz = 2.4;
  uint32_t* out;
  CHK(hipMalloc(&out, size_t(cus) * 4 * 256 * 4));
  std::printf("device %s, %d CUs, cycles at %.1f GHz\n", p.gcnArchName, cus, ghz);
  run<0, 8>("V0 dpp mov + alignbit", cus, out, ghz);
  run<1, 8>("V1 dpp fused into v_or (VOP2)", cus, out, ghz);
  run<2, 8>("V2 carry trick l, dpp r", cus, out, ghz);
  run<3, 8>("V3 carry trick l and r", cus, out, ghz);
  run<4, 8>("V4 ds_bpermute", cus, out, ghz);
  run<5, 8>("V5 no cross-lane (alignbit)", cus, out, ghz);
  run<6, 8>("V6 no cross-lane (shift-or)", cus, out, ghz);
  run<7, 8>("V7 dpp grouped back-to-back", cus, out, ghz);
  run<0, 4>("V0 dpp mov + alignbit", cus, out, ghz);
  run<7, 4>("V7 dpp grouped back-to-back", cus, out, ghz);
  CHK(hipFree(out));
  return 0;
}
