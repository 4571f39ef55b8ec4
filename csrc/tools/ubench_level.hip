// Microbenchmark: cost of one life_block "level body" (hsum + rule + flag,
// 14 VALU ops) with N independent chains per wave, and variants with the
// cross-lane DPP moves and/or the v_alignbit funnel shifts replaced by
// full-rate ops, to attribute the kernel's VALU time.
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
                  EQ_NE = uint8_t(~(A ^ B) & (A ^ C)), SEL = uint8_t((A & B) | (~A & C)), OR_XOR = uint8_t(A | (B ^ C));

template <int V>
__device__ __forceinline__ uint32_t body(uint32_t cur, uint32_t& a0, uint32_t& a1, uint32_t& b0, uint32_t& b1,
                                         uint32_t& ctr, uint32_t& acc) {
  uint32_t lw, rw, l, r;
  if constexpr (V & 4) {  // ds_bpermute (LDS crossbar) instead of DPP
    const int lane = threadIdx.x & 63;
    lw = __builtin_amdgcn_ds_bpermute((lane - 1) * 4, cur);
    rw = __builtin_amdgcn_ds_bpermute((lane + 1) * 4, cur);
  } else if constexpr (V & 1) {  // no DPP
    lw = cur ^ 0x1234u;
    rw = cur ^ 0x4321u;
  } else {
    lw = __builtin_amdgcn_mov_dpp(cur, 0x138, 0xF, 0xF, true);
    rw = __builtin_amdgcn_mov_dpp(cur, 0x130, 0xF, 0xF, true);
  }
  if constexpr (V & 2) {  // no alignbit
    l = bop3<0x96>(cur, lw, a0);
    r = bop3<0x96>(rw, cur, a1);
  } else {
    l = __builtin_amdgcn_alignbit(cur, lw, 31);
    r = __builtin_amdgcn_alignbit(rw, cur, 1);
  }
  const uint32_t h0 = bop3<XOR3>(l, cur, r), h1 = bop3<MAJ>(l, cur, r);
  const uint32_t x0 = bop3<XOR3>(a0, b0, h0), x1 = bop3<MAJ>(a0, b0, h0);
  const uint32_t y0 = bop3<XOR3>(a1, b1, h1), y1 = bop3<MAJ>(a1, b1, h1);
  const uint32_t s3 = bop3<ANDN_XOR>(y1, x1, y0), s4 = bop3<EQ_NE>(x1, y0, y1);
  const uint32_t nxt = bop3<SEL>(x0, s3, ctr & s4);
  acc = bop3<OR_XOR>(acc, nxt, ctr);
  a0 = b0; a1 = b1; b0 = h0; b1 = h1; ctr = cur;
  return nxt;
}

// Two words per lane: one DPP pair serves both words.
template <int V>
__device__ __forceinline__ void body2(uint32_t& c0, uint32_t& c1, uint32_t* st) {
  uint32_t lw, rw;
  if constexpr (V & 4) {
    const int lane = threadIdx.x & 63;
    lw = __builtin_amdgcn_ds_bpermute((lane - 1) * 4, c1);
    rw = __builtin_amdgcn_ds_bpermute((lane + 1) * 4, c0);
  } else {
    lw = __builtin_amdgcn_mov_dpp(c1, 0x138, 0xF, 0xF, true);
    rw = __builtin_amdgcn_mov_dpp(c0, 0x130, 0xF, 0xF, true);
  }
  const uint32_t l0 = __builtin_amdgcn_alignbit(c0, lw, 31), r0 = __builtin_amdgcn_alignbit(c1, c0, 1);
  const uint32_t l1 = __builtin_amdgcn_alignbit(c1, c0, 31), r1 = __builtin_amdgcn_alignbit(rw, c1, 1);
  uint32_t n[2];
  const uint32_t cc[2] = {c0, c1}, ll[2] = {l0, l1}, rr[2] = {r0, r1};
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    uint32_t* q = st + 6 * w;  // a0 a1 b0 b1 ctr acc
    const uint32_t h0 = bop3<XOR3>(ll[w], cc[w], rr[w]), h1 = bop3<MAJ>(ll[w], cc[w], rr[w]);
    const uint32_t x0 = bop3<XOR3>(q[0], q[2], h0), x1 = bop3<MAJ>(q[0], q[2], h0);
    const uint32_t y0 = bop3<XOR3>(q[1], q[3], h1), y1 = bop3<MAJ>(q[1], q[3], h1);
    const uint32_t s3 = bop3<ANDN_XOR>(y1, x1, y0), s4 = bop3<EQ_NE>(x1, y0, y1);
    n[w] = bop3<SEL>(x0, s3, q[4] & s4);
    q[5] = bop3<OR_XOR>(q[5], n[w], q[4]);
    q[0] = q[2]; q[1] = q[3]; q[2] = h0; q[3] = h1; q[4] = cc[w];
  }
  c0 = n[0];
  c1 = n[1];
}

template <int V, int N>
__global__ __launch_bounds__(256) void bench2(uint32_t* out, int iters, uint32_t seed) {
  uint32_t c0[N], c1[N], st[N][12];
#pragma unroll
  for (int c = 0; c < N; ++c) {
    c0[c] = seed * (threadIdx.x + 3 * c + 1);
    c1[c] = c0[c] * 13;
#pragma unroll
    for (int k = 0; k < 12; ++k) st[c][k] = c0[c] * (k + 3);
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < N; ++c) body2<V>(c0[c], c1[c], st[c]);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < N; ++c) s ^= c0[c] ^ c1[c] ^ st[c][5] ^ st[c][11];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V, int N>
void run2(const char* name, int cus, uint32_t* out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int iters = 1024;
  for (int wps : {1, 2, 4}) {
    const int blocks = cus * wps;
    hipLaunchKernelGGL((bench2<V, N>), dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
    CHK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((bench2<V, N>), dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double words = double(wps) * iters * N * 2 * 5;  // word-bodies per SIMD
    std::printf("%-26s chains=%2d waves/SIMD=%d  %.2f ns/word-body/SIMD = %.1f cyc@2.3GHz\n", name, N, wps,
                ms * 1e6 / words, ms * 1e6 / words * 2.3);
  }
}

template <int V, int N>
__global__ __launch_bounds__(256) void bench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t cur[N], a0[N], a1[N], b0[N], b1[N], ctr[N], acc[N];
#pragma unroll
  for (int c = 0; c < N; ++c) {
    cur[c] = seed * (threadIdx.x + 3 * c + 1);
    a0[c] = cur[c] * 3; a1[c] = cur[c] * 5; b0[c] = cur[c] * 7; b1[c] = cur[c] * 9; ctr[c] = cur[c] * 11; acc[c] = 0;
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < N; ++c) cur[c] = body<V>(cur[c], a0[c], a1[c], b0[c], b1[c], ctr[c], acc[c]);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < N; ++c) s ^= acc[c] ^ cur[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V, int N>
void run(const char* name, int cus, uint32_t* out) {
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
    std::printf("%-26s chains=%2d waves/SIMD=%d  %.2f ns/body/SIMD = %.1f cyc@2.3GHz (%.2f cyc/op)\n", name, N, wps,
                ms * 1e6 / bodies, ms * 1e6 / bodies * 2.3, ms * 1e6 / bodies * 2.3 / 14);
  }
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  CHK(hipMalloc(&out, size_t(cus) * 4 * 256 * 4));
  run<0, 1>("full level body", cus, out);
  run<0, 4>("full level body", cus, out);
  run<0, 8>("full level body", cus, out);
  run<1, 8>("no DPP", cus, out);
  run<2, 8>("no alignbit", cus, out);
  run<3, 8>("no DPP, no alignbit", cus, out);
  run<4, 8>("ds_bpermute", cus, out);
  run2<0, 4>("2 words/lane DPP", cus, out);
  run2<4, 4>("2 words/lane bpermute", cus, out);
  return 0;
}
