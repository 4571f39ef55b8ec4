"""Generates csrc/tools/ubench_body.hip: one full B3/S23 level body (window,
horizontal sum, rule, change flag) as a dependent chain - the shape of the
temporal-blocking kernel's inner loop - for the DPP+alignbit window and the
add-with-carry window, with N independent chains either kept body-by-body
(chain-major) or interleaved instruction by instruction.  Physical registers
are named directly (clobbered) so nothing is rescheduled.  Prints cycles per
level body per SIMD at 2.4 GHz after a clock ramp."""

XOR3, MAJ, ANDN_XOR, EQ_NE, SEL, OR_XOR = 0x96, 0xE8, 0x06, 0x42, 0xCA, 0xF6


def body(kind, j):
    b = 64 + 16 * j
    c, a0, a1, b0, b1, ctr, acc, t1, t2, l1, l2, h0, h1, x0, x1, y0 = [f"v{b + k}" for k in range(16)]
    m1, m2 = f"s[{40 + 4 * j}:{41 + 4 * j}]", f"s[{42 + 4 * j}:{43 + 4 * j}]"
    bo = lambda d, x, y, z, tt: f"v_bitop3_b32 {d}, {x}, {y}, {z} bitop3:{tt:#x}"
    if kind == "dpp":
        w = [f"v_mov_b32_dpp {t1}, {c} wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
             f"v_mov_b32_dpp {t2}, {c} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
             f"v_alignbit_b32 {l1}, {c}, {t1}, 31",
             f"v_alignbit_b32 {l2}, {t2}, {c}, 1"]
    else:
        w = [f"v_add_co_u32_e64 {t1}, {m1}, {c}, {c}",
             f"v_add_co_u32_e64 {t2}, {m2}, {t1}, {t1}",
             f"s_lshl_b64 {m1}, {m1}, 1",
             f"s_lshl_b64 {m2}, {m2}, 1",
             f"v_addc_co_u32_e64 {l1}, {m1}, {t1}, 0, {m1}",
             f"v_addc_co_u32_e64 {l2}, {m2}, {l1}, {l1}, {m2}"]
    r = [bo(h0, l2, l1, c, XOR3), bo(h1, l2, l1, c, MAJ),
         bo(x0, a0, b0, h0, XOR3), bo(x1, a0, b0, h0, MAJ),
         bo(y0, a1, b1, h1, XOR3), bo(t1, a1, b1, h1, MAJ),
         bo(t2, t1, x1, y0, ANDN_XOR), bo(l2, x1, y0, t1, EQ_NE),
         f"v_and_b32_e32 {l2}, {ctr}, {l2}",
         bo(c, x0, t2, l2, SEL), bo(acc, acc, c, ctr, OR_XOR)]
    return w + r


cases = []
for kind in ("dpp", "add"):
    for n in (1, 2, 4):
        for order in ("chain-major", "interleaved"):
            if n == 1 and order == "interleaved":
                continue
            bodies = [body(kind, j) for j in range(n)]
            reps = 4 // n  # 4 bodies per asm block
            ins = []
            for _ in range(reps):
                if order == "chain-major":
                    for bd in bodies:
                        ins += bd
                else:
                    for k in range(len(bodies[0])):
                        ins += [bd[k] for bd in bodies]
            cases.append((f"{kind} chains={n} {order}", ins, 4))

out = ['''#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s line %d\\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)
#define CLOB ''' + ", ".join([f'"v{r}"' for r in range(64, 128)] + [f'"s{r}"' for r in range(40, 56)] + ['"scc"', '"vcc"']) + '''
__global__ __launch_bounds__(256) void warm(unsigned* o, int iters) {
  unsigned x = threadIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
  o[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
''']
init = " ".join(f'"v_mov_b32 v{r}, %0\\n"' for r in range(64, 128))
for k, (label, ins, nb) in enumerate(cases):
    body_s = " ".join(f'"{s}\\n"' for s in ins)
    out.append(f'''__global__ __launch_bounds__(256) void k{k}(unsigned* o, int iters) {{
  asm volatile({init} :: "v"(threadIdx.x * 2654435761u) : CLOB);
  for (int it = 0; it < iters; ++it) asm volatile({body_s} ::: CLOB);
  unsigned s; asm volatile("v_xor_b32 %0, v70, v86" : "=v"(s) :: CLOB);
  o[blockIdx.x * blockDim.x + threadIdx.x] = s;
}}
''')
out.append('''int main(){ setvbuf(stdout, nullptr, _IOLBF, 0); hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p,0)); int cus=p.multiProcessorCount;
 unsigned* o; CHK(hipMalloc(&o, size_t(cus)*8*256*4)); hipEvent_t a,b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
 for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(warm, dim3(cus*8), dim3(256), 0, 0, o, 200000);
 CHK(hipDeviceSynchronize());
 const int iters = 4096; const double ghz = 2.4;
''')
for k, (label, ins, nb) in enumerate(cases):
    out.append(f''' for (int w : {{1,2,3,4}}) {{ int blocks=cus*w; hipLaunchKernelGGL(k{k}, dim3(blocks), dim3(256),0,0,o,iters);
   CHK(hipEventRecord(a)); for(int r=0;r<4;++r) hipLaunchKernelGGL(k{k}, dim3(blocks), dim3(256),0,0,o,iters); CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
   float ms; CHK(hipEventElapsedTime(&ms,a,b)); double bodies=double(w)*iters*{nb}*4; printf("%-34s waves/SIMD=%d  %6.1f cyc/body/SIMD\\n", "{label}", w, ms*1e6/bodies*ghz); }}
''')
out.append(' return 0; }\n')
open("csrc/tools/ubench_body.hip", "w").write("".join(out))
