"""Generates csrc/tools/ubench_dpp_raw.hip: cost of a DPP wave shift as a
function of the distance (in instructions) to the VALU op that wrote its
source, alone and mixed with v_bitop3 at several ratios."""
# generates a DPP read-after-write latency microbenchmark
Ds=[1,2,3,4,6,8,12,16]
Ps=[1,2,4,8,0]   # 0 = no DPP (all bitop3)
N=48
out=[]
out.append('''#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s line %d\\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)
''')
kern=[]
for D in Ds:
    for P in Ps:
        lines=[]
        for i in range(N):
            k=i%D
            if P and i%P==0:
                lines.append(f'"v_mov_b32_dpp %{k}, %{k} wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\\n"')
            else:
                lines.append(f'"v_bitop3_b32 %{k}, %{k}, %{D}, %{k} bitop3:0x96\\n"')
        ops=", ".join(f'"+v"(r[{k}])' for k in range(D))
        name=f"k_d{D}_p{P}"
        out.append(f'''__global__ __launch_bounds__(256) void {name}(unsigned* o, int iters) {{
  unsigned r[{D}]; unsigned c = threadIdx.x * 7u + 1u;
  for (int k = 0; k < {D}; ++k) r[k] = threadIdx.x * (k + 3u);
  for (int it = 0; it < iters; ++it) {{
    asm volatile({" ".join(lines)} : {ops} : "v"(c));
  }}
  unsigned s = 0; for (int k = 0; k < {D}; ++k) s ^= r[k];
  o[blockIdx.x * blockDim.x + threadIdx.x] = s;
}}
''')
        kern.append((name,D,P))
out.append('''int main(){ hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p,0)); int cus=p.multiProcessorCount;
 unsigned* o; CHK(hipMalloc(&o, size_t(cus)*8*256*4)); hipEvent_t a,b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
 const int iters=4096; const double ghz=2.4;
''')
for name,D,P in kern:
    out.append(f''' for (int w : {{1,2,4}}) {{ int blocks=cus*w; hipLaunchKernelGGL({name}, dim3(blocks), dim3(256),0,0,o,iters);
   CHK(hipEventRecord(a)); for(int r=0;r<3;++r) hipLaunchKernelGGL({name}, dim3(blocks), dim3(256),0,0,o,iters); CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
   float ms; CHK(hipEventElapsedTime(&ms,a,b)); double ins=double(w)*iters*{N}*3; printf("dist=%2d dpp_every=%d waves/SIMD=%d  %.2f cyc/instr/SIMD\\n", {D}, {P}, w, ms*1e6/ins*ghz); }}
''')
out.append(' return 0; }\n')
open('csrc/tools/ubench_dpp_raw.hip','w').write("".join(out))
