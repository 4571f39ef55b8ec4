"""Generates csrc/tools/ubench_dpp_mix.hip: what a DPP wave shift costs inside
a v_bitop3 stream, as a function of its source/destination VGPR banks and of
the distance to the instruction that wrote its source / reads its result.
Physical VGPRs v64..v127 are named directly (clobbered), so register banks
(index mod 4) are fixed.  Each pattern is 48 instructions = 6 x (1 DPP + 7
v_bitop3); cycles are per instruction per SIMD at 2.4 GHz after a clock ramp."""
N = 48


def dpp(d, s):
    return f"v_mov_b32_dpp v{d}, v{s} wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"


def bop(d, a, b, c):
    return f"v_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x96"


pats = []  # (label, [instr])


def pure_bop():
    ins = []
    for i in range(N):
        r = 80 + (i % 12)
        ins.append(bop(r, r, 96, 97))
    return ins


pats.append(("bitop3 only (12 independent chains)", pure_bop()))

# A: DPP source never written in the loop (no RAW), vary src/dst bank.
for sb in range(4):
    for db in range(4):
        ins = []
        for g in range(N // 8):
            ins.append(dpp(64 + 4 * (g % 2) + db + 8, 64 + sb))
            for j in range(7):
                r = 80 + (7 * g + j) % 12
                ins.append(bop(r, r, 96, 97))
        pats.append((f"A no-RAW dpp src bank {sb} dst bank {db}", ins))

# B: DPP source written by a bitop3 `dist` instructions earlier (1..7).
for dist in (1, 2, 3, 4, 7):
    ins = []
    for g in range(N // 8):
        blk = []
        src = 100 + 4 * (g % 2)  # bank 0
        for j in range(7):
            r = 80 + (7 * g + j) % 12
            if j == 7 - dist:
                blk.append(bop(src, r, 96, 97))
            else:
                blk.append(bop(r, r, 96, 97))
        ins.extend(blk)
        ins.append(dpp(110 + (g % 2) * 4, src))
    pats.append((f"B dpp reads a bitop3 result {dist} instr earlier", ins))

# C: DPP result read by a bitop3 `dist` instructions later (1..7).
for dist in (1, 2, 3, 4, 7):
    ins = []
    for g in range(N // 8):
        dst = 110 + (g % 2) * 4
        ins.append(dpp(dst, 64))
        for j in range(1, 8):
            r = 80 + (7 * g + j) % 12
            if j == dist:
                ins.append(bop(r, dst, 96, r))
            else:
                ins.append(bop(r, r, 96, 97))
    pats.append((f"C dpp result read by a bitop3 {dist} instr later", ins))

# D: kernel-like: 2 DPPs (shr, shl) of the same fresh value per 15 ops.
ins = []
for g in range(3):
    src = 100 + g
    blk = [bop(src, src, 96, 97)]
    blk.append(dpp(110 + g, src))
    blk.append(dpp(114 + g, src).replace("wave_shr", "wave_shl"))
    for j in range(13):
        r = 80 + (13 * g + j) % 12
        blk.append(bop(r, r, 96, 97))
    ins.extend(blk)
pats.append(("D 2 dpp right after their producer + 13 bitop3", ins))


# F: run-1 style in-place chains: n registers in rotation, every instruction
# rewrites the register of its slot; DPP (in place) every P instructions.
for n in (2, 3, 4, 5, 6, 8, 12):
    for P in (4, 8):
        ins = []
        for i in range(N):
            r = 80 + i % n
            ins.append(dpp(r, r) if i % P == 0 else bop(r, r, 96, r))
        pats.append((f"F in-place n={n} dpp every {P}", ins))
# G: same rotation, DPP reads a register never written in the loop.
for n in (4, 8):
    ins = []
    for i in range(N):
        r = 80 + i % n
        ins.append(dpp(r, 64) if i % 8 == 0 else bop(r, r, 96, r))
    pats.append((f"G n={n} dpp from a constant reg every 8", ins))
# H: same rotation, DPP writes a register never read in the loop.
for n in (4, 8):
    ins = []
    for i in range(N):
        r = 80 + i % n
        ins.append(dpp(64, r) if i % 8 == 0 else bop(r, r, 96, r))
    pats.append((f"H n={n} dpp into a dead reg every 8", ins))
# I: pure bitop3 with n-register rotation (reference for F).
for n in (4, 8):
    ins = [bop(80 + i % n, 80 + i % n, 96, 80 + i % n) for i in range(N)]
    pats.append((f"I bitop3 only n={n}", ins))


# J: candidate DPP-free ways to move a lane's edge bit: VOPC compares and
# add-with-carry writing lane masks to SGPR pairs, SALU shifts of those masks.
def grp(first, nb=7):
    ins = []
    for g in range(N // (len(first) + nb)):
        ins += [f.format(g=g, s=40 + 2 * (g % 4), t=48 + 2 * (g % 4), x=100 + g % 4, y=104 + g % 4) for f in first]
        for j in range(nb):
            r = 80 + ((nb * g + j) % 12)
            ins.append(bop(r, r, 96, 97))
    return ins
J = {
    "v_cmp_lt_i32_e64": ["v_cmp_lt_i32_e64 s[{s}:{s1}], v{x}, 0"],
    "v_add_co_u32_e64": ["v_add_co_u32_e64 v{y}, s[{s}:{s1}], v{x}, v{x}"],
    "v_addc_co_u32_e64": ["v_addc_co_u32_e64 v{y}, s[{t}:{t1}], v{x}, v{x}, s[{s}:{s1}]"],
    "v_alignbit_b32": ["v_alignbit_b32 v{y}, v{x}, v{y}, 31"],
    "v_cndmask_b32_e64": ["v_cndmask_b32_e64 v{y}, v{x}, v{y}, s[{s}:{s1}]"],
    "v_lshlrev_b32": ["v_lshlrev_b32 v{y}, 1, v{x}"],
    "v_lshl_or_b32": ["v_lshl_or_b32 v{y}, v{x}, 1, v{y}"],
    "s_lshl_b64": ["s_lshl_b64 s[{s}:{s1}], s[{s}:{s1}], 1"],
    "v_mov_b32 (VOP1)": ["v_mov_b32 v{y}, v{x}"],
}
for name, f in J.items():
    f = [x.replace("{s1}", "{s1}") for x in f]
    ins = grp([x.replace("{s1}", "SONE").replace("{t1}", "TONE") for x in f])
    ins = [i for i in ins]
    pats.append((f"J 1 {name} + 7 bitop3", ins))
# K: the full DPP-free left window for one word: cmp, s_lshl, addc, cmp,
# s_lshl, addc (+ 10 bitop3 = the rest of a level body), 3 per 48.
k = ["v_cmp_lt_i32_e64 s[{s}:SONE], v{x}, 0", "s_lshl_b64 s[{s}:SONE], s[{s}:SONE], 1",
     "v_addc_co_u32_e64 v{y}, s[{t}:TONE], v{x}, v{x}, s[{s}:SONE]",
     "v_cmp_lt_i32_e64 s[{s}:SONE], v{y}, 0", "s_lshl_b64 s[{s}:SONE], s[{s}:SONE], 1",
     "v_addc_co_u32_e64 v{y}, s[{t}:TONE], v{y}, v{y}, s[{s}:SONE]"]
pats.append(("K carry window (4 VALU + 2 SALU) + 10 bitop3", grp(k, 10)))
# K2: same body with the 2 DPP + 2 alignbit window (today's kernel).
k2 = ["v_mov_b32_dpp v{y}, v{x} wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
      "v_alignbit_b32 v{y}, v{x}, v{y}, 31",
      "v_mov_b32_dpp v{x}, v{y} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
      "v_alignbit_b32 v{x}, v{x}, v{y}, 1"]
pats.append(("K2 dpp window (2 DPP + 2 alignbit) + 11 bitop3", grp(k2, 11)))

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
import re as _re
def _fix(s):
    s = _re.sub(r"s\[(\d+):SONE\]", lambda m: f"s[{m.group(1)}:{int(m.group(1))+1}]", s)
    return _re.sub(r"s\[(\d+):TONE\]", lambda m: f"s[{m.group(1)}:{int(m.group(1))+1}]", s)
NN = {}
for k, (label, ins) in enumerate(pats):
    ins[:] = [_fix(i) for i in ins]
    NN[k] = len(ins)
    body = " ".join(f'"{s}\\n"' for s in ins)
    out.append(f'''__global__ __launch_bounds__(256) void k{k}(unsigned* o, int iters) {{
  asm volatile("v_mov_b32 v96, %0\\n v_mov_b32 v97, %1\\n" :: "v"(threadIdx.x), "v"(threadIdx.x * 3u) : CLOB);
  for (int it = 0; it < iters; ++it) asm volatile({body} ::: CLOB);
  unsigned s; asm volatile("v_xor_b32 %0, v80, v110" : "=v"(s) :: CLOB);
  o[blockIdx.x * blockDim.x + threadIdx.x] = s;
}}
''')
out.append('''int main(){ setvbuf(stdout, nullptr, _IOLBF, 0); hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p,0)); int cus=p.multiProcessorCount;
 unsigned* o; CHK(hipMalloc(&o, size_t(cus)*8*256*4)); hipEvent_t a,b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
 for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(warm, dim3(cus*8), dim3(256), 0, 0, o, 200000);
 CHK(hipDeviceSynchronize());
 const int iters = 8192; const double ghz = 2.4;
''')
for k, (label, ins) in enumerate(pats):
    out.append(f''' for (int w : {{2,4}}) {{ int blocks=cus*w; hipLaunchKernelGGL(k{k}, dim3(blocks), dim3(256),0,0,o,iters);
   CHK(hipEventRecord(a)); for(int r=0;r<4;++r) hipLaunchKernelGGL(k{k}, dim3(blocks), dim3(256),0,0,o,iters); CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
   float ms; CHK(hipEventElapsedTime(&ms,a,b)); double ins=double(w)*iters*{NN[k]}*4; printf("%-52s waves/SIMD=%d  %.2f cyc/instr/SIMD\\n", "{label}", w, ms*1e6/ins*ghz); }}
''')
out.append(' return 0; }\n')
open("csrc/tools/ubench_dpp_mix.hip", "w").write("".join(out))
