"""Generates csrc/tools/ubench_vop3.hip: issue cost of the VALU instruction
forms the level body is built from, with hand-placed VGPR operands.

The question it answers: why does v_bitop3_b32 issue at about half the rate
of a two-source VOP2 op (profiles/ubench_valu.txt)?  Candidates: the VOP3
encoding itself, a third VGPR source (register-file read ports), or VGPR
bank conflicts between the sources (bank = register index mod 4).  Every
variant is a block of 32 independent instructions (sources v0-v15, never
written; destinations v16-v31) repeated in a loop, at 1, 2, 4 and 8 waves per
SIMD.  Each wave reads s_memtime (shader clock) and s_memrealtime (100 MHz)
around its loop.

Run: python scripts/gen_ubench_vop3.py && hipcc --offload-arch=gfx950 -O3
csrc/tools/ubench_vop3.hip -o bin/ubench_vop3
"""
from __future__ import annotations

from pathlib import Path

N = 32  # instructions per block


def v(i: int) -> str:
    return f"v{i}"


def dst(i: int) -> str:
    return v(16 + i % 16)


def distinct3(i):  # three sources in three different banks
    return v(i % 16), v((i + 1) % 16), v((i + 2) % 16)


def same_bank3(i):  # three sources in one bank
    b = i % 4
    return v(b), v(b + 4), v(b + 8)


VARIANTS = [
    ("v_xor_b32 (VOP2, 2 src)", lambda i: f"v_xor_b32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}"),
    ("v_xor_b32_e64 (VOP3, 2 src)", lambda i: f"v_xor_b32_e64 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}"),
    ("v_bitop3 3 src, distinct banks", lambda i: "v_bitop3_b32 {}, {}, {}, {} bitop3:0x96".format(dst(i), *distinct3(i))),
    ("v_bitop3 3 src, one bank", lambda i: "v_bitop3_b32 {}, {}, {}, {} bitop3:0x96".format(dst(i), *same_bank3(i))),
    ("v_bitop3 2 vgpr + sgpr", lambda i: f"v_bitop3_b32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}, s40 bitop3:0x96"),
    ("v_bitop3 2 vgpr + const", lambda i: f"v_bitop3_b32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}, 1 bitop3:0x96"),
    ("v_bitop3 a,b,a (2 regs)", lambda i: f"v_bitop3_b32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}, {v(i % 16)} bitop3:0x96"),
    ("v_or3_b32 distinct banks", lambda i: "v_or3_b32 {}, {}, {}, {}".format(dst(i), *distinct3(i))),
    ("v_and_or_b32 distinct banks", lambda i: "v_and_or_b32 {}, {}, {}, {}".format(dst(i), *distinct3(i))),
    ("v_add3_u32 distinct banks", lambda i: "v_add3_u32 {}, {}, {}, {}".format(dst(i), *distinct3(i))),
    ("v_alignbit_b32 2 src + const", lambda i: f"v_alignbit_b32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}, 31"),
    ("v_add_co_u32_e64 (sgpr carry out)", lambda i: f"v_add_co_u32_e64 {dst(i)}, s[42:43], {v(i % 16)}, {v((i + 1) % 16)}"),
    ("v_addc_co_u32_e64 (sgpr carry in/out)",
     lambda i: f"v_addc_co_u32_e64 {dst(i)}, s[42:43], {v(i % 16)}, {v((i + 1) % 16)}, s[44:45]"),
    ("v_add_u32 (VOP2)", lambda i: f"v_add_u32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}"),
    ("v_add_co_u32_e32 (vcc carry out)", lambda i: f"v_add_co_u32_e32 {dst(i)}, vcc, {v(i % 16)}, {v((i + 1) % 16)}"),
    ("v_addc_co_u32_e32 (vcc in/out)", lambda i: f"v_addc_co_u32_e32 {dst(i)}, vcc, {v(i % 16)}, {v((i + 1) % 16)}, vcc"),
    ("v_addc_co_u32_e32 (vcc in/out, src0 0)", lambda i: f"v_addc_co_u32_e32 {dst(i)}, vcc, 0, {v(i % 16)}, vcc"),
    ("v_cmp_gt_i32_e32 (vcc)", lambda i: f"v_cmp_gt_i32_e32 vcc, 0, {v(i % 16)}"),
    ("v_cmp_gt_i32_e64 (sgpr pair)", lambda i: f"v_cmp_gt_i32_e64 s[42:43], 0, {v(i % 16)}"),
    ("v_cndmask_b32_e32 (vcc)", lambda i: f"v_cndmask_b32_e32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}, vcc"),
    ("v_cndmask_b32_e64 (sgpr pair)", lambda i: f"v_cndmask_b32_e64 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}, s[44:45]"),
    ("v_lshlrev_b32_e32", lambda i: f"v_lshlrev_b32_e32 {dst(i)}, 1, {v(i % 16)}"),
    ("v_lshrrev_b32_e32", lambda i: f"v_lshrrev_b32_e32 {dst(i)}, 31, {v(i % 16)}"),
    ("v_lshl_or_b32 (VOP3 3 src)", lambda i: f"v_lshl_or_b32 {dst(i)}, {v(i % 16)}, 1, {v((i + 1) % 16)}"),
    ("v_add_u32_e64 with sgpr source", lambda i: f"v_add_u32_e64 {dst(i)}, s40, {v(i % 16)}"),
    ("v_xor_b32_e32 with sgpr source", lambda i: f"v_xor_b32_e32 {dst(i)}, s40, {v(i % 16)}"),
    ("v_mov_b32_dpp row_shr:1", lambda i: f"v_mov_b32_dpp {dst(i)}, {v(i % 16)} row_shr:1 row_mask:0xf bank_mask:0xf"),
    ("v_or_b32_dpp row_shr:1", lambda i: f"v_or_b32_dpp {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)} row_shr:1 row_mask:0xf bank_mask:0xf"),
    ("v_mov_b32_dpp wave_shr:1", lambda i: f"v_mov_b32_dpp {dst(i)}, {v(i % 16)} wave_shr:1 row_mask:0xf bank_mask:0xf"),
    ("v_or_b32_dpp wave_shr:1", lambda i: f"v_or_b32_dpp {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)} wave_shr:1 row_mask:0xf bank_mask:0xf"),
    ("v_mov_b32_dpp row_bcast / quad_perm", lambda i: f"v_mov_b32_dpp {dst(i)}, {v(i % 16)} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"),
    ("v_permlane32_swap", lambda i: f"v_permlane32_swap_b32_e32 {v(16 + (2 * i) % 16)}, {v(17 + (2 * i) % 16)}"),
    ("v_and_b32 (VOP2) + v_bitop3 alternating",
     lambda i: (f"v_and_b32 {dst(i)}, {v(i % 16)}, {v((i + 1) % 16)}" if i % 2 == 0 else
                "v_bitop3_b32 {}, {}, {}, {} bitop3:0x96".format(dst(i), *distinct3(i)))),
]


def main() -> None:
    out = Path(__file__).resolve().parents[1] / "csrc" / "tools" / "ubench_vop3.hip"
    lines = [
        "// GENERATED by scripts/gen_ubench_vop3.py - do not edit.",
        "// Issue cost of VALU instruction forms with hand-placed VGPR operands",
        "// (sources v0-v15, destinations v16-v31), 1-8 waves per SIMD.",
        "#include <hip/hip_runtime.h>",
        "",
        "#include <cstdint>",
        "#include <cstdio>",
        "#include <cstdlib>",
        "#include <algorithm>",
        "#include <map>",
        "#include <vector>",
        "",
        "#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf(\"HIP error %s line %d\\n\", "
        "hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)",
        "",
        "#define CLOB \"v0\",\"v1\",\"v2\",\"v3\",\"v4\",\"v5\",\"v6\",\"v7\",\"v8\",\"v9\",\"v10\",\"v11\",\"v12\",\"v13\","
        "\"v14\",\"v15\",\"v16\",\"v17\",\"v18\",\"v19\",\"v20\",\"v21\",\"v22\",\"v23\",\"v24\",\"v25\",\"v26\",\"v27\","
        "\"v28\",\"v29\",\"v30\",\"v31\",\"s40\",\"s42\",\"s43\",\"s44\",\"s45\",\"vcc\"",
        "",
        "constexpr int kRec = 5;",
        "",
        "template <int V>",
        "__global__ __launch_bounds__(256) void bench(uint64_t* rec, uint32_t* sink, int iters, uint32_t seed) {",
        "  const uint32_t x = seed * (threadIdx.x + 1);",
        "  // Sources v0-v15 from the lane's seed; s40 and the carry-in pair too.",
        "  asm volatile(",
    ]
    init = [f"\"v_add_u32 v{r}, {r + 1}, %0\\n\\t\"" for r in range(16)]
    init += [f"\"v_mov_b32 v{r}, 0\\n\\t\"" for r in range(16, 32)]
    init += ["\"s_mov_b32 s40, 0x5a5a5a5a\\n\\t\"", "\"s_mov_b64 s[44:45], -1\\n\\t\""]
    lines += ["      " + s for s in init]
    lines += ["      :: \"v\"(x) : CLOB);"]
    lines += [
        "  uint64_t t0, r0, t1, r1;",
        "  asm volatile(\"s_memtime %0\\n\\ts_memrealtime %1\\n\\ts_waitcnt lgkmcnt(0)\" : \"=s\"(t0), \"=s\"(r0));",
        "  for (int it = 0; it < iters; ++it) {",
    ]
    for k, (_, fn) in enumerate(VARIANTS):
        body = "\\n\\t".join(fn(i) for i in range(N))
        lines.append(f"    if constexpr (V == {k}) asm volatile(\"{body}\" ::: CLOB);")
    lines += [
        "  }",
        "  asm volatile(\"s_memtime %0\\n\\ts_memrealtime %1\\n\\ts_waitcnt lgkmcnt(0)\" : \"=s\"(t1), \"=s\"(r1));",
        "  uint32_t acc;",
        "  asm volatile(\"v_bitop3_b32 %0, v16, v17, v18 bitop3:0x96\\n\\tv_bitop3_b32 %0, %0, v19, v31 bitop3:0x96\" : \"=v\"(acc) :: CLOB);",
        "  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;",
        "  // Where the wave ran: HW_ID (wave, SIMD, CU, SH, SE) and the XCC.",
        "  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));",
        "  const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));",
        "  if ((threadIdx.x & 63) == 0) {",
        "    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;",
        "    rec[kRec * w + 0] = t0;",
        "    rec[kRec * w + 1] = t1;",
        "    rec[kRec * w + 2] = r0;",
        "    rec[kRec * w + 3] = r1;",
        "    rec[kRec * w + 4] = (uint64_t(xcc) << 32) | hw;",
        "  }",
        "}",
        "",
        f"static const char* kNames[] = {{{', '.join(repr(n).replace(chr(39), chr(34)) for n, _ in VARIANTS)}}};",
        f"constexpr int kVariants = {len(VARIANTS)};",
        "",
        "template <int V>",
        "void run(int cus, int iters) {",
        "  for (int w : {1, 2, 4, 8}) {",
        "    const int blocks = cus * w, waves = blocks * 4;",
        "    uint64_t* rec;",
        "    uint32_t* sink;",
        "    CHK(hipMalloc(&rec, sizeof(uint64_t) * kRec * waves));",
        "    CHK(hipMalloc(&sink, sizeof(uint32_t) * 256 * blocks));",
        "    hipLaunchKernelGGL(bench<V>, dim3(blocks), dim3(256), 0, 0, rec, sink, iters / 8, 7u);  // warm",
        "    hipLaunchKernelGGL(bench<V>, dim3(blocks), dim3(256), 0, 0, rec, sink, iters, 7u);",
        "    CHK(hipDeviceSynchronize());",
        "    std::vector<uint64_t> h(size_t(kRec) * waves);",
        "    CHK(hipMemcpy(h.data(), rec, sizeof(uint64_t) * kRec * waves, hipMemcpyDeviceToHost));",
        "    // Per SIMD (XCC, SE, SH, CU, SIMD): waves it ran, the span from the first",
        "    // start to the last end (100 MHz realtime), and the clock (memtime ticks",
        "    // per realtime tick) -> cycles per wave-instruction on that SIMD.",
        "    struct S { int n = 0; uint64_t r0 = ~0ull, r1 = 0; double clk = 0; int conc = 0; };",
        "    std::map<uint64_t, S> simds;",
        "    for (int i = 0; i < waves; ++i) {",
        "      const uint64_t* q = &h[size_t(kRec) * i];",
        "      const uint64_t hwid = q[4] & 0xffffffffull, xcc = q[4] >> 32;",
        "      const uint64_t key = (xcc << 32) | (hwid & 0xff30u);  // SIMD [5:4], CU [11:8], SH/SE [15:12]",
        "      S& s = simds[key];",
        "      s.n++;",
        "      s.r0 = std::min(s.r0, q[2]);",
        "      s.r1 = std::max(s.r1, q[3]);",
        "      s.clk += double(q[1] - q[0]) / double(std::max<uint64_t>(1, q[3] - q[2]));",
        "    }",
        "    double cpi = 0, clk = 0, nw = 0;",
        "    for (auto& [k, s] : simds) {",
        f"      const double instrs = double(iters) * {N} * s.n;",
        "      const double c = s.clk / s.n;  // memtime ticks per 10 ns",
        "      cpi += double(s.r1 - s.r0) * c / instrs;",
        "      clk += c;",
        "      nw += s.n;",
        "    }",
        "    const double ns = double(simds.size());",
        "    std::printf(\"%-40s waves/SIMD=%d (%4zu SIMDs, %.2f waves each)  %.2f cycles per wave-instruction per SIMD  (clock %.2f GHz)\\n\",",
        "                kNames[V], w, simds.size(), nw / ns, cpi / ns, clk / ns / 10.0);",
        "    CHK(hipFree(rec));",
        "    CHK(hipFree(sink));",
        "  }",
        "}",
        "",
        "template <int... Vs>",
        "void run_all(int cus, int iters, std::integer_sequence<int, Vs...>) {",
        "  (run<Vs>(cus, iters), ...);",
        "}",
        "",
        "int main(int argc, char** argv) {",
        "  const int iters = argc > 1 ? std::atoi(argv[1]) : 4096;",
        "  hipDeviceProp_t prop;",
        "  CHK(hipGetDeviceProperties(&prop, 0));",
        "  std::printf(\"device %s, %d CUs, %d instructions per wave per variant\\n\", prop.gcnArchName,",
        f"              prop.multiProcessorCount, iters * {N});",
        "  run_all(prop.multiProcessorCount, iters, std::make_integer_sequence<int, kVariants>{});",
        "  return 0;",
        "}",
    ]
    out.write_text("\n".join(lines) + "\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
