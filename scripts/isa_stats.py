#!/usr/bin/env python3
"""Instruction mix of each life_block kernel instance in a hipcc --save-temps .s file."""
import re
import sys

src = open(sys.argv[1]).read()
parts = re.split(r"\n(?=_Z\S+:\s*;)", src)
for f in parts[1:]:
    name = f.split(":")[0].replace("_ZN3gol4hipk12_GLOBAL__N_117life_block_kernel", "")[:28]
    body = f.split(".Lfunc_end")[0]
    ins = [l.strip() for l in body.split("\n")[1:]]
    ins = [l for l in ins if l and not l.startswith((".", ";")) and not l.endswith(":")]
    c = lambda p: sum(1 for l in ins if l.startswith(p))
    nops = sum(int(l.split()[1], 0) + 1 for l in ins if l.startswith("s_nop"))
    print(f"{name:30s} n={len(ins):6d} dpp={sum('_dpp' in l for l in ins):5d} bitop3={c('v_bitop3'):5d} "
          f"align={c('v_alignbit'):5d} nop_cyc={nops:4d} vmov={c('v_mov_b32 '):4d} acc={sum('accvgpr' in l for l in ins)}"
          f" glob={c('global_'):4d} bperm={c('ds_bpermute'):4d}")
