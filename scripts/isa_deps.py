#!/usr/bin/env python3
"""Dependency distance profile of the hottest loop of each kernel in a
hipcc --save-temps .s file: for every VALU instruction, how many
instructions back its nearest VGPR producer is (in-order issue stalls when
that distance is small)."""
import re
import statistics
import sys

src = open(sys.argv[1]).read()
filt = sys.argv[2] if len(sys.argv) > 2 else ""
funcs = re.split(r"\n(?=_Z\S+:\s*;)", src)[1:]
vreg = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def regs(s):
    out = []
    for m in vreg.finditer(s):
        if m.group(1):
            out.append(int(m.group(1)))
        else:
            out += list(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


for f in funcs:
    name = f.split(":")[0]
    if filt and filt not in name:
        continue
    lines = f.split(".Lfunc_end")[0].split("\n")
    # find largest loop: label ... s_cbranch to that label
    labels = {}
    best = None
    for i, l in enumerate(lines):
        l = l.strip()
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
        m = re.match(r"^s_cbranch_\w+\s+(\.LBB\S+)", l) or re.match(r"^s_branch\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels:
            a = labels[m.group(1)]
            if best is None or i - a > best[1] - best[0]:
                best = (a, i)
    if not best:
        continue
    body = [l.strip() for l in lines[best[0]:best[1]] if l.strip() and not l.strip().startswith((".", ";"))]
    body = [l for l in body if not l.endswith(":")]
    last_def = {}
    dists = []
    nvalu = 0
    for i, l in enumerate(body):
        op = l.split()[0]
        if not op.startswith("v_"):
            continue
        nvalu += 1
        parts = l.split(None, 1)[1] if " " in l else ""
        ops = [x.strip() for x in parts.split(",")]
        dst = regs(ops[0]) if ops else []
        srcs = [r for x in ops[1:] for r in regs(x)]
        d = [i - last_def[r] for r in srcs if r in last_def]
        if d:
            dists.append(min(d))
        for r in dst:
            last_def[r] = i
    if dists:
        short = sum(1 for x in dists if x <= 2)
        print(f"{name[-70:]}: loop {len(body)} instr, {nvalu} VALU, median dep distance "
              f"{statistics.median(dists)}, <=2: {short / len(dists):.0%}")
