#!/usr/bin/env python3
"""Per-kernel statistics of a hipcc -save-temps gfx950 .s file: instruction
counts, SGPR spill traffic (v_writelane / v_readlane), scratch accesses, and
every loop (a label with a later backward branch to it) with its VALU / SALU
/ memory instruction mix, so a hot loop's cost can be compared between
kernels without a GPU.

    python scripts/asm_stats.py FILE.s [NAME_SUBSTRING ...]
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        yield m.group(1), text[start:end]


def instrs(body):
    out = []
    for ln in body.splitlines():
        t = ln.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            out.append(("label", t[:-1]) if t.endswith(":") else None)
            continue
        out.append(("op", t))
    return [x for x in out if x]


def mix(ops):
    c = {"valu": 0, "salu": 0, "vmem": 0, "lds": 0, "readlane": 0, "writelane": 0, "scratch": 0, "waitcnt": 0,
         "total": 0}
    for o in ops:
        op = o.split()[0]
        c["total"] += 1
        if op.startswith("v_readlane"):
            c["readlane"] += 1
        if op.startswith("v_writelane"):
            c["writelane"] += 1
        if op.startswith("scratch_"):
            c["scratch"] += 1
        if op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        if op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
    return c


def main():
    text = open(sys.argv[1]).read()
    pats = sys.argv[2:]
    for name, body in kernels(text):
        if pats and not any(p in name for p in pats):
            continue
        seq = instrs(body)
        ops = [x[1] for x in seq if x[0] == "op"]
        print(f"{name[:110]}\n  whole: {mix(ops)}")
        labels = {x[1]: i for i, x in enumerate(seq) if x[0] == "label"}
        for i, x in enumerate(seq):
            if x[0] != "op" or not x[1].startswith("s_cbranch") and not x[1].startswith("s_branch"):
                continue
            tgt = x[1].split()[-1]
            j = labels.get(tgt)
            if j is None or j >= i:
                continue
            loop = [y[1] for y in seq[j:i + 1] if y[0] == "op"]
            if len(loop) < 40:
                continue
            print(f"  loop {tgt}: {mix(loop)}")


if __name__ == "__main__":
    main()
