#!/usr/bin/env python3
"""Experiment builds: the default bit-layout kernel TU (life_block_bits_w1_dpp)
recompiled with extra -D flags and linked into alt_so/<name>/_gol.so beside the
regular objects.  bench.py loads one with GOL_NATIVE_SO=alt_so/<name>/_gol.so,
so several kernel builds can be A/B-timed in one GPU call on one device.

    python scripts/build_alt.py epi4 -DGOL_EPI_SCHED=4 -DGOL_GROUP_T16_WAVES=3
    python scripts/build_alt.py add12 --tu=kernels/life_block_bits_w1_add.hip -DGOL_GROUP_T16_ADD_WAVES=4
    python scripts/build_alt.py sync1 --tu=kernels/life_resident_rw1.hip --tu=kernels/life_resident_rw3.hip -DGOL_RES_SYNC=1
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
from gol_amd import native_build as nb  # noqa: E402


def main() -> int:
    name, args = sys.argv[1], sys.argv[2:]
    tus = [a[5:] for a in args if a.startswith("--tu=")] or ["kernels/life_block_bits_w1_dpp.hip"]
    flags = [a for a in args if not a.startswith("--tu=")]
    nb.build()
    alt = {}
    for tu in tus:  # every listed translation unit recompiled with the flags
        obj = nb.BUILD / f"alt_{name}_{tu.replace('/', '_')}.o"
        cmd = nb._compile_cmd(nb.CSRC / tu, obj)
        i = cmd.index("-c")
        cmd[i:i] = flags
        nb._run(cmd, True)
        alt[tu] = obj
    objs = [str(alt[s]) if s in alt else str(nb.BUILD / (s.replace("/", "_") + ".o"))
            for s in nb.HOST_SRCS + nb.HIP_SRCS + nb.BIND_SRCS]
    out = REPO / "alt_so" / name / "_gol.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    libs = [f"-L{nb.ROCM / 'lib'}", "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx",
            f"-Wl,-rpath,{nb.ROCM / 'lib'}", "-pthread"]
    nb._run([nb._hipcc(), "-shared", "-fPIC", *objs, "-o", str(out), *libs], False)
    print(out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
