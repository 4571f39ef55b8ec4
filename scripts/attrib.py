#!/usr/bin/env python3
"""Per-wave attribution table of the grouped kernel from the PMC passes of
scripts/gpu_attrib.sh (occ_<run> and iss_<run> directories of one OUTDIR):
instructions per wave, and how a wave's resident time splits into cycles
with a VALU instruction in flight and cycles waiting (dependency / memory /
barrier waits, SQ_WAIT_INST_ANY and SQ_WAIT_ANY), as fractions of its
resident cycles (SQ_WAVE_CYCLES; the SQ wave-cycle counters share one unit,
so the fractions are unit-free).  Ideal VALU per wave: 15 per level body
(the DPP window's body, scripts/asm_stats.py on the main loop) times the
level bodies of the wave's output rows.

    attrib.py OUTDIR > attrib.md
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from occupancy import SIMDS, XCDS, load  # noqa: E402

RUNS = {"tile8ring": (32768, 4096, "ring tile 32768 x 4096 (8-GPU share), DPP T = 16"),
        "fulldpp16": (32768, 32768, "full grid 32768^2, DPP T = 16 forced (long waves)"),
        "s8192": (8192, 8192, "config 2's grid 8192^2 (bits), DPP T = 8")}


def main(out: str) -> None:
    print("| run | kernel | launches | µs / launch | waves | VALU / wave | ideal VALU / wave | VALU overhead |"
          " SALU / wave | LDS / wave | waves / SIMD | cycles / VALU / SIMD | VALU-active share of resident |"
          " waiting on an instruction | waiting on anything |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for run, (W, H, desc) in RUNS.items():
        occ = load(os.path.join(out, f"occ_{run}"))
        iss = load(os.path.join(out, f"iss_{run}"))
        for k, d in sorted(occ.items(), key=lambda kv: -kv[1]["dur"]):
            if "life_group_kernel" not in k or d["n"] < 4:
                continue
            c, i = d["ctr"], iss.get(k, {"ctr": {}})["ctr"]
            n, waves = d["n"], c["SQ_WAVES"]
            T = int(k.split("<")[1].split(",")[0])
            # Level bodies per launch: 32-cell words x rows x T, 64 lanes a wave-instruction.
            ideal = 15.0 * (W / 32) * H * T / 64 / (waves / n)
            valu = c["SQ_INSTS_VALU"] / waves
            xcd = c["GRBM_GUI_ACTIVE"] / XCDS
            occ_w = 4.0 * c["SQ_WAVE_CYCLES"] / xcd / SIMDS
            cpi = xcd * SIMDS / c["SQ_INSTS_VALU"]
            res = c["SQ_WAVE_CYCLES"]
            frac = lambda key: (i.get(key, 0.0) / res) if res else float("nan")  # noqa: E731
            print(f"| {desc} | `{k[:60]}` | {n} | {d['dur'] / n:.1f} | {waves / n:.0f} | {valu:.0f} | {ideal:.0f} | "
                  f"{valu / ideal:.2f}x | {i.get('SQ_INSTS_SALU', 0) / waves:.0f} | {i.get('SQ_INSTS_LDS', 0) / waves:.0f} | "
                  f"{occ_w:.2f} | {cpi:.2f} | {frac('SQ_ACTIVE_INST_VALU'):.2f} | {frac('SQ_WAIT_INST_ANY'):.2f} | "
                  f"{frac('SQ_WAIT_ANY'):.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
