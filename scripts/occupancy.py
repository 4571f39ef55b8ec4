#!/usr/bin/env python3
"""Measured occupancy (mean resident waves per SIMD) per kernel from one
rocprofv3 PMC pass of SQ_WAVES, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE (plus
optional VALU / LDS counters), and the VGPR-derived ceiling.

  waves/SIMD = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / XCDs) / SIMDs

SQ_WAVE_CYCLES counts quad-cycles of resident waves summed over the chip
(MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units"); GRBM_GUI_ACTIVE is
summed over the 8 XCDs.  The formula is calibrated on csrc/tools/
ubench_clock.hip, whose launches hold exactly 1, 2 and 4 waves per SIMD for
hundreds of milliseconds (the `calibration` rows): the script prints the
measured/expected ratio it found there.  (SQ_LEVEL_WAVES / SQ_ACCUM_PREV_HIRES
read 0 on this ROCm / gfx950 pool, profiles/rocprof_lds_u8_8192.md, hence this
derivation.)

    occupancy.py DIR_OR_CSV [--label NAME] ...  >> profiles/r03/occupancy.md
"""
from __future__ import annotations

import argparse
import collections
import csv
import os
import sys

SIMDS = 1024
XCDS = 8
VGPR_FILE = 512  # VGPRs per SIMD lane on CDNA3/4
# rocprofv3's VGPR_Count on gfx950 is half the compiler's count
# (-Rpass-analysis=kernel-resource-usage: life_group_kernel<12, adder> 120,
# rocprofv3 60).
VGPR_SCALE = 2


def short(name: str) -> str:
    n = name.replace("gol::hipk::", "").replace("(anonymous namespace)::", "").replace("lb::", "")
    n = n.replace("void ", "")
    for k in ("HIP_vector_type", "(gol::hipk::"):
        n = n.split(k)[0]
    return n[:100]


def load(path: str):
    f = path if path.endswith(".csv") else os.path.join(path, "run_counter_collection.csv")
    per = collections.defaultdict(lambda: {"n": 0, "ctr": collections.defaultdict(float), "vgpr": 0, "agpr": 0,
                                           "lds": 0, "wg": 0, "dur": 0.0})
    seen = set()
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        d = per[k]
        d["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in seen:
            seen.add(r["Dispatch_Id"])
            d["n"] += 1
            d["dur"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
            d["vgpr"] = int(r["VGPR_Count"])
            d["agpr"] = int(r.get("Accum_VGPR_Count", 0) or 0)
            d["lds"] = int(r["LDS_Block_Size"])
            d["wg"] = int(r["Workgroup_Size"])
    return per


def ceiling(vgpr: int, agpr: int, lds: int, wg: int, waves: float) -> float:
    """Resident waves per SIMD the launch could reach: register file, LDS,
    and the launch's own size (waves / SIMDs)."""
    regs = max(1, VGPR_SCALE * (vgpr + agpr))
    by_vgpr = min(8, VGPR_FILE // regs)
    waves_per_wg = max(1, wg // 64)
    c = float(by_vgpr)
    if lds > 0:
        wgs = max(1, (160 * 1024) // lds)
        c = min(c, wgs * waves_per_wg / 4.0)
    return min(c, waves / SIMDS)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("runs", nargs="+", help="LABEL=DIR pairs (rocprofv3 -d DIR with -o run)")
    ap.add_argument("--min-calls", type=int, default=2)
    ap.add_argument("--scale", type=float, default=1.0, help="calibration factor (measured/expected)")
    a = ap.parse_args()
    print("| run | kernel | calls | avg µs | VGPRs | LDS B / WG | waves / launch | ceiling waves/SIMD "
          "(regs, LDS, launch size) | measured waves/SIMD | VALU / wave | cycles per VALU per SIMD |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for spec in a.runs:
        label, _, path = spec.partition("=")
        for k, d in sorted(load(path).items(), key=lambda kv: -kv[1]["dur"]):
            c = d["ctr"]
            if d["n"] < a.min_calls or "SQ_WAVE_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
                continue
            n = d["n"]
            xcd_cycles = c["GRBM_GUI_ACTIVE"] / XCDS
            occ = 4.0 * c["SQ_WAVE_CYCLES"] / xcd_cycles / SIMDS / a.scale if xcd_cycles else 0.0
            valu = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_WAVES"] if c.get("SQ_WAVES") else float("nan")
            nvalu = c.get("SQ_INSTS_VALU", 0.0)
            cpi = xcd_cycles * SIMDS / nvalu if nvalu else float("nan")
            waves = c.get("SQ_WAVES", 0) / n
            print(f"| {label} | `{k}` | {n} | {d['dur'] / n:.1f} | {VGPR_SCALE * d['vgpr']}"
                  f"{'+' + str(VGPR_SCALE * d['agpr']) if d['agpr'] else ''}"
                  f" | {d['lds']} | {waves:.0f} | {ceiling(d['vgpr'], d['agpr'], d['lds'], d['wg'], waves):.2f}"
                  f" | {occ:.2f} | {valu:.0f} | {cpi:.2f} |")


if __name__ == "__main__":
    sys.exit(main())
