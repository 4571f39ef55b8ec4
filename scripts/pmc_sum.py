#!/usr/bin/env python3
"""Per-kernel sums of every counter in rocprofv3 --pmc CSV runs (one column per
counter, one row per kernel and run directory), for quick A/B tables of passes
that occupancy.py / attrib.py do not model (TLB, L2, DRAM).

    pmc_sum.py LABEL=DIR [LABEL=DIR ...] [--kernel SUBSTRING]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("runs", nargs="+")
    ap.add_argument("--kernel", default="life_group_kernel")
    a = ap.parse_args()
    rows = []
    names: list[str] = []
    for spec in a.runs:
        label, _, path = spec.partition("=")
        files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
        tot = collections.defaultdict(float)
        disp = set()
        for f in files:
            for r in csv.DictReader(open(f)):
                if a.kernel not in r["Kernel_Name"]:
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
        for k in tot:
            if k not in names:
                names.append(k)
        rows.append((label, len(disp), tot))
    print("| run | dispatches | " + " | ".join(names) + " |")
    print("|---|---:|" + "---:|" * len(names))
    for label, n, tot in rows:
        print(f"| {label} | {n} | " + " | ".join(f"{tot.get(k, 0):.4g}" for k in names) + " |")


if __name__ == "__main__":
    main()
