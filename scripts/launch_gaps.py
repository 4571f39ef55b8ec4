#!/usr/bin/env python3
"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace
(*_kernel_trace.csv): how much of the generation loop the GPU spends between
launches rather than in them.  Usage: launch_gaps.py <kernel_trace.csv> [name-filter]"""
import csv
import statistics
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the timed loop: from the first life kernel to the last
    life = [i for i, r in enumerate(rows) if "life_" in r["Kernel_Name"]]
    rows = rows[life[len(life) // 4]:life[-1] + 1]  # skip warmup-ish first quarter
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
    by = {}
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
        by.setdefault(n, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"kernels {len(rows)} span {span / 1e3:.1f} us busy {busy / 1e3:.1f} us "
          f"({100 * busy / span:.1f}%) gaps median {statistics.median(gaps) / 1e3:.2f} us "
          f"max {max(gaps) / 1e3:.2f} us total {sum(gaps) / 1e3:.1f} us")
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:40s} n={len(v):5d} total {sum(v) / 1e3:9.1f} us  mean {statistics.mean(v) / 1e3:7.2f} us")


if __name__ == "__main__":
    main()
