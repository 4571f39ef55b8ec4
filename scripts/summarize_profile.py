#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (kernel stats + PMC counter CSVs) into a
markdown table for profiles/.  Usage: summarize_profile.py PROF_DIR > out.md"""
import collections
import csv
import os
import sys


def short(name: str) -> str:
    n = name.replace("gol::hipk::", "").replace("(anonymous namespace)::", "").replace("lb::", "")
    keep = any(k in n for k in ("life_block_kernel", "life_group_kernel", "life_short_kernel"))
    return n[:110] if keep else n.split("(")[0][:90]


def from_db(db_path: str) -> None:
    """rocprofv3 >= 7 writes a rocpd SQLite database (run_results.db): kernel
    time per kernel, and the device's busy share of the traced span."""
    import sqlite3  # noqa: PLC0415

    cur = sqlite3.connect(db_path).cursor()
    rows = cur.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                       "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    print("## Kernel time (rocprofv3 --kernel-trace --stats)\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for name, n, s_ns, a_ns in rows:
        print(f"| `{short(name)}` | {n} | {s_ns / 1e6:.3f} | {a_ns / 1e3:.2f} | {100.0 * s_ns / tot:.2f} |")
    ks = cur.execute("select start, end from kernels order by start").fetchall()
    if ks:
        busy, end = 0, ks[0][0]
        for a, b in ks:  # union of kernel intervals
            if b > end:
                busy += b - max(a, end)
                end = b
        span = ks[-1][1] - ks[0][0]
        print(f"\nDevice busy {100.0 * busy / span:.1f} % of the traced span ({span / 1e6:.2f} ms, "
              f"{len(ks)} dispatches).\n")


def main(d: str) -> None:
    db = os.path.join(d, "run_results.db")
    if os.path.exists(db):
        from_db(db)
        return
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        rows = list(csv.DictReader(open(stats)))
        print("## Kernel time (rocprofv3 --kernel-trace --stats)\n")
        print("| kernel | calls | total ms | avg us | % |")
        print("|---|---:|---:|---:|---:|")
        for r in rows:
            print(f"| `{short(r['Name'])}` | {r['Calls']} | {int(r['TotalDurationNs'])/1e6:.3f} | "
                  f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.2f} |")
        print()
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if not any(k in r["Kernel_Name"] for k in ("life_block_kernel", "life_group_kernel", "life_short_kernel",
                                                       "life_step_lds")):
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        if not agg:
            continue
        print(f"## PMC set `{sub}` (summed over all temporal-block kernel dispatches)\n")
        print("| counter | value |")
        print("|---|---:|")
        for k, v in sorted(agg.items()):
            print(f"| {k} | {v:.4g} |")
        print()
        derived = []
        if "SQ_INSTS_VALU" in agg and "SQ_WAVES" in agg:
            derived.append(("VALU instructions per wave", agg["SQ_INSTS_VALU"] / agg["SQ_WAVES"]))
        if "SQ_ACTIVE_INST_VALU" in agg and "SQ_BUSY_CYCLES" in agg:
            derived.append(("SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES", agg["SQ_ACTIVE_INST_VALU"] / agg["SQ_BUSY_CYCLES"]))
        if "SQ_WAIT_INST_ANY" in agg and "SQ_WAVE_CYCLES" in agg:
            derived.append(("wave cycles waiting on any instruction (fraction)",
                            agg["SQ_WAIT_INST_ANY"] / agg["SQ_WAVE_CYCLES"]))
        if "SQC_ICACHE_HITS" in agg and "SQC_ICACHE_MISSES" in agg:
            derived.append(("instruction cache hit rate",
                            agg["SQC_ICACHE_HITS"] / max(1.0, agg["SQC_ICACHE_HITS"] + agg["SQC_ICACHE_MISSES"])))
        if "FETCH_SIZE" in agg:
            derived.append(("HBM fetch, GB (FETCH_SIZE is KB)", agg["FETCH_SIZE"] / 1e6))
        if derived:
            print("| derived | value |")
            print("|---|---:|")
            for k, v in derived:
                print(f"| {k} | {v:.4g} |")
            print()


if __name__ == "__main__":
    main(sys.argv[1])
