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


def from_trace(path: str) -> None:
    """rocprofv3 --kernel-trace --output-format csv: per-kernel time of the
    framework's own dispatches (the fp32 PyTorch oracle of bench.py's verify
    step is left out), and how busy the device was between the first and the
    last temporal-block kernel."""
    rows = list(csv.DictReader(open(path)))
    ours = [r for r in rows if not r["Kernel_Name"].startswith(("void at::", "at::"))]
    life = [r for r in ours if "life_" in r["Kernel_Name"]]
    if not life:
        return
    # The timed steps (with the prewarm and warmup before them) are one run of
    # back-to-back temporal-block dispatches; the verify step and the setup are
    # separated from it by host work.  Take the longest run with gaps < 20 ms.
    life.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], [life[0]]
    for r in life[1:]:
        if int(r["Start_Timestamp"]) - int(cur[-1]["End_Timestamp"]) > 20_000_000:
            runs.append(cur)
            cur = []
        cur.append(r)
    runs.append(cur)
    best = max(runs, key=len)
    t0 = int(best[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in best)
    win = [r for r in ours if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
    agg = collections.OrderedDict()
    for r in sorted(win, key=lambda r: int(r["Start_Timestamp"])):
        k = short(r["Kernel_Name"])
        a = agg.setdefault(k, {"n": 0, "ns": 0, "lds": r["LDS_Block_Size"],
                               "grid": int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))})
        a["n"] += 1
        a["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(a["ns"] for a in agg.values()) or 1
    print("## Kernel time over the generation loop (rocprofv3 --kernel-trace: the longest run of "
          "back-to-back temporal-block dispatches, i.e. prewarm + warmup + timed steps)\n")
    print("| kernel | calls | total ms | avg us | % | LDS B / WG | workgroups |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        print(f"| `{k}` | {a['n']} | {a['ns'] / 1e6:.3f} | {a['ns'] / a['n'] / 1e3:.2f} | "
              f"{100.0 * a['ns'] / tot:.2f} | {a['lds']} | {a['grid']} |")
    busy, end = 0, t0
    for r in sorted(win, key=lambda r: int(r["Start_Timestamp"])):
        a_, b_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if b_ > end:
            busy += b_ - max(a_, end)
            end = b_
    print(f"\nWindow {(t1 - t0) / 1e6:.2f} ms, {len(win)} dispatches; some kernel running "
          f"{100.0 * busy / max(1, t1 - t0):.1f} % of it (linked launches overlap, so summed kernel "
          f"time can exceed the window).\n")


def main(d: str) -> None:
    db = os.path.join(d, "run_results.db")
    if os.path.exists(db):
        from_db(db)
        return
    trace = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(trace):
        from_trace(trace)
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
