#!/usr/bin/env python3
"""Timeline of the epoch boundaries in a rocprofv3 kernel trace of a
multi-rank schedule (bench.py --rehearse-rccl): for every RCCL kernel, when
it started relative to the end of the temporal-block launches before it, how
long it ran, and how long after it the next block launch started.  Separates
the exchange's own time from the hops around it (docs/PERFORMANCE.md, "The
exchange").  Usage: epoch_gaps.py <kernel_trace.csv>"""
import csv
import statistics
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    life = [r for r in rows if "life_" in r["Kernel_Name"]]
    comm = [r for r in rows if "nccl" in r["Kernel_Name"].lower() or "rccl" in r["Kernel_Name"].lower()]
    t = lambda r, k: int(r[k])  # noqa: E731
    pre, dur, post, span = [], [], [], []
    for c in comm[len(comm) // 4:]:  # skip the warm-up quarter
        s, e = t(c, "Start_Timestamp"), t(c, "End_Timestamp")
        before = [x for x in life if t(x, "Start_Timestamp") < s]
        after = [x for x in life if t(x, "Start_Timestamp") >= e]
        if not before or not after:
            continue
        last_end = max(t(x, "End_Timestamp") for x in before[-3:])
        nxt = t(after[0], "Start_Timestamp")
        pre.append(s - last_end)  # < 0: the exchange started before the last block ended
        dur.append(e - s)
        post.append(nxt - e)
        span.append(nxt - last_end)
    if not pre:
        print("no RCCL kernels between temporal blocks")
        return
    med = lambda v: statistics.median(v) / 1e3  # noqa: E731
    print(f"RCCL kernels at epoch boundaries: {len(pre)}")
    print(f"  start - end of the blocks before it : median {med(pre):8.2f} us  (negative = overlapped)")
    print(f"  RCCL kernel duration                : median {med(dur):8.2f} us")
    print(f"  next block start - RCCL end         : median {med(post):8.2f} us")
    print(f"  gap between blocks across the epoch : median {med(span):8.2f} us")


if __name__ == "__main__":
    main()
