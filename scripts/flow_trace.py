#!/usr/bin/env python3
"""Summary of a GOL_FLOW_TRACE csv (one persistent dataflow launch,
life_flow_impl.hpp): how long items waited for the block before them, how
long they ran, how many ran at once, and the workgroups' idle time between
items.  Ticks are s_memrealtime (100 MHz, 10 ns).

    python scripts/flow_trace.py TRACE.csv [...]
"""
import sys

import numpy as np


def summarize(path):
    head = open(path).readline().strip()
    d = np.genfromtxt(path, delimiter=",", names=True, skip_header=1, dtype=np.int64)
    t0 = d["t_deq"].min()
    span = (d["t_done"].max() - t0) / 100.0  # us
    wait = (d["t_ready"] - d["t_deq"]) / 100.0
    run = (d["t_done"] - d["t_ready"]) / 100.0
    nblk = int(d["block"].max()) + 1
    print(f"{path}: {head}")
    print(f"  items {len(d)}  blocks {nblk}  span {span:.1f} us  ({span / nblk:.2f} us per block)")
    print(f"  wait  mean {wait.mean():.2f} us  p50 {np.median(wait):.2f}  p90 {np.percentile(wait, 90):.2f}  max {wait.max():.2f}")
    print(f"  run   mean {run.mean():.2f} us  p50 {np.median(run):.2f}  p90 {np.percentile(run, 90):.2f}  max {run.max():.2f}")
    print(f"  mean items running {run.sum() / span:.1f}, waiting {wait.sum() / span:.1f}, "
          f"workgroups {len(np.unique(d['wg']))}")
    gaps = []
    for wg in np.unique(d["wg"]):
        e = np.sort(d[d["wg"] == wg], order="t_deq")
        gaps.extend((e["t_deq"][1:] - e["t_done"][:-1]) / 100.0)
    if gaps:
        g = np.array(gaps)
        print(f"  gap between a workgroup's items: mean {g.mean():.2f} us  max {g.max():.2f}")
    first = d[d["block"] == 0]
    last = d[d["block"] == nblk - 1]
    print(f"  ramp: first item ready after {(first['t_ready'].min() - t0) / 100:.2f} us; "
          f"tail: last block's items end {(last['t_done'].max() - last['t_done'].min()) / 100:.1f} us apart")
    for b in sorted({0, nblk // 2, nblk - 1}):
        sel = d["block"] == b
        print(f"  block {b}: run mean {run[sel].mean():.2f} us, wait mean {wait[sel].mean():.2f} us")


for p in sys.argv[1:]:
    summarize(p)
