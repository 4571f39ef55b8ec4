#!/usr/bin/env python3
"""Summarise a GOL_WG_TRACE CSV (one grouped-kernel launch, one record per
wave: block, wave, XCC_ID, HW_ID, start/end in 100 MHz ticks).

Reports the launch span, the busy-time distribution per CU and per SIMD
(how many waves each ran, and whether some CUs took two workgroups while
others idled), and the spread of wave durations.  HW_ID fields (gfx9):
wave 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13.
"""
import collections
import csv
import statistics
import sys


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    t0 = min(int(r["t_start"]) for r in rows)
    t1 = max(int(r["t_end"]) for r in rows)
    per_cu = collections.defaultdict(list)
    per_simd = collections.Counter()
    blocks_cu = collections.defaultdict(set)
    dur = []
    for r in rows:
        hw, xcc = int(r["hw_id"]), int(r["xcc_id"]) & 0xF
        simd, cu, sh, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
        key = (xcc, se, sh, cu)
        s, e = int(r["t_start"]) - t0, int(r["t_end"]) - t0
        per_cu[key].append((s, e))
        per_simd[key + (simd,)] += 1
        blocks_cu[key].add(int(r["block"]))
        dur.append(e - s)
    tick_us = 0.01
    print(f"{path}: T={rows[0]['T']} rows={rows[0]['rows']} waves={len(rows)} "
          f"blocks={len({r['block'] for r in rows})} span={(t1 - t0) * tick_us:.2f} us")
    print(f"CUs used {len(per_cu)}; workgroups per CU: "
          f"{dict(sorted(collections.Counter(len(b) for b in blocks_cu.values()).items()))}")
    print(f"waves per SIMD: {dict(sorted(collections.Counter(per_simd.values()).items()))}")
    q = statistics.quantiles(dur, n=10)
    print(f"wave duration us: min {min(dur) * tick_us:.2f} p10 {q[0] * tick_us:.2f} median "
          f"{statistics.median(dur) * tick_us:.2f} p90 {q[-1] * tick_us:.2f} max {max(dur) * tick_us:.2f}")
    ends = sorted(max(e for _, e in v) for v in per_cu.values())
    starts = sorted(min(s for s, _ in v) for v in per_cu.values())
    print(f"CU first start us: median {statistics.median(starts) * tick_us:.2f} max {starts[-1] * tick_us:.2f}")
    print(f"CU last end us: min {ends[0] * tick_us:.2f} median {statistics.median(ends) * tick_us:.2f} "
          f"max {ends[-1] * tick_us:.2f}")
    busy = sum(e - s for v in per_cu.values() for s, e in v) / 8  # ~8 waves in flight per CU when packed
    print(f"mean CU occupancy over the span: {busy / (len(per_cu) * (t1 - t0)):.2f} workgroups")


def pair(path: str) -> None:
    """Two consecutive launches traced with GOL_WG_TRACE=N:path:pair: how far
    the second (linked) launch overlapped the first."""
    rows = list(csv.DictReader(open(path)))
    tick_us = 0.01
    by = collections.defaultdict(list)
    for r in rows:
        by[int(r["launch"])].append((int(r["t_start"]), int(r["t_end"])))
    t0 = min(s for v in by.values() for s, _ in v)
    (a, b) = (by[0], by[1])
    a0, a1 = min(s for s, _ in a) - t0, max(e for _, e in a) - t0
    b0, b1 = min(s for s, _ in b) - t0, max(e for _, e in b) - t0
    early = sum(1 for s, _ in b if s - t0 < a1)
    print(f"{path}: linked={rows[-1]['linked']} T={rows[0]['T']}/{rows[-1]['T']}")
    print(f"launch 0: {len(a)} waves, {a0 * tick_us:.2f} .. {a1 * tick_us:.2f} us")
    print(f"launch 1: {len(b)} waves, {b0 * tick_us:.2f} .. {b1 * tick_us:.2f} us")
    print(f"overlap: launch 1 starts {(a1 - b0) * tick_us:.2f} us before launch 0 ends; "
          f"{early} of its {len(b)} waves ({100.0 * early / max(1, len(b)):.0f} %) start before that end; "
          f"two launches in {(b1 - a0) * tick_us:.2f} us vs {((a1 - a0) + (b1 - b0)) * tick_us:.2f} us back to back")


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--pair":
        for p in args[1:]:
            pair(p)
    else:
        for p in args:
            main(p)
