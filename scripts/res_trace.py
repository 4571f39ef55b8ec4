#!/usr/bin/env python3
"""Summarise a resident-kernel refresh trace (GOL_RES_TRACE=<launch>:<csv>).

Per refresh m, over all workgroups: the spread of the refresh start times
(how far apart the workgroups arrive), and the median / max of each phase:
store drain (t_stored - t_start), neighbour wait (t_flags - t_stored) and the
halo loads (t_loaded - t_flags).  s_memrealtime ticks at 100 MHz."""
import csv
import statistics as st
import sys


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    k0 = [r for r in rows if r["refresh"] == "0"]
    rows = [r for r in rows if r["refresh"] != "0"]
    if k0:  # refresh 0 = the kernel: start, state loaded, loop done, end
        t = lambda r, c: int(r[c]) * 0.01
        s0 = min(t(r, "t_start") for r in k0)
        print(f"kernel: first start -> last start {max(t(r, 't_start') for r in k0) - s0:.2f} us, "
              f"-> last loaded {max(t(r, 't_stored') for r in k0) - s0:.2f}, -> last loop end "
              f"{max(t(r, 't_flags') for r in k0) - s0:.2f}, -> last end {max(t(r, 't_loaded') for r in k0) - s0:.2f}")
    by_m: dict[int, list[dict]] = {}
    for r in rows:
        by_m.setdefault(int(r["refresh"]), []).append(r)
    us = 0.01  # 100 MHz ticks -> us
    print(f"{path}: k={rows[0]['k']} rw={rows[0]['rw']} T={rows[0]['T']} regions={len({r['region'] for r in rows})}")
    print(" m  start_spread  store_med store_max  wait_med wait_max  load_med load_max  total_med total_max  gap_from_prev")
    prev_end = None
    for m in sorted(by_m):
        rs = by_m[m]
        t0 = [int(r["t_start"]) for r in rs]
        d1 = [(int(r["t_stored"]) - int(r["t_start"])) * us for r in rs]
        d2 = [(int(r["t_flags"]) - int(r["t_stored"])) * us for r in rs]
        d3 = [(int(r["t_loaded"]) - int(r["t_flags"])) * us for r in rs]
        tot = [(int(r["t_loaded"]) - int(r["t_start"])) * us for r in rs]
        gap = (min(t0) - prev_end) * us if prev_end else float("nan")
        prev_end = max(int(r["t_loaded"]) for r in rs)
        print(f"{m:2d}  {(max(t0) - min(t0)) * us:11.2f}  {st.median(d1):9.2f} {max(d1):9.2f}  {st.median(d2):8.2f} "
              f"{max(d2):8.2f}  {st.median(d3):8.2f} {max(d3):8.2f}  {st.median(tot):9.2f} {max(tot):9.2f}  {gap:10.2f}")


def compute(path: str) -> None:
    """Per workgroup, the k generations between two refreshes: wall time and
    shader clock (s_memtime cycles / s_memrealtime time)."""
    rows = [r for r in csv.DictReader(open(path)) if r["refresh"] != "0"]
    by: dict[int, dict[int, dict]] = {}
    for r in rows:
        by.setdefault(int(r["region"]), {})[int(r["refresh"])] = r
    us, ghz = [], []
    for ms in by.values():
        for m in sorted(ms):
            if m + 1 in ms:
                dt = (int(ms[m + 1]["t_start"]) - int(ms[m]["t_loaded"])) * 0.01
                dc = int(ms[m + 1]["clk_start"]) - int(ms[m]["clk_loaded"])
                us.append(dt)
                if dt > 0:
                    ghz.append(dc / dt / 1e3)
    k = int(rows[0]["k"])
    print(f"compute between refreshes ({k} generations): median {st.median(us):.2f} us ({st.median(us) / k:.3f} us/gen), "
          f"min {min(us):.2f}, max {max(us):.2f}; shader clock median {st.median(ghz):.2f} GHz "
          f"(min {min(ghz):.2f}, max {max(ghz):.2f})")


if __name__ == "__main__":
    main(sys.argv[1])
    compute(sys.argv[1])
