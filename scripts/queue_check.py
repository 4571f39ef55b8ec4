#!/usr/bin/env python3
"""Hardware queues and overlap of the temporal-block launches in rocprofv3
kernel traces (round 6): for each trace, the (Queue_Id, Stream_Id) pairs the
grouped kernels ran on, how many consecutive launches overlapped (the next
started before the previous ended: linking at work), and the median launch
period, next to the bench line's ms per step.  Two linked streams that share
one hardware queue serialise their launches.

    queue_check.py DIR [DIR ...]     (each: rocprofv3 -d DIR -o run, DIR.json the bench line)
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        print(d, "no trace")
        continue
    rows = [r for r in csv.DictReader(open(f[0])) if "life_group_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    qs = collections.Counter((r["Queue_Id"], r["Stream_Id"]) for r in rows)
    s = [int(r["Start_Timestamp"]) for r in rows]
    e = [int(r["End_Timestamp"]) for r in rows]
    over = sum(1 for i in range(1, len(rows)) if s[i] < e[i - 1])
    period = statistics.median(s[i] - s[i - 1] for i in range(1, len(rows))) / 1e3 if len(rows) > 1 else 0
    ms = "?"
    try:
        ms = "%.3f" % json.loads(open(d + ".json").read().strip().splitlines()[-1])["ms_per_step"]
    except Exception:  # noqa: BLE001
        pass
    print(f"{os.path.basename(d)}: ms/step {ms}; launches {len(rows)}, overlapped {over}; median period "
          f"{period:.1f} us; (queue, stream): {dict(qs)}")
