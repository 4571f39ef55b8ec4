#!/usr/bin/env python3
"""In-process A/B of termination-poll intervals (round 6): engines with
different poll_gens on the same grid, alternating 1000-generation runs with
termination polls (Engine.run_until) in one process, so process-level
run-to-run spread (memory placement, clocks) is shared by both.

    python scripts/poll_ab.py [SIZE] [LAYOUT] [ROUNDS] [POLLS...]
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import gol_amd  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
layout = sys.argv[2] if len(sys.argv) > 2 else "bits"
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 30
polls = [int(x) for x in sys.argv[4:]] or [256, 1024]
sims = {}
for p in polls:
    s = gol_amd.Simulation(gol_amd.LifeConfig(S, S, gen_limit=10**9, layout=layout, poll_gens=p,
                                              check_similarity=False), engine="hip")
    s.init_random(1, 0.5)
    s.native_engine.run_until(s.generation + 4000)  # warm-up
    sims[p] = s
ms = {p: [] for p in polls}
for _ in range(rounds):
    for p, s in sims.items():
        eng = s.native_engine
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_until(eng.generation + 1000)
        torch.cuda.synchronize()
        ms[p].append((time.perf_counter() - t0) * 1e3)
for p in polls:
    v = ms[p]
    print(f"{S}^2 {layout} poll {p}: median {statistics.median(v):.3f} ms, min {min(v):.3f}, max {max(v):.3f} "
          f"({len(v)} runs)")
