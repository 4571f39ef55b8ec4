#!/usr/bin/env python3
"""In-process check of engines created one after another (round 6): N engines
of the same configuration on one grid, alternating 1000-generation runs with
termination polls (Engine.run_until), so an engine that runs slower only
because of its place in the process shows up beside the others.  Found with
it: HIP maps streams round-robin onto GPU_MAX_HW_QUEUES hardware queues (4 by
default), so the second engine's two linked compute streams shared a queue
and its linked launches serialised (8192^2 2.83 vs 1.48-1.51 ms; with 8
queues 1.50 for all three).  Fixed since: a backend created while another
lives on its device gives its second linked stream a hardware queue of its own
(tuning link_queue = -1, a stream CU-masked to the whole device): 1.49-1.55 ms
for all three with 4 queues; link_queue=0 shows the old behaviour.

    python scripts/engines_ab.py [SIZE] [ENGINES] [ROUNDS]
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import gol_amd  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 20
sims = []
for i in range(n):
    s = gol_amd.Simulation(gol_amd.LifeConfig(S, S, gen_limit=10**9, check_similarity=False), engine="hip")
    s.init_random(1, 0.5)
    s.native_engine.run_until(s.generation + 4000)
    sims.append(s)
ms = [[] for _ in sims]
for _ in range(rounds):
    for i, s in enumerate(sims):
        eng = s.native_engine
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_until(eng.generation + 1000)
        torch.cuda.synchronize()
        ms[i].append((time.perf_counter() - t0) * 1e3)
q = os.environ.get("GPU_MAX_HW_QUEUES", "default")
for i, v in enumerate(ms):
    print(f"{S}^2 GPU_MAX_HW_QUEUES={q} engine {i} (ring {sims[i].native_engine.row_ring}, Dv "
          f"{sims[i].native_engine.geom.Dv}): median {statistics.median(v):.3f} ms, min {min(v):.3f}, max {max(v):.3f}")
