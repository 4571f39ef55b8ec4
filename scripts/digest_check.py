#!/usr/bin/env python3
"""Final-grid digests of the single-rank default path, for comparing two
trees bit for bit ("bench.py output is bit-identical
before and after"): each case initialises the bench's random grid (seed 1,
density 0.5) on the device, advances N generations with the default schedule
and prints the sha256 of the owned cells (0/1 bytes, row-major).

    python scripts/digest_check.py [TREE]    # TREE: a checkout holding gol_amd
"""
import hashlib
import os
import sys
import time

tree = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, tree)
import numpy as np  # noqa: E402

import gol_amd  # noqa: E402

CASES = [("32768^2 bits", 32768, "bits", 2000), ("32768^2 u8", 32768, "u8", 2000),
         ("8192^2 u8", 8192, "u8", 3000), ("8192^2 bits", 8192, "bits", 3000)]
print(f"tree {tree}: module {gol_amd.native().__file__}", flush=True)
for name, S, layout, gens in CASES:
    sim = gol_amd.Simulation(gol_amd.LifeConfig(S, S, gen_limit=10**9, layout=layout), engine="hip")
    sim.init_random(1, 0.5)
    t0 = time.perf_counter()
    sim.advance(gens)
    dt = time.perf_counter() - t0
    g = np.ascontiguousarray(sim.tile(), dtype=np.uint8)
    print(f"{name} x {gens}: sha256 {hashlib.sha256(g.tobytes()).hexdigest()}  alive {int(g.sum())}  "
          f"({dt * 1e3:.0f} ms incl. warm-up)", flush=True)
    del sim
