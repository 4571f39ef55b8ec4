#!/usr/bin/env python3
"""GPU debug probe for the T = 48 pipelined byte pass: one 48-generation
block on tiles of several heights / wave-count targets, compared with the
fp32 conv oracle; prints where the mismatching rows are."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from gol_amd import LifeConfig, Simulation, random_grid  # noqa: E402
from gol_amd.ops.life_ops import life_step_torch  # noqa: E402


def main() -> int:
    T = int(os.environ.get("PROBE_T", "48"))
    for W in (6400, 1999, 32768):
        for H in (700, 1500, 8000):
            for target in ("0", "3000", "100000"):
                os.environ["GOL_TARGET_WAVES"] = target
                g = random_grid(W, H, W + H)
                want = life_step_torch(g, T, device="cuda")
                sim = Simulation(LifeConfig(W, H, gen_limit=T, layout="u8", tmax=T, epoch=T), engine="hip")
                if sim.describe()["tmax"] != T:
                    print(f"W={W} H={H}: tmax {sim.describe()['tmax']}", flush=True)
                    continue
                sim.load(g)
                sim.advance(T)
                got = sim.tile()
                bad = np.nonzero((got != want).any(axis=1))[0]
                cols = np.nonzero((got != want).any(axis=0))[0]
                msg = "ok" if bad.size == 0 else (f"{bad.size} bad rows: {bad[:8].tolist()}...{bad[-4:].tolist()} "
                                                  f"cols {cols.size}: {cols[:6].tolist()}...{cols[-3:].tolist()}")
                print(f"W={W} H={H} target={target}: {msg}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
