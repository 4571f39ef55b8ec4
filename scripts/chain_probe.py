#!/usr/bin/env python3
"""GPU probe of the chained-group hand-off: forced chained launches (set
GOL_CHAIN=1 in the environment) on the shapes whose waits gave up in the r03
GPU tier; prints per attempt ok / the give-up diagnostics and the time."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gol_amd import life_step, random_grid  # noqa: E402
from gol_amd.ops.life_ops import life_step_torch  # noqa: E402


def main() -> int:
    attempts = int(os.environ.get("PROBE_N", "4"))
    bad = 0
    for layout, W, H, T in (("bits", 6400, 700, 8), ("u8", 6400, 700, 4), ("bits", 6400, 700, 4),
                            ("bits", 2048, 333, 4)):
        g = random_grid(W, H, T)
        want = life_step_torch(g, 2 * T + 3, device="cuda")
        for i in range(attempts):
            t0 = time.time()
            try:
                got = life_step(g, 2 * T + 3, engine="hip", layout=layout, tmax=T)
                msg = "ok" if (got == want).all() else "WRONG"
            except Exception as e:  # noqa: BLE001
                msg = f"ERR {e}"
            bad += msg != "ok"
            print(f"{layout} {W}x{H} T={T} #{i}: {msg} ({time.time() - t0:.2f} s)", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
