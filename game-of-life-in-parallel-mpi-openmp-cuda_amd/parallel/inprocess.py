"""In-process ranks: P subdomains driven by P host threads in one process.

Two uses:

* T3 tests: a 1-GPU box cannot host two RCCL ranks (RCCL
  refuses duplicate devices), so decomposition, halo routing, deep halos and
  the distributed termination logic are exercised with several subdomains on
  one device through the native ``ThreadTransport`` (device-to-device copies).
* Single-process multi-GPU runs (``devices=[0..7]``), the analogue of the
  reference's hybrid "ranks x threads" build (src/game_openmp.c) - one host
  driver thread per GPU.
"""
from __future__ import annotations

import threading
from typing import Callable, Optional, Sequence

import numpy as np

from .._native import native
from ..models.life import LifeConfig, RunReport, Simulation, make_backend, make_tuning


class InProcessGroup:
    def __init__(self, config: LifeConfig, nranks: int, engine: str = "auto",
                 devices: Optional[Sequence[int]] = None, threads_per_rank: int = 1):
        C = native()
        self.config = config
        self.nranks = int(nranks)
        self.hub = C.ThreadHub(self.nranks)
        devs = list(devices) if devices else [0]
        self.sims: list[Simulation] = []
        self.backends = []
        # Every backend before any engine, so that all ranks' devices are set
        # up before any schedule is decided.  (Several engines on one device
        # share its hardware queues: their linked launches may serialise,
        # docs/PERFORMANCE.md "Open problems"; results are exact either way.)
        self.backends = [make_backend(engine, devs[r % len(devs)], threads_per_rank, config.tune)
                         for r in range(self.nranks)]
        for r, be in enumerate(self.backends):
            tr = C.thread_transport(self.hub, r, be, tune=make_tuning(config.tune))
            self.sims.append(Simulation(config, transport=tr, backend=be))

    def parallel(self, fn: Callable[[Simulation], object]) -> list:
        out: list = [None] * self.nranks
        errs: list = [None] * self.nranks

        def work(r):
            try:
                # A new thread starts on device 0: bind this rank's GPU first
                # (every backend entry point also switches to its device).
                self.backends[r].bind_thread()
                out[r] = fn(self.sims[r])
            except BaseException as e:  # noqa: BLE001
                errs[r] = e

        ts = [threading.Thread(target=work, args=(r,)) for r in range(self.nranks)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for e in errs:
            if e is not None:
                raise e
        return out

    def load(self, grid: np.ndarray) -> None:
        g = np.ascontiguousarray(grid, dtype=np.uint8)
        self.parallel(lambda s: s.load(g))

    def init_random(self, seed: int, density: float = 0.5) -> None:
        self.parallel(lambda s: s.init_random(seed, density))

    def run(self) -> list[RunReport]:
        return self.parallel(lambda s: s.run())

    def advance(self, n: int) -> list[RunReport]:
        return self.parallel(lambda s: s.advance(n))

    def gather(self) -> np.ndarray:
        out = np.zeros((self.config.height, self.config.width), dtype=np.uint8)
        for s in self.sims:
            (r0, r1), (c0, c1) = s.rows, s.cols
            out[r0:r1, c0:c1] = s.tile()
        return out
