"""High-level simulation API over the native engine.

The "model" of this framework is the B3/S23 cellular automaton on a periodic
W x H torus - the single model family of the reference (README.md:4-10): six
programs (serial, MPI x3, MPI+OpenMP, CUDA) that all evolve the same
automaton.  Here those six programs are one engine with pluggable pieces:

======================  ==========================================  ==================================
reference program       this framework                              how to select it
======================  ==========================================  ==================================
src/game.c              ``engine="ref"`` (exact eager serial loop)   ``Simulation(..., engine="ref")``
src/game_openmp.c       ``engine="cpu"`` (threaded bit-sliced)       ``engine="cpu", threads=N``
src/game_cuda.cu        ``engine="hip"`` (CDNA4 temporal blocking)   ``engine="hip"``
src/game_mpi*.c         any engine x ``transport=thread|rccl|torch`` ``Simulation.distributed(...)``
======================  ==========================================  ==================================
"""
from __future__ import annotations

import dataclasses
import time
from typing import Any, Optional

import numpy as np

from .._native import native


@dataclasses.dataclass
class LifeConfig:
    """Runtime configuration; defaults equal the reference's compile-time
    constants (GEN_LIMIT 1000, CHECK_SIMILARITY on, SIMILARITY_FREQUENCY 3:
    src/game.c:6-9)."""

    width: int
    height: int
    gen_limit: int = 1000
    check_similarity: bool = True
    sim_freq: int = 3
    layout: str = "auto"        # auto | bits | u8
    decomp: str = "auto"        # auto | PxQ
    tmax: int = 0               # generations per kernel launch (0 = the backend's choice: bits 12 adder /
                                # 16 DPP; u8 32 / 24 / 16 by tile size)
    epoch: int = 0              # generations per halo exchange (0 = 8*tmax, 16*tmax with several ranks)
    poll_gens: int = 0          # generations between termination polls (0: 256; 512 with several ranks;
                                # 1024 on single-rank device tiles whose polls join the compute streams)
    overlap: str = "auto"       # auto | on (= trigger) | off | trigger: overlap the row halo exchange with compute
    lagged_poll: bool = True    # check termination polls one window late (no queue drain)
    graphs: str = "off"         # auto | on | off: replay full epochs as captured HIP graphs
    start_gen: int = 0          # resume: generation number of the initial state
    sim_phase: int = 0          # resume: similarity counter at start_gen
    timing_barriers: bool = True  # barrier + sync around each run's loop (off: the caller brackets it)
    self_exchange: bool = False   # rehearse the multi-rank row-halo schedule on one rank (transport to self)
    watchdog_s: float = 0.0       # fail when a termination poll waits longer (0 = GOL_WATCHDOG_S or 900 s)
    u8_compute: str = "auto"      # auto | bits | bytes: byte-layout epochs on bit words (packed once per epoch)
                                  # or on the bytes themselves; auto = bits on the GPU with the plain schedule
    # Runtime tuning, key -> value (``native().tuning_keys()``; csrc/include/gol/tuning.hpp): kernel and
    # schedule knobs over the GOL_* environment overrides.  Used by the engine and by the backend this
    # Simulation creates (an explicitly passed backend keeps the tuning it was created with).
    tune: dict = dataclasses.field(default_factory=dict)

    def resolved_layout(self) -> str:
        if self.layout == "auto":
            return "bits" if self.width % 32 == 0 else "u8"
        if self.layout not in ("bits", "u8"):
            raise ValueError(f"unknown layout {self.layout!r}")
        return self.layout

    def to_native(self):
        C = native()
        c = C.EngineConfig()
        c.W = int(self.width)
        c.H = int(self.height)
        c.layout = C.Layout.Bits if self.resolved_layout() == "bits" else C.Layout.U8
        c.decomp = self.decomp
        c.gen_limit = int(self.gen_limit)
        c.check_similarity = bool(self.check_similarity)
        c.sim_freq = int(self.sim_freq)
        c.tmax = int(self.tmax)
        c.epoch = int(self.epoch)
        c.poll_gens = int(self.poll_gens)
        c.overlap = {"auto": -1, "off": 0, "on": 3, "trigger": 3}[self.overlap]
        c.lagged_poll = bool(self.lagged_poll)
        c.graphs = {"auto": -1, "off": 0, "on": 1}[self.graphs]
        c.start_gen = int(self.start_gen)
        c.sim_phase = int(self.sim_phase)
        c.timing_barriers = bool(self.timing_barriers)
        c.self_exchange = bool(self.self_exchange)
        c.watchdog_s = float(self.watchdog_s)
        c.u8_compute = {"auto": -1, "bytes": 0, "bits": 1}[self.u8_compute]
        c.tune = make_tuning(self.tune)
        return c


def make_tuning(tune=None):
    """A native ``Tuning``: the table's defaults, the GOL_* environment, then
    ``tune`` (a dict key -> value, a list of ``"key=value"`` strings, or a
    ``Tuning``, returned as a copy).  Unknown keys and non-integer values of
    integer keys raise."""
    C = native()
    if isinstance(tune, C.Tuning):
        return tune.copy()
    t = C.Tuning.from_env()
    items = tune.items() if isinstance(tune, dict) else (kv.split("=", 1) for kv in (tune or []))
    for k, v in items:
        t.set(str(k), str(int(v)) if isinstance(v, bool) else str(v))
    return t


def parse_tune_args(pairs) -> dict:
    """``["key=value", ...]`` (CLI --tune, repeatable) -> dict, validated."""
    out = {}
    for kv in pairs or []:
        if "=" not in kv:
            raise ValueError(f"--tune {kv!r}: expected key=value")
        k, v = kv.split("=", 1)
        out[k] = v
    make_tuning(out)  # unknown keys / bad values fail here, before any device work
    return out


def make_backend(engine: str = "auto", device: int = 0, threads: int = 0, tune=None):
    """``hip`` -> MI355X backend on ``device``; ``cpu`` -> threaded host backend.
    ``tune``: runtime tuning (see make_tuning), read once, here."""
    C = native()
    if engine == "auto":
        engine = "hip" if C.hip_available() else "cpu"
    if engine == "hip":
        return C.hip_backend(int(device), tune=make_tuning(tune))
    if engine == "cpu":
        return C.cpu_backend(int(threads), tune=make_tuning(tune))
    raise ValueError(f"unknown engine {engine!r} (want hip, cpu or auto)")


# Tuning keys the engine reads from EngineConfig::tune (engine.cpp); the rest
# are read by the backend (or the transports) at construction.
_ENGINE_KEYS = frozenset({"u8_via_bits", "side_poll", "poll_copy_side", "watchdog_s", "overlap_auto",
                          "cpu_side_poll"})


@dataclasses.dataclass
class RunReport:
    generations: int
    executed: int
    stop_reason: str
    loop_ms: float
    first_unchanged: int = -1
    extinct: bool = False
    exchanges: int = 0
    polls: int = 0
    kernel_launches: int = 0
    cells: int = 0
    overlapped: bool = False
    graph_launches: int = 0
    halo_bytes: int = 0
    linked_launches: int = 0  # launches that overlapped the previous one (GOL_LINK)
    # Per-phase device time (Simulation.phase_timing).
    phase_timed: bool = False
    compute_ms: float = 0.0
    halo_ms: float = 0.0
    fill_ms: float = 0.0
    allreduce_ms: float = 0.0

    @property
    def cell_updates_per_s(self) -> float:
        return self.cells * self.executed / (self.loop_ms * 1e-3) if self.loop_ms > 0 else 0.0

    def as_dict(self) -> dict[str, Any]:
        d = dataclasses.asdict(self)
        d["cell_updates_per_s"] = self.cell_updates_per_s
        return d


class Simulation:
    """One rank's view of a (possibly decomposed) Game of Life run.

    Single GPU / CPU::

        sim = Simulation(LifeConfig(1024, 1024), engine="hip")
        sim.load(grid)                    # numpy uint8 H x W (0/1 or ASCII)
        report = sim.run()                # reference termination semantics
        out = sim.gather()                # final grid (rank-local tile if distributed)
    """

    def __init__(self, config: LifeConfig, engine: str = "auto", device: int = 0, threads: int = 0,
                 transport=None, backend=None):
        C = native()
        self.config = config
        self.engine_name = engine
        self.backend = backend if backend is not None else make_backend(engine, device, threads, config.tune)
        self.transport = transport if transport is not None else C.self_transport()
        self._eng = C.Engine(config.to_native(), self.backend, self.transport)
        self.last_report: Optional[RunReport] = None

    # -- geometry --------------------------------------------------------
    @property
    def rank(self) -> int:
        return self._eng.rank

    @property
    def rows(self) -> tuple[int, int]:
        r = self._eng.rows
        return (r.begin, r.end)

    @property
    def cols(self) -> tuple[int, int]:
        c = self._eng.cols
        return (c.begin, c.end)

    @property
    def generation(self) -> int:
        return self._eng.generation

    @property
    def native_engine(self):
        return self._eng

    @property
    def epoch_depth(self) -> int:
        return self._eng.epoch_depth

    @property
    def phase_timing(self) -> bool:
        """Per-phase device timing of the following runs (RunReport.*_ms)."""
        return bool(self._eng.phase_timing)

    @phase_timing.setter
    def phase_timing(self, on: bool) -> None:
        self._eng.phase_timing = bool(on)

    def describe(self) -> dict[str, Any]:
        d = self._eng.decomp
        g = self._eng.compute_geom  # the tile the temporal blocks run on (halos)
        return {"backend": self.backend.name(), "transport": self.transport.name(),
                "layout": self.config.resolved_layout(), "decomp": d.describe(),
                "rank": self.rank, "ranks": d.nranks(), "tile_rows": g.H, "tile_cols": g.W,
                "halo_rows": g.Dv, "halo_words": g.hw, "tmax": self._eng.tmax,
                "epoch": self._eng.epoch_depth, "pitch": self._eng.geom.pitch, "overlap": self._eng.overlap(),
                "graphs": self._eng.graphs(), "overlap_mode": self._eng.overlap_mode(),
                "overlap_trial_ms_plain": self._eng.trial_ms_plain,
                "overlap_trial_ms_trigger": self._eng.trial_ms_trigger,
                "poll_mode": self._eng.poll_mode(),
                "poll_trial_ms_per_window": {"joined": self._eng.poll_trial_ms_joined,
                                             "side": self._eng.poll_trial_ms_side,
                                             "side_steady": self._eng.poll_trial_ms_side_steady},
                "triggered_sends": self._eng.triggered_sends(),
                "u8_compute": ("bits" if self._eng.via_bits else "bytes") if self.config.resolved_layout() == "u8" else None,
                "row_ring": bool(self._eng.row_ring), "row_ring_fallback": self._eng.row_ring_fallback or None,
                "kernel": self._kernel_name(),
                "tuning": self.tuning(), "tuning_changed": self.tuning_changed()}

    def tuning(self) -> dict[str, str]:
        """Effective value of every tuning key of class ``tune`` (the default
        build's knobs): the backend's for its keys, the engine's for the keys
        it reads."""
        be, eng = self.backend.tuning().values(), self._eng.config.tune.values()
        keys = [k for k in native().tuning_keys() if k["class"] == "tune"]
        return {k["key"]: (eng if k["key"] in _ENGINE_KEYS else be)[k["key"]] for k in keys}

    def tuning_changed(self) -> dict[str, str]:
        """Every key off its default, any class: ``value (source)``, source
        ``env`` (a GOL_* variable) or ``set`` (LifeConfig.tune / --tune)."""
        out = {}
        for t in (self.backend.tuning(), self._eng.config.tune):
            for k, v in t.changed().items():
                out.setdefault(k, f"{v} ({t.source(k)})")
        return out

    def _kernel_name(self) -> str:
        """What the temporal blocks run, for reports (bench.py config.kernel)."""
        e = self._eng
        lay = self.config.resolved_layout()
        be = self.backend.name()
        if lay == "u8" and not e.via_bits and "lds-tiled" in be:
            return "LDS-tiled byte kernel (" + be.split("; u8 ")[-1].rstrip("]").strip() + ")"
        window = "adder window (drifting frame)" if e.drifting else "symmetric window"
        parts = [f"bit-sliced temporal blocks, T={e.tmax}", window]
        if lay == "u8":
            parts.append("byte grid packed to bit words once per run" if e.via_bits else "byte-layout kernels")
        if e.row_ring:
            parts.append("row ring (no halo fills)")
        return ", ".join(parts)

    # -- state -----------------------------------------------------------
    def load(self, grid: np.ndarray) -> None:
        """Load the full global grid (each rank copies out its own tile)."""
        g = np.ascontiguousarray(grid, dtype=np.uint8)
        self._eng.load_global(g)

    def load_tile(self, tile: np.ndarray) -> None:
        self._eng.load_cells(np.ascontiguousarray(tile, dtype=np.uint8))

    def load_text(self, path: str) -> None:
        """Parallel subarray read of a text grid (MPI-IO view equivalent)."""
        self._eng.read_text(str(path))

    def init_random(self, seed: int = 1, density: float = 0.5) -> None:
        """Counter-based random init on the device (independent of layout and
        decomposition; equal to ``gol_gen`` / ``generate_text``)."""
        self._eng.init_random(int(seed), float(density))

    def tile(self, ascii: bool = False) -> np.ndarray:
        return self._eng.store_cells(ascii)

    def write_text(self, path: str, create: bool = True) -> None:
        self._eng.write_text(str(path), create)

    def alive_count(self) -> int:
        return int(self._eng.alive_count())

    # -- running ---------------------------------------------------------
    def _report(self, r) -> RunReport:
        rep = RunReport(generations=r.generations, executed=r.executed, stop_reason=r.stop_reason,
                        loop_ms=r.loop_ms, first_unchanged=r.first_unchanged, extinct=r.extinct,
                        exchanges=r.exchanges, polls=r.polls, kernel_launches=r.kernel_launches,
                        cells=self.config.width * self.config.height, overlapped=r.overlapped,
                        graph_launches=r.graph_launches, halo_bytes=r.halo_bytes,
                        linked_launches=r.linked_launches, phase_timed=r.phase_timed,
                        compute_ms=r.compute_ms, halo_ms=r.halo_ms, fill_ms=r.fill_ms,
                        allreduce_ms=r.allreduce_ms)
        self.last_report = rep
        return rep

    def run(self) -> RunReport:
        """Evolve up to ``gen_limit`` with the reference's termination rules."""
        return self._report(self._eng.run())

    def advance(self, n: int) -> RunReport:
        """Evolve exactly ``n`` generations (no early stop)."""
        return self._report(self._eng.advance(int(n)))


def simulate(grid: np.ndarray, gens: int, engine: str = "auto", layout: str = "auto",
             check_similarity: bool = True, sim_freq: int = 3, **kw) -> tuple[np.ndarray, RunReport]:
    """Convenience: run a grid to ``gens`` (reference semantics) on one rank."""
    grid = np.ascontiguousarray(grid, dtype=np.uint8)
    H, W = grid.shape
    cfg = LifeConfig(W, H, gen_limit=gens, check_similarity=check_similarity, sim_freq=sim_freq,
                     layout=layout, **kw)
    sim = Simulation(cfg, engine=engine)
    sim.load(grid)
    rep = sim.run()
    return sim.tile(), rep


def reference_run(grid: np.ndarray, gen_limit: int = 1000, check_similarity: bool = True,
                  sim_freq: int = 3, threads: int = 1) -> tuple[np.ndarray, int, float]:
    """Exact eager serial loop of src/game.c (native).  Returns (grid, gens, ms)."""
    gens, ms, out = native().cpu_reference_run(np.ascontiguousarray(grid, dtype=np.uint8), int(gen_limit),
                                               bool(check_similarity), int(sim_freq), int(threads))
    return out, int(gens), float(ms)


def timed(fn, *a, **kw):
    t0 = time.perf_counter()
    r = fn(*a, **kw)
    return r, (time.perf_counter() - t0) * 1e3
