"""Checkpoint / resume.

Reference: no explicit checkpointing, but the output file is in exactly the
input format, so ``./a.out N N game_output.out`` resumes from the last
generation - losing the generation counter and the similarity-counter phase
(src/game.c:171).  Here a checkpoint is

* ``grid.txt``  - the text grid, written by every rank at its subarray
  offsets (same path as the output writer, so it stays a valid input), and
* ``meta.json`` - generation number, similarity phase and run config,

so a resumed run reproduces an uninterrupted one exactly (same final grid,
same "Generations" line).
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Optional

from ..models.life import LifeConfig, RunReport, Simulation
from .termination import reported_generations, sim_phase_at


def save_checkpoint(sim: Simulation, directory: str, is_root: bool = True, barrier=None) -> Path:
    d = Path(directory)
    if is_root:
        d.mkdir(parents=True, exist_ok=True)
    if barrier:
        barrier()
    cfg = sim.config
    gen = sim.generation
    meta = {
        "format": "gol-mi355x-checkpoint-v1",
        "width": cfg.width, "height": cfg.height, "generation": gen,
        "sim_phase": sim_phase_at(gen, cfg.start_gen, cfg.sim_phase, cfg.sim_freq),
        "gen_limit": cfg.gen_limit, "check_similarity": cfg.check_similarity,
        "sim_freq": cfg.sim_freq, "layout": cfg.resolved_layout(),
    }
    grid = d / "grid.txt"
    if is_root:
        from .io import create_text_file  # noqa: PLC0415
        create_text_file(str(grid), cfg.width, cfg.height)
    if barrier:
        barrier()
    sim.write_text(str(grid), create=False)
    if barrier:
        barrier()
    if is_root:
        tmp = d / "meta.json.tmp"
        tmp.write_text(json.dumps(meta, indent=1))
        os.replace(tmp, d / "meta.json")
    return d


def load_checkpoint(directory: str, **overrides) -> tuple[LifeConfig, Path]:
    d = Path(directory)
    meta = json.loads((d / "meta.json").read_text())
    cfg = LifeConfig(meta["width"], meta["height"], gen_limit=meta["gen_limit"],
                     check_similarity=meta["check_similarity"], sim_freq=meta["sim_freq"],
                     layout=meta.get("layout", "auto"), start_gen=meta["generation"],
                     sim_phase=meta["sim_phase"])
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg, d / "grid.txt"


def run_with_checkpoints(sim: Simulation, every: int, directory: Optional[str], is_root: bool = True,
                         barrier=None) -> RunReport:
    """Run to gen_limit, writing a checkpoint every ``every`` generations."""
    cfg = sim.config
    limit = cfg.gen_limit
    eng = sim.native_engine
    total_ms, executed, exch, polls, launches = 0.0, 0, 0, 0, 0
    while True:
        target = min(limit, sim.generation + every) if every > 0 else limit
        r = eng.run_until(target)
        total_ms += r.loop_ms
        executed += r.executed
        exch += r.exchanges
        polls += r.polls
        launches += r.kernel_launches
        if r.first_unchanged >= 0 or sim.generation >= limit:
            gens, reason = reported_generations(r.first_unchanged, r.extinct, limit, cfg.start_gen,
                                                cfg.check_similarity, cfg.sim_freq, cfg.sim_phase)
            return RunReport(gens, executed, reason, total_ms, r.first_unchanged, r.extinct, exch,
                             polls, launches, cfg.width * cfg.height)
        if directory:
            save_checkpoint(sim, directory, is_root, barrier)
