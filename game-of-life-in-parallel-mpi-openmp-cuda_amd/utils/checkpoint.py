"""Checkpoint / resume.

Reference: no explicit checkpointing, but the output file is in exactly the
input format, so ``./a.out N N game_output.out`` resumes from the last
generation - losing the generation counter and the similarity-counter phase
(src/game.c:171).  Here a checkpoint is

* ``grid-<gen>[b].txt`` - the text grid, written by every rank at its
  subarray offsets (same path as the output writer, so it stays a valid
  input), and
* ``meta.json`` - generation number, similarity phase, run config and the
  name of its grid file,

so a resumed run reproduces an uninterrupted one exactly (same final grid,
same "Generations" line).  A new checkpoint writes a grid file the committed
one does not use, fsyncs it, then replaces meta.json atomically and only
then deletes the old grid: a crash at any point leaves one complete
checkpoint (csrc/include/gol/checkpoint.hpp, same format).
"""
from __future__ import annotations

import json
import os
import re
from pathlib import Path
from typing import Optional

from ..models.life import LifeConfig, RunReport, Simulation
from .termination import reported_generations, sim_phase_at


_GRID_NAME = re.compile(r"grid-[0-9]+b?\.txt")
# Grids a checkpoint created that no commit has taken over yet (one name per
# line; the same file as csrc/src/checkpoint.cpp's kInflightName).
INFLIGHT = ".gol-inflight"


def grid_name_ok(name) -> bool:
    """Whether ``name`` may be a checkpoint's grid file: the plain basename
    ``grid-<digits>[b].txt`` or the legacy ``grid.txt`` - never a path, "..",
    or meta.json, so a tampered meta.json cannot make a resume read, or a
    commit delete, anything else (checkpoint.cpp:checkpoint_grid_name_ok)."""
    return isinstance(name, str) and (name == "grid.txt" or _GRID_NAME.fullmatch(name) is not None)


def _meta_grid(meta: dict, directory) -> str:
    name = meta.get("grid", "grid.txt")
    if not grid_name_ok(name):
        raise ValueError(f"checkpoint '{directory}': bad grid file name {name!r} "
                         "(expected grid-<generation>[b].txt)")
    return name


def committed_grid(directory) -> Optional[str]:
    """Grid file name of the committed checkpoint in ``directory`` (None: none)."""
    meta = Path(directory) / "meta.json"
    if not meta.exists():
        return None
    return _meta_grid(json.loads(meta.read_text()), directory)


def _fsync(path: Path, directory: bool = False) -> None:
    fd = os.open(str(path), os.O_RDONLY | (os.O_DIRECTORY if directory else 0))
    try:
        os.fsync(fd)
    except OSError:
        if not directory:
            raise
    finally:
        os.close(fd)


def save_checkpoint(sim: Simulation, directory: str, is_root: bool = True, barrier=None) -> Path:
    d = Path(directory)
    if is_root:
        d.mkdir(parents=True, exist_ok=True)
    if barrier:
        barrier()
    cfg = sim.config
    gen = sim.generation
    # Every rank picks the same fresh name (nobody commits before the last
    # barrier below), never the committed checkpoint's file.
    previous = committed_grid(d)
    name = f"grid-{gen}.txt"
    if name == previous:
        name = f"grid-{gen}b.txt"
    meta = {
        "format": "gol-mi355x-checkpoint-v1",
        "width": cfg.width, "height": cfg.height, "generation": gen,
        "sim_phase": sim_phase_at(gen, cfg.start_gen, cfg.sim_phase, cfg.sim_freq),
        "gen_limit": cfg.gen_limit, "check_similarity": cfg.check_similarity,
        "sim_freq": cfg.sim_freq, "layout": cfg.resolved_layout(), "grid": name,
    }
    grid = d / name
    if is_root:
        from .io import create_text_file  # noqa: PLC0415
        # Recorded before it exists: a commit sweeps only grids a checkpoint
        # of ours created, never a user's file named like one.
        with open(d / INFLIGHT, "a") as f:
            f.write(name + "\n")
        create_text_file(str(grid), cfg.width, cfg.height)
    if barrier:
        barrier()
    sim.write_text(str(grid), create=False)
    if barrier:
        barrier()
    if is_root:
        if os.environ.get("GOL_FAULT_CHECKPOINT_CRASH_PY") == str(gen):  # fault injection (tests)
            os._exit(86)
        _fsync(grid)
        tmp = d / "meta.json.tmp"
        tmp.write_text(json.dumps(meta, indent=1))
        _fsync(tmp)
        os.replace(tmp, d / "meta.json")
        _fsync(d, directory=True)
        if previous and previous != name and (d / previous).exists():
            (d / previous).unlink()
        # Grids an interrupted checkpoint of ours left behind (crash before
        # commit): the names in the in-flight list, which is then cleared.
        inflight = d / INFLIGHT
        if inflight.exists():
            for orphan in inflight.read_text().split():
                if orphan != name and grid_name_ok(orphan):
                    (d / orphan).unlink(missing_ok=True)
            inflight.unlink(missing_ok=True)
    if barrier:
        barrier()
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
    return cfg, d / _meta_grid(meta, d)


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
