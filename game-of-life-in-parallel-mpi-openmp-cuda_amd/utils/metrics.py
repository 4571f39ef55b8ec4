"""Metrics and reporting.

The reference reports only ``Generations`` / ``Execution time`` (and, for
MPI, ``Reading file`` / ``Writing file``) via printf on rank 0
(src/game.c:201-203, src/game_mpi.c:264-265, 426-427, 466).
These helpers keep those exact lines and add a JSON record with throughput,
per-phase times and the parallel layout.
"""
from __future__ import annotations

import json
from typing import Any, Optional


def stdout_lines(style: str, generations: int, loop_ms: float, read_ms: float = 0.0,
                 write_ms: float = 0.0, nranks: int = 1) -> str:
    """The exact stdout of the matching reference build."""
    if style in ("mpi", "async", "collective", "openmp"):
        s = (f"Reading file:\t{read_ms:.2f} msecs\n"
             f"Generations:\t{generations}\n"
             f"Execution time:\t{loop_ms:.2f} msecs\n"
             f"Writing file:\t{write_ms:.2f} msecs\n")
        if style != "openmp":  # every MPI process prints it (src/game_mpi.c:514)
            s += "Finished\n" * nranks
        return s
    if style == "cuda":
        return f"Generations:\t{generations}\nExecution time:\t{loop_ms:.2f} msecs\nFinished\n"
    return f"Finished.\n\nGenerations:\t{generations}\nExecution time:\t{loop_ms:.2f} msecs\nFinished\n"


def write_json(path: Optional[str], record: dict[str, Any]) -> None:
    if not path:
        return
    with open(path, "w") as f:
        json.dump(record, f, indent=1, sort_keys=True)
        f.write("\n")
