"""Text-grid I/O (native, byte-compatible with the reference's format).

Format: H lines of W '0'/'1' characters plus '\\n' (README.md:61).  Readers
are parallel subarray preads (the MPI-IO view math of
src/game_mpi_async.c:168-221) with an fgetc-compatible fallback; a short
file raises instead of hanging (reference quirk Q8).
"""
from __future__ import annotations

import numpy as np

from .._native import native


def read_grid(path: str, width: int, height: int) -> np.ndarray:
    return native().read_text_grid(str(path), int(width), int(height))


def read_tile(path: str, width: int, height: int, rows: tuple[int, int], cols: tuple[int, int]) -> np.ndarray:
    return native().read_text_tile(str(path), int(width), int(height), int(rows[0]), int(rows[1]),
                                   int(cols[0]), int(cols[1]))


def write_grid(path: str, grid: np.ndarray) -> None:
    native().write_text_grid(str(path), np.ascontiguousarray(grid, dtype=np.uint8))


def create_text_file(path: str, width: int, height: int) -> None:
    native().create_text_file(str(path), int(width), int(height))


def write_tile(path: str, width: int, height: int, row0: int, col0: int, tile: np.ndarray) -> None:
    native().write_text_tile(str(path), int(width), int(height), int(row0), int(col0),
                             np.ascontiguousarray(tile, dtype=np.uint8))


def generate(path: str, width: int, height: int, seed: int = 1, density: float = 0.5) -> None:
    """Random text grid (replaces generate.sh; same RNG as device init)."""
    native().generate_text_file(str(path), int(width), int(height), int(seed), float(density))


def parse_text(text: str, width: int, height: int) -> np.ndarray:
    """Pure-Python parser with the reference's fgetc semantics (tests)."""
    cells = [1 if ch == "1" else 0 for ch in text if ch not in "\r\n"]
    if len(cells) < width * height:
        raise ValueError(f"input holds {len(cells)} cells, need {width * height}")
    return np.array(cells[: width * height], dtype=np.uint8).reshape(height, width)


def format_text(grid: np.ndarray) -> str:
    g = np.asarray(grid)
    return "".join("".join("1" if v else "0" for v in row) + "\n" for row in g)


def show_text(grid: np.ndarray) -> str:
    """The reference's VT100 viewer (src/game.c:42-58): cursor home, then per
    row two reverse-video spaces for every live cell and two plain spaces for
    every dead one, and a next-line escape.  (The MPI copy tests truthiness,
    so it shows every cell as live, quirk Q3; here a cell is live if it is
    1 or '1'.)"""
    g = np.asarray(grid)
    live = (g == 1) | (g == ord("1"))
    out = ["\033[H"]
    for row in live:
        out.append("".join("\033[07m  \033[m" if v else "  " for v in row))
        out.append("\033[E")
    return "".join(out)
