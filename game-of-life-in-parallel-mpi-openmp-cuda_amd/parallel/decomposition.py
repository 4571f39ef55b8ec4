"""Pure-Python mirror of the native decomposition (csrc/src/decomp.cpp).

Used by tests as an independent statement of the topology contract:
periodic Px x Py torus, rank = py*Px + px, "north" = previous rows.  The
reference computes N = row+1 / S = row-1 (src/game_mpi.c:293-294), which is
only right for q <= 2; this mirror pins the corrected
orientation.
"""
from __future__ import annotations

from dataclasses import dataclass

NORTH, SOUTH, WEST, EAST, NW, NE, SW, SE = range(8)


def split_range(n: int, p: int, i: int) -> tuple[int, int]:
    base, rem = divmod(n, p)
    b = i * base + min(i, rem)
    return b, b + base + (1 if i < rem else 0)


@dataclass(frozen=True)
class PyDecomposition:
    W: int
    H: int
    Px: int
    Py: int
    col_unit: int = 1

    def coords(self, rank: int) -> tuple[int, int]:
        return rank % self.Px, rank // self.Px

    def rank_of(self, px: int, py: int) -> int:
        return (py % self.Py) * self.Px + (px % self.Px)

    def rows(self, rank: int) -> tuple[int, int]:
        return split_range(self.H, self.Py, self.coords(rank)[1])

    def cols(self, rank: int) -> tuple[int, int]:
        b, e = split_range(self.W // self.col_unit, self.Px, self.coords(rank)[0])
        return b * self.col_unit, e * self.col_unit

    def neighbors(self, rank: int) -> list[int]:
        px, py = self.coords(rank)
        d = [(0, -1), (0, 1), (-1, 0), (1, 0), (-1, -1), (1, -1), (-1, 1), (1, 1)]
        return [self.rank_of(px + dx, py + dy) for dx, dy in d]
