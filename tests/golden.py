"""Golden patterns and expected reference outcomes.

The expected "Generations" values were established against the reference's
serial build (src/game.c): a still-life block reports 2, a single cell 1, an
empty grid 0, and a glider on an 8x8 torus runs 1000 generations ending
displaced by (+2, +2) (1000 gens = 250 glider periods of (+1,+1) per 4).
"""
import numpy as np


def pattern(rows):
    return np.array([[1 if c == "1" else 0 for c in r] for r in rows], dtype=np.uint8)


BLOCK = pattern(["000000", "000000", "001100", "001100", "000000", "000000"])
SINGLE = pattern(["000000", "000000", "001000", "000000", "000000", "000000"])
EMPTY = np.zeros((6, 6), dtype=np.uint8)
BLINKER = pattern(["00000", "00100", "00100", "00100", "00000"])
GLIDER = pattern(["00000000", "00100000", "00010000", "01110000", "00000000", "00000000",
                  "00000000", "00000000"])

# (name, grid, expected Generations)
CASES = [("block", BLOCK, 2), ("single", SINGLE, 1), ("empty", EMPTY, 0), ("blinker", BLINKER, 1000),
         ("glider", GLIDER, 1000)]

# Random grids that reach a fixed point before GEN_LIMIT: (W, H, seed, density)
CONVERGING = [(16, 16, 1, 0.2), (16, 16, 3, 0.5), (20, 12, 4, 0.2), (20, 12, 6, 0.2), (33, 17, 4, 0.35),
              (40, 40, 14, 0.2), (64, 32, 11, 0.2), (64, 32, 21, 0.5)]
