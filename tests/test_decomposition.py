"""T0: decomposition math (native vs an independent Python statement)."""
import itertools

import pytest

from gol_amd.parallel.decomposition import EAST, NORTH, SOUTH, WEST, PyDecomposition, split_range


@pytest.mark.parametrize("n,p", [(10, 3), (96, 4), (7, 7), (1000, 8), (33, 5)])
def test_split_range_balanced(native, n, p):
    parts = [split_range(n, p, i) for i in range(p)]
    assert parts[0][0] == 0 and parts[-1][1] == n
    for (b0, e0), (b1, _) in zip(parts, parts[1:]):
        assert e0 == b1
    sizes = [e - b for b, e in parts]
    assert max(sizes) - min(sizes) <= 1
    for i in range(p):
        e = native.split_range(n, p, i)
        assert (e.begin, e.end) == parts[i]


@pytest.mark.parametrize("Px,Py", [(1, 1), (1, 8), (8, 1), (2, 4), (4, 2), (3, 3), (2, 2), (5, 1)])
def test_neighbors_and_extents(native, Px, Py):
    W, H, unit = 32 * 20, 97, 32
    d = native.Decomposition(W, H, Px, Py, unit)
    pd = PyDecomposition(W, H, Px, Py, unit)
    covered = set()
    for r in range(Px * Py):
        assert list(d.neighbors(r)) == pd.neighbors(r)
        rr, cc = d.rows(r), d.cols(r)
        assert (rr.begin, rr.end) == pd.rows(r)
        assert (cc.begin, cc.end) == pd.cols(r)
        assert cc.begin % unit == 0 and cc.end % unit == 0
        covered.add((rr.begin, cc.begin))
    assert len(covered) == Px * Py


def test_north_is_previous_rows(native):
    # The reference swaps N/S (src/game_mpi.c:293-294, quirk Q1); here north
    # is the tile that holds the rows just above ours, with periodic wrap.
    d = native.Decomposition(64, 90, 1, 3, 1)
    for r in range(3):
        nb = d.neighbors(r)
        assert d.rows(nb[NORTH]).end % 90 == d.rows(r).begin
        assert d.rows(nb[SOUTH]).begin == d.rows(r).end % 90
    d2 = native.Decomposition(96, 10, 3, 1, 32)
    for r in range(3):
        nb = d2.neighbors(r)
        assert d2.cols(nb[WEST]).end % 96 == d2.cols(r).begin
        assert d2.cols(nb[EAST]).begin == d2.cols(r).end % 96


def test_make_specs(native):
    assert native.Decomposition.make(64, 64, 8, "auto", 32).describe() == "1x8"
    assert native.Decomposition.make(64, 64, 8, "2x4", 32).describe() == "2x4"
    assert native.Decomposition.make(256, 4, 8, "auto", 32).describe() == "8x1"  # too few rows
    with pytest.raises(RuntimeError):
        native.Decomposition.make(64, 64, 8, "3x3", 32)
    with pytest.raises(RuntimeError):
        native.Decomposition.make(64, 64, 8, "bogus", 32)


def test_non_square_process_counts_supported(native):
    # The reference aborts for non-square P (quirk Q4); every P works here.
    for P in range(1, 9):
        for Px, Py in itertools.product(range(1, P + 1), repeat=2):
            if Px * Py == P:
                d = native.Decomposition(32 * 16, 64, Px, Py, 32)
                assert d.nranks() == P
