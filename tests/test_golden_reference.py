"""T2 golden semantics against the reference itself: the
reference's serial src/game.c is compiled in a scratch directory (never
vendored) and run on the same input file as `bin/gol`; the output file must
be byte-identical and the "Generations:" line equal.  The serial reference
indexes [y][x] and is only correct for square grids (README.md:61), so the
grids are square."""
import gzip
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from gol_amd.utils import io

from conftest import generations_line, run_reference_serial
from golden import CASES

GRIDS = [(96, 1, 0.5), (256, 2, 0.5), (64, 11, 0.2), (40, 14, 0.2), (48, 7, 0.3), (33, 4, 0.35)]


def _run_ours(gol_bin, workdir, N, path, *extra):
    r = subprocess.run([str(gol_bin), str(N), str(N), str(path), *map(str, extra)], cwd=workdir,
                       capture_output=True, text=True, timeout=300, check=True)
    return r.stdout, (workdir / "game_output.out").read_bytes()


def _compare(reference_serial, gol_bin, tmp_path, N, grid_file, *extra):
    ref_dir, our_dir = tmp_path / "ref", tmp_path / "ours"
    ref_dir.mkdir(exist_ok=True)
    our_dir.mkdir(exist_ok=True)
    ref_out, ref_bytes = run_reference_serial(reference_serial, ref_dir, N, N, grid_file)
    our_out, our_bytes = _run_ours(gol_bin, our_dir, N, grid_file, *extra)
    assert generations_line(our_out) == generations_line(ref_out)
    assert our_bytes == ref_bytes
    assert len(our_bytes) == N * (N + 1)


@pytest.mark.parametrize("N,seed,density", GRIDS)
@pytest.mark.parametrize("engine", ["cpu", "ref"])
def test_output_bytes_match_reference_game_c(reference_serial, gol_bin, tmp_path, N, seed, density, engine):
    f = tmp_path / "in.txt"
    io.generate(str(f), N, N, seed=seed, density=density)
    _compare(reference_serial, gol_bin, tmp_path, N, f, "--engine", engine)


@pytest.mark.parametrize("name,grid,gens", [c for c in CASES if c[1].shape[0] == c[1].shape[1]])
def test_golden_patterns_match_reference_game_c(reference_serial, gol_bin, tmp_path, name, grid, gens):
    N = grid.shape[0]
    f = tmp_path / "in.txt"
    io.write_grid(str(f), np.asarray(grid))
    _compare(reference_serial, gol_bin, tmp_path, N, f, "--engine", "cpu")


def test_stdout_contract_serial(reference_serial, gol_bin, tmp_path):
    """Same stdout lines as game.c (only the timing value differs)."""
    f = tmp_path / "in.txt"
    io.generate(str(f), 32, 32, seed=3)
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    ref_out, _ = run_reference_serial(reference_serial, tmp_path / "a", 32, 32, f)
    our_out, _ = _run_ours(gol_bin, tmp_path / "b", 32, f, "--engine", "cpu")
    strip = lambda s: [ln.split("\t")[0] for ln in s.splitlines()]  # noqa: E731
    assert strip(our_out) == strip(ref_out)


@pytest.mark.gpu
@pytest.mark.parametrize("N,seed,density", GRIDS)
def test_output_bytes_match_reference_game_c_on_gpu(reference_serial, gol_bin, tmp_path, N, seed, density):
    f = tmp_path / "in.txt"
    io.generate(str(f), N, N, seed=seed, density=density)
    _compare(reference_serial, gol_bin, tmp_path, N, f, "--engine", "hip")


# Recorded outputs of the same reference build on the same GRIDS inputs
# (tests/make_game_c_fixtures.py), for boxes without the reference mount.
FIXTURES = Path(__file__).resolve().parent / "fixtures" / "game_c"


def _fixture(N, seed, density):
    key = f"{N}_{seed}_{density}"
    gens = json.loads((FIXTURES / "generations.json").read_text())[key]
    return gens, gzip.decompress((FIXTURES / f"{key}.out.gz").read_bytes())


def _compare_fixture(gol_bin, tmp_path, N, seed, density, engine):
    f = tmp_path / "in.txt"
    io.generate(str(f), N, N, seed=seed, density=density)
    our_out, our_bytes = _run_ours(gol_bin, tmp_path, N, f, "--engine", engine)
    gens, want = _fixture(N, seed, density)
    assert generations_line(our_out) == gens
    assert our_bytes == want


@pytest.mark.parametrize("N,seed,density", GRIDS)
def test_output_bytes_match_recorded_game_c(gol_bin, tmp_path, N, seed, density):
    _compare_fixture(gol_bin, tmp_path, N, seed, density, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("N,seed,density", GRIDS)
def test_output_bytes_match_recorded_game_c_on_gpu(gol_bin, tmp_path, N, seed, density):
    _compare_fixture(gol_bin, tmp_path, N, seed, density, "hip")


@pytest.mark.parametrize("N,seed,density", GRIDS)
def test_recorded_game_c_fixtures_are_current(reference_serial, tmp_path, N, seed, density):
    f = tmp_path / "in.txt"
    io.generate(str(f), N, N, seed=seed, density=density)
    ref_out, ref_bytes = run_reference_serial(reference_serial, tmp_path, N, N, f)
    assert _fixture(N, seed, density) == (generations_line(ref_out), ref_bytes)
