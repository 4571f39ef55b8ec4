"""T1/T2 on the CPU backend: kernels vs oracles, termination semantics vs the
exact serial loop (src/game.c), temporal blocking / epoch / layout variants."""
import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, life_step, life_step_numpy, life_step_torch, random_grid, \
    reference_run, simulate
from gol_amd.utils.termination import reported_generations

from golden import CASES, CONVERGING, GLIDER


@pytest.mark.parametrize("W,H", [(1, 1), (2, 2), (3, 5), (31, 7), (33, 33), (64, 3), (65, 40), (100, 1)])
def test_life_step_u8_awkward_sizes_vs_oracles(native, W, H):
    g = random_grid(W, H, W * 131 + H)
    for gens in (1, 5):
        want = life_step_numpy(g, gens)
        assert (life_step_torch(g, gens) == want).all()
        assert (life_step(g, gens, engine="cpu", layout="u8") == want).all()


@pytest.mark.parametrize("W,H", [(32, 1), (32, 32), (64, 5), (96, 70), (160, 33)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_life_step_word_sizes(native, W, H, layout):
    g = random_grid(W, H, W + 7 * H)
    assert (life_step(g, 7, engine="cpu", layout=layout) == life_step_numpy(g, 7)).all()


@pytest.mark.parametrize("tmax", [1, 2, 4, 8, 16, 32])
@pytest.mark.parametrize("epoch", [0, 1, 5, 33, 100])
def test_temporal_block_and_epoch_variants(native, tmax, epoch):
    g = random_grid(64, 48, 17)
    got = life_step(g, 77, engine="cpu", tmax=tmax, epoch=epoch)
    assert (got == life_step_numpy(g, 77)).all()


@pytest.mark.parametrize("epoch", [0, 50, 96, 200])
def test_deep_byte_schedule_t32(native, epoch):
    """The byte layout's deep schedule (kTSizes 32 / 24 / 16 ... split of an
    epoch) on the CPU backend, with and without an early-stop poll."""
    g = random_grid(70, 120, 5)
    got = life_step(g, 211, engine="cpu", layout="u8", tmax=32, epoch=epoch)
    assert (got == life_step_numpy(g, 211)).all()


@pytest.mark.parametrize("name,grid,gens", CASES)
@pytest.mark.parametrize("layout", ["auto", "u8"])
def test_golden_patterns(native, name, grid, gens, layout):
    out, rep = simulate(grid, 1000, engine="cpu", layout=layout)
    ref, rgens, _ = reference_run(grid)
    assert rep.generations == gens == rgens
    assert (out == ref).all()


def test_glider_displacement(native):
    out, rep = simulate(GLIDER, 1000, engine="cpu")
    assert rep.generations == 1000
    assert (out == np.roll(np.roll(GLIDER, 2, 0), 2, 1)).all()


@pytest.mark.parametrize("W,H,seed,density", CONVERGING)
def test_lazy_termination_matches_eager_reference(native, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    assert rgens < 1000
    for tmax, epoch, poll in [(16, 0, 0), (4, 7, 5), (1, 1, 1), (32, 64, 1000)]:
        out, rep = simulate(g, 1000, engine="cpu", tmax=tmax, epoch=epoch, poll_gens=poll)
        assert rep.generations == rgens, (tmax, epoch, poll)
        assert (out == ref).all()


@pytest.mark.parametrize("freq", [1, 2, 3, 5, 7])
@pytest.mark.parametrize("sim", [True, False])
def test_similarity_frequency_and_switch(native, freq, sim):
    g = random_grid(20, 12, 4, 0.2)
    ref, rgens, _ = reference_run(g, 1000, sim, freq)
    out, rep = simulate(g, 1000, engine="cpu", check_similarity=sim, sim_freq=freq)
    assert rep.generations == rgens
    assert (out == ref).all()


@pytest.mark.parametrize("limit", [0, 1, 2, 3, 10, 37, 200])
def test_generation_limits(native, limit):
    g = random_grid(33, 17, 4, 0.35)
    ref, rgens, _ = reference_run(g, limit)
    out, rep = simulate(g, limit, engine="cpu")
    assert rep.generations == rgens
    assert (out == ref).all()


def test_reported_generations_function():
    # extinction at g_f-1; similarity at the first check >= g_f; else limit
    assert reported_generations(5, True, 1000) == (4, "extinction")
    assert reported_generations(5, False, 1000) == (5, "similarity")
    assert reported_generations(6, False, 1000) == (5, "similarity")
    assert reported_generations(7, False, 1000) == (8, "similarity")
    assert reported_generations(7, False, 8) == (8, "fixed_point")
    assert reported_generations(7, False, 1000, check_similarity=False) == (1000, "fixed_point")
    assert reported_generations(-1, False, 1000) == (1000, "limit")
    assert reported_generations(7, False, 1000, start_gen=1, sim_phase=0) == (6, "similarity")


def test_advance_exact_and_generation_counter(native):
    g = random_grid(64, 64, 3)
    sim = Simulation(LifeConfig(64, 64), engine="cpu")
    sim.load(g)
    sim.advance(10)
    sim.advance(13)
    assert sim.generation == 23
    assert (sim.tile() == life_step_numpy(g, 23)).all()
    assert sim.alive_count() == int(life_step_numpy(g, 23).sum())


@pytest.mark.parametrize("first", [("run_until", 1), ("run_until", 2), ("advance", 1), ("advance", 5)])
@pytest.mark.parametrize("layout", ["u8", "bits"])
def test_run_after_partial_run_keeps_similarity_phase(native, first, layout):
    """the similarity phase is anchored at start_gen, so run() after
    an earlier advance()/run_until() on the same engine reports the same
    Generations as one uninterrupted reference loop (48x40, seed 20 -> 875)."""
    g = random_grid(64, 40, 15, 0.3) if layout == "bits" else random_grid(48, 40, 20)
    ref, rgens, _ = reference_run(g)
    assert rgens < 1000
    sim = Simulation(LifeConfig(g.shape[1], g.shape[0], layout=layout), engine="cpu")
    sim.load(g)
    kind, n = first
    if kind == "run_until":
        sim.native_engine.run_until(n)
    else:
        sim.advance(n)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()


def test_random_init_is_layout_and_decomposition_independent(native):
    a = Simulation(LifeConfig(96, 40, layout="bits"), engine="cpu")
    b = Simulation(LifeConfig(96, 40, layout="u8"), engine="cpu")
    a.init_random(77, 0.4)
    b.init_random(77, 0.4)
    assert (a.tile() == b.tile()).all()
    assert (a.tile() == random_grid(96, 40, 77, 0.4)).all()


def test_bits_layout_rejects_ragged_width(native):
    with pytest.raises(RuntimeError):
        Simulation(LifeConfig(33, 10, layout="bits"), engine="cpu")
