"""Resident-epoch schedule of the engine on the CPU (GOL_CPU_RESIDENT=1).

On the GPU, Backend::resident_epoch lets a whole-width bit tile that fits the
register file run every halo epoch as ONE launch (life_resident_impl.hpp):
the engine then picks T = the epoch's remaining generations for every block
(no T <= 16 blocks), never splits an epoch for overlap, and accounts one
block's drift per epoch.  The CPU backend can emulate that schedule (its
run_block evaluates any T), so the engine side of it - epoch depth, partial
epochs, flags of long blocks, termination, multi-rank row strips, the byte
layout on bit words - is checked here against the exact serial loop
(src/game.c semantics) without a GPU.  The kernel itself is covered by the
GPU tier (tests/test_gpu.py::test_resident_*)."""
import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, life_step_numpy, random_grid, reference_run
from gol_amd.models.life import make_tuning
from gol_amd.parallel import InProcessGroup

from golden import CONVERGING


@pytest.fixture
def resident_env(tune):
    tune["cpu_resident"] = "1"


def _sim(native, cfg, drift=0):
    return Simulation(cfg, backend=native.cpu_backend(2, drift, tune=make_tuning(cfg.tune)))


@pytest.mark.parametrize("epoch", [0, 40, 100])
@pytest.mark.parametrize("drift", [0, 1])
def test_resident_schedule_matches_reference(native, tune, resident_env, epoch, drift):
    W, H = 256, 90
    g = random_grid(W, H, 5 + epoch)
    ref, rgens, _ = reference_run(g, 300)
    sim = _sim(native, LifeConfig(W, H, gen_limit=300, epoch=epoch, tune=tune), drift)
    assert sim.native_engine.resident
    D = sim.native_engine.epoch_depth
    assert D == (epoch if epoch else 128) and sim.native_engine.tmax == D
    sim.load(g)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()
    # one block per epoch (a partial one at the end)
    assert rep.kernel_launches == -(-rep.executed // D)


@pytest.mark.parametrize("case", [c for c in CONVERGING if c[0] % 32 == 0] + [(256, 512, 77, 0.5)])
def test_resident_termination(native, tune, resident_env, case):
    W, H, seed, density = case
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    sim = _sim(native, LifeConfig(W, H, epoch=48, poll_gens=96, tune=tune))
    assert sim.native_engine.resident
    sim.load(g)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()


def test_resident_chunked_partial_epochs(native, tune, resident_env):
    W, H = 128, 64
    g = random_grid(W, H, 9)
    sim = _sim(native, LifeConfig(W, H, gen_limit=2000, check_similarity=False, epoch=64, tune=tune))
    sim.load(g)
    want = g
    for n in (30, 97, 64, 5, 200):
        sim.advance(n)
        want = life_step_numpy(want, n)
        assert (sim.tile() == want).all(), n


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("1x4", 4)])
def test_resident_row_strips(native, tune, resident_env, spec, P):
    """Multi-rank row strips: every rank takes the same resident decision and
    epoch depth (exchanges in lockstep), halos D rows deep."""
    W, H = 256, 512
    g = random_grid(W, H, 31, 0.4)
    ref, rgens, _ = reference_run(g)
    grp = InProcessGroup(LifeConfig(W, H, decomp=spec, epoch=64, poll_gens=128, tune=tune), P, engine="cpu")
    assert all(s.native_engine.resident for s in grp.sims)
    assert {s.native_engine.epoch_depth for s in grp.sims} == {64}
    grp.load(g)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


def test_resident_u8_on_bit_words(native, resident_env, tune):
    tune["u8_via_bits"] = "1"
    W, H = 192, 80
    g = random_grid(W, H, 4)
    ref, rgens, _ = reference_run(g, 500)
    sim = _sim(native, LifeConfig(W, H, gen_limit=500, layout="u8", epoch=50, tune=tune))
    assert sim.native_engine.resident and sim.native_engine.via_bits
    sim.load(g)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()


def test_resident_not_for_column_splits_or_overlap(native, tune, resident_env):
    W, H = 256, 256
    grp = InProcessGroup(LifeConfig(W, H, decomp="2x2", tune=tune), 4, engine="cpu")
    assert not any(s.native_engine.resident for s in grp.sims)
    sim = _sim(native, LifeConfig(W, H, overlap="on", tune=tune))
    assert not sim.native_engine.resident
