"""Drifting storage frame (csrc/kernels/life_kernels.hpp kXlaneAdd) on the CPU.

The HIP adder window evaluates B3/S23 with a one-sided horizontal window and
stores generation t+1's cell x-1 at column x, so every temporal block leaves
the tile rotated T cells to the right.  The engine tracks that drift, sizes
the left halo for the one-sided light cone, and rotates it out before every
read-out (Engine::normalize).  The CPU backend emulates the same frame
(``cpu_backend(drift=1)``), so this bookkeeping is tested here against the
exact serial loop (src/game.c semantics), independently of the GPU."""
import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, random_grid, reference_run
from gol_amd.models.life import make_tuning
from gol_amd.parallel import InProcessGroup

from golden import CONVERGING


def sim_with(native, cfg, drift):
    return Simulation(cfg, backend=native.cpu_backend(2, drift, tune=make_tuning(cfg.tune)))


@pytest.mark.parametrize("layout", ["bits", "u8"])
@pytest.mark.parametrize("tmax,epoch", [(16, 0), (8, 24), (4, 12), (3, 7)])
def test_drift_frame_matches_reference(native, tune, layout, tmax, epoch):
    W, H = 256, 90
    g = random_grid(W, H, 17 + tmax)
    ref, rgens, _ = reference_run(g, 300)
    sim = sim_with(native, LifeConfig(W, H, gen_limit=300, layout=layout, tmax=tmax, epoch=epoch, tune=tune), 1)
    sim.load(g)
    rep = sim.run()
    assert sim.native_engine.drift == rep.executed % W  # every block drifted
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()
    assert sim.native_engine.drift == 0  # the read-out rotated it out


def test_drift_accumulates_and_wraps(native, tune):
    W, H = 64, 40
    g = random_grid(W, H, 3)
    sim = sim_with(native, LifeConfig(W, H, gen_limit=10_000, tmax=16, epoch=32, tune=tune), 1)
    sim.load(g)
    eng = sim.native_engine
    for n in (5, 16, 59, 64, 100):
        before = eng.drift
        sim.advance(n)
        assert eng.drift == (before + n) % W
    want = g
    for _ in range(5 + 16 + 59 + 64 + 100):
        want = np.asarray(reference_run(want, 1, check_similarity=False)[0])
    assert (sim.tile() == want).all()


def test_drift_needs_whole_width_tiles(native, tune):
    """Column decompositions (Px > 1) keep the symmetric kernel: a drift would
    move cells across rank boundaries."""
    tune["cpu_drift"] = "1"
    W, H = 128, 64
    g = random_grid(W, H, 8)
    ref, rgens, _ = reference_run(g, 150)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=150, decomp="2x2", tmax=8, tune=tune), 4, engine="cpu")
    assert all("drift" in s.backend.name() for s in grp.sims)
    grp.load(g)
    reps = grp.run()
    assert all(s.native_engine.drift == 0 for s in grp.sims)
    assert (grp.gather() == ref).all() and {r.generations for r in reps} == {rgens}


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("1x3", 3), ("1x4", 4)])
@pytest.mark.parametrize("overlap", ["off", "trigger"])
def test_drift_row_strips_and_overlap(native, tune, spec, P, overlap):
    """Row strips (the multi-GPU default) drift in lockstep on every rank;
    the boundary-trigger launches drift with the rest."""
    tune["cpu_drift"] = "1"
    tune["cpu_trigger"] = "1"
    W, H = 192, 120
    g = random_grid(W, H, P + 40)
    ref, rgens, _ = reference_run(g, 200)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=200, decomp=spec, tmax=4, epoch=12, overlap=overlap, tune=tune), P,
                         engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert all(s.native_engine.drift == r.executed % W for s, r in zip(grp.sims, reps))
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


@pytest.mark.parametrize("W,H,seed,density", [c for c in CONVERGING if c[0] % 32 == 0][:4])
def test_drift_termination_exact(native, tune, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    sim = sim_with(native, LifeConfig(W, H, tmax=8, epoch=16, poll_gens=16, tune=tune), 1)
    sim.load(g)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()


def test_rotate_cols_matches_numpy(native, tune):
    """The rotated-out drifted buffer equals the non-drifting backend's tile."""
    W, H = 96, 20
    g = random_grid(W, H, 21)
    a = sim_with(native, LifeConfig(W, H, gen_limit=50, tmax=4, epoch=8, tune=tune), 1)
    b = sim_with(native, LifeConfig(W, H, gen_limit=50, tmax=4, epoch=8, tune=tune), 0)
    for s in (a, b):
        s.load(g)
        s.advance(37)
    assert a.native_engine.drift == 37 and b.native_engine.drift == 0
    assert (a.tile() == b.tile()).all()
