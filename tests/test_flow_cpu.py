"""Persistent dataflow launches (EngineConfig::flow, Backend::run_flow) on
the CPU: GOL_CPU_FLOW=1 makes the CPU backend accept runs of equal blocks,
which the base class evaluates block by block, so the engine's flow
bookkeeping - which blocks go into one run, buffer parity, drift, flags,
the ring's poll-window epochs and the trapezoid of a deep-halo epoch - is
checked here against the exact serial loop and the numpy oracle.  The HIP
kernel itself (life_flow_impl.hpp) is checked in tests/test_gpu_flow.py."""
import pytest

from gol_amd import LifeConfig, Simulation, life_step_numpy, random_grid, reference_run
from gol_amd.parallel import InProcessGroup

from golden import CONVERGING


@pytest.fixture
def tune():
    """Tuning passed through LifeConfig.tune (gol/tuning.hpp): the CPU backend accepts flow runs."""
    return {"cpu_flow": "1"}


@pytest.mark.parametrize("ring", ["0", "1"])
@pytest.mark.parametrize("drift", ["0", "1"])
@pytest.mark.parametrize("layout,u8c", [("bits", "auto"), ("u8", "bits")])
def test_flow_single_rank_matches_oracle(native, tune, ring, drift, layout, u8c):
    tune["cpu_ring"] = ring
    tune["cpu_drift"] = drift
    W, H = 256, 128
    sim = Simulation(LifeConfig(W, H, layout=layout, u8_compute=u8c, tmax=8, gen_limit=2000, poll_gens=64, tune=tune),
                     engine="cpu")
    d = sim.describe()
    assert d["flow"] is True
    assert d["row_ring"] is (ring == "1")
    if ring == "1":
        assert d["epoch"] == 64  # a ring's epoch is the poll window: one flow run per window
    g = random_grid(W, H, 17)
    sim.load(g)
    want = g
    for n in (150, 37, 8, 3):  # full windows, partial ones, a single block, below one block
        rep = sim.advance(n)
        want = life_step_numpy(want, n)
        assert (sim.tile() == want).all(), n
    assert sim.last_report.flow_launches == 0  # 3 generations: no run of two blocks


def test_flow_counts_blocks(native, tune):
    tune["cpu_ring"] = "1"
    sim = Simulation(LifeConfig(128, 64, tmax=8, gen_limit=1000, poll_gens=64, tune=tune), engine="cpu")
    sim.load(random_grid(128, 64, 3))
    rep = sim.advance(200)  # 3 windows of 64 (8 blocks each) + 8: three flow runs and one block
    assert rep.flow_launches == 3
    assert rep.flow_blocks == 24
    assert rep.kernel_launches == 4


def test_flow_off(native, tune):
    tune["cpu_ring"] = "1"
    sim = Simulation(LifeConfig(128, 64, tmax=8, gen_limit=100, flow="off", tune=tune), engine="cpu")
    assert sim.describe()["flow"] is False
    sim.load(random_grid(128, 64, 3))
    assert sim.advance(64).flow_launches == 0


@pytest.mark.parametrize("W,H,seed,density", [c for c in CONVERGING if c[1] % 16 == 0][:4])
@pytest.mark.parametrize("ring", ["0", "1"])
def test_flow_termination_is_exact(native, tune, W, H, seed, density, ring):
    tune["cpu_ring"] = ring
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    sim = Simulation(LifeConfig(W, H, tmax=4, poll_gens=32, tune=tune), engine="cpu")
    sim.load(g)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("1x4", 4), ("2x2", 4), ("2x3", 6)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
@pytest.mark.parametrize("overlap", ["off", "on"])
def test_flow_multirank_trapezoid_epochs(native, tune, spec, P, layout, overlap):
    """Deep-halo epochs of several ranks: one flow run per epoch whose blocks
    shrink by T rows per side (the early-boundary schedule keeps its split
    last block out of the run)."""
    W, H = 192, 160
    g = random_grid(W, H, 77)
    ref, rgens, _ = reference_run(g, 150)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=150, decomp=spec, layout=layout, tmax=4, epoch=16,
                                    overlap=overlap, tune=tune), P, engine="cpu")
    assert all(s.describe()["flow"] for s in grp.sims)
    grp.load(g)
    reps = grp.run()
    assert all(r.generations == rgens for r in reps)
    assert (grp.gather() == ref).all()
    assert all(r.flow_launches > 0 for r in reps)


def test_flow_self_exchange_rehearsal(native, tune):
    W, H = 128, 96
    g = random_grid(W, H, 4)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=100, tmax=4, epoch=16, self_exchange=True, tune=tune), 1,
                         engine="cpu")
    grp.load(g)
    rep = grp.sims[0].advance(70)
    assert rep.flow_launches >= 4
    assert (grp.gather() == life_step_numpy(g, 70)).all()
