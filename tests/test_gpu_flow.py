"""GPU tier (experimental builds: the kernel measured slower than the grouped
launches, docs/PERFORMANCE.md): the persistent dataflow kernel
(life_flow_impl.hpp) against the PyTorch fp32 oracle.  Every plan dimension the planner can pick is forced
here: T = 8 / 12 / 16, the adder and DPP windows, 4- and 8-wave items, few
and many groups per strip (rotation, dependency wrap on rings), folded and
unfolded last strips, ring tiles (dependencies across the torus seam) and
trapezoid epochs (periodic fills, blocks shrinking per side), the byte layout
on bit words, exact termination, and back-to-back launches of different
plans on one backend (monotonic tickets and completion words)."""
import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, life_step_torch, random_grid, reference_run
from gol_amd.models.life import make_tuning

from golden import CONVERGING

pytestmark = [pytest.mark.gpu, pytest.mark.experimental]


@pytest.fixture
def tune():
    """Tuning passed through LifeConfig.tune: flow launches on."""
    return {"flow": "1"}


def _sim(tune, W, H, **kw):
    kw.setdefault("gen_limit", 100_000)
    return Simulation(LifeConfig(W, H, tune=tune, **kw), engine="hip")


def _check(sim, g, chunks):
    want = g
    sim.load(g)
    for n in chunks:
        sim.advance(n)
        want = life_step_torch(want, n, device="cuda")
        assert (sim.tile() == want).all(), n
    return sim.last_report


@pytest.mark.parametrize("xlane,tmax", [(3, 8), (3, 12), (0, 8), (0, 12), (0, 16)])
@pytest.mark.parametrize("m", [4, 8])
@pytest.mark.parametrize("W,H", [(4096, 512), (2016, 384), (8192, 256)])
def test_flow_ring_plans_vs_torch(gpu, tune, xlane, tmax, m, W, H):
    tune["xlane"] = str(xlane)
    tune["flow_m"] = str(m)
    sim = _sim(tune, W, H, tmax=tmax, poll_gens=8 * tmax)
    d = sim.describe()
    assert d["flow"] and d["row_ring"], d
    g = random_grid(W, H, W + H + tmax + m)
    rep = _check(sim, g, [20 * tmax + 5, 3 * tmax, 7])
    assert "flow" in sim.backend.flow_desc()
    assert f"M={m}" in sim.backend.flow_desc()


@pytest.mark.parametrize("nseg", [1, 2, 3, 7])
@pytest.mark.parametrize("xlane", [0, 3])
def test_flow_groups_per_strip_vs_torch(gpu, tune, nseg, xlane):
    """Few groups per strip: every item waits across the ring's seam (one
    group: its own previous block), rotation over 2-7 positions."""
    tune["xlane"] = str(xlane)
    tune["flow_m"] = "4"
    tune["flow_nseg"] = str(nseg)
    W, H = 4096, 1024
    sim = _sim(tune, W, H, tmax=8, poll_gens=96)
    g = random_grid(W, H, 31 * nseg + xlane)
    _check(sim, g, [96 * 3, 40])
    assert f"groups/strip={nseg}" in sim.backend.flow_desc()


@pytest.mark.parametrize("fold", ["0", "1"])
def test_flow_fold_vs_torch(gpu, tune, fold):
    tune["fold"] = fold
    tune["xlane"] = "3"
    W, H = 32768, 256  # 16 strips of 63 words + a 16-word strip folded three times
    sim = _sim(tune, W, H, tmax=8, poll_gens=64)
    _check(sim, random_grid(W, H, 5), [130])


@pytest.mark.parametrize("xlane,tmax", [(3, 8), (0, 16), (3, 12)])
def test_flow_trapezoid_epochs_vs_torch(gpu, tune, xlane, tmax):
    """No ring: epochs of D generations after a periodic fill, one flow
    launch whose blocks shrink by T rows per side."""
    tune["row_ring"] = "0"
    tune["xlane"] = str(xlane)
    W, H = 4096, 700
    sim = _sim(tune, W, H, tmax=tmax, epoch=8 * tmax)
    d = sim.describe()
    assert d["flow"] and not d["row_ring"]
    rep = _check(sim, random_grid(W, H, 3 + tmax), [8 * tmax * 3 + tmax + 3])
    assert rep.flow_launches >= 3


def test_flow_u8_on_bit_words_vs_torch(gpu, tune):
    tune["u8_via_bits"] = "1"
    W, H = 4096, 512
    sim = _sim(tune, W, H, layout="u8", tmax=8, poll_gens=64)
    assert sim.describe()["u8_compute"] == "bits" and sim.describe()["flow"]
    _check(sim, random_grid(W, H, 8), [150, 22])


@pytest.mark.parametrize("W,H,seed,density", [c for c in CONVERGING if c[0] % 32 == 0 and c[1] % 8 == 0][:4])
def test_flow_termination_is_exact(gpu, tune, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    sim = Simulation(LifeConfig(W, H, tmax=8, poll_gens=64, tune=tune), engine="hip")
    sim.load(g)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()


def test_flow_back_to_back_plans_share_counters(gpu, tune):
    """Two engines of different tiles on ONE backend alternate flow launches:
    their plans differ (items per block, groups), the ticket counter and the
    completion words are shared and monotonic."""
    native = gpu
    be = native.hip_backend(0, tune=make_tuning(tune))
    sims = [Simulation(LifeConfig(W, H, tmax=8, poll_gens=64, gen_limit=10_000, tune=tune), backend=be)
            for W, H in ((4096, 512), (2048, 1024))]
    grids = [random_grid(s.config.width, s.config.height, i + 40) for i, s in enumerate(sims)]
    wants = list(grids)
    for s, g in zip(sims, grids):
        s.load(g)
    for rnd in range(4):
        for i, s in enumerate(sims):
            n = 64 + 8 * rnd
            s.advance(n)
            wants[i] = life_step_torch(wants[i], n, device="cuda")
    for s, w in zip(sims, wants):
        assert (s.tile() == w).all()
        assert s.last_report.flow_launches >= 1


def test_flow_rank_tile_shape_vs_torch(gpu, tune):
    """The 8-GPU rank tile's shape (32768 wide) with the rehearsal's epochs
    shortened: trapezoid epochs through the self-exchange path."""
    tune["xlane"] = "3"
    W, H = 32768, 512
    native = gpu
    sim = Simulation(LifeConfig(W, H, tmax=8, epoch=64, gen_limit=10_000, self_exchange=True, tune=tune), engine="hip",
                     transport=native.rccl_transport(native.rccl_unique_id(), 0, 1, 0, tune=make_tuning(tune)))
    assert sim.describe()["flow"]
    g = random_grid(W, H, 11)
    rep = _check(sim, g, [64 * 3 + 8])
    assert rep.flow_launches >= 3


@pytest.mark.parametrize("xlane,nseg", [(3, 0), (0, 2), (3, 5)])
def test_flow_late_seam_producers_vs_torch(gpu, tune, xlane, nseg):
    """GOL_FAULT_DELAY_SPINS: the items at the torus seam (first and last row
    position, folded items) publish ~1 ms late, so any item that read their
    rows without waiting for them would see the previous generation."""
    tune["xlane"] = str(xlane)
    tune["fault_delay_spins"] = "300"
    if nseg:
        tune["flow_nseg"] = str(nseg)
    W, H = 32768, 512
    sim = _sim(tune, W, H, tmax=8, poll_gens=64)
    _check(sim, random_grid(W, H, 21 + nseg), [64 * 2 + 8])

