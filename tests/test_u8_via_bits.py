"""Byte layout computed on bit words (EngineConfig::u8_compute = bits,
Engine::epoch_via_bits): the byte-per-cell grid stays the storage, each epoch
packs its owned rows into bit words in the spare byte buffer, exchanges or
fills the halos there and runs the bit-layout temporal blocks, then unpacks.
On the CPU backend (default: bytes) it is selected explicitly; every result is
checked against the exact serial loop (src/game.c semantics) or the numpy
oracle.  The GPU tier repeats the core cases in test_gpu.py."""
import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, life_step_numpy, random_grid, reference_run
from gol_amd.models.life import make_tuning
from gol_amd.parallel import InProcessGroup

from golden import CONVERGING


# Converging random grids of whole 32-cell words (stop before GEN_LIMIT).
WORD_CONVERGING = [(32, 16, 1, 0.2), (32, 40, 3, 0.2), (64, 20, 1, 0.2), (96, 24, 11, 0.2), (128, 12, 11, 0.2)] + \
    [c for c in CONVERGING if c[0] % 32 == 0]


def u8_bits(W, H, **kw):
    return LifeConfig(W, H, layout="u8", u8_compute="bits", **kw)


@pytest.mark.parametrize("W,H", [(32, 1), (32, 32), (64, 5), (96, 70), (160, 33)])
@pytest.mark.parametrize("tmax,epoch", [(0, 0), (4, 5), (8, 33), (16, 100), (2, 1)])
def test_via_bits_matches_oracle(native, W, H, tmax, epoch):
    g = random_grid(W, H, W + 3 * H + tmax)
    sim = Simulation(u8_bits(W, H, gen_limit=77, tmax=tmax, epoch=epoch), engine="cpu")
    d = sim.describe()
    assert d["layout"] == "u8" and d["u8_compute"] == "bits"
    sim.load(g)
    sim.advance(77)
    assert (sim.tile() == life_step_numpy(g, 77)).all()
    assert sim.alive_count() == int(life_step_numpy(g, 77).sum())


def test_selection_rules(native, tune):
    # CPU default: the byte kernels; a ragged width cannot use bit words.
    assert Simulation(LifeConfig(64, 8, layout="u8", tune=tune), engine="cpu").describe()["u8_compute"] == "bytes"
    assert Simulation(LifeConfig(100, 8, layout="u8", u8_compute="bits", tune=tune),
                      engine="cpu").describe()["u8_compute"] == "bytes"
    assert Simulation(LifeConfig(64, 8, layout="bits", tune=tune), engine="cpu").describe()["u8_compute"] is None
    tune["u8_via_bits"] = "1"
    assert Simulation(LifeConfig(64, 8, layout="u8", tune=tune), engine="cpu").describe()["u8_compute"] == "bits"
    # An explicit choice wins over the environment.
    assert Simulation(LifeConfig(64, 8, layout="u8", u8_compute="bytes", tune=tune),
                      engine="cpu").describe()["u8_compute"] == "bytes"


def test_epoch_depth_and_scratch_sharing(native):
    # The bit layout's epoch depth; a large tile keeps its bit words in the
    # spare byte buffer (results stay exact across many epochs, runs and
    # read-outs: each run packs the byte tile once and unpacks it once).
    W, H = 256, 200
    g = random_grid(W, H, 8)
    sim = Simulation(u8_bits(W, H, gen_limit=1000, tmax=4), engine="cpu")
    assert sim.epoch_depth == 8 * 4
    d = sim.describe()
    assert d["halo_rows"] == 32 and sim.native_engine.geom.Dv == 0  # halos live on the bit tile only
    sim.load(g)
    sim.advance(300)
    mid = sim.tile()
    assert (mid == life_step_numpy(g, 300)).all()
    sim.advance(129)
    assert (sim.tile() == life_step_numpy(mid, 129)).all()


@pytest.mark.parametrize("W,H,seed,density", WORD_CONVERGING)
def test_via_bits_termination_matches_reference(native, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    for tmax, epoch, poll in [(0, 0, 0), (4, 7, 5), (1, 1, 1), (8, 64, 1000)]:
        sim = Simulation(u8_bits(W, H, tmax=tmax, epoch=epoch, poll_gens=poll), engine="cpu")
        sim.load(g)
        rep = sim.run()
        assert rep.generations == rgens, (tmax, epoch, poll)
        assert (sim.tile() == ref).all()


@pytest.mark.parametrize("tmax,epoch", [(16, 0), (8, 24), (3, 7)])
def test_via_bits_drifting_frame(native, tune, tmax, epoch):
    """A drifting bit kernel leaves the byte grid drifted by the same amount;
    the read-out rotates it out (Engine::normalize on the byte grid)."""
    W, H = 256, 90
    g = random_grid(W, H, 17 + tmax)
    ref, rgens, _ = reference_run(g, 300)
    sim = Simulation(u8_bits(W, H, gen_limit=300, tmax=tmax, epoch=epoch, tune=tune),
                     backend=native.cpu_backend(2, 1, tune=make_tuning(tune)))
    assert sim.native_engine.drifting
    sim.load(g)
    rep = sim.run()
    assert sim.native_engine.drift == rep.executed % W
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()
    assert sim.native_engine.drift == 0


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("2x1", 2), ("2x2", 4), ("1x4", 4), ("2x4", 8), ("3x3", 9)])
def test_via_bits_decompositions(native, spec, P):
    """Halo exchanges (columns, then rows) run on the bit tile: 8x fewer bytes
    than the byte tile's."""
    W, H = 192, 96
    g = random_grid(W, H, 1234)
    ref, rgens, _ = reference_run(g, 120)
    grp = InProcessGroup(u8_bits(W, H, gen_limit=120, decomp=spec, tmax=8, epoch=16), P, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert all(r.generations == rgens for r in reps)
    assert (grp.gather() == ref).all()
    assert all(s.native_engine.via_bits for s in grp.sims)


@pytest.mark.parametrize("spec", ["1x2", "2x1"])
def test_via_bits_exchanges_bit_rows(native, tune, spec):
    """The same run on the byte tiles sends ~8x the halo bytes (4x at least
    after the 256-byte pitch rounding of both)."""
    W, H = 2048, 64
    g = random_grid(W, H, 77)
    want = life_step_numpy(g, 40)
    sent = {}
    for mode in ("bits", "bytes"):
        grp = InProcessGroup(LifeConfig(W, H, gen_limit=40, decomp=spec, tmax=4, epoch=8, layout="u8",
                                        u8_compute=mode, check_similarity=False, tune=tune), 2, engine="cpu")
        grp.load(g)
        reps = grp.parallel(lambda s: s.advance(40))
        assert (grp.gather() == want).all()
        sent[mode] = sum(r.halo_bytes for r in reps)
    assert 0 < 4 * sent["bits"] <= sent["bytes"]


@pytest.mark.parametrize("W,H,seed,density", WORD_CONVERGING)
def test_via_bits_distributed_termination(native, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    spec = "2x2" if W % 64 == 0 else "1x2"
    grp = InProcessGroup(u8_bits(W, H, decomp=spec, epoch=3, poll_gens=2), int(spec[0]) * int(spec[2]), engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


def test_via_bits_phase_timing_and_counters(native):
    W, H = 128, 64
    sim = Simulation(u8_bits(W, H, gen_limit=200, tmax=4, epoch=20), engine="cpu")
    sim.phase_timing = True
    sim.load(random_grid(W, H, 2))
    rep = sim.advance(200)
    assert rep.exchanges == 10  # one fill of the bit tile per epoch
    assert rep.phase_timed and rep.compute_ms > 0
    assert (sim.tile() == life_step_numpy(random_grid(W, H, 2), 200)).all()
    assert np.array_equal(sim.tile(), sim.tile())


@pytest.mark.parametrize("drift", [0, 1])
def test_bit_image_stays_live_across_runs(native, drift):
    """A run leaves its result in the bit image and unpacks it only when the
    byte tile is next read (Engine::sync_bytes): back-to-back runs, reads
    between them (tile, alive count, row bands, raw buffer), a reload and a
    random init in the middle, all against the numpy oracle; with the CPU
    backend's drifting frame the unpacked bytes are rotated on read."""
    W, H = 256, 96
    g = random_grid(W, H, 21)
    sim = Simulation(u8_bits(W, H, gen_limit=10_000, tmax=8, epoch=16),
                     backend=native.cpu_backend(2, drift))
    sim.load(g)
    want = g
    for n in (40, 17, 64):  # three runs with nothing read in between
        sim.advance(n)
        want = life_step_numpy(want, n)
    assert sim.alive_count() == int(want.sum())  # counted on the live bit image
    assert (sim.tile() == want).all()
    sim.advance(33)
    want = life_step_numpy(want, 33)
    rows = np.asarray(sim.native_engine.store_rows(20, 10, False)).reshape(10, W)
    assert (rows == want[20:30]).all()
    sim.advance(9)
    want = life_step_numpy(want, 9)
    assert sim.native_engine.current_buffer() != 0  # a raw view syncs the bytes first
    assert (sim.tile() == want).all()
    g2 = random_grid(W, H, 22)  # a reload makes the byte tile the state again
    sim.advance(12)
    sim.load(g2)
    sim.advance(25)
    assert (sim.tile() == life_step_numpy(g2, 25)).all()
    sim.init_random(5, 0.3)  # so does an init on the device
    g3 = sim.tile()
    sim.advance(30)
    sim.advance(2)
    assert (sim.tile() == life_step_numpy(g3, 32)).all()
