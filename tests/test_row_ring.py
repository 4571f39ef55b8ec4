"""Row ring (Backend::row_ring_halo / alloc_row_ring): a single-rank torus
whose top and bottom halo rows are second virtual mappings of its last and
first owned rows, so the periodic row halos are never filled and every
temporal block covers exactly the owned rows.  The CPU backend emulates the
HIP backend's VMM mapping with a memfd mapped three times (GOL_CPU_RING=1),
so the engine's ring schedule is checked here against the exact serial loop
and the fp32 oracle; tests/test_gpu.py covers the device rings."""
import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, life_step_numpy, random_grid, reference_run

from golden import CONVERGING


@pytest.fixture
def tune():
    """Tuning passed through LifeConfig.tune (gol/tuning.hpp): the CPU backend emulates row rings."""
    return {"cpu_ring": "1"}


def _sim(tune, W, H, **kw):
    sim = Simulation(LifeConfig(W, H, tune=tune, **kw), engine="cpu")
    return sim


@pytest.mark.parametrize("layout", ["bits", "u8"])
@pytest.mark.parametrize("W,H,tmax", [(128, 64, 4), (256, 160, 8), (96, 48, 16), (512, 256, 12)])
def test_ring_matches_oracle(native, tune, layout, W, H, tmax):
    sim = _sim(tune, W, H, layout=layout, tmax=tmax, gen_limit=300)
    assert sim.describe()["row_ring"] is True
    assert sim.describe()["epoch"] == sim.describe()["tmax"]
    g = random_grid(W, H, W + H + tmax)
    sim.load(g)
    want = g
    for n in (37, 100, 3):  # chunks: partial epochs, read-outs in between
        sim.advance(n)
        want = life_step_numpy(want, n)
        assert (sim.tile() == want).all(), n
    rep = sim.last_report
    assert rep.exchanges > 0


@pytest.mark.parametrize("drift", ["0", "1"])
def test_ring_with_drifting_frame_and_u8_compute(native, tune, drift):
    tune["cpu_drift"] = drift
    W, H = 256, 128
    g = random_grid(W, H, 5)
    for layout, u8c in (("bits", "auto"), ("u8", "bits"), ("u8", "bytes")):
        sim = _sim(tune, W, H, layout=layout, u8_compute=u8c, tmax=8, gen_limit=500)
        assert sim.describe()["row_ring"] is True, (layout, u8c)
        sim.load(g)
        sim.advance(77)
        assert (sim.tile() == life_step_numpy(g, 77)).all(), (layout, u8c)


@pytest.mark.parametrize("W,H,seed,density", [c for c in CONVERGING if c[1] % 16 == 0])
def test_ring_termination_is_exact(native, tune, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    sim = _sim(tune, W, H, tmax=4)
    sim.load(g)
    rep = sim.run()
    assert rep.generations == rgens
    assert (sim.tile() == ref).all()


def test_ring_off_for_geometries_the_pages_do_not_fit(native, tune):
    # 30 rows of 256-byte bit rows: 7680 bytes is not a whole number of pages.
    sim = _sim(tune, 128, 30, tmax=4)
    assert sim.describe()["row_ring"] is False
    g = random_grid(128, 30, 1)
    sim.load(g)
    sim.advance(20)
    assert (sim.tile() == life_step_numpy(g, 20)).all()


def test_ring_halo_rows_alias_owned_rows(native, tune):
    """The mapping itself: the top halo reads the last owned rows and the
    bottom halo the first ones, through the engine's current buffer."""
    import ctypes

    W, H = 128, 64
    sim = _sim(tune, W, H, layout="u8", u8_compute="bytes", tmax=4)
    g = random_grid(W, H, 9)
    sim.load(g)
    eng = sim.native_engine
    geo = eng.geom
    base = eng.current_buffer()
    buf = (ctypes.c_uint8 * int(geo.bytes())).from_address(base)
    a = np.frombuffer(buf, dtype=np.uint8).reshape(geo.R(), geo.pitch)
    Dv = geo.Dv
    assert (a[:Dv] == a[H:H + Dv]).all()          # top halo == last Dv owned rows
    assert (a[Dv + H:] == a[Dv:2 * Dv]).all()     # bottom halo == first Dv owned rows
    assert not (a[Dv:Dv + H] == 0).all()


def test_ring_allocation_failure_falls_back_to_fills(native, tune, capfd):
    """A backend that promises a ring but cannot map it (GOL_CPU_RING=fail):
    the engine warns, allocates plain buffers and fills the row halos."""
    tune["cpu_ring"] = "fail"
    sim = _sim(tune, 128, 64, tmax=4, gen_limit=100)
    assert sim.describe()["row_ring"] is False
    assert "row ring unavailable" in capfd.readouterr().err
    g = random_grid(128, 64, 3)
    sim.load(g)
    sim.advance(50)
    assert (sim.tile() == life_step_numpy(g, 50)).all()
