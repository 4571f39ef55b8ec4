"""T3 on CPU: several subdomains in one process (ThreadTransport), covering
pack/unpack, neighbour routing, deep halos and distributed lazy termination.
The same tests run on one GPU in test_gpu.py."""
import pytest

from gol_amd import LifeConfig, random_grid, reference_run
from gol_amd.parallel import InProcessGroup

from golden import CONVERGING

DECOMPS = [("1x2", 2), ("2x1", 2), ("1x4", 4), ("2x2", 4), ("1x8", 8), ("2x4", 8), ("4x2", 8), ("3x3", 9)]


@pytest.mark.parametrize("spec,P", DECOMPS)
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_decompositions_match_serial(native, spec, P, layout):
    W, H = 160, 96
    g = random_grid(W, H, 1234)
    ref, rgens, _ = reference_run(g, 120)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=120, decomp=spec, layout=layout, tmax=8), P, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert all(r.generations == rgens for r in reps)
    assert (grp.gather() == ref).all()


@pytest.mark.parametrize("W,H,seed,density", CONVERGING[:4])
@pytest.mark.parametrize("spec,P", [("1x2", 2), ("2x2", 4)])
def test_distributed_termination(native, W, H, seed, density, spec, P):
    if spec == "2x2" and W < 64:
        pytest.skip("tiles narrower than 32 cells")
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    grp = InProcessGroup(LifeConfig(W, H, decomp=spec, layout="u8", epoch=3, poll_gens=2), P, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


def test_uneven_tiles_u8(native):
    W, H = 100, 37  # 100 not a multiple of 32 -> u8 with cell-granular splits
    g = random_grid(W, H, 5)
    ref, rgens, _ = reference_run(g, 64)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=64, decomp="1x3", layout="u8", epoch=12), 3, engine="cpu")
    grp.load(g)
    grp.run()
    assert (grp.gather() == ref).all()


def test_random_init_decomposition_independent(native):
    grp = InProcessGroup(LifeConfig(128, 64, decomp="2x2"), 4, engine="cpu")
    grp.init_random(99)
    assert (grp.gather() == random_grid(128, 64, 99)).all()


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("1x3", 3), ("2x2", 4), ("2x3", 6)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
@pytest.mark.parametrize("tmax,epoch", [(4, 8), (8, 8), (4, 12), (2, 5)])
def test_overlapped_exchange_matches_serial(native, spec, P, layout, tmax, epoch):
    """Overlapped epochs (interior during the row exchange, edge strips in
    scratch tiles) are bit-identical to the serial reference, including a
    short final epoch (gens not a multiple of the epoch depth)."""
    W, H = 192, 150
    g = random_grid(W, H, 77 + tmax)
    gens = 3 * epoch + epoch // 2 + 1
    ref, _, _ = reference_run(g, gens)
    cfg = LifeConfig(W, H, gen_limit=gens, decomp=spec, layout=layout, tmax=tmax, epoch=epoch, overlap="on")
    grp = InProcessGroup(cfg, P, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert all(r.overlapped for r in reps)
    assert (grp.gather() == ref).all()


@pytest.mark.parametrize("W,H,seed,density", CONVERGING)
@pytest.mark.parametrize("lagged", [True, False])
def test_overlapped_termination(native, W, H, seed, density, lagged):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    cfg = LifeConfig(W, H, decomp="1x2", layout="u8", tmax=2, epoch=3, poll_gens=4, overlap="on",
                     lagged_poll=lagged)
    grp = InProcessGroup(cfg, 2, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert all(r.overlapped == (H // 2 >= 7) for r in reps)
    assert (grp.gather() == ref).all()


def test_overlap_is_opt_in(native):
    """auto = off (the edge strips are latency-bound small launches that cost
    more than the exchange they hide); on requires H > 2D."""
    auto = InProcessGroup(LifeConfig(64, 512, decomp="1x2", tmax=4, epoch=16), 2, engine="cpu")
    assert not auto.sims[0].native_engine.overlap()
    on = InProcessGroup(LifeConfig(64, 512, decomp="1x2", tmax=4, epoch=16, overlap="on"), 2, engine="cpu")
    assert on.sims[0].native_engine.overlap()
    short = InProcessGroup(LifeConfig(64, 40, decomp="1x2", tmax=4, epoch=16, overlap="on"), 2, engine="cpu")
    assert not short.sims[0].native_engine.overlap()


@pytest.mark.parametrize("overlap", ["off", "on"])
def test_random_transport_delays_do_not_change_results(native, monkeypatch, overlap):
    """Fault injection: random delays before every publish and
    consume shake the message interleaving; results must stay exact."""
    monkeypatch.setenv("GOL_FAULT_DELAY_US", "300")
    W, H = 128, 120
    g = random_grid(W, H, 8)
    ref, _, _ = reference_run(g, 40)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=40, decomp="2x3", layout="u8", tmax=2, epoch=6,
                                    overlap=overlap), 6, engine="cpu")
    grp.load(g)
    grp.run()
    assert (grp.gather() == ref).all()


def test_garbled_halo_is_detected(native, monkeypatch):
    """Fault injection: a corrupted halo message must show up as
    a mismatch against the serial reference - the golden comparison catches
    communication faults."""
    monkeypatch.setenv("GOL_FAULT_GARBLE", "3")
    W, H = 96, 96
    g = random_grid(W, H, 21)
    ref, _, _ = reference_run(g, 30)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=30, decomp="1x2", layout="u8", tmax=2, epoch=4,
                                    overlap="off"), 2, engine="cpu")
    grp.load(g)
    grp.run()
    assert (grp.gather() != ref).any()


def test_thread_transport_pair_matching_two_ranks(native):
    """The row-phase op order of Engine::halo_exchange (engine.cpp) with
    Py = 2, where north and south are the same peer: messages between a pair
    must match in issue order (send N <-> recv S, send S <-> recv N), the
    contract RCCL's grouped send/recv also follows."""
    import threading

    import numpy as np

    C = native
    hub = C.ThreadHub(2)
    bes = [C.cpu_backend(1) for _ in range(2)]
    trs = [C.thread_transport(hub, r, bes[r]) for r in range(2)]
    n = 4096
    rng = np.random.default_rng(0)
    top = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(2)]
    bot = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(2)]
    halo_s = [np.zeros(n, np.uint8) for _ in range(2)]
    halo_n = [np.zeros(n, np.uint8) for _ in range(2)]

    def run(r):
        p = 1 - r
        trs[r].exchange([(True, p, top[r].ctypes.data, n), (False, p, halo_s[r].ctypes.data, n),
                         (True, p, bot[r].ctypes.data, n), (False, p, halo_n[r].ctypes.data, n)], 0)

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(30)
    for r in range(2):
        assert (halo_s[r] == top[1 - r]).all()  # south neighbour's top rows -> my bottom halo
        assert (halo_n[r] == bot[1 - r]).all()  # north neighbour's bottom rows -> my top halo
