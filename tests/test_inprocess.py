"""T3 on CPU: several subdomains in one process (ThreadTransport), covering
pack/unpack, neighbour routing, deep halos and distributed lazy termination.
The same tests run on one GPU in test_gpu.py."""
import pytest

from gol_amd import LifeConfig, random_grid, reference_run
from gol_amd.models.life import make_tuning
from gol_amd.parallel import InProcessGroup

from golden import CONVERGING

DECOMPS = [("1x2", 2), ("2x1", 2), ("1x4", 4), ("2x2", 4), ("1x8", 8), ("2x4", 8), ("4x2", 8), ("3x3", 9)]


@pytest.mark.parametrize("spec,P", DECOMPS)
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_decompositions_match_serial(native, tune, spec, P, layout):
    W, H = 160, 96
    g = random_grid(W, H, 1234)
    ref, rgens, _ = reference_run(g, 120)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=120, decomp=spec, layout=layout, tmax=8, tune=tune), P,
                         engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert all(r.generations == rgens for r in reps)
    assert (grp.gather() == ref).all()


@pytest.mark.parametrize("W,H,seed,density", CONVERGING[:4])
@pytest.mark.parametrize("spec,P", [("1x2", 2), ("2x2", 4)])
def test_distributed_termination(native, tune, W, H, seed, density, spec, P):
    if spec == "2x2" and W < 64:
        pytest.skip("tiles narrower than 32 cells")
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    grp = InProcessGroup(LifeConfig(W, H, decomp=spec, layout="u8", epoch=3, poll_gens=2, tune=tune), P, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


def test_uneven_tiles_u8(native, tune):
    W, H = 100, 37  # 100 not a multiple of 32 -> u8 with cell-granular splits
    g = random_grid(W, H, 5)
    ref, rgens, _ = reference_run(g, 64)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=64, decomp="1x3", layout="u8", epoch=12, tune=tune), 3,
                         engine="cpu")
    grp.load(g)
    grp.run()
    assert (grp.gather() == ref).all()


def test_random_init_decomposition_independent(native, tune):
    grp = InProcessGroup(LifeConfig(128, 64, decomp="2x2", tune=tune), 4, engine="cpu")
    grp.init_random(99)
    assert (grp.gather() == random_grid(128, 64, 99)).all()


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("1x3", 3), ("2x2", 4), ("2x3", 6)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
@pytest.mark.parametrize("tmax,epoch", [(4, 8), (8, 8), (4, 12), (2, 5)])
def test_overlapped_exchange_matches_serial(native, tune, spec, P, layout, tmax, epoch):
    """Overlapped (trigger) epochs are bit-identical to the serial reference,
    including a short final epoch (gens not a multiple of the epoch depth):
    the last block's boundary rows are sent once the groups writing them are
    done (row strips, Px == 1; the CPU backend emulates the counter, tuning
    cpu_trigger)."""
    tune["cpu_trigger"] = "1"
    W, H = 192, 150
    g = random_grid(W, H, 77 + tmax)
    gens = 3 * epoch + epoch // 2 + 1
    ref, _, _ = reference_run(g, gens)
    cfg = LifeConfig(W, H, gen_limit=gens, decomp=spec, layout=layout, tmax=tmax, epoch=epoch, overlap="trigger", tune=tune)
    grp = InProcessGroup(cfg, P, engine="cpu")
    grp.load(g)
    reps = grp.run()
    want = spec.startswith("1x")
    assert all(r.overlapped == want for r in reps)
    assert all(s.native_engine.triggered_sends() == (3 if want else 0) for s in grp.sims)
    assert (grp.gather() == ref).all()


@pytest.mark.parametrize("W,H,seed,density", CONVERGING)
@pytest.mark.parametrize("lagged", [True, False])
def test_overlapped_termination(native, tune, W, H, seed, density, lagged):
    tune["cpu_trigger"] = "1"
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    cfg = LifeConfig(W, H, decomp="1x2", layout="u8", tmax=2, epoch=3, poll_gens=4, overlap="trigger",
                     lagged_poll=lagged, tune=tune)
    grp = InProcessGroup(cfg, 2, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    # The trigger needs no interior (H > 2D): only a second epoch in the run.
    assert all(r.overlapped == (r.executed > 3) for r in reps)
    assert (grp.gather() == ref).all()


def test_overlap_modes(native, tune):
    """trigger (= on) = the boundary rows sent once the groups writing them
    are done, on row strips of a backend that counts boundary groups done;
    auto decides on the ranks; column decompositions do not overlap."""
    def ov(**kw):
        cfg = dict(decomp="1x2", tmax=4, epoch=16)
        cfg.update(kw)
        H = cfg.pop("H", 512)
        eng = InProcessGroup(LifeConfig(64, H, **cfg, tune=tune), 2, engine="cpu").sims[0].native_engine
        return eng.overlap(), eng.overlap_mode()
    assert ov(overlap="trigger") == (False, "off")  # no counter on this backend
    assert ov() == (False, "off")
    tune["cpu_trigger"] = "1"
    assert ov(overlap="trigger") == (True, "trigger") and ov(H=40, overlap="trigger")[0]
    assert ov(overlap="on") == (True, "trigger")
    assert ov() == (False, "auto:trial") and ov(overlap="off") == (False, "off")
    assert not ov(decomp="2x1", overlap="trigger")[0]


@pytest.mark.parametrize("lagged", [True, False])
def test_trigger_across_runs_and_readouts(native, tune, lagged):
    """Chunked runs (run_until) and read-outs between them: an exchange sent at
    the end of one run is consumed by the next, and a read-out in between
    (tile(), which may rotate a drift out) never sees stale halos."""
    tune["cpu_trigger"] = "1"
    W, H = 128, 160
    g = random_grid(W, H, 5)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=10_000, decomp="1x2", tmax=4, epoch=8, poll_gens=8,
                                    overlap="trigger", lagged_poll=lagged, tune=tune), 2, engine="cpu")
    grp.load(g)
    want = g
    done = 0
    for n in (20, 3, 40, 16, 9):
        grp.parallel(lambda s: s.native_engine.run_until(s.generation + n))
        done += n
        want = reference_run(want, n, check_similarity=False)[0] if n else want
        assert (grp.gather() == want).all(), done


@pytest.mark.parametrize("overlap,decomp", [("off", "2x3"), ("trigger", "1x3")])
def test_random_transport_delays_do_not_change_results(native, tune, overlap, decomp):
    """Fault injection: random delays before every publish and
    consume shake the message interleaving; results must stay exact."""
    tune["fault_delay_us"] = "300"
    tune["cpu_trigger"] = "1"
    W, H = 128, 120
    g = random_grid(W, H, 8)
    ref, _, _ = reference_run(g, 40)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=40, decomp=decomp, layout="u8", tmax=2, epoch=6,
                                    overlap=overlap, tune=tune), 6 if decomp == "2x3" else 3, engine="cpu")
    grp.load(g)
    grp.run()
    assert (grp.gather() == ref).all()


def test_garbled_halo_is_detected(native, tune):
    """Fault injection: a corrupted halo message must show up as
    a mismatch against the serial reference - the golden comparison catches
    communication faults."""
    tune["fault_garble"] = "3"
    W, H = 96, 96
    g = random_grid(W, H, 21)
    ref, _, _ = reference_run(g, 30)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=30, decomp="1x2", layout="u8", tmax=2, epoch=4,
                                    overlap="off", tune=tune), 2, engine="cpu")
    grp.load(g)
    grp.run()
    assert (grp.gather() != ref).any()


def test_thread_transport_pair_matching_two_ranks(native, tune):
    """The row-phase op order of Engine::halo_exchange (engine.cpp) with
    Py = 2, where north and south are the same peer: messages between a pair
    must match in issue order (send N <-> recv S, send S <-> recv N), the
    contract RCCL's grouped send/recv also follows."""
    import threading

    import numpy as np

    C = native
    hub = C.ThreadHub(2)
    bes = [C.cpu_backend(1, tune=make_tuning(tune)) for _ in range(2)]
    trs = [C.thread_transport(hub, r, bes[r], tune=make_tuning(tune)) for r in range(2)]
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


@pytest.mark.parametrize("mode", ["auto", "trigger"])
def test_overlap_decision_is_global_on_uneven_tiles(native, tune, mode):
    """37 rows over 3 ranks = tiles of 12, 12, 13 rows.  Every rank must take
    the same schedule (a rank that sends from its last block while the others
    reduce flags would deadlock), so the decision depends on the
    decomposition, not on this rank's tile."""
    tune["cpu_trigger"] = "1"
    W, H = 96, 37
    g = random_grid(W, H, 3)
    ref, rgens, _ = reference_run(g, 50)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=50, decomp="1x3", layout="u8", tmax=2, epoch=6, overlap=mode,
                                    tune=tune), 3, engine="cpu")
    assert len({s.native_engine.overlap() for s in grp.sims}) == 1
    grp.load(g)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


@pytest.mark.parametrize("overlap", ["off", "on", "trigger"])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_self_exchange_rehearsal(native, tune, overlap, layout):
    """One rank rehearsing the multi-rank row-strip schedule (bench.py
    --rehearse-rccl): halos go through the transport to itself, with the
    multi-rank epoch depth and overlap; results equal the serial loop."""
    tune["cpu_trigger"] = "1"
    W, H = 128, 200
    g = random_grid(W, H, 12)
    ref, rgens, _ = reference_run(g, 120)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=120, layout=layout, tmax=4, epoch=16, overlap=overlap,
                                    self_exchange=True, tune=tune), 1, engine="cpu")
    grp.load(g)
    (rep,) = grp.run()
    assert rep.generations == rgens
    assert rep.exchanges >= 120 // 16 and rep.halo_bytes > 0
    assert rep.overlapped == (overlap != "off")
    assert (grp.gather() == ref).all()
