"""GPU tier (MI355X): the CDNA4 kernels against the PyTorch fp32 oracle and the
CPU backend, golden semantics on the device, multi-subdomain runs on one GPU
(T3) and the RCCL / torch.distributed transport plumbing."""
import gc
import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, life_step, life_step_numpy, life_step_torch, random_grid, \
    reference_run, simulate
from gol_amd.models.life import make_tuning
from gol_amd.parallel import InProcessGroup

from golden import CASES, CONVERGING, GLIDER

pytestmark = pytest.mark.gpu


@pytest.fixture
def tune():
    """Runtime tuning each test passes through LifeConfig.tune and the
    backends it makes (gol/tuning.hpp).  The byte-layout tests here exercise
    the byte kernels themselves; the GPU's default byte-layout path (bit
    words, EngineConfig::u8_compute auto) has its own tests at the end of this
    file (test_u8_via_bits_*), which drop the key."""
    return {"u8_via_bits": "0"}


def test_hip_backend_is_native_gfx950(gpu, tune):
    be = gpu.hip_backend(0, tune=make_tuning(tune))
    assert be.is_device()
    assert "gfx950" in be.name()


@pytest.mark.parametrize("W,H", [(1, 1), (2, 2), (3, 5), (31, 7), (33, 33), (65, 40), (100, 1), (257, 129)])
def test_u8_kernel_awkward_sizes_vs_torch(gpu, W, H):
    g = random_grid(W, H, W * 7 + H)
    for gens in (1, 3, 17):
        want = life_step_torch(g, gens, device="cuda")
        assert (life_step(g, gens, engine="hip", layout="u8") == want).all(), gens


@pytest.mark.parametrize("W,H", [(32, 1), (32, 32), (64, 5), (96, 70), (2048, 40), (4000 - 4000 % 32, 130)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_kernel_word_sizes_vs_torch(gpu, W, H, layout):
    g = random_grid(W, H, W + H)
    want = life_step_torch(g, 21, device="cuda")
    assert (life_step(g, 21, engine="hip", layout=layout) == want).all()


@pytest.mark.parametrize("tmax", [1, 2, 4, 8, 16, 32])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_every_temporal_block_size(gpu, tmax, layout):
    # Wide enough for several column waves (62 words each) and tall enough
    # for several row segments per wave.
    W, H = 32 * 200, 700
    g = random_grid(W, H, tmax)
    want = life_step_torch(g, 2 * tmax + 3, device="cuda")
    got = life_step(g, 2 * tmax + 3, engine="hip", layout=layout, tmax=tmax)
    assert (got == want).all()


@pytest.mark.parametrize("xlane", [0, 3])
@pytest.mark.parametrize("tmax", [1, 4, 8, 12, 16])
def test_kernel_variants_vs_torch(gpu, tune, xlane, tmax):
    """Every compiled life_block variant (DPP | adder window) against the fp32
    conv oracle, including the changed-flag termination."""
    tune["xlane"] = str(xlane)
    # 4000 cells wide: 125 words -> tail handling in the last column wave.
    W, H = 4000 - 4000 % 32, 333
    g = random_grid(W, H, 11 + tmax)
    gens = 3 * tmax + 1
    want = life_step_torch(g, gens, device="cuda")
    assert (life_step(g, gens, engine="hip", layout="bits", tmax=tmax) == want).all()
    for cw, ch, seed, density in [c for c in CONVERGING if c[0] % 32 == 0]:
        grid = random_grid(cw, ch, seed, density)
        out, rep = simulate(grid, 1000, engine="hip", layout="bits", tmax=tmax)
        ref, rgens, _ = reference_run(grid)
        assert rep.generations == rgens, seed
        assert (out == ref).all(), seed


@pytest.mark.parametrize("xlane", [0, 3])
@pytest.mark.parametrize("tmax", [1, 8, 16])
def test_u8_kernel_variants_vs_torch(gpu, tune, xlane, tmax):
    tune["xlane"] = str(xlane)
    W, H = 1999, 301
    g = random_grid(W, H, 5 + tmax)
    gens = 2 * tmax + 5
    want = life_step_torch(g, gens, device="cuda")
    assert (life_step(g, gens, engine="hip", layout="u8", tmax=tmax) == want).all()


@pytest.mark.parametrize("tmax", [24, 32])
@pytest.mark.parametrize("xlane", [0, 3])
def test_deep_byte_passes_vs_torch(gpu, tune, tmax, xlane):
    """T = 24 / 32 byte-layout passes (life_block_u8_w1_*_t24/_t32.hip, the
    HBM-bound layout's deep passes) in every byte variant and schedule,
    against the fp32 conv oracle, and the exact Generations count."""
    tune["xlane"] = str(xlane)
    for group in ("8", "4", "0"):
        tune["group"] = group
        for W, H in [(32 * 200, 900), (1999, 777)]:
            g = random_grid(W, H, W + H + tmax)
            gens = 2 * tmax + 7
            want = life_step_torch(g, gens, device="cuda")
            sim = Simulation(LifeConfig(W, H, gen_limit=gens, layout="u8", tmax=tmax, tune=tune), engine="hip")
            assert sim.describe()["tmax"] == tmax
            sim.load(g)
            sim.advance(gens)
            assert (sim.tile() == want).all(), (group, W, H)
    grid = np.zeros((1024, 512), dtype=np.uint8)
    W, H, seed, density = CONVERGING[5]
    grid[500:500 + H, 200:200 + W] = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(grid)
    out, rep = simulate(grid, 1000, engine="hip", layout="u8", tmax=tmax)
    assert rep.generations == rgens
    assert (out == ref).all()


@pytest.mark.parametrize("group", ["0", "4", "8", "-1"])
@pytest.mark.parametrize("tmax", [4, 8, 12, 16])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_grouped_schedule_vs_torch(gpu, tune, group, tmax, layout):
    """Grouped schedule (csrc/kernels/life_group_impl.hpp: the M waves of a
    workgroup share their segment boundaries through LDS, so only group
    boundaries keep the redundant triangle) against the fp32 conv oracle:
    several groups per strip, uneven group sizes, last-wave remainders, tail
    words.  GOL_GROUP=0 is the classic schedule, -1 the model's choice."""
    tune["group"] = group
    for W, H in [(32 * 200, 700), (4000 - 4000 % 32, 1111), (2048, 333)]:
        g = random_grid(W, H, W + H + tmax)
        gens = 2 * tmax + 3
        want = life_step_torch(g, gens, device="cuda")
        assert (life_step(g, gens, engine="hip", layout=layout, tmax=tmax) == want).all(), (W, H)


@pytest.mark.parametrize("group", ["0", "4", "8", "-1"])
@pytest.mark.parametrize("tmax", [2, 4, 8, 12, 16])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_adder_window_vs_torch(gpu, tune, group, tmax, layout):
    """The DPP-free adder window (GOL_XLANE=3, kXlaneAdd: one-sided horizontal
    window from add-with-carry lane masks, storage frame drifting T cells per
    block) in every schedule, against the fp32 conv oracle; the drift is
    rotated out by the read-out."""
    tune["xlane"] = "3"
    tune["group"] = group
    for W, H in [(32 * 200, 700), (4000 - 4000 % 32, 1111), (2048, 333), (64, 40), (32, 3)]:
        g = random_grid(W, H, W + H + tmax)
        gens = 2 * tmax + 3
        want = life_step_torch(g, gens, device="cuda")
        sim = Simulation(LifeConfig(W, H, gen_limit=gens, layout=layout, tmax=tmax, tune=tune), engine="hip")
        sim.load(g)
        sim.advance(gens)
        assert sim.native_engine.drift == gens % W, (W, H)
        assert (sim.tile() == want).all(), (W, H)


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("1x4", 4), ("1x8", 8)])
@pytest.mark.parametrize("overlap", ["off", "trigger"])
def test_adder_window_row_strips_and_termination(gpu, tune, spec, P, overlap):
    """Row-strip subdomains on one GPU (the multi-GPU default decomposition)
    with the drifting adder window: lockstep drift, the trigger schedule's
    boundary sends, exact Generations."""
    tune["xlane"] = "3"
    for W, H, seed, density in [c for c in CONVERGING if c[0] % 32 == 0][:3] + [(256, 512, 77, 0.5)]:
        if H < 8 * P:
            continue
        g = random_grid(W, H, seed, density)
        ref, rgens, _ = reference_run(g)
        grp = InProcessGroup(LifeConfig(W, H, decomp=spec, tmax=8, epoch=16, poll_gens=32, overlap=overlap,
                                        tune=tune), P, engine="hip")
        grp.load(g)
        reps = grp.run()
        assert {r.generations for r in reps} == {rgens}, (W, H, seed)
        assert (grp.gather() == ref).all(), (W, H, seed)


@pytest.mark.parametrize("group", ["4", "8"])
def test_grouped_schedule_many_groups_and_termination(gpu, tune, group):
    """As many groups as the rows allow (GOL_TARGET_WAVES), and the exact
    Generations count when the grid settles inside a grouped launch."""
    tune["group"] = group
    tune["target_waves"] = "1000000"
    g = random_grid(2048, 1500, 9)
    for tmax in (8, 16):
        want = life_step_torch(g, 3 * tmax + 1, device="cuda")
        assert (life_step(g, 3 * tmax + 1, engine="hip", tmax=tmax) == want).all(), tmax
    grid = np.zeros((1024, 512), dtype=np.uint8)
    W, H, seed, density = CONVERGING[5]
    grid[500:500 + H, 200:200 + W] = random_grid(W, H, seed, density)  # settles after a while
    ref, rgens, _ = reference_run(grid)
    for layout in ("bits", "u8"):
        out, rep = simulate(grid, 1000, engine="hip", layout=layout, tmax=16)
        assert rep.generations == rgens, layout
        assert (out == ref).all(), layout


@pytest.mark.parametrize("W,H", [(32 * 200, 700), (4000 - 4000 % 32, 1111), (2048, 333), (4096, 2100),
                                 (32768, 600)])
@pytest.mark.parametrize("xlane,tmax", [(0, 16), (3, 12), (0, 8), (3, 4), (0, 12)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_chained_groups_vs_torch(gpu, tune, W, H, xlane, tmax, layout):
    """Chained groups (GOL_CHAIN=1, life_group_impl.hpp chain_fetch: the last
    wave of every group but a strip's last ends with the inverted triangle fed
    by the next group's wave 0 through global memory and a per-launch flag)
    against the fp32 conv oracle; few, many (several dispatch rounds) and a
    middle number of groups via the wave-count target."""
    tune["chain"] = "1"
    tune["xlane"] = str(xlane)
    g = random_grid(W, H, W * 7 + H)
    gens = 2 * tmax + 11
    want = life_step_torch(g, gens, device="cuda")
    for target in ("0", "100000", "3000"):
        tune["target_waves"] = target
        sim = Simulation(LifeConfig(W, H, gen_limit=gens, layout=layout, tmax=tmax, tune=tune), engine="hip")
        assert " chain" in sim.describe()["backend"]
        sim.load(g)
        sim.advance(gens)
        assert (sim.tile() == want).all(), target


def test_chain_autotuning_is_exact(gpu, tune, capfd):
    """Default launch-shape autotuning (GOL_CHAIN=-1): trial launches of both
    options (timed with events) and the settled choice give the same rows as
    the fp32 conv oracle, and every launch shape reaches a decision."""
    tune["chain"] = "-1"
    tune["tune_log"] = "1"
    W, H, gens = 8192, 1024, 16 * 12
    g = random_grid(W, H, 4242)
    want = life_step_torch(g, gens, device="cuda")
    sim = Simulation(LifeConfig(W, H, gen_limit=gens, tmax=16, epoch=32, tune=tune), engine="hip")
    assert "chain=tuned" in sim.describe()["backend"]
    sim.load(g)
    sim.advance(gens // 2)  # the trials (6 launches per shape); returns with the device idle
    sim.advance(gens - gens // 2)  # collects them and runs the settled choice
    assert (sim.tile() == want).all()
    err = capfd.readouterr().err
    assert "gol autotune:" in err and ("-> plain" in err or "-> chained" in err), err[-2000:]


@pytest.mark.parametrize("graphs", ["off", "on"])
def test_chained_groups_termination_and_row_strips(gpu, tune, graphs):
    """Exact Generations with chained groups, in graph capture (where the
    chain is off) and on 1x4 row-strip subdomains of one GPU."""
    tune["chain"] = "1"
    tune["target_waves"] = "100000"
    grid = np.zeros((1024, 512), dtype=np.uint8)
    W, H, seed, density = CONVERGING[5]
    grid[500:500 + H, 200:200 + W] = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(grid)
    for layout in ("bits", "u8"):
        out, rep = simulate(grid, 1000, engine="hip", layout=layout, tmax=16, graphs=graphs)
        assert rep.generations == rgens, layout
        assert (out == ref).all(), layout
    grp = InProcessGroup(LifeConfig(512, 1024, decomp="1x4", tmax=16, epoch=64, poll_gens=64, graphs=graphs,
                                    tune=tune), 4, engine="hip")
    grp.load(grid)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


@pytest.mark.parametrize("words", [79, 93, 136, 1024])
@pytest.mark.parametrize("xlane,tmax", [(0, 16), (3, 12), (0, 8), (3, 4)])
@pytest.mark.parametrize("wrap,fold", [("1", "1"), ("1", "0"), ("0", "0")])
def test_wrap_and_folded_strip_vs_torch(gpu, tune, words, xlane, tmax, wrap, fold):
    """Wrap mode (whole-width tiles read owned words mod the width, no halo
    columns; csrc/kernels/life_block_impl.hpp lane_cols) and the folded last
    strip (life_group_kernel: the narrow last strip's lanes packed 2-4 times
    into one wave, each sub-strip running another group's rows) against the
    fp32 conv oracle.  Widths: 79 / 93 / 136 words leave a last strip of
    16 / 30 / 10 words (fold 3 / 2 / 4); several group counts, including ones
    that leave a partial fold and unequal group sizes."""
    tune["xlane"] = str(xlane)
    tune["wrap"] = wrap
    tune["fold"] = fold
    W, H = 32 * words, 613 if words < 1024 else 300
    g = random_grid(W, H, words * 7 + tmax)
    gens = 2 * tmax + 5
    want = life_step_torch(g, gens, device="cuda")
    for target in ("0", "2000", "100000"):
        tune["target_waves"] = target
        sim = Simulation(LifeConfig(W, H, gen_limit=gens, tmax=tmax, tune=tune), engine="hip")
        sim.load(g)
        sim.advance(gens)
        assert (sim.tile() == want).all(), target


@pytest.mark.parametrize("words", [1, 2, 3, 31, 32, 33, 62, 63, 64, 65, 94, 125, 126, 127, 129, 190])
@pytest.mark.parametrize("xlane", [0, 3])
def test_wrap_mode_widths_vs_torch(gpu, tune, words, xlane):
    """Wrap mode across torus widths: narrower than one strip (lanes wrap
    several times around the row), one word either side of a strip boundary,
    and every fold factor of the last strip (1-4)."""
    tune["xlane"] = str(xlane)
    W, H = 32 * words, 97 + words
    g = random_grid(W, H, words * 13 + xlane)
    for tmax in (16, 12, 4):
        gens = tmax + 7
        want = life_step_torch(g, gens, device="cuda")
        sim = Simulation(LifeConfig(W, H, gen_limit=gens, tmax=tmax, tune=tune), engine="hip")
        sim.load(g)
        sim.advance(gens)
        assert (sim.tile() == want).all(), tmax


@pytest.mark.parametrize("xlane", [0, 3])
def test_folded_strip_termination_and_row_strips(gpu, tune, xlane):
    """Exact Generations with a folded last strip (the change flags of every
    sub-strip), and row-strip subdomains (Px = 1, so wrap mode on every rank)."""
    tune["xlane"] = str(xlane)
    tune["target_waves"] = "3000"
    grid = np.zeros((700, 32 * 79), dtype=np.uint8)
    W, H, seed, density = CONVERGING[5]
    grid[300:300 + H, 2500 - W:2500] = random_grid(W, H, seed, density)  # straddles the folded strip
    ref, rgens, _ = reference_run(grid)
    out, rep = simulate(grid, 1000, engine="hip", tmax=12 if xlane == 3 else 16)
    assert rep.generations == rgens
    assert (out == ref).all()
    grp = InProcessGroup(LifeConfig(32 * 79, 700, decomp="1x3", tmax=8, epoch=16, poll_gens=32, tune=tune), 3,
                         engine="hip")
    grp.load(grid)
    reps = grp.run()
    assert {r.generations for r in reps} == {rgens}
    assert (grp.gather() == ref).all()


def test_grouped_schedule_is_the_default(gpu, tune):
    sim = Simulation(LifeConfig(4096, 2048, tune=tune), engine="hip")
    assert "group=8" in sim.describe()["backend"]


@pytest.mark.parametrize("W,H", [(1, 1), (5, 3), (100, 70), (1023, 65), (1025, 200), (3000, 129), (32, 40),
                                 (2048, 333), (3072, 97), (8192, 130)])
@pytest.mark.parametrize("lds_rows", [32, 64])
def test_u8_lds_single_step_kernel_vs_torch(gpu, tune, W, H, lds_rows):
    """The LDS-tiled single-step byte kernel (GOL_U8_KERNEL=lds, T = 1); widths
    that are multiples of 32 run the torus-wrap loads (no halo columns, no
    fills: one launch per generation)."""
    tune["u8_kernel"] = "lds"
    tune["lds_rows"] = str(lds_rows)
    tune["lds_t"] = "1"
    g = random_grid(W, H, W ^ H)
    want = life_step_torch(g, 9, device="cuda")
    assert (life_step(g, 9, engine="hip", layout="u8") == want).all()
    sim = Simulation(LifeConfig(W, H, layout="u8", tune=tune), engine="hip")
    assert "lds" in sim.describe()["backend"] and sim.describe()["tmax"] == 1


@pytest.mark.parametrize("W,H", [(1, 1), (5, 3), (100, 70), (1023, 65), (1025, 200), (3000, 129), (32, 40),
                                 (2048, 333), (3072, 97), (8192, 130), (992, 56), (1984, 113)])
@pytest.mark.parametrize("lds_T,pack", [(2, 0), (4, 0), (8, 0), (8, 1), (16, 1), (32, 1), (32, 2),
                                         (8, 3), (32, 3)])
def test_u8_lds_multi_generation_kernel_vs_torch(gpu, tune, W, H, lds_T, pack):
    """The LDS-tiled byte kernel with T generations per launch: on the bytes
    (992-cell tiles with a 16-byte halo chunk per side) or packed to bit words
    in LDS (1984-cell tiles with a halo word per side); torus-wrap tiles
    (width % 32 == 0) and halo-column tiles, 45 generations (partial blocks
    at the end).  Packed tiles run 16-wave workgroups on these small grids;
    pack == 2: with the XCD-aware tile order (GOL_LDS_XCD=1), pack == 3:
    8-wave workgroups (the large-grid choice)."""
    tune["u8_kernel"] = "lds"
    tune["lds_t"] = str(lds_T)
    tune["lds_pack"] = str(min(pack, 1))
    tune["lds_xcd"] = str(int(pack == 2))
    tune["lds_waves"] = "8" if pack == 3 else "0"
    g = random_grid(W, H, W * 3 + H + lds_T)
    want = life_step_torch(g, 45, device="cuda")
    assert (life_step(g, 45, engine="hip", layout="u8") == want).all()
    sim = Simulation(LifeConfig(W, H, layout="u8", tune=tune), engine="hip")
    assert f"lds-tiled T={lds_T}" in sim.describe()["backend"] and sim.describe()["tmax"] == lds_T


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("2x1", 2), ("2x2", 4)])
def test_u8_lds_kernel_multi_subdomain(gpu, tune, spec, P):
    """LDS kernel with row exchanges (column wrap on 1xN strips) and column
    exchanges (halo columns), several subdomains on one GPU."""
    tune["u8_kernel"] = "lds"
    W, H = 32 * 40, 210
    g = random_grid(W, H, 8)
    want = life_step_torch(g, 40, device="cuda")
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=40, layout="u8", decomp=spec, tune=tune), P, engine="hip",
                         devices=[0])
    grp.load(g)
    grp.advance(40)
    assert (grp.gather() == want).all()


@pytest.mark.parametrize("W,H,seed,density", CONVERGING)
def test_u8_lds_termination(gpu, tune, W, H, seed, density):
    tune["u8_kernel"] = "lds"
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    out, rep = simulate(g, 1000, engine="hip", layout="u8")
    assert rep.generations == rgens
    assert (out == ref).all()


@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_graph_replay_matches_plain_launches(gpu, tune, layout):
    """Full epochs replayed from captured HIP graphs (device-side generation
    offset for the flags) == plain launches, incl. exact termination."""
    for W, H, seed, density in CONVERGING:
        g = random_grid(W, H, seed, density)
        ref, rgens, _ = reference_run(g)
        outs = {}
        for mode in ("on", "off"):
            lay = layout if (layout == "u8" or W % 32 == 0) else "u8"
            sim = Simulation(LifeConfig(W, H, layout=lay, tmax=4, epoch=8, poll_gens=16, graphs=mode, tune=tune),
                             engine="hip")
            sim.load(g)
            rep = sim.run()
            assert rep.generations == rgens, (mode, seed)
            assert (mode == "on") == (rep.graph_launches > 0) or rgens < 8
            outs[mode] = sim.tile()
        assert (outs["on"] == ref).all() and (outs["off"] == ref).all()
    g = random_grid(1000 - 1000 % 32, 300, 5)
    a = Simulation(LifeConfig(992, 300, gen_limit=500, epoch=64, graphs="on", tune=tune), engine="hip")
    a.load(g)
    r = a.run()
    assert r.graph_launches >= 7 and a.describe()["graphs"]
    assert (a.tile() == life_step_torch(g, 500, device="cuda")).all()


def test_hip_matches_cpu_backend_long_run(gpu):
    g = random_grid(1024, 512, 5)
    a = life_step(g, 300, engine="hip")
    b = life_step(g, 300, engine="cpu")
    assert (a == b).all()


@pytest.mark.parametrize("name,grid,gens", CASES)
@pytest.mark.parametrize("layout", ["auto", "u8"])
def test_golden_patterns_gpu(gpu, name, grid, gens, layout):
    out, rep = simulate(grid, 1000, engine="hip", layout=layout)
    ref, rgens, _ = reference_run(grid)
    assert rep.generations == gens == rgens
    assert (out == ref).all()


def test_glider_gpu(gpu):
    out, rep = simulate(GLIDER, 1000, engine="hip")
    assert (out == np.roll(np.roll(GLIDER, 2, 0), 2, 1)).all()


@pytest.mark.parametrize("W,H,seed,density", CONVERGING)
def test_termination_gpu(gpu, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    for tmax, epoch, poll in [(16, 0, 0), (4, 7, 5), (32, 64, 1000)]:
        out, rep = simulate(g, 1000, engine="hip", tmax=tmax, epoch=epoch, poll_gens=poll)
        assert rep.generations == rgens
        assert (out == ref).all()


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("1x4", 4), ("2x2", 4), ("2x4", 8), ("3x3", 9)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
@pytest.mark.parametrize("overlap", ["off", "trigger"])
def test_multi_subdomain_one_gpu(gpu, tune, spec, P, layout, overlap):
    W, H = 32 * 12, 300
    g = random_grid(W, H, 42)
    want = life_step_numpy(g, 150)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=150, decomp=spec, layout=layout, tmax=16, epoch=16,
                                    overlap=overlap, tune=tune), P, engine="hip", devices=[0])
    grp.load(g)
    reps = grp.run()
    assert all(r.generations == 150 for r in reps)
    assert all(r.overlapped == (overlap == "trigger" and spec.startswith("1x")) for r in reps)
    assert (grp.gather() == want).all()


def test_random_init_on_device_matches_host(gpu, tune):
    s = Simulation(LifeConfig(4096, 100, tune=tune), engine="hip")
    s.init_random(11, 0.5)
    assert (s.tile() == random_grid(4096, 100, 11, 0.5)).all()
    assert s.alive_count() == int(random_grid(4096, 100, 11, 0.5).sum())


def test_text_io_on_device(gpu, tune, tmp_path):
    from gol_amd.utils import io

    p = tmp_path / "in.txt"
    io.generate(str(p), 300, 200, seed=3)
    s = Simulation(LifeConfig(300, 200, gen_limit=50, tune=tune), engine="hip")
    s.load_text(str(p))
    s.run()
    out = tmp_path / "out.txt"
    s.write_text(str(out))
    ref, _, _ = reference_run(io.read_grid(str(p), 300, 200), 50)
    assert out.read_text() == io.format_text(ref)


def test_rccl_single_rank_self_exchange(gpu, tune):
    """RCCL transport plumbing on one GPU: a 1-rank communicator with
    send/recv to itself and a MAX all-reduce."""
    import torch

    C = gpu
    tr = C.rccl_transport(C.rccl_unique_id(), 0, 1, 0, tune=make_tuning(tune))
    assert tr.size() == 1 and tr.name() == "rccl"
    tr.barrier()
    # The engine's row-phase op order (send N, recv S, send S, recv N) with
    # every neighbour = self: pairs match in issue order, as between two ranks.
    n = 256 * 4160  # 256 halo rows of a 32768-cell bit tile's pitch
    top = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    bot = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    halo_s = torch.zeros_like(top)
    halo_n = torch.zeros_like(top)
    s = torch.cuda.current_stream().cuda_stream
    tr.exchange([(True, 0, top.data_ptr(), n), (False, 0, halo_s.data_ptr(), n),
                 (True, 0, bot.data_ptr(), n), (False, 0, halo_n.data_ptr(), n)], s)
    flags = torch.tensor([3, 0, 7], dtype=torch.int32, device="cuda")
    tr.allreduce_max_u32(flags.data_ptr(), 3, s)
    torch.cuda.synchronize()
    assert torch.equal(halo_s, top) and torch.equal(halo_n, bot)
    assert flags.tolist() == [3, 0, 7]


@pytest.mark.parametrize("overlap,side", [("off", "1"), ("off", "0"), ("trigger", "1"), ("trigger", "-1"), ("off", "-1")])
@pytest.mark.parametrize("xlane", [0, -1])
def test_rccl_self_exchange_rehearsal(gpu, tune, overlap, side, xlane):
    """The multi-rank row-strip schedule on one GPU (bench.py --rehearse-rccl):
    row halos through a 1-rank RCCL communicator sending to itself, the
    boundary-trigger sends, termination polls reduced on the side stream
    through the transport's flags communicator (GOL_SIDE_POLL = 1, or timed
    on the ranks with -1), against the fp32 conv oracle and the exact
    Generations."""
    tune["xlane"] = str(xlane)
    tune["side_poll"] = side
    C = gpu
    W, H = 32 * 96, 1200
    g = random_grid(W, H, 31)
    gens = 300
    want = life_step_torch(g, gens, device="cuda")
    tr = C.rccl_transport(C.rccl_unique_id(), 0, 1, 0, tune=make_tuning(tune))
    sim = Simulation(LifeConfig(W, H, gen_limit=gens, tmax=12 if xlane else 16, epoch=96, overlap=overlap,
                                self_exchange=True, tune=tune),
                     transport=tr, backend=C.hip_backend(0, tune=make_tuning(tune)))
    sim.load(g)
    rep = sim.advance(gens)
    assert rep.exchanges >= gens // 96 and rep.overlapped == (overlap != "off")
    assert (sim.tile() == want).all()
    for cw, ch, seed, density in [c for c in CONVERGING if c[0] % 32 == 0]:
        grid = random_grid(cw, ch, seed, density)
        ref, rgens, _ = reference_run(grid)
        s2 = Simulation(LifeConfig(cw, ch, tmax=4, epoch=8, poll_gens=16, overlap=overlap, self_exchange=True,
                                   tune=tune),
                        transport=tr, backend=C.hip_backend(0, tune=make_tuning(tune)))
        s2.load(grid)
        assert s2.run().generations == rgens
        assert (s2.tile() == ref).all()


def test_torch_tensor_views_of_engine_buffers(gpu):
    import torch

    from gol_amd.parallel.dist import tensor_view

    x = torch.arange(256, dtype=torch.uint8, device="cuda")
    v = tensor_view(x.data_ptr(), 256, True)
    assert v.device.type == "cuda" and v.data_ptr() == x.data_ptr()
    v[0] = 7
    torch.cuda.synchronize()
    assert int(x[0].item()) == 7


@pytest.mark.parametrize("W,H,epoch", [(64, 5, 32), (96, 70, 64), (2048, 40, 128), (32, 1, 16)])
def test_fused_periodic_fill_matches_cpu_buffer(gpu, tune, W, H, epoch):
    """Single-rank halo_exchange is one fused launch (fill_all_bits): the whole
    padded buffer (column halos, halo rows and corners, multi-wrap when Dv > H)
    must equal the CPU backend's two-pass fill.  Halo mode (GOL_WRAP=0): in
    wrap mode the engine fills no column halos."""
    import torch

    tune["wrap"] = "0"
    tune["row_ring"] = "0"  # a row ring has no row halos to fill

    from gol_amd.parallel.dist import tensor_view

    g = random_grid(W, H, W * 3 + H)
    bufs = []
    for engine in ("hip", "cpu"):
        sim = Simulation(LifeConfig(W, H, gen_limit=64, layout="bits", epoch=epoch, tune=tune), engine=engine)
        sim.load(g)
        eng = sim.native_engine
        eng.halo_exchange()
        sim.backend.synchronize()
        geo = eng.geom
        raw = tensor_view(eng.current_buffer(), geo.R() * geo.pitch, engine == "hip").cpu().numpy().copy()
        used = 4 * (2 * geo.hw + W // 32)  # bytes per row that hold cells (pitch padding excluded)
        bufs.append((raw.reshape(geo.R(), geo.pitch)[:, :used], geo.Dv, geo.hw))
        torch.cuda.synchronize()
    (a, dva, hwa), (b, dvb, hwb) = bufs
    assert (dva, hwa) == (dvb, hwb) and dva > 0 and hwa > 0
    assert np.array_equal(a, b)


def test_inprocess_ranks_keep_device_affinity(gpu, tune, tmp_path):
    """Single-process multi-rank run from fresh Python threads with
    GOL_CHECK_DEVICE=1: every backend entry point asserts its device is
    current and that its staging / chain / scratch buffers and the launch
    operands live on it.  Drives load_text, the autotuned chained-group
    launches, halo exchanges and store_cells (gather)."""
    from gol_amd.utils import io

    tune["check_device"] = "1"
    tune["chain"] = "-1"
    W, H, gens = 32 * 64, 4 * 640, 300
    p = tmp_path / "in.txt"
    io.generate(str(p), W, H, seed=9)
    g = io.read_grid(str(p), W, H)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=gens, decomp="1x4", epoch=96, tune=tune), 4, engine="hip",
                         devices=[0, 0, 0, 0])
    grp.parallel(lambda s: s.load_text(str(p)))
    reps = grp.advance(gens)
    assert all(r.executed == gens for r in reps)
    assert (grp.gather() == life_step_torch(g, gens, device="cuda")).all()


@pytest.mark.parametrize("W,H", [(32768, 1024), (4096, 700), (2048 * 3, 333), (32 * 100, 1000)])
@pytest.mark.parametrize("xlane,tmax", [(0, 16), (0, 8), (3, 12), (0, 12)])
def test_linked_launches_vs_torch(gpu, tune, W, H, xlane, tmax):
    """Linked launches (GOL_LINK=1, LifeBlockParams::link_*): consecutive
    grouped launches of an epoch run on two streams at once and order their
    rows through per-group completion words; against the fp32 conv oracle,
    with several epochs, the drifting adder window and partial epochs."""
    tune["link"] = "1"
    tune["row_ring"] = "0"  # ring epochs are single blocks: nothing to link
    tune["xlane"] = str(xlane)
    g = random_grid(W, H, W + 3 * H + tmax)
    gens = 10 * tmax + 7
    want = life_step_torch(g, gens, device="cuda")
    sim = Simulation(LifeConfig(W, H, gen_limit=gens, tmax=tmax, tune=tune), engine="hip")
    sim.load(g)
    rep = sim.advance(gens)
    assert (sim.tile() == want).all()
    assert rep.linked_launches > 0


def test_linked_launches_termination_and_subdomains(gpu, tune):
    tune["row_ring"] = "0"
    tune["link"] = "1"
    grid = np.zeros((1024, 2048), dtype=np.uint8)
    W, H, seed, density = CONVERGING[5]
    grid[500:500 + H, 200:200 + W] = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(grid)
    out, rep = simulate(grid, 1000, engine="hip", tmax=16)
    assert rep.generations == rgens
    assert (out == ref).all()
    W, H, gens = 32 * 64, 4 * 300, 400
    g = random_grid(W, H, 12)
    want = life_step_torch(g, gens, device="cuda")
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=gens, decomp="1x4", tmax=16, tune=tune), 4, engine="hip",
                         devices=[0])
    grp.load(g)
    grp.advance(gens)
    assert (grp.gather() == want).all()


# ---- byte layout on bit words (Engine::epoch_via_bits), the GPU default ----

@pytest.mark.parametrize("W,H,gens,tmax", [(32, 1, 40, 0), (96, 70, 77, 4), (2048, 40, 200, 0), (6400, 700, 131, 8),
                                           (8192, 1024, 1000, 0)])
def test_u8_via_bits_default_vs_torch(gpu, tune, W, H, gens, tmax):
    tune.pop("u8_via_bits", None)
    g = random_grid(W, H, W + H + gens)
    sim = Simulation(LifeConfig(W, H, gen_limit=gens, layout="u8", tmax=tmax, tune=tune), engine="hip")
    d = sim.describe()
    assert d["u8_compute"] == "bits" and d["layout"] == "u8"
    sim.load(g)
    sim.advance(gens)
    assert (sim.tile() == life_step_torch(g, gens, device="cuda")).all()


def test_u8_via_bits_ragged_width_falls_back(gpu, tune):
    tune.pop("u8_via_bits", None)
    W, H = 1000, 64
    g = random_grid(W, H, 3)
    sim = Simulation(LifeConfig(W, H, gen_limit=50, layout="u8", tune=tune), engine="hip")
    assert sim.describe()["u8_compute"] == "bytes"
    sim.load(g)
    sim.advance(50)
    assert (sim.tile() == life_step_torch(g, 50, device="cuda")).all()


@pytest.mark.parametrize("W,H,seed,density", [(32, 16, 1, 0.2), (64, 20, 1, 0.2), (128, 12, 11, 0.2)] +
                         [c for c in CONVERGING if c[0] % 32 == 0])
def test_u8_via_bits_termination(gpu, tune, W, H, seed, density):
    g = random_grid(W, H, seed, density)
    ref, rgens, _ = reference_run(g)
    for tmax, epoch in [(0, 0), (4, 7), (1, 1)]:
        sim = Simulation(LifeConfig(W, H, layout="u8", u8_compute="bits", tmax=tmax, epoch=epoch, tune=tune),
                         engine="hip")
        sim.load(g)
        rep = sim.run()
        assert rep.generations == rgens, (tmax, epoch)
        assert (sim.tile() == ref).all()


@pytest.mark.parametrize("spec,P", [("1x2", 2), ("2x2", 4), ("1x4", 4)])
def test_u8_via_bits_subdomains_one_gpu(gpu, tune, spec, P):
    W, H = 4096, 512
    g = random_grid(W, H, 41)
    want = life_step_torch(g, 300, device="cuda")
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=300, decomp=spec, layout="u8", u8_compute="bits",
                                    check_similarity=False, tune=tune), P, engine="hip")
    grp.load(g)
    grp.parallel(lambda s: s.advance(300))
    assert all(s.native_engine.via_bits for s in grp.sims)
    assert (grp.gather() == want).all()


def test_u8_via_bits_graphs_and_chunked_runs(gpu, tune):
    """Captured epochs alternate over the bit-word pair (graphs keyed by its
    parity); each run packs and unpacks once, so chunked runs and read-outs in
    between stay exact."""
    W, H = 4096, 1024
    g = random_grid(W, H, 12)
    sim = Simulation(LifeConfig(W, H, gen_limit=2000, layout="u8", u8_compute="bits", graphs="on",
                                check_similarity=False, tune=tune), engine="hip")
    assert sim.native_engine.graphs()
    sim.load(g)
    want = g
    graphs = 0
    for n in (300, 517, 96):
        sim.advance(n)
        graphs += sim.last_report.graph_launches  # a run shorter than an epoch replays none
        want = life_step_torch(want, n, device="cuda")
        assert (sim.tile() == want).all(), n
    assert graphs > 0


def test_u8_via_bits_graphs_survive_drift_rotation(gpu, tune):
    """A drifting (adder-window) kernel leaves the byte tile drifted; every
    read-out rotates the drift out, which flips the byte buffer pair and so
    moves the bit scratch.  Equal-length chunks must not replay a graph
    captured against the other buffer (graphs are keyed by both parities)."""
    tune["xlane"] = "3"  # kXlaneAdd: the drifting adder window
    W, H = 4096, 1024
    g = random_grid(W, H, 21)
    sim = Simulation(LifeConfig(W, H, gen_limit=4000, layout="u8", u8_compute="bits", graphs="on",
                                check_similarity=False, tune=tune), engine="hip")
    eng = sim.native_engine
    assert eng.graphs() and eng.drifting
    sim.load(g)
    want = g
    graphs = 0
    drifted = 0
    for _ in range(4):
        sim.advance(2 * eng.epoch_depth)
        graphs += sim.last_report.graph_launches
        drifted += eng.drift != 0
        want = life_step_torch(want, 2 * eng.epoch_depth, device="cuda")
        assert (sim.tile() == want).all()
    assert graphs > 0 and drifted > 0


# ---- row ring (Backend::row_ring_halo, hipMemMap'd halos) -------------------

@pytest.mark.parametrize("W,H", [(8192, 4096), (32768, 1024), (16384, 2048), (4096, 8192)])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_row_ring_vs_torch(gpu, tune, W, H, layout):
    """Single-rank tiles whose row halos are second mappings of their own
    owned rows (three physical pieces mapped [C | A B C | A]; B may be empty):
    no fills, every block over exactly the owned rows.  Chunked runs with
    read-outs (drift rotations) in between, against the fp32 oracle."""
    g = random_grid(W, H, W // 32 + H)
    sim = Simulation(LifeConfig(W, H, layout=layout, gen_limit=1000, tune=tune), engine="hip")
    d = sim.describe()
    assert d["row_ring"] is True, d
    sim.load(g)
    want = g
    for n in (45, 100):
        sim.advance(n)
        want = life_step_torch(want, n, device="cuda")
        assert (sim.tile() == want).all(), n
    assert sim.last_report.exchanges > 0


def test_row_ring_termination_and_off_switch(gpu, tune):
    """Exact Generations through the ring: a block split by the wrap row is a
    still life only if the halos alias correctly (reference: 2 generations);
    a lone cell dies (1).  Same with the ring off."""
    for ring in ("1", "0"):
        tune["row_ring"] = ring
        for cells, want in (([(4095, 10), (4095, 11), (0, 10), (0, 11)], 2), ([(0, 8191)], 1)):
            grid = np.zeros((4096, 8192), dtype=np.uint8)
            for r, c in cells:
                grid[r, c] = 1
            sim = Simulation(LifeConfig(8192, 4096, poll_gens=16, tune=tune), engine="hip")
            assert sim.describe()["row_ring"] is (ring == "1")
            sim.load(grid)
            rep = sim.run()
            assert rep.generations == want, (ring, cells)
            assert (sim.tile() == (grid if want == 2 else 0)).all(), (ring, cells)


def test_row_ring_graphs(gpu, tune):
    W, H = 8192, 4096
    g = random_grid(W, H, 77)
    sim = Simulation(LifeConfig(W, H, gen_limit=400, graphs="on", check_similarity=False, tune=tune), engine="hip")
    assert sim.describe()["row_ring"] is True and sim.native_engine.graphs()
    sim.load(g)
    sim.advance(200)
    assert sim.last_report.graph_launches > 0
    assert (sim.tile() == life_step_torch(g, 200, device="cuda")).all()


def test_rank_tile_multirank_schedule_links_by_default(gpu, tune):
    """The 8-GPU rank tile (32768 x 4096) in the multi-rank schedule (row
    halos through a 1-rank RCCL communicator, epoch trapezoids): the blocks of
    an epoch run linked by default, every exchange and poll joins the two
    streams first, and the result is exact against the fp32 oracle."""
    C = gpu
    W, H = 32768, 4096
    g = random_grid(W, H, 17)
    gens = 600  # past two epochs of 16T = 256 and two termination polls
    want = life_step_torch(g, gens, device="cuda")
    tr = C.rccl_transport(C.rccl_unique_id(), 0, 1, 0, tune=make_tuning(tune))
    sim = Simulation(LifeConfig(W, H, gen_limit=gens, self_exchange=True, tune=tune), transport=tr,
                     backend=C.hip_backend(0, tune=make_tuning(tune)))
    d = sim.describe()
    assert d["tmax"] == 16 and d["row_ring"] is False
    sim.load(g)
    rep = sim.advance(gens)
    assert rep.exchanges >= 2 and rep.linked_launches > 0
    assert (sim.tile() == want).all()


def test_small_ring_tiles_link_launches_by_default(gpu, tune):
    """Small single-rank ring tiles (the small-tile T rule, >= 1.5 waves per
    SIMD per launch) run consecutive blocks linked by default
    (KernelChoice::link): exact against the fp32 oracle, bits and u8 (the
    GPU default for bytes: computed on bit words)."""
    tune.pop("u8_via_bits", None)
    W = H = 8192
    g = random_grid(W, H, 88)
    want = life_step_torch(g, 200, device="cuda")
    for layout in ("bits", "u8"):
        sim = Simulation(LifeConfig(W, H, layout=layout, gen_limit=1000, tune=tune), engine="hip")
        assert sim.describe()["row_ring"] is True and sim.describe()["tmax"] == 8
        sim.load(g)
        rep = sim.advance(200)
        assert rep.linked_launches > 0, layout
        assert (sim.tile() == want).all(), layout


@pytest.mark.parametrize("seed,density", [(5, 0.5), (77, 0.004), (3, 0.01)])
def test_linked_chain_continues_across_polls(gpu, tune, seed, density):
    """Termination polls of a single-rank run copy their flag window on a side
    stream that waits for both compute streams' tails (Backend::poll_side),
    so a linked chain is not restarted at every poll: a run that reaches its
    limit is one chain (every launch but the first linked).  Exact against
    the same run with linking off (whose termination the serial-loop tests
    pin) - sparse soups settle or die inside the run - and, at the limit,
    against the fp32 oracle."""
    tune.pop("u8_via_bits", None)
    W = H = 8192
    g = random_grid(W, H, seed, density)
    reps, tiles = [], []
    for link in ("-1", "0"):
        t = dict(tune, link=link, poll_copy_side="1")  # forced: auto keeps T <= 8 tiles on the join path
        sim = Simulation(LifeConfig(W, H, gen_limit=600, poll_gens=64, tune=t), engine="hip")
        assert sim.describe()["tmax"] == 8
        sim.load(g)
        reps.append(sim.run())
        tiles.append(sim.tile())
    (a, b), (ta, tb) = reps, tiles
    assert (a.generations, a.stop_reason) == (b.generations, b.stop_reason)
    assert (ta == tb).all()
    assert b.linked_launches == 0
    if a.stop_reason == "limit":
        assert (ta == life_step_torch(g, 600, device="cuda")).all()
        # 75 launches of T = 8, 9 polls every 64 generations: one chain.
        assert a.kernel_launches == 75 and a.linked_launches == 74 and a.polls >= 9, a


@pytest.mark.parametrize("seed,density", [(77, 0.004), (3, 0.01), (5, 0.5)])
def test_default_poll_interval_termination_exact(gpu, tune, seed, density):
    """A single-rank tile whose polls join the linked streams (T <= 8) polls
    every 1024 generations by default (round 6): the stop is still exact -
    the same Generations, reason and final grid as polling every 64 - and a
    run to the limit makes one poll per 1024 generations (plus the last)."""
    tune.pop("u8_via_bits", None)
    W = H = 8192
    g = random_grid(W, H, seed, density)
    out = []
    for poll in (0, 64):
        sim = Simulation(LifeConfig(W, H, gen_limit=2500, poll_gens=poll, tune=tune), engine="hip")
        assert sim.describe()["tmax"] == 8
        sim.load(g)
        out.append((sim.run(), sim.tile()))
    (a, ta), (b, tb) = out
    assert (a.generations, a.stop_reason) == (b.generations, b.stop_reason)
    assert (ta == tb).all()
    if a.stop_reason == "limit":
        assert a.polls == 3 and b.polls > 30, (a.polls, b.polls)


@pytest.mark.parametrize("part", ["0/2", "1/4", "3/8"])
def test_cu_partition_single_process(gpu, tune, part):
    """tuning cu_partition=k/n (ranks sharing a GPU): the backend's streams
    are CU-masked to the k-th of n slices, launches are planned for the
    slice's CUs, and chained groups and linked launches stay off (a time-
    sliced queue could outlast their bounded waits).  Exact against the fp32
    oracle on a small ring tile that links by default and on the rank tile's
    multi-rank schedule."""
    from gol_amd import native
    tune.pop("u8_via_bits", None)
    t = dict(tune, cu_partition=part)
    W = H = 8192
    g = random_grid(W, H, 13)
    sim = Simulation(LifeConfig(W, H, gen_limit=1000, tune=t), engine="hip")
    assert "cu-partition=" + part in sim.backend.name()
    assert sim.describe()["tuning"]["cu_partition"] == part
    sim.load(g)
    rep = sim.advance(160)
    assert rep.linked_launches == 0
    assert (sim.tile() == life_step_torch(g, 160, device="cuda")).all()
    C = native()
    W2, H2 = 32768, 1024
    g2 = random_grid(W2, H2, 14)
    tr = C.rccl_transport(C.rccl_unique_id(), 0, 1, 0, tune=make_tuning(t))
    sim2 = Simulation(LifeConfig(W2, H2, gen_limit=1000, self_exchange=True, tune=t), transport=tr,
                      backend=C.hip_backend(0, tune=make_tuning(t)))
    sim2.load(g2)
    rep2 = sim2.advance(300)
    assert rep2.linked_launches == 0 and rep2.exchanges > 0
    assert (sim2.tile() == life_step_torch(g2, 300, device="cuda")).all()
    # Masked streams are HIP queues of their own: release them here, not at
    # an arbitrary later collection.
    del sim, sim2, tr
    gc.collect()


def test_linked_ring_late_seam_producers_vs_torch(gpu, tune):
    """Linked launches on a row ring (the round-4 race): with
    GOL_FAULT_DELAY_SPINS the first and last groups of every launch publish
    ~1 ms late, so a group at the other end of the torus that read their rows
    without waiting for them (link_wait before it wrapped the rows) would see
    the previous generation."""
    tune["link"] = "1"
    tune["fault_delay_spins"] = "300"
    W, H = 8192, 8192
    sim = Simulation(LifeConfig(W, H, tmax=8, gen_limit=10_000, tune=tune), engine="hip")
    assert sim.describe()["row_ring"]
    g = random_grid(W, H, 8)
    sim.load(g)
    rep = sim.advance(8 * 12 + 3)
    assert rep.linked_launches > 0
    assert (sim.tile() == life_step_torch(g, 8 * 12 + 3, device="cuda")).all()


@pytest.mark.parametrize("side", ["0", "1"])
def test_rank_tile_links_only_without_comm_stream_work(gpu, tune, side):
    """Linked launches assume the device to themselves (the "two launches
    fit" cap counts only the pair): the engine links blocks of
    the multi-rank schedule only while no transport work can run beside them
    on the comm stream.  The 8-GPU rank tile's schedule, rehearsed with a
    1-rank RCCL communicator: linked with polls on the compute stream, never
    with side polls (tuning side_poll = 1) - and exact either way."""
    native = gpu
    tune["side_poll"] = side
    W, H = 32768, 4096
    tr = native.rccl_transport(native.rccl_unique_id(), 0, 1, 0, tune=make_tuning(tune))
    sim = Simulation(LifeConfig(W, H, gen_limit=600, overlap="off", self_exchange=True, epoch=256, tune=tune),
                     engine="hip", transport=tr)
    g = random_grid(W, H, 77)
    sim.load(g)
    rep = sim.run()  # with termination polls
    if side == "0":
        assert rep.linked_launches > 0
    else:
        assert rep.linked_launches == 0
    assert (sim.tile() == life_step_torch(g, 600, device="cuda")).all()


@pytest.mark.parametrize("layout,delay", [("bits", "0"), ("bits", "300"), ("u8", "0")])
def test_rank_tile_trigger_schedule(gpu, tune, layout, delay):
    """The boundary-trigger schedule on the 8-GPU rank tile (32768 x 4096,
    multi-rank epochs against a 1-rank RCCL communicator): the last block of
    every full epoch is a linked launch whose boundary groups count
    themselves done on a device counter, the comm stream waits on it
    (hipStreamWaitValue64) and sends the rows while the interior groups run.
    With GOL_FAULT_DELAY_SPINS the first and last groups - exactly the
    boundary groups - publish ~1 ms late, so a send that did not wait for
    them would ship the previous generation.  Byte tiles run it on their bit
    image.  Exact against the fp32 oracle."""
    tune.pop("u8_via_bits", None)
    tune["fault_delay_spins"] = delay
    C = gpu
    W, H = 32768, 4096
    g = random_grid(W, H, 23)
    gens = 600  # two full epochs followed by another: two triggered sends
    want = life_step_torch(g, gens, device="cuda")
    tr = C.rccl_transport(C.rccl_unique_id(), 0, 1, 0, tune=make_tuning(tune))
    sim = Simulation(LifeConfig(W, H, layout=layout, gen_limit=gens, self_exchange=True, overlap="trigger",
                                tune=tune),
                     transport=tr, backend=C.hip_backend(0, tune=make_tuning(tune)))
    d = sim.describe()
    assert d["overlap_mode"] == "trigger" and d["epoch"] == 256
    sim.load(g)
    rep = sim.advance(gens)
    assert rep.overlapped and rep.linked_launches > 0
    assert sim.native_engine.triggered_sends() == 2
    assert (sim.tile() == want).all()


def test_ring_stress_tool_keep_policy(gpu, repo):
    """bin/ring_stress (VERDICT r05 Weak 6): 200 rings of mixed geometry with
    allocation churn, mapped exactly as HipBackend::alloc_row_ring does, every
    address range kept reserved after release (the backend's policy): no
    hipMemSetAccess failure and every halo alias reads its owned row.  (With
    ranges freed or reused the same tool finds stale aliases,
    profiles/r06/ring_stress.txt - why the backend never reuses a range.)"""
    import subprocess

    r = subprocess.run([str(repo / "bin" / "ring_stress"), "200", "keep"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    line = next(ln for ln in r.stdout.splitlines() if ln.startswith("keep"))
    assert "setaccess failures 0 " in line and "alias failures 0 " in line, line


def test_many_ring_engines_in_one_process_keep_their_rings(gpu, tune):
    """Engines with row rings created and dropped one after another in one
    process (a test session, repeated Simulation construction) all get their
    rings - no silent fallback to fills - and stay exact."""
    tune.pop("u8_via_bits", None)
    for i in range(40):
        W, H = (4096, 2048) if i % 2 else (8192, 1024)
        sim = Simulation(LifeConfig(W, H, gen_limit=100, tune=tune), engine="hip")
        d = sim.describe()
        assert d["row_ring"] is True and d["row_ring_fallback"] is None, (i, d["row_ring_fallback"])
        if i % 10 == 0:
            g = random_grid(W, H, i)
            sim.load(g)
            sim.advance(40)
            assert (sim.tile() == life_step_torch(g, 40, device="cuda")).all(), i
        del sim
        gc.collect()
