"""bench.py's launch contract, per-phase timing and the overlap auto trial on
the CPU (gloo / thread transports).

* ``bench.py --gpus N`` with no launcher starts N rank processes itself
  (the reference's ``mpiexec -n P``, README.md:56) and reports n_gpus = N;
  a launcher whose WORLD_SIZE differs from --gpus is refused.
* Per-phase device times are present and account for the
  generation loop.
* ``overlap=auto`` alternates the plain and trigger schedules, decides
  at the same epoch on every rank, and is exact in both outcomes and across
  the switch.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, random_grid, reference_run
from gol_amd.parallel import InProcessGroup

REPO = Path(__file__).resolve().parents[1]


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    env["PYTHONPATH"] = str(REPO) + os.pathsep + env.get("PYTHONPATH", "")
    env["GOL_HOST_THREADS"] = "2"
    env["OMP_NUM_THREADS"] = "1"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *map(str, args)], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


SMALL = ["--engine", "cpu", "--size", 256, "--steps", 3, "--warmup", 1, "--gens-per-step", 100, "--prewarm", 16,
         "--verify", 40]


@pytest.mark.parametrize("gpus", [1, 4, 8])
def test_bench_gpus_n_launches_n_ranks_itself(native, gpus):
    r = _bench(["--gpus", gpus, *SMALL])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == gpus and rec["steps"] == 3 and rec["warmup"] == 1
    cfg = rec["config"]
    assert cfg["generations_timed"] == 300 and cfg["step_stop_reasons"] == ["limit"]
    assert cfg["parallelism"].startswith("1x1" if gpus == 1 else f"1x{gpus}")
    assert rec["verified"] is True
    assert cfg["verify"]["vs_torch_fp32_oracle"] and cfg["verify"]["vs_u8_layout"]
    assert cfg["verify"]["generations"] == 40
    ph = cfg["phase_ms_one_step"]
    assert ph["generations"] == 100 and ph["compute_ms"] > 0 and ph["allreduce_ms"] >= 0
    if gpus > 1:
        assert ph["halo_ms"] > 0 and cfg["halo_bytes_per_step"] > 0
    # What the communicator saw: every rank reported, on the CPU engine.
    assert rec["rccl_nranks"] == gpus
    assert sorted(d["rank"] for d in rec["devices"]) == list(range(gpus))
    assert all(d["device"] == "cpu" for d in rec["devices"])
    # 256^2 is BASELINE config 1's grid, not the headline metric.
    assert rec["headline"] is False and rec["config_id"] == 1
    assert rec["metric"] == "cell-updates/sec (whole node), 256^2 x 100 gens"


@pytest.mark.parametrize("height,drift", [(256, "0"), (192, "1")])
def test_bench_band_verification_reads_rows_from_the_device(native, height, drift):
    """The check of grids beyond 2^30 cells: row bands and
    their light cones read straight from the engine (Engine.store_rows, no
    whole-grid host copy), wrapped around the torus, against the fp32 oracle;
    --verify-bands forces it on a small grid, with a drifting frame too."""
    r = _bench([*SMALL[:4], "--height", height, *SMALL[4:], "--verify-bands"], env_extra={"GOL_CPU_DRIFT": drift})
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    v = rec["config"]["verify"]
    assert rec["verified"] is True and v["vs_torch_fp32_oracle"] is True and v["vs_u8_layout"] is None
    assert "read from the device" in v["oracle"] and v["generations"] == 40


def test_store_rows_matches_the_tile(native):
    from gol_amd import LifeConfig, Simulation, random_grid

    for drift in ("0", "1"):
        os.environ["GOL_CPU_DRIFT"] = drift
        try:
            sim = Simulation(LifeConfig(128, 96, tmax=4, gen_limit=100), engine="cpu")
        finally:
            os.environ.pop("GOL_CPU_DRIFT")
        sim.load(random_grid(128, 96, 5))
        sim.advance(13)
        t = sim.tile()
        eng = sim.native_engine
        for r0, n in ((0, 96), (5, 17), (90, 6), (40, 0)):
            assert (eng.store_rows(r0, n) == t[r0:r0 + n]).all(), (r0, n)


def _bench_module():
    import importlib.util  # noqa: PLC0415
    spec = importlib.util.spec_from_file_location("gol_bench", REPO / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_metric_label_names_the_grid():
    b = _bench_module()
    m, head, cid = b.metric_label(32768, 32768, 1000)
    assert m == b.METRIC and head is True and cid == 3
    m, head, cid = b.metric_label(8192, 8192, 1000)
    assert "32768" not in m and "8192^2 x 1000 gens" in m and head is False and cid == 2
    m, head, cid = b.metric_label(32768, 4096, 1000)
    assert "32768x4096" in m and head is False and cid is None
    assert b.metric_label(32768, 32768, 200)[1] is False
    assert b.metric_label(65536, 65536, 1000)[2] == 4 and b.metric_label(1048576, 1048576, 1000)[2] == 5


def test_bench_rehearsal_is_never_a_headline():
    """VERDICT r04 Weak 5: 8 rank processes on one GPU (--share-gpus) or the
    one-rank RCCL self-exchange carry their own metric string, headline false
    and no BASELINE config id, even on the headline grid."""
    b = _bench_module()
    infos = [{"rank": r, "host": "n0", "device": 0, "pci_bus_id": "0000:05:00.0", "uuid": "ab"} for r in range(8)]
    reh = b.rehearsal_label(8, True, False, infos)
    assert reh == "8 ranks on 1 GPU"
    m, head, cid = b.metric_label(32768, 32768, 1000, reh)
    assert head is False and cid is None and m != b.METRIC and "rehearsal: 8 ranks on 1 GPU" in m
    assert b.rehearsal_label(1, False, True, infos[:1]) == "1 rank exchanging with itself through RCCL"
    m, head, cid = b.metric_label(32768, 32768, 1000, b.rehearsal_label(1, False, True, infos[:1]))
    assert head is False and cid is None and "rehearsal" in m
    two = [dict(i, uuid=str(i["rank"] % 2), pci_bus_id=f"0000:0{i['rank'] % 2}:00.0") for i in infos]
    assert b.rehearsal_label(8, True, False, two) == "8 ranks on 2 GPUs"
    real = [dict(i, uuid=str(i["rank"]), pci_bus_id=f"0000:{i['rank'] + 5:02x}:00.0") for i in infos]
    assert b.rehearsal_label(8, False, False, real) is None


def test_bench_check_ranks_refuses_what_rccl_did_not_see():
    """A fake communicator view: the refusal cases of bench.py's rank check
    (rccl_nranks != WORLD_SIZE, a rank missing, two ranks on one physical GPU
    without --share-gpus)."""
    b = _bench_module()
    infos = [{"rank": r, "host": "n0", "device": r, "pci_bus_id": f"0000:{r + 5:02x}:00.0", "uuid": f"u{r}"}
             for r in range(8)]
    assert b.check_ranks(8, False, 8, infos) is None
    assert "7 ranks" in b.check_ranks(8, False, 7, infos)
    assert "7 of 8" in b.check_ranks(8, False, 8, infos[:7])
    same = [dict(i, pci_bus_id="0000:05:00.0", uuid="u0", device=0) for i in infos]  # eight ranks on one device
    assert "share GPU" in b.check_ranks(8, False, 8, same)
    assert b.check_ranks(8, True, 8, same) is None  # --share-gpus: a declared rehearsal
    # one GPU seen under different process-local ordinals (per-rank
    # HIP_VISIBLE_DEVICES) is still one GPU.
    renamed = [dict(i, pci_bus_id="0000:05:00.0", uuid="u0") for i in infos]
    assert "share GPU" in b.check_ranks(8, False, 8, renamed)
    # Partitions of one physical GPU may share a bus id but have UUIDs of their own.
    parts = [dict(i, pci_bus_id="0000:05:00.0") for i in infos]
    assert b.check_ranks(8, False, 8, parts) is None


def test_bench_refuses_a_launcher_with_another_world_size(native):
    r = _bench(["--gpus", 4, *SMALL], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert r.stdout.strip() == ""
    assert "WORLD_SIZE=2" in r.stderr


def test_phase_times_account_for_the_loop(native):
    g = random_grid(512, 384, 3)
    sim = Simulation(LifeConfig(512, 384, gen_limit=300, tmax=8, epoch=32), engine="cpu")
    sim.load(g)
    assert sim.advance(50).phase_timed is False
    sim.phase_timing = True
    rep = sim.advance(250)
    assert rep.phase_timed
    total = rep.compute_ms + rep.halo_ms + rep.fill_ms + rep.allreduce_ms
    assert rep.compute_ms > 0 and rep.fill_ms > 0
    # Synchronous backend: the phases tile the loop (host bookkeeping aside).
    assert 0.6 * rep.loop_ms <= total <= 1.01 * rep.loop_ms, (total, rep.loop_ms)


def test_phase_times_with_ranks(native):
    W, H = 256, 512
    g = random_grid(W, H, 5)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=200, decomp="2x2", tmax=8, epoch=16), 4, engine="cpu")
    grp.load(g)
    for s in grp.sims:
        s.phase_timing = True
    reps = grp.run()  # with termination polls: flag all-reduces
    for r in reps:
        assert r.phase_timed and r.compute_ms > 0 and r.halo_ms > 0 and r.allreduce_ms > 0
        assert r.compute_ms + r.halo_ms + r.fill_ms + r.allreduce_ms <= 1.01 * r.loop_ms
    want, gens, _ = reference_run(g, 200)
    assert all(r.generations == gens for r in reps)
    assert (grp.gather() == want).all()


@pytest.mark.parametrize("pick", ["plain", "trigger", ""])
@pytest.mark.parametrize("layout", ["bits", "u8"])
def test_overlap_auto_trial_is_exact(native, monkeypatch, pick, layout):
    """Trial epochs alternate the plain schedule and the boundary trigger
    (the CPU backend emulates its counter with cpu_trigger), then every rank
    keeps the decided one; forced either way (and measured) the final grid
    and Generations equal the serial loop's."""
    monkeypatch.setenv("GOL_OVERLAP_AUTO", pick)
    monkeypatch.setenv("GOL_CPU_TRIGGER", "1")
    W, H, gens = 256, 3 * 200, 700
    g = random_grid(W, H, 7)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=gens, decomp="1x3", layout=layout, tmax=8, epoch=32,
                                    check_similarity=False), 3, engine="cpu")
    grp.load(g)
    reps = grp.advance(gens)
    modes = {s.describe()["overlap_mode"] for s in grp.sims}
    assert len(modes) == 1
    mode = modes.pop()
    if pick:
        assert mode == f"auto:{pick}"
    else:
        assert mode in ("auto:plain", "auto:trigger")
    d = grp.sims[0].describe()
    assert d["overlap_trial_ms_plain"] > 0 and d["overlap_trial_ms_trigger"] > 0
    assert all(r.overlapped for r in reps)  # the trial ran trigger epochs
    assert d["triggered_sends"] > 0
    want, _, _ = reference_run(g, gens, check_similarity=False)
    assert (grp.gather() == want).all()


def test_overlap_auto_with_termination(native, monkeypatch):
    """A run that stops at a fixed point during the trial keeps the exact
    Generations line, and the next run continues the trial."""
    monkeypatch.setenv("GOL_OVERLAP_AUTO", "trigger")
    monkeypatch.setenv("GOL_CPU_TRIGGER", "1")
    W, H = 32, 96
    g = random_grid(W, H, 95, 0.1)
    ref, rgens, _ = reference_run(g)
    assert rgens < 1000
    grp = InProcessGroup(LifeConfig(W, H, decomp="1x3", tmax=2, epoch=4, poll_gens=8), 3, engine="cpu")
    grp.load(g)
    reps = grp.run()
    assert all(r.generations == rgens for r in reps)
    assert (grp.gather() == ref).all()


def test_overlap_auto_is_off_without_row_exchange(native):
    sim = Simulation(LifeConfig(256, 256, gen_limit=100), engine="cpu")
    sim.load(random_grid(256, 256, 1))
    sim.run()
    assert sim.describe()["overlap_mode"] == "off"


def test_python_cli_show_prints_the_vt100_view(native, tmp_path):
    from gol_amd.utils import io

    g = np.array([[0, 1, 0], [1, 1, 0]], dtype=np.uint8)
    want = "\033[H" + "  \033[07m  \033[m  " + "\033[E" + "\033[07m  \033[m\033[07m  \033[m  " + "\033[E"
    assert io.show_text(g) == want
    assert io.show_text(np.where(g == 1, ord("1"), ord("0")).astype(np.uint8)) == want
    grid = random_grid(8, 6, 2)
    inp = tmp_path / "in.txt"
    io.write_grid(str(inp), grid)
    env = dict(os.environ, PYTHONPATH=str(REPO))
    r = subprocess.run([sys.executable, "-m", "gol_amd", "8", "6", str(inp), "--engine", "cpu", "--gens", "5",
                        "--output", "none", "--show"], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    ref, gens, _ = reference_run(grid, 5)
    assert r.stdout.startswith(f"Finished.\n\nGenerations:\t{gens}\n")
    assert r.stdout.endswith(io.show_text(ref))


def test_native_cli_metrics_carry_phases_and_comm(gol_bin, tmp_path):
    """bin/gol --metrics-json: per-phase device times (with --phase-timing
    only, so the timed loop carries no events by default), the resolved
    in-process transport (auto -> thread for CPU ranks) and the overlap mode."""
    m = tmp_path / "m.json"
    args = [str(gol_bin), "256", "600", "--random", "3", "--engine", "cpu", "--ranks", "3", "--decomp", "1x3",
            "--gens", "500", "--tmax", "8", "--epoch", "32", "--output", "none", "--metrics-json", str(m)]
    r = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(m.read_text())["phase_timed"] is False
    r = subprocess.run(args + ["--phase-timing"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rec = json.loads(m.read_text())
    assert rec["comm"] == "thread" and rec["ranks"] == 3
    assert rec["phase_timed"] is True and rec["compute_ms"] > 0 and rec["halo_ms"] > 0
    assert rec["compute_ms"] + rec["halo_ms"] + rec["fill_ms"] + rec["allreduce_ms"] <= 1.01 * rec["loop_ms"]
    assert rec["overlap_mode"] == "off"  # no trigger counter on the CPU backend


def test_native_cli_rccl_needs_a_gpu_per_rank(gol_bin, tmp_path):
    r = subprocess.run([str(gol_bin), "64", "64", "--random", "1", "--engine", "cpu", "--ranks", "2", "--comm", "rccl",
                        "--output", "none"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "rccl" in r.stderr


def test_native_cli_resume_rejects_another_sim_freq(gol_bin, tmp_path):
    ck = tmp_path / "ck"
    r = subprocess.run([str(gol_bin), "64", "64", "--random", "1", "--engine", "cpu", "--gens", "40",
                        "--checkpoint-every", "10", "--checkpoint-dir", str(ck), "--output", "none"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(gol_bin), "--resume", str(ck), "--engine", "cpu", "--sim-freq", "5", "--output", "none"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--sim-freq" in r.stderr


def test_band_oracle_matches_whole_grid_oracle():
    """bench.py checks grids beyond 2^30 cells on row bands with their light
    cones (no 2^32-element fp32 tensor): each band equals the same rows of the
    whole-grid fp32 oracle, at the torus's top, middle and bottom."""
    import numpy as np

    from gol_amd import random_grid
    from gol_amd.ops.life_ops import life_step_torch_roll

    b = _bench_module()
    H, W, g = 300, 64, 23
    snap = random_grid(W, H, 9)
    want = life_step_torch_roll(snap, g)
    starts = b.band_starts(H)
    assert starts[0] == 0 and starts[-1] == H - b.ORACLE_BAND_ROWS and len(starts) == 3
    for r0 in starts + [7]:
        rows = np.arange(r0, r0 + b.ORACLE_BAND_ROWS) % H
        assert np.array_equal(b.band_oracle(snap, r0, g, "cpu"), want[rows]), r0


def test_band_oracle_small_grid_is_whole_grid():
    """A torus shorter than one band: a single band covering every row."""
    import numpy as np

    from gol_amd import random_grid
    from gol_amd.ops.life_ops import life_step_torch_roll

    b = _bench_module()
    H, W, g = 40, 32, 9
    snap = random_grid(W, H, 3)
    assert b.band_starts(H) == [0]
    assert np.array_equal(b.band_oracle(snap, 0, g, "cpu"), life_step_torch_roll(snap, g))


@pytest.mark.parametrize("layout,u8c,want", [("bits", "auto", "u1 bit-packed"),
                                             ("u8", "bits", "u8 storage, computed on a live bit image"),
                                             ("u8", "bytes", "u8 byte-per-cell, computed on the bytes")])
def test_bench_dtype_label_says_what_the_loop_computes_on(native, layout, u8c, want):
    """VERDICT r05 Weak 5: a byte-layout record whose epochs ran on the bit
    image must not claim byte-per-cell compute."""
    env = dict(os.environ, PYTHONPATH=str(REPO), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--engine", "cpu", "--size", "128", "--steps", "1",
                        "--warmup", "0", "--gens-per-step", "32", "--prewarm", "0", "--verify", "16",
                        "--layout", layout, "--u8-compute", u8c], capture_output=True, text=True, timeout=300,
                       env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["dtype"].startswith(want), rec["dtype"]
    assert rec["config"]["u8_compute"] == (None if layout == "bits" else u8c)
    assert rec["config"]["row_ring_fallback"] is None


@pytest.mark.parametrize("overlap", ["off", "auto"])
def test_poll_placement_trial_is_exact(native, monkeypatch, overlap):
    """side_poll = -1 (default): after the overlap trial the ranks alternate
    poll windows whose flag all-reduce joins the compute stream and windows
    whose all-reduce runs on a side stream through the flags communicator,
    time them, MAX-reduce the medians and keep the faster - the same decision
    on every rank, with termination exact throughout (the thread transport
    claims a flags communicator with cpu_side_poll)."""
    monkeypatch.setenv("GOL_CPU_SIDE_POLL", "1")
    W, H = 128, 3 * 64
    g = random_grid(W, H, 21)
    grp = InProcessGroup(LifeConfig(W, H, gen_limit=1200, decomp="1x3", tmax=4, epoch=8, poll_gens=16,
                                    overlap=overlap, check_similarity=False), 3, engine="cpu")
    grp.load(g)
    modes0 = {s.describe()["poll_mode"] for s in grp.sims}
    assert modes0 == {"auto:trial"}
    reps = grp.run()  # termination polls every 16 generations
    d = [s.describe() for s in grp.sims]
    assert len({x["poll_mode"] for x in d}) == 1 and d[0]["poll_mode"] in ("auto:joined", "auto:side")
    pt = d[0]["poll_trial_ms_per_window"]
    assert pt["joined"] > 0 and pt["side"] > 0
    # a side win in the alternation is checked on a run of side windows and kept only if it holds
    if pt["side"] < 0.98 * pt["joined"]:
        assert pt["side_steady"] > 0 and (d[0]["poll_mode"] == "auto:side") == (pt["side_steady"] < pt["joined"])
    else:
        assert pt["side_steady"] == -1 and d[0]["poll_mode"] == "auto:joined"
    want, gens, _ = reference_run(g, 1200, check_similarity=False)
    assert all(r.generations == gens for r in reps)
    assert (grp.gather() == want).all()
    # a terminating run while the trial is still open stops exactly where the serial loop does
    g2 = random_grid(W, H, 95, 0.1)
    ref, rgens, _ = reference_run(g2)
    grp2 = InProcessGroup(LifeConfig(W, H, decomp="1x3", tmax=2, epoch=4, poll_gens=8, overlap=overlap), 3,
                          engine="cpu")
    grp2.load(g2)
    assert all(r.generations == rgens for r in grp2.run())
    assert (grp2.gather() == ref).all()
