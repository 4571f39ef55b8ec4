"""Multi-process runs on the CPU: one process per rank, torch.distributed
(gloo) process group, halos through the engine's torch.distributed callback
transport - the same code path the GPU uses with nccl=RCCL.  Compared
byte-for-byte with the exact serial loop."""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from gol_amd import random_grid, reference_run
from gol_amd.utils import io

REPO = Path(__file__).resolve().parents[1]



def _torchrun(nproc: int, args: list[str], cwd: Path, timeout: int = 300) -> subprocess.CompletedProcess:
    env = dict(os.environ)
    env["PYTHONPATH"] = str(REPO) + os.pathsep + env.get("PYTHONPATH", "")
    env["GOL_HOST_THREADS"] = "2"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}",
           "--standalone", "--local-addr=127.0.0.1", *args]
    return subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("nproc,decomp,layout", [(2, "1x2", "bits"), (2, "2x1", "u8"), (4, "2x2", "bits"),
                                                 (3, "1x3", "u8"), (8, "1x8", "bits"), (8, "2x4", "u8")])
def test_torchrun_cli_matches_serial(native, tmp_path, nproc, decomp, layout):
    W, H = 128, 96
    g = random_grid(W, H, 31)
    inp = tmp_path / "in.txt"
    io.write_grid(str(inp), g)
    r = _torchrun(nproc, ["-m", "gol_amd", str(W), str(H), str(inp), "--engine", "cpu", "--gens", "200",
                          "--decomp", decomp, "--layout", layout, "--comm", "torch", "--epoch", "9",
                          "--output", str(tmp_path / "out.txt"), "--style", "mpi"], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    ref, gens, _ = reference_run(g, 200)
    assert f"Generations:\t{gens}" in r.stdout
    assert r.stdout.count("Finished") == nproc
    assert (tmp_path / "out.txt").read_text() == io.format_text(ref)


def test_torchrun_terminating_run(native, tmp_path):
    W, H = 64, 32
    g = random_grid(W, H, 11, 0.2)
    ref, gens, _ = reference_run(g)
    assert gens < 1000
    inp = tmp_path / "in.txt"
    io.write_grid(str(inp), g)
    r = _torchrun(2, ["-m", "gol_amd", str(W), str(H), str(inp), "--engine", "cpu", "--comm", "torch",
                      "--poll", "8", "--output", str(tmp_path / "out.txt")], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert f"Generations:\t{gens}" in r.stdout
    assert (tmp_path / "out.txt").read_text() == io.format_text(ref)


def test_bench_cpu_dry_run_two_ranks(native, tmp_path):
    r = _torchrun(2, [str(REPO / "bench.py"), "--gpus", "2", "--engine", "cpu", "--comm", "torch",
                      "--size", "256", "--steps", "3", "--warmup", "1", "--gens-per-step", "100",
                      "--prewarm", "16"], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    import json

    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1 and rec["value"] > 0
    assert rec["higher_is_better"] is True and rec["scaling"] == "strong"
    cfg = rec["config"]
    # one step = one --gens-per-step run; exactly steps x that many timed
    assert cfg["gens_per_step"] == 100 and cfg["generations_timed"] == 300
    assert cfg["step_stop_reasons"] == ["limit"]
    assert cfg["exchanges_per_step"] >= 1 and cfg["polls_per_step"] >= 1
    assert abs(rec["value"] - 256 * 256 * 300 / (rec["ms_per_step"] * 3e-3)) < 1e-6 * rec["value"]


@pytest.mark.parametrize("nproc,layout", [(2, "bits"), (4, "u8")])
def test_torchrun_trigger_schedule_matches_serial(native, tmp_path, nproc, layout):
    """The boundary-trigger schedule (overlap trigger: each epoch's new
    boundary rows sent as soon as the groups writing them are done) across
    real rank processes over gloo, the CPU backend emulating the device
    counter (tuning cpu_trigger): byte-identical output and Generations."""
    W, H = 128, 160
    g = random_grid(W, H, 47)
    inp = tmp_path / "in.txt"
    io.write_grid(str(inp), g)
    r = _torchrun(nproc, ["-m", "gol_amd", str(W), str(H), str(inp), "--engine", "cpu", "--gens", "300",
                          "--decomp", f"1x{nproc}", "--layout", layout, "--comm", "torch", "--epoch", "8",
                          "--tmax", "4", "--overlap", "trigger", "--tune", "cpu_trigger=1",
                          "--output", str(tmp_path / "out.txt"), "--style", "mpi"], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    ref, gens, _ = reference_run(g, 300)
    assert f"Generations:\t{gens}" in r.stdout
    assert (tmp_path / "out.txt").read_text() == io.format_text(ref)


@pytest.mark.parametrize("nproc,layout,overlap", [(2, "bits", "off"), (3, "u8", "trigger"), (4, "bits", "auto")])
def test_bench_multirank_band_verifier(native, tmp_path, nproc, layout, overlap):
    """bench.py --verify-bands on several ranks: every rank checks the top,
    middle and bottom row bands of its own tile against the fp32 oracle, the
    light-cone rows beyond its tile sent by its north and south neighbours
    (parallel/dist.py verify_row_bands) - the path config 5's 2^40-cell grid
    takes, where no host can gather the grid."""
    args = [str(REPO / "bench.py"), "--gpus", str(nproc), "--engine", "cpu", "--comm", "torch",
            "--size", "256", "--height", str(96 * nproc), "--layout", layout, "--steps", "1", "--warmup", "0",
            "--gens-per-step", "64", "--prewarm", "0", "--verify", "40", "--verify-bands", "--overlap", overlap,
            "--tune", "cpu_trigger=1"]
    r = _torchrun(nproc, args, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    v = rec["config"]["verify"]
    assert rec["verified"] is True and v["vs_torch_fp32_oracle"] is True, v
    assert "no gather" in v["oracle"] and v["generations"] == 40


def test_multirank_band_verifier_catches_a_wrong_cell(native, tmp_path):
    """The verifier is not vacuous: a few wrong cells on one rank, introduced
    between the snapshot and the run, fails every rank (AND over ranks)."""
    script = tmp_path / "flip.py"
    script.write_text(f'''
import sys
sys.path.insert(0, {str(REPO)!r})
import numpy as np
import gol_amd
from gol_amd.parallel.dist import init_process_group, make_transport, verify_row_bands, env_rank
rank, world, local = env_rank()
dist = init_process_group("gloo")
be = gol_amd.make_backend("cpu", 0)
sim = gol_amd.Simulation(gol_amd.LifeConfig(128, 64 * world, gen_limit=200, check_similarity=False),
                         transport=make_transport("torch", be, 0), backend=be)
sim.init_random(5, 0.5)
sim.advance(10)
ok = verify_row_bands(sim, 16, 32)["ok"]
def flip(s):  # wrong cells in the middle band of rank 1 tile, after the snapshot
    if rank == 1:
        t = s.tile()
        t[28:32, 58:62] ^= 1
        s.load_tile(t)
bad = verify_row_bands(sim, 16, 32, after_snapshot=flip)["ok"]
sys.stdout.write(f"RESULT {{ok}} {{bad}}" + chr(10))
sys.stdout.flush()
dist.destroy_process_group()
''')
    r = _torchrun(2, [str(script)], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("RESULT True False") == 2, r.stdout
