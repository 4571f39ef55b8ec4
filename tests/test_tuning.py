"""Runtime tuning (csrc/include/gol/tuning.hpp): one table of knobs, defaults
under GOL_* environment overrides under explicit settings (LifeConfig.tune,
``--tune key=value`` on bin/gol, gol_amd.cli and bench.py); the engine and
the backends read it once, at construction; describe() and bench.py's record
list the effective values.  The reference has no runtime tuning (its launch
geometry is compile-time, src/game_cuda.cu:12-14), so there is nothing to
pin against it: these tests pin the contract itself."""
import json
import os
import re
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from gol_amd import LifeConfig, Simulation, random_grid, reference_run
from gol_amd.models.life import make_tuning, parse_tune_args

REPO = Path(__file__).resolve().parents[1]


def test_table_defaults_and_classes(native):
    keys = native.tuning_keys()
    t = native.Tuning()
    assert t.changed() == {} and t.summary() == "defaults"
    assert len({k["key"] for k in keys}) == len(keys) and len({k["env"] for k in keys}) == len(keys)
    assert {k["class"] for k in keys} == {"tune", "diag", "fault", "emul"}
    for k in keys:
        assert k["env"].startswith("GOL_") and t.get(k["key"]) == k["default"] and t.source(k["key"]) == "default"
    # the measured-slower variants and their probes are gone
    cls = {k["key"]: k["class"] for k in keys}
    for gone in ("flow", "resident", "split", "short", "pipe", "skew", "wpl", "lds_add", "link_force", "pitch_pad",
                 "chain_acquire", "link_events"):
        assert gone not in cls, gone


def test_precedence_default_env_set(native, monkeypatch):
    monkeypatch.delenv("GOL_HOST_THREADS", raising=False)  # conftest's CPU-tier setting
    monkeypatch.setenv("GOL_GROUP", "4")
    monkeypatch.setenv("GOL_XLANE", "")  # empty: unset
    t = native.Tuning.from_env()
    assert t.get("group") == "4" and t.source("group") == "env"
    assert t.get("xlane") == "-1" and t.source("xlane") == "default"
    t.set("group", "2")
    assert t.get("group") == "2" and t.source("group") == "set"
    assert t.changed() == {"group": "2"}
    assert "group=2[set]" in t.summary()
    # make_tuning: environment first, then the dict / list / Tuning
    assert make_tuning({"group": 6}).get("group") == "6"
    assert make_tuning(["chain=0", "wrap=0"]).changed() == {"group": "4", "chain": "0", "wrap": "0"}
    assert make_tuning({"fold": True}).get("fold") == "1"
    c = make_tuning(t)
    c.set("group", "9")
    assert t.get("group") == "2"  # a copy


def test_bad_settings_fail_loudly(native, monkeypatch):
    t = native.Tuning()
    with pytest.raises(Exception, match="unknown tuning key 'gruop'"):
        t.set("gruop", "4")
    with pytest.raises(Exception, match="expected an integer"):
        t.set("group", "four")
    with pytest.raises(ValueError):
        parse_tune_args(["group"])
    with pytest.raises(Exception, match="unknown tuning key"):
        parse_tune_args(["nope=1"])
    monkeypatch.setenv("GOL_TARGET_WAVES", "lots")
    with pytest.raises(Exception, match="GOL_TARGET_WAVES"):
        native.Tuning.from_env()


def test_watchdog_accepts_fractional_seconds(native, monkeypatch):
    """GOL_WATCHDOG_S is a number of seconds (0.5 was accepted
    before the table was typed); a malformed value names its variable."""
    monkeypatch.setenv("GOL_WATCHDOG_S", "0.5")
    assert native.Tuning.from_env().get("watchdog_s") == "0.5"
    Simulation(LifeConfig(64, 32), engine="cpu")  # a default EngineConfig reads it
    monkeypatch.setenv("GOL_WATCHDOG_S", "soon")
    with pytest.raises(Exception, match="GOL_WATCHDOG_S.*expected a number"):
        native.Tuning.from_env()


def test_config_tuning_reaches_engine_and_backend(native):
    """LifeConfig.tune steers the backend the Simulation makes (cpu_ring: the
    CPU backend's row rings) and the engine (u8_via_bits), with no
    environment involved; describe() reports both."""
    W, H = 256, 96
    g = random_grid(W, H, 4)
    ref, rgens, _ = reference_run(g, 200)
    plain = Simulation(LifeConfig(W, H, gen_limit=200, layout="u8"), engine="cpu")
    tuned = Simulation(LifeConfig(W, H, gen_limit=200, layout="u8", tune={"cpu_ring": 1, "u8_via_bits": 1}),
                       engine="cpu")
    d0, d1 = plain.describe(), tuned.describe()
    assert not d0["row_ring"] and d0["u8_compute"] == "bytes"
    assert d1["row_ring"] and d1["u8_compute"] == "bits"
    assert d1["tuning_changed"]["cpu_ring"] == "1 (set)" and d1["tuning_changed"]["u8_via_bits"] == "1 (set)"
    assert d1["tuning"]["u8_via_bits"] == "1" and set(d1["tuning"]) == {
        k["key"] for k in native.tuning_keys() if k["class"] == "tune"}
    for s in (plain, tuned):
        s.load(g)
        assert s.run().generations == rgens
        assert np.array_equal(s.tile(), ref)


def test_an_explicit_backend_keeps_its_own_tuning(native):
    be = native.cpu_backend(2, tune=make_tuning({"cpu_ring": "1"}))
    assert be.tuning().get("cpu_ring") == "1"
    sim = Simulation(LifeConfig(128, 64, tune={"cpu_ring": "0"}), backend=be)
    assert sim.describe()["row_ring"]  # the backend decides what it can do


def test_knobs_are_read_in_one_place():
    """The framework reads its GOL_* knobs through Tuning::from_env only; the
    remaining environment reads are the build (arch, scheduler strategy),
    the module loader and the Python checkpoint writer's fault hook."""
    sites = []
    for p in list((REPO / "csrc").rglob("*.[ch]pp")) + list((REPO / "csrc").rglob("*.hip")):
        for i, ln in enumerate(p.read_text().splitlines()):
            if "getenv(" in ln:
                sites.append(f"{p.relative_to(REPO)}:{i + 1}")
    assert [s for s in sites if not s.startswith(("csrc/src/tuning.cpp", "csrc/tools/gol_selftest.cpp"))] == [], sites
    py = []
    for p in list((REPO / "gol_amd").rglob("*.py")) + [REPO / "bench.py"]:
        for i, ln in enumerate(p.read_text().splitlines()):
            if re.search(r"os\.environ(\.get)?\(?\[?\"GOL_", ln):
                py.append(f"{p.name}:{i + 1}")
    assert len(sites) + len(py) <= 15, (sites, py)


def test_gol_cli_tune(gol_bin, tmp_path):
    h = subprocess.run([str(gol_bin), "--tune", "help"], capture_output=True, text=True, timeout=60)
    assert h.returncode == 0 and "GOL_XLANE" in h.stdout and "cpu_ring" in h.stdout
    bad = subprocess.run([str(gol_bin), "64", "64", "--random", "1", "--engine", "cpu", "--tune", "nope=1"],
                         capture_output=True, text=True, timeout=60)
    assert bad.returncode != 0 and "unknown tuning key" in bad.stderr
    outs = []
    for extra in ([], ["--tune", "cpu_ring=1", "--tune", "cpu_drift=1"]):
        o = tmp_path / f"out{len(extra)}.txt"
        r = subprocess.run([str(gol_bin), "128", "64", "--random", "3", "--engine", "cpu", "--gens", "150",
                            "--output", str(o), *extra], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append((o.read_bytes(), r.stdout.split("Generations:")[-1].split()[0]))
    assert outs[0] == outs[1]
    # --metrics-json stays valid JSON whatever text a string-valued key holds
    # (trace paths with quotes or backslashes).
    m = tmp_path / "m.json"
    odd = 'x:/tmp/a"b\\c'
    r = subprocess.run([str(gol_bin), "64", "64", "--random", "1", "--engine", "cpu", "--gens", "5",
                        "--tune", f"wg_trace={odd}", "--metrics-json", str(m)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rec = json.loads(m.read_text())
    assert rec["tuning_changed"]["wg_trace"] == odd and odd in rec["tuning"]


def test_python_cli_tune_help():
    env = dict(os.environ, PYTHONPATH=str(REPO))
    r = subprocess.run([sys.executable, "-m", "gol_amd.cli", "--tune", "help"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=REPO)
    assert r.returncode == 0 and "GOL_ROW_RING" in r.stdout


def test_bench_records_tuning(native):
    env = dict(os.environ, PYTHONPATH=str(REPO), OMP_NUM_THREADS="1")
    env.pop("GOL_HOST_THREADS", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--engine", "cpu", "--size", "256", "--steps", "2",
                        "--warmup", "1", "--gens-per-step", "64", "--prewarm", "0", "--verify", "32",
                        "--tune", "cpu_ring=1", "--tune", "host_threads=2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    cfg = rec["config"]
    assert cfg["env_knobs"] == {}
    assert cfg["tuning_changed"] == {"cpu_ring": "1 (set)", "host_threads": "2 (set)"}
    assert cfg["tuning"]["row_ring"] == "1" and rec["verified"] is True


def test_tuning_doc_lists_every_key(native):
    """docs/TUNING.md is generated from the table; a key added without
    regenerating it fails here."""
    doc = (REPO / "docs" / "TUNING.md").read_text()
    for k in native.tuning_keys():
        assert f"| `{k['key']}` | `{k['env']}` |" in doc, k["key"]
