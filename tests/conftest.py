"""Test configuration.

Markers: ``gpu`` - needs a real MI355X (run on the GPU box with ``-m gpu``);
everything else runs on the CPU (``-m "not gpu"``), including the
multi-process ``gloo`` tests.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X, gfx950)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_terminal_summary(terminalreporter):
    """GPU sessions: how many HIP errors the native release paths ignored
    (destructors, frees; reported one by one on the tests' stderr)."""
    mod = next((m for n, m in sys.modules.items() if n.endswith("._gol") and hasattr(m, "hip_release_errors")), None)
    if mod is not None and mod.hip_available():
        terminalreporter.write_line(f"gol: HIP errors ignored by native release paths: {mod.hip_release_errors()}")


@pytest.fixture(scope="session")
def native():
    import gol_amd  # noqa: PLC0415

    return gol_amd.native()


@pytest.fixture(scope="session")
def gpu(native):
    if not native.hip_available():
        pytest.skip("no HIP device")
    return native


@pytest.fixture
def tune() -> dict:
    """Runtime tuning a test passes through LifeConfig.tune and the backends
    it makes (csrc/include/gol/tuning.hpp); test modules override it with
    their own defaults."""
    return {}


@pytest.fixture(scope="session")
def repo() -> Path:
    return REPO


@pytest.fixture(scope="session")
def gol_bin(native) -> Path:
    return REPO / "bin" / "gol"


@pytest.fixture(scope="session")
def reference_serial(tmp_path_factory):
    """The reference's serial src/game.c compiled in a scratch dir (never
    vendored); skipped when the read-only reference mount is absent."""
    src = Path("/root/reference/src/game.c")
    cc = shutil.which("gcc")
    if not src.exists() or cc is None:
        pytest.skip("reference source or gcc unavailable")
    d = tmp_path_factory.mktemp("refbuild")
    exe = d / "game_serial"
    subprocess.run([cc, "-std=c99", "-O3", str(src), "-o", str(exe)], check=True, capture_output=True)
    return exe


def run_reference_serial(exe: Path, workdir: Path, W: int, H: int, grid_path: Path):
    r = subprocess.run([str(exe), str(W), str(H), str(grid_path)], cwd=workdir, capture_output=True,
                       text=True, timeout=300, check=True)
    return r.stdout, (workdir / "game_output.out").read_bytes()


def generations_line(stdout: str) -> str:
    return next(line for line in stdout.splitlines() if line.startswith("Generations:"))


os.environ.setdefault("GOL_HOST_THREADS", "4")
