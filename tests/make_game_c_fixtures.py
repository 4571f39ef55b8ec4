#!/usr/bin/env python3
"""Regenerate tests/fixtures/game_c/: outputs of the reference's serial
src/game.c (compiled here from the read-only mount, never vendored) on the
GRIDS inputs of test_golden_reference.py, so that the GPU tier can compare
against them on a box without the reference mount.

    python tests/make_game_c_fixtures.py
"""
import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

from gol_amd.utils import io  # noqa: E402
from test_golden_reference import GRIDS  # noqa: E402


def main() -> int:
    src = Path("/root/reference/src/game.c")
    out_dir = HERE / "fixtures" / "game_c"
    out_dir.mkdir(parents=True, exist_ok=True)
    index = {}
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        exe = d / "game_serial"
        subprocess.run([shutil.which("gcc"), "-std=c99", "-O3", str(src), "-o", str(exe)], check=True)
        for N, seed, density in GRIDS:
            key = f"{N}_{seed}_{density}"
            f = d / f"{key}.txt"
            io.generate(str(f), N, N, seed=seed, density=density)
            r = subprocess.run([str(exe), str(N), str(N), str(f)], cwd=d, capture_output=True, text=True,
                               check=True)
            gens = next(ln for ln in r.stdout.splitlines() if ln.startswith("Generations:"))
            data = (d / "game_output.out").read_bytes()
            with gzip.GzipFile(out_dir / f"{key}.out.gz", "wb", mtime=0) as g:
                g.write(data)
            index[key] = gens
    (out_dir / "generations.json").write_text(json.dumps(index, indent=1) + "\n")
    print(f"wrote {len(index)} fixtures to {out_dir}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
