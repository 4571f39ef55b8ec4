"""T0: text I/O contract."""
import os

import numpy as np
import pytest

from gol_amd.ops.life_ops import random_grid
from gol_amd.utils import io


def test_roundtrip_and_size(tmp_path, native):
    g = random_grid(37, 21, 3)
    p = tmp_path / "g.txt"
    io.write_grid(str(p), g)
    assert os.path.getsize(p) == 21 * (37 + 1)  # H*(W+1) bytes
    txt = p.read_text()
    assert txt == io.format_text(g)
    assert (io.read_grid(str(p), 37, 21) == g).all()
    assert (io.parse_text(txt, 37, 21) == g).all()


def test_subarray_reads_match_full(tmp_path, native):
    W, H = 100, 60
    p = tmp_path / "g.txt"
    io.generate(str(p), W, H, seed=9)
    full = io.read_grid(str(p), W, H)
    for rows, cols in [((0, H), (0, W)), ((7, 31), (5, 77)), ((59, 60), (99, 100)), ((0, 1), (0, 1))]:
        t = io.read_tile(str(p), W, H, rows, cols)
        assert (t == full[rows[0]:rows[1], cols[0]:cols[1]]).all()


def test_generator_matches_device_rng(tmp_path, native):
    p = tmp_path / "g.txt"
    io.generate(str(p), 64, 16, seed=42, density=0.3)
    assert (io.read_grid(str(p), 64, 16) == random_grid(64, 16, 42, 0.3)).all()
    d = random_grid(512, 512, 1, 0.3).mean()
    assert 0.27 < d < 0.33


def test_short_file_is_an_error_not_a_hang(tmp_path, native):
    # The reference's fgetc loop spins forever on a short file (quirk Q8).
    p = tmp_path / "short.txt"
    p.write_text("0101\n0101\n")
    with pytest.raises(RuntimeError, match="cells"):
        io.read_grid(str(p), 4, 3)


def test_fgetc_semantics_and_crlf(tmp_path, native):
    # Non-exact layouts are read like the reference's sequential parser: the
    # first W*H non-newline bytes in order, '1' alive, anything else dead.
    p = tmp_path / "odd.txt"
    p.write_text("0110\r\n1x01\r\n0011\r\n")
    g = io.read_grid(str(p), 4, 3)
    assert g.tolist() == [[0, 1, 1, 0], [1, 0, 0, 1], [0, 0, 1, 1]]
    q = tmp_path / "flat.txt"
    q.write_text("011010010011")  # one line holding all 12 cells
    assert (io.read_grid(str(q), 4, 3) == g).all()


@pytest.mark.parametrize("body", [
    "1" * 10 + "0" * 15 + "\n\n",          # 25 cells + 2 newlines = 27 B = exact size of 8x3
    "10110011\n0110\n1001\n01100110\n",    # exact size, misplaced line breaks
    "10110011\n01101001\n01100110",        # exact size - 1, no trailing newline
    "10110011\n01101001\n01100110\n",      # exact layout
])
def test_column_tiles_take_the_same_path_as_the_full_read(tmp_path, native, body):
    """Every column rank of a decomposed read sees the same layout decision,
    so the tiles assemble to the full-width read."""
    p = tmp_path / "g.txt"
    p.write_bytes(body.encode())
    W, H = 8, 3
    full = io.read_grid(str(p), W, H)
    for cols in [(0, 4), (4, 8), (0, 3), (3, 8), (2, 6)]:
        for rows in [(0, H), (1, 3), (0, 1)]:
            t = io.read_tile(str(p), W, H, rows, cols)
            assert (t == full[rows[0]:rows[1], cols[0]:cols[1]]).all(), (cols, rows)


def test_line_break_inside_an_exact_row_reads_fixed_offsets(tmp_path, native):
    # Exact size and every row's '\n' in place, but a '\r' among the cells:
    # the reference's serial fgetc loop would come up one cell short and spin
    # (quirk Q8); its MPI-IO builds read fixed offsets, which every tile does
    # here too - the stray byte is a dead cell and all ranks agree.
    p = tmp_path / "g.txt"
    p.write_bytes(b"0110\n1\r01\n0011\n")
    full = io.read_grid(str(p), 4, 3)
    assert full.tolist() == [[0, 1, 1, 0], [1, 0, 0, 1], [0, 0, 1, 1]]
    for cols in [(0, 2), (2, 4), (1, 3)]:
        assert (io.read_tile(str(p), 4, 3, (0, 3), cols) == full[:, cols[0]:cols[1]]).all()


def test_tile_writes_assemble_the_file(tmp_path, native):
    W, H = 70, 45
    g = random_grid(W, H, 5)
    p = tmp_path / "out.txt"
    io.create_text_file(str(p), W, H)
    # 2x3 decomposition, written in a scrambled order like independent ranks
    rows = [(0, 20), (20, 45)]
    cols = [(0, 30), (30, 50), (50, 70)]
    for (r0, r1) in rows[::-1]:
        for (c0, c1) in cols[::-1]:
            io.write_tile(str(p), W, H, r0, c0, g[r0:r1, c0:c1])
    assert p.read_text() == io.format_text(g)


def test_ascii_and_binary_inputs_equivalent(native):
    g = random_grid(40, 10, 2)
    ascii_grid = (g + ord("0")).astype(np.uint8)
    from gol_amd import reference_run

    a = reference_run(g, 50)[0]
    b = reference_run(ascii_grid, 50)[0]
    assert (a == b).all()


_FSIZE_CHILD = r"""
import resource, sys
sys.path.insert(0, {repo!r})
from gol_amd.utils import io
resource.setrlimit(resource.RLIMIT_FSIZE, (1 << 20, 1 << 20))
for what, call in [("create", lambda: io.create_text_file({p1!r}, 2048, 2048)),
                   ("generate", lambda: io.generate({p2!r}, 2048, 2048, seed=1))]:
    try:
        call()
    except Exception as e:
        print(what, "raised", "RLIMIT_FSIZE" in str(e))
    else:
        print(what, "returned")
"""


def test_output_beyond_file_size_limit_raises_not_signals(tmp_path, native, repo):
    """outputs are written through shared mappings; a file the
    process may not grow must fail with an error (SIGXFSZ / SIGBUS would kill
    a Python caller without a message)."""
    import subprocess
    import sys

    code = _FSIZE_CHILD.format(repo=str(repo), p1=str(tmp_path / "a.txt"), p2=str(tmp_path / "b.txt"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.split("\n")[:2] == ["create raised True", "generate raised True"], r.stdout


def test_mapped_writes_reserve_their_blocks(tmp_path, native):
    """A tile written through a mapping is backed by disk blocks first
    (fallocate), so a full file system reports an error instead of SIGBUS."""
    W, H = 4096, 64
    p = tmp_path / "s.txt"
    io.create_text_file(str(p), W, H)  # sized by ftruncate: sparse
    g = random_grid(W, H, 5)
    io.write_tile(str(p), W, H, 0, 0, g)
    st = os.stat(p)
    if st.st_blocks * 512 < st.st_size:
        pytest.skip("this file system does not reserve ranges (fallocate unsupported): the pwrite path ran")
    assert (io.read_grid(str(p), W, H) == g).all()
