"""Host sanitizer tier: the runtime's host code - engine,
CPU backend, thread pool, in-process thread transport, text I/O - built
with AddressSanitizer + UBSan and with ThreadSanitizer, checked against the
serial oracle (csrc/tools/gol_selftest.cpp).  GPU code is not involved (GPU
sanitizers are not available for this target)."""
import os
import subprocess

import pytest

from gol_amd import native_build


@pytest.mark.parametrize("kind", ["address", "thread"])
def test_selftest_under_sanitizer(kind, tmp_path):
    exe = native_build.build_selftest(kind)
    env = dict(os.environ, TMPDIR=str(tmp_path), ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               TSAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "SELFTEST OK" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
