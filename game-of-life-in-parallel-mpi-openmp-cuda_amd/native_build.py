"""Native build driver: compiles the C++ runtime and the CDNA4 HIP kernels.

Everything is built in-tree so the artefacts travel with the repository:

* ``gol_amd/_gol.so`` - pybind11 module (engine, backends, transports, I/O)
* ``bin/gol``         - CLI with the reference's ``./a.out W H file`` contract
* ``bin/gol_gen``     - text-grid generator (replaces generate.sh)

Reference build: one compiler call per program, ``-std=c99 -Wall -O3``, nvcc
with no flags at all (Makefile:7-31).  Here: host C++17 with g++, HIP sources
with ``hipcc --offload-arch=gfx950`` (CDNA4 only, no other targets), parallel
incremental compilation, link against HIP + RCCL.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BIN = REPO / "bin"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("GOL_OFFLOAD_ARCH", "gfx950")
BUILD = REPO / "build" / "obj"

HOST_SRCS = ["src/decomp.cpp", "src/parallel.cpp", "src/backend_cpu.cpp", "src/transport.cpp",
             "src/engine.cpp", "src/io.cpp", "src/cpu_ref.cpp", "src/checkpoint.cpp", "src/tuning.cpp",
             "src/numa.cpp"]
# One translation unit per compiled kernel variant (layout x cross-lane
# window), so the build compiles them in parallel.  The variants measured
# slower than these (resident epochs, persistent dataflow launches, short
# segments, split / skewed schedules, ds_bpermute and carry-chain windows, two
# words per lane, the byte layout's T = 48 pipelined pass) were removed in round 6; their code is in git history
# (docs/HISTORY.md) and their numbers in docs/HISTORY.md / PERFORMANCE.md.
LIFE_VARIANTS = ["bits_w1_dpp", "bits_w1_add", "u8_w1_dpp", "u8_w1_add",
                 *[f"u8_w1_dpp_t{t}" for t in (24, 32)]]  # deep byte passes
HIP_SRCS = ["src/backend_hip.hip", "src/transport_rccl.hip", "kernels/life_block.hip",
            *[f"kernels/life_block_{v}.hip" for v in LIFE_VARIANTS], "kernels/life_step_lds.hip",
            "kernels/tile_ops.hip"]
BIND_SRCS = ["src/bindings.cpp"]
CLI_MAIN = "tools/gol_main.cpp"
GEN_MAIN = "tools/gol_gen.cpp"
# Stand-alone HIP tools (no engine code): the row-ring VMM stress test.
TOOLS = ["tools/ring_stress.hip"]

MODULE = PKG_DIR / "_gol.so"


def _hipcc() -> str:
    for c in (ROCM / "bin" / "hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return str(c)
    raise RuntimeError("hipcc not found: the native build needs ROCm (hipcc --offload-arch=gfx950)")


def _headers_mtime() -> float:
    m = 0.0
    for p in list(CSRC.rglob("*.hpp")) + list(CSRC.rglob("*.h")):
        m = max(m, p.stat().st_mtime)
    return m


def _compile_cmd(src: Path, obj: Path) -> list[str]:
    inc = [f"-I{CSRC / 'include'}", f"-I{CSRC}"]
    if src.suffix == ".hip":
        extra = []
        if src.name.startswith("life_block_"):
            # Scheduler for the temporal-blocking kernels: max-ILP interleaves the
            # independent generation levels.  Measured on MI355X it is on par
            # with the default strategy (the kernel is VALU-throughput bound);
            # GOL_SCHED_STRATEGY selects another one for experiments.
            extra = ["-mllvm", f"-amdgpu-sched-strategy={os.environ.get('GOL_SCHED_STRATEGY', 'max-ilp')}"]
        return [_hipcc(), "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                "-Wall", "-Wno-unused-result", "-munsafe-fp-atomics", *inc, f"-I{ROCM / 'include'}",
                *extra, "-MMD", "-MF", str(obj.with_suffix(".d")), "-c", str(src), "-o", str(obj)]
    extra = []
    if src.name == "bindings.cpp":
        import pybind11  # noqa: PLC0415
        extra = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
                 "-fvisibility=hidden"]
    return ["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-pthread", *inc, *extra,
            "-MMD", "-MF", str(obj.with_suffix(".d")), "-c", str(src), "-o", str(obj)]


def _deps(obj: Path) -> list[Path] | None:
    """Headers the object was built from (the compiler's -MMD file), or None."""
    d = obj.with_suffix(".d")
    if not d.exists():
        return None
    text = d.read_text().replace("\\\n", " ")
    _, _, rest = text.partition(":")
    return [Path(t) for t in rest.split() if t.endswith((".hpp", ".h", ".hip", ".inc"))]


def _needs(obj: Path, src: Path, hdr_mtime: float) -> bool:
    if not obj.exists():
        return True
    om = obj.stat().st_mtime
    if om < src.stat().st_mtime:
        return True
    deps = _deps(obj)
    if deps is None:  # no dependency record: any header change rebuilds
        return om < hdr_mtime
    return any((not p.exists()) or om < p.stat().st_mtime for p in deps if str(p).startswith(str(CSRC)))


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> dict[str, Path]:
    """Compile (incrementally) and link the module and the CLI tools."""
    BUILD.mkdir(parents=True, exist_ok=True)
    BIN.mkdir(parents=True, exist_ok=True)
    hdr = _headers_mtime()
    srcs = HOST_SRCS + HIP_SRCS + BIND_SRCS + [CLI_MAIN, GEN_MAIN] + TOOLS
    objs = {s: BUILD / (s.replace("/", "_") + ".o") for s in srcs}
    todo = [s for s in srcs if force or _needs(objs[s], CSRC / s, hdr)]
    # Longest compiles first (deep byte passes, then the kernel variants), so
    # the pool does not end on one long translation unit.
    todo.sort(key=lambda s: 0 if any(f"_t{t}" in s for t in (24, 32, 48, 64)) else
              1 if "life_block_" in s else 2)
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_run, _compile_cmd(CSRC / s, objs[s]), verbose) for s in todo]
        for f in futs:
            f.result()
    core = [str(objs[s]) for s in HOST_SRCS + HIP_SRCS]
    rocm_libs = [f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM / 'lib'}",
                 "-pthread"]
    outs = {
        "module": MODULE,
        "gol": BIN / "gol",
        "gol_gen": BIN / "gol_gen",
    }
    relink = bool(todo) or force or any(not p.exists() for p in outs.values())
    if relink:
        _run([_hipcc(), "-shared", "-fPIC", *core, str(objs[BIND_SRCS[0]]), "-o", str(MODULE), *rocm_libs],
             verbose)
        _run([_hipcc(), *core, str(objs[CLI_MAIN]), "-o", str(outs["gol"]), *rocm_libs], verbose)
        _run([_hipcc(), *core, str(objs[GEN_MAIN]), "-o", str(outs["gol_gen"]), *rocm_libs], verbose)
    for t in TOOLS:
        exe = BIN / Path(t).stem
        if relink or not exe.exists() or exe.stat().st_mtime < objs[t].stat().st_mtime:
            _run([_hipcc(), str(objs[t]), "-o", str(exe), f"-L{ROCM / 'lib'}", "-lamdhip64",
                  f"-Wl,-rpath,{ROCM / 'lib'}"], verbose)
    LAST_BUILD.clear()
    LAST_BUILD.update(compiled=len(todo), up_to_date=len(srcs) - len(todo), relinked=relink)
    return outs


# What the last build() in this process did (compiled vs up-to-date objects).
LAST_BUILD: dict = {}


def gfx950_code_objects(path: Path = MODULE) -> int:
    """Number of gfx950 device code objects bundled in a built library (the
    offload bundle entries name their target)."""
    return path.read_bytes().count(b"amdgcn-amd-amdhsa--" + ARCH.encode())


SELFTEST_MAIN = "tools/gol_selftest.cpp"
SANITIZERS = {
    "address": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
    "thread": ["-fsanitize=thread"],
    "none": [],
}


def build_selftest(kind: str = "address", verbose: bool = False, jobs: int | None = None) -> Path:
    """Host-only self test (engine + CPU backend + thread transport + text
    I/O vs the serial oracle) built with a sanitizer: bin/gol_selftest_<kind>.
    No HIP code is involved, so ASan/UBSan/TSan apply to the whole binary."""
    flags = SANITIZERS[kind]
    obj_dir = REPO / "build" / f"san_{kind}"
    obj_dir.mkdir(parents=True, exist_ok=True)
    BIN.mkdir(parents=True, exist_ok=True)
    inc = [f"-I{CSRC / 'include'}", f"-I{CSRC}"]
    srcs = HOST_SRCS + [SELFTEST_MAIN]
    hdr = _headers_mtime()
    objs = {s: obj_dir / (s.replace("/", "_") + ".o") for s in srcs}
    cmds = [["g++", "-O1", "-g", "-std=c++17", "-pthread", *flags, *inc, "-c", str(CSRC / s), "-o", str(objs[s])]
            for s in srcs if _needs(objs[s], CSRC / s, hdr)]
    with cf.ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 4)) as ex:
        for f in [ex.submit(_run, c, verbose) for c in cmds]:
            f.result()
    out = BIN / f"gol_selftest_{kind}"
    if cmds or not out.exists():
        _run(["g++", *flags, "-pthread", *[str(objs[s]) for s in srcs], "-o", str(out)], verbose)
    return out


def is_built() -> bool:
    if not MODULE.exists():
        return False
    hdr = _headers_mtime()
    newest = max([(CSRC / s).stat().st_mtime for s in HOST_SRCS + HIP_SRCS + BIND_SRCS] + [hdr])
    return MODULE.stat().st_mtime >= newest


if __name__ == "__main__":
    if "--selftest" in sys.argv:
        kind = sys.argv[sys.argv.index("--selftest") + 1]
        print(build_selftest(kind, verbose="-v" in sys.argv))
        sys.exit(0)
    out = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    for k, v in out.items():
        print(f"{k}: {v}")
