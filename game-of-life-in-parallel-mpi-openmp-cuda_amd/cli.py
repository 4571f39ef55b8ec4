"""Python front end: ``python -m gol_amd W H input_file [options]``.

Same positional contract as the reference (``./a.out <width> <height>
<input_file>``, README.md:50-57) and the native ``bin/gol``; additionally
runs under ``torchrun`` with one process per GPU (the equivalent of
``mpiexec -n P ./a.out``, src/game_mpi.c:2), every rank reading and writing
its own subarray of the text file.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m gol_amd 32768 32768 in.txt --style mpi
"""
from __future__ import annotations

import argparse
import os
import sys
import time

from .models.life import LifeConfig, Simulation, make_backend, parse_tune_args, reference_run
from .utils.metrics import stdout_lines, write_json


def parse_args(argv=None):
    p = argparse.ArgumentParser(prog="gol_amd", description=__doc__.split("\n\n")[0])
    p.add_argument("width", nargs="?", type=int, default=0)
    p.add_argument("height", nargs="?", type=int, default=0)
    p.add_argument("input_file", nargs="?", default=None)
    p.add_argument("--engine", default="auto", choices=["auto", "hip", "cpu", "ref"])
    p.add_argument("--layout", default="auto", choices=["auto", "bits", "u8"])
    p.add_argument("--u8-compute", default="auto", choices=["auto", "bits", "bytes"],
                   help="byte layout: epochs on bit words packed once per epoch (auto: on the GPU) or on the bytes")
    p.add_argument("--gens", type=int, default=1000, help="GEN_LIMIT")
    p.add_argument("--sim-freq", type=int, default=None, help="SIMILARITY_FREQUENCY (default 3)")
    p.add_argument("--no-similarity", action="store_true")
    p.add_argument("--random", default=None, help="SEED[:DENSITY] random init instead of a file")
    p.add_argument("--output", default=None,
                   help="output path or 'none' (default: the reference build's name for --style)")
    p.add_argument("--decomp", default="auto")
    p.add_argument("--comm", default="auto", choices=["auto", "rccl", "torch"])
    p.add_argument("--tmax", type=int, default=0)
    p.add_argument("--epoch", "--halo-depth", dest="epoch", type=int, default=0,
                   help="generations per halo exchange (deep halo depth)")
    p.add_argument("--poll", "--poll-every", dest="poll", type=int, default=0,
                   help="generations between termination polls")
    p.add_argument("--overlap", default="auto", choices=["auto", "on", "off", "trigger"],
                   help="trigger (= on) = an epoch's boundary rows sent once the groups writing them are done; "
                        "off = no overlap; auto = time plain against trigger epochs on the ranks and keep the "
                        "faster (row strips only)")
    p.add_argument("--graphs", default="off", choices=["auto", "on", "off"],
                   help="replay full epochs as captured HIP graphs")
    p.add_argument("--threads", type=int, default=0)
    p.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                   help="runtime tuning (repeatable; --tune help lists the keys, their GOL_* overrides and defaults)")
    p.add_argument("--style", default="serial", choices=["serial", "mpi", "async", "collective", "openmp", "cuda"])
    p.add_argument("--metrics-json", default=None,
                   help="write run metrics as JSON (per-phase device times with --phase-timing)")
    p.add_argument("--phase-timing", action="store_true",
                   help="time kernels / halos / fills / reductions (adds event pairs inside the timed loop)")
    p.add_argument("--show", action="store_true",
                   help="print the final grid with VT100 escapes (src/game.c:42-58)")
    p.add_argument("--checkpoint-every", type=int, default=0)
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--resume", default=None, help="checkpoint directory to resume from")
    a = p.parse_args(argv)
    a.sim_freq_given = a.sim_freq is not None
    if a.sim_freq is None:
        a.sim_freq = 3
    if a.output is None:  # src/game.c:27, src/game_mpi.c:29, ... src/game_cuda.cu:37
        a.output = f"./{'game' if a.style == 'serial' else a.style}_output.out"
    if a.width <= 0:
        a.width = 30
    if a.height <= 0:
        a.height = 30
    return a


def print_tuning_keys() -> None:
    from ._native import native  # noqa: PLC0415

    for k in native().tuning_keys():
        print(f"{k['key']:<22} {k['class']:<13} {k['env']:<27} default {k['default'] or repr(''):<6} {k['doc']}")


def main(argv=None) -> int:
    a = parse_args(argv)
    if "help" in a.tune:
        print_tuning_keys()
        return 0
    if a.input_file is None and a.random is None and a.resume is None:
        print("Finished")
        return 0
    seed, density = 1, 0.5
    if a.random is not None:
        s, _, d = a.random.partition(":")
        seed, density = int(s), float(d) if d else 0.5

    if a.engine == "ref":
        import numpy as np  # noqa: PLC0415

        from .ops.life_ops import random_grid  # noqa: PLC0415
        from .utils.io import read_grid, write_grid  # noqa: PLC0415

        t0 = time.perf_counter()
        grid = random_grid(a.width, a.height, seed, density) if a.random else read_grid(a.input_file, a.width, a.height)
        read_ms = (time.perf_counter() - t0) * 1e3
        out, gens, ms = reference_run(np.asarray(grid), a.gens, not a.no_similarity, a.sim_freq, max(1, a.threads))
        t1 = time.perf_counter()
        if a.output != "none":
            write_grid(a.output, out)
        sys.stdout.write(stdout_lines(a.style, gens, ms, read_ms, (time.perf_counter() - t1) * 1e3))
        if a.show:
            from .utils.io import show_text  # noqa: PLC0415

            sys.stdout.write(show_text(out))
            sys.stdout.flush()
        return 0

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    tune = parse_tune_args(a.tune)
    backend = make_backend(a.engine, local, a.threads, tune)
    if world > 1:
        from .parallel.dist import init_process_group, make_transport  # noqa: PLC0415

        init_process_group("nccl" if backend.is_device() else "gloo",
                           device=int(backend.device()) if backend.is_device() else None)
        transport = make_transport(a.comm, backend, local, tune=tune)
    else:
        from ._native import native  # noqa: PLC0415

        transport = native().self_transport()

    cfg = LifeConfig(a.width, a.height, gen_limit=a.gens, check_similarity=not a.no_similarity,
                     sim_freq=a.sim_freq, layout=a.layout, decomp=a.decomp, tmax=a.tmax,
                     epoch=a.epoch, poll_gens=a.poll, overlap=a.overlap, graphs=a.graphs,
                     u8_compute=a.u8_compute, tune=tune)
    src = a.input_file
    if a.resume:
        from .utils.checkpoint import load_checkpoint  # noqa: PLC0415

        cfg, grid_path = load_checkpoint(a.resume, layout=a.layout, decomp=a.decomp, tmax=a.tmax,
                                         epoch=a.epoch, poll_gens=a.poll, gen_limit=a.gens)
        if a.sim_freq_given and not a.no_similarity and a.sim_freq != cfg.sim_freq:
            raise SystemExit(f"--resume: checkpoint was taken with --sim-freq {cfg.sim_freq}; resuming with "
                             f"--sim-freq {a.sim_freq} would shift the similarity checks")
        src = str(grid_path)
    sim = Simulation(cfg, transport=transport, backend=backend)
    # Opt-in only: the event pairs would sit inside the loop that loop_ms and
    # the reference-style timing line report.
    sim.phase_timing = bool(a.phase_timing)
    t0 = time.perf_counter()
    if a.random is not None and not a.resume:
        sim.init_random(seed, density)
    else:
        sim.load_text(src)
    transport.barrier()
    read_ms = (time.perf_counter() - t0) * 1e3

    if a.checkpoint_every > 0:
        from .utils.checkpoint import run_with_checkpoints  # noqa: PLC0415

        rep = run_with_checkpoints(sim, a.checkpoint_every, a.checkpoint_dir, rank == 0, transport.barrier)
    else:
        rep = sim.run()

    write_ms = 0.0
    tiles = None
    if a.show:  # every rank's tile, gathered on rank 0 (the viewer prints the whole grid)
        from .parallel.dist import gather_grid  # noqa: PLC0415

        tiles = gather_grid(sim) if world > 1 else sim.tile()
    if a.output != "none":
        t1 = time.perf_counter()
        if rank == 0:
            from .utils.io import create_text_file  # noqa: PLC0415

            create_text_file(a.output, a.width, a.height)
        transport.barrier()
        sim.write_text(a.output, create=False)
        transport.barrier()
        write_ms = (time.perf_counter() - t1) * 1e3
    if rank == 0:
        sys.stdout.write(stdout_lines(a.style, rep.generations, rep.loop_ms, read_ms, write_ms, world))
        sys.stdout.flush()
        rec = rep.as_dict()
        rec.update(sim.describe())
        rec.update({"read_ms": read_ms, "write_ms": write_ms, "width": a.width, "height": a.height})
        write_json(a.metrics_json, rec)
        if tiles is not None:
            from .utils.io import show_text  # noqa: PLC0415

            sys.stdout.write(show_text(tiles))
            sys.stdout.flush()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
