#!/usr/bin/env python3
"""Headline benchmark: whole-node cell-updates/s on a 32768^2 torus.

BASELINE.json metric: "cell-updates/sec (whole node), 32768^2 x 1000 gens;
scaling at 1/2/4/8 GPUs" - cell-updates/s = W * H * Generations / loop time,
exactly as the reference times its generation loop (src/game.c:175-199,
src/game_mpi.c:385-424, src/game_cuda.cu:219-279).

One *step* = one run of the reference's benchmark unit: GEN_LIMIT = 1000
generations of the full 32768^2 grid (--gens-per-step), B3/S23 on a torus
with the reference's termination checks on (per-generation change flags
fused into the kernel, polled every 256 generations and resolved exactly at
the end of the step) and every halo exchange the decomposition needs.  Each
step continues the same grid (a random 32768^2 soup never reaches a fixed
point within the run; if it did, the step would stop there exactly as the
reference does and `generations_timed` would say so).  `--steps K` times
exactly K such runs after `--warmup W` untimed ones, bracketed by a barrier +
device synchronisation on both sides; the slowest rank's time counts.
Strong scaling: the grid is fixed, N GPUs split it into 1 x N row strips,
one process per GPU, halos and flag reductions over RCCL/xGMI.

    python bench.py                                   # 1 GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

Data: synthetic - counter-based RNG random init at density 0.5 (the same
distribution as generate.sh's $((RANDOM % 2))), generated on the device.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "cell-updates/sec (whole node), 32768^2 x 1000 gens; scaling at 1/2/4/8 GPUs"
# no published numbers; best reference run measured there is
# game_mpi_collective/async.c, 4 ranks, 2048^2: ~8.9e8 cell-updates/s.
BASELINE_VALUE = 8.9e8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _claim_stdout() -> int:
    """Route fd 1 to stderr for the whole run and return a private duplicate
    of the real stdout.  The driver reads exactly one JSON line from rank 0's
    stdout, but RCCL prints a version banner ("RCCL version : ...") to stdout
    when a communicator is created (ours and torch.distributed's), and other
    native libraries may print too; only the result line goes to the
    duplicate."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    return real


def main() -> int:
    out_fd = _claim_stdout()
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed steps (one step = --gens-per-step generations)")
    ap.add_argument("--warmup", type=int, default=2, help="untimed steps before the timed ones")
    ap.add_argument("--gens-per-step", type=int, default=1000,
                    help="generations per step: GEN_LIMIT of the reference's benchmark run (src/game.c:6)")
    ap.add_argument("--prewarm", type=int, default=8192,
                    help="extra untimed generations before the warmup: the GPU clock needs ~10 ms of load to ramp "
                         "(100 warmup gens = 1.3 ms left the first timed run 6%% slow, profiles/sweep_warmup.jsonl)")
    ap.add_argument("--size", type=int, default=32768, help="grid side (cells)")
    ap.add_argument("--height", type=int, default=0, help="grid height if not square (experiments only)")
    ap.add_argument("--layout", default="bits", choices=["bits", "u8"])
    ap.add_argument("--engine", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--comm", default="rccl", choices=["rccl", "torch"])
    ap.add_argument("--decomp", default="auto")
    ap.add_argument("--tmax", type=int, default=0)
    ap.add_argument("--epoch", type=int, default=0)
    ap.add_argument("--poll", type=int, default=0)
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off", "edges"])
    ap.add_argument("--graphs", default="off", choices=["auto", "on", "off"])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--repeats", type=int, default=1, help="timed repetitions (best is reported)")
    ap.add_argument("--rehearse-rccl", action="store_true",
                    help="one GPU: run the multi-rank row-strip schedule (epoch depth, early-boundary overlap, "
                         "RCCL send/recv + all-reduce) against a 1-rank RCCL communicator that exchanges with "
                         "itself; use with --height H/N to rehearse one rank of an N-GPU run")
    a = ap.parse_args()

    import torch  # noqa: PLC0415

    from gol_amd import LifeConfig, Simulation, make_backend, native  # noqa: PLC0415
    from gol_amd.parallel.dist import allreduce_max_float, env_rank  # noqa: PLC0415

    rank, world, local = env_rank()
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    on_gpu = a.engine == "hip"
    if on_gpu:
        if not torch.cuda.is_available():
            raise SystemExit("bench.py: no GPU visible (use --engine cpu for a CPU dry run)")
        torch.cuda.set_device(local)
    backend = make_backend(a.engine, local)
    dist = None
    if world > 1:
        from gol_amd.parallel.dist import init_process_group, make_transport  # noqa: PLC0415

        dist = init_process_group("nccl" if on_gpu else "gloo")
        transport = make_transport(a.comm, backend, local)
    elif a.rehearse_rccl and on_gpu:
        C = native()
        transport = C.rccl_transport(C.rccl_unique_id(), 0, 1, local)
    else:
        transport = native().self_transport()

    S = a.size
    Hg = a.height or S
    gps = max(1, a.gens_per_step)
    total = a.prewarm + (a.warmup + a.steps * a.repeats) * gps
    cfg = LifeConfig(S, Hg, gen_limit=total, layout=a.layout, decomp=a.decomp, tmax=a.tmax, epoch=a.epoch,
                     poll_gens=a.poll, overlap=a.overlap, graphs=a.graphs, timing_barriers=False,
                     self_exchange=bool(a.rehearse_rccl and world == 1),
                     watchdog_s=300.0)  # a stuck rank or kernel fails the run instead of hanging it
    sim = Simulation(cfg, transport=transport, backend=backend)
    eng = sim.native_engine
    sim.init_random(a.seed, 0.5)

    def sync():
        if dist is not None:
            dist.barrier()
        if on_gpu:
            torch.cuda.synchronize()
        backend.synchronize()

    def step():
        """One reference benchmark run: gps generations with termination checks."""
        return eng.run_until(sim.generation + gps)

    if a.prewarm > 0:
        eng.run_until(sim.generation + a.prewarm)
    for _ in range(a.warmup):
        step()
    best = None
    for _ in range(a.repeats):
        sync()
        t0 = time.perf_counter()
        g0 = sim.generation
        rs = [step() for _ in range(a.steps)]
        sync()
        dt = time.perf_counter() - t0
        dt = allreduce_max_float(dt)
        executed = sim.generation - g0
        if best is None or dt < best[0]:
            best = (dt, executed, rs)
    dt, executed, rs = best
    gens = max(1, executed)
    value = float(S) * float(Hg) * gens / dt
    stops = sorted({r.stop_reason for r in rs})
    desc = sim.describe()
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": value,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3 / max(1, a.steps),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": value / BASELINE_VALUE,
            "dtype": "u1 bit-packed cells (exact boolean B3/S23; reference stores u8 chars)"
                     if a.layout == "bits" else "u8 byte-per-cell (exact)",
            "data": "synthetic: on-device counter-based RNG random grid, density 0.5 (generate.sh distribution)",
            "config": {
                "model": f"Game of Life B3/S23 torus {S}x{Hg}",
                "global_batch": 1,
                "seq_len": S * Hg,
                "parallelism": f"{desc['decomp']} row/col tiles, "
                               f"{'rccl' if world > 1 else 'rccl-self (rehearsal)' if a.rehearse_rccl else 'single'} halos",
                "grid": f"{S}x{Hg}",
                "layout": a.layout,
                "engine": backend.name(),
                "kernel": desc["kernel"],
                "tmax": desc["tmax"],
                "epoch": desc["epoch"],
                "gens_per_step": gps,
                "generations_timed": gens,
                "step_stop_reasons": stops,
                "prewarm_generations": a.prewarm,
                "warmup_generations": a.warmup * gps,
                "loop_ms_engine_per_step": sum(r.loop_ms for r in rs) / max(1, len(rs)),
                "exchanges_per_step": rs[-1].exchanges if rs else 0,
                "polls_per_step": rs[-1].polls if rs else 0,
                "kernel_launches_per_step": rs[-1].kernel_launches if rs else 0,
                "halo_bytes_per_step": rs[-1].halo_bytes if rs else 0,
                "overlapped_halo_exchange": bool(rs and rs[-1].overlapped),
                "graph_epochs": sum(r.graph_launches for r in rs),
                "baseline": "8.9e8 cell-updates/s (best reference run in BASELINE.md: MPI, 4 ranks, 2048^2, CPU)",
            },
        }
        os.write(out_fd, (json.dumps(rec) + "\n").encode())
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
