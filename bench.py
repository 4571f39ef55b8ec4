#!/usr/bin/env python3
"""Headline benchmark: whole-node cell-updates/s on a 32768^2 torus.

BASELINE.json metric: "cell-updates/sec (whole node), 32768^2 x 1000 gens;
scaling at 1/2/4/8 GPUs" - cell-updates/s = W * H * Generations / loop time,
exactly as the reference times its generation loop (src/game.c:175-199,
src/game_mpi.c:385-424, src/game_cuda.cu:219-279).

One *step* = one run of the reference's benchmark unit: GEN_LIMIT = 1000
generations of the full 32768^2 grid (--gens-per-step), B3/S23 on a torus
with the reference's termination checks on (per-generation change flags
fused into the kernel, polled every 256-1024 generations and resolved exactly at
the end of the step) and every halo exchange the decomposition needs.  Each
step continues the same grid (a random 32768^2 soup never reaches a fixed
point within the run; if it did, the step would stop there exactly as the
reference does and `generations_timed` would say so).  `--steps K` times
exactly K such runs after `--warmup W` untimed ones, bracketed by a barrier +
device synchronisation on both sides; the slowest rank's time counts.
Strong scaling: the grid is fixed, N GPUs split it into 1 x N row strips,
one process per GPU, halos and flag reductions over RCCL/xGMI.

    python bench.py                                   # 1 GPU
    python bench.py --gpus 8                          # launches 8 rank processes itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

`--gpus N` is the reference's `mpiexec -n P` (README.md:56, src/game_mpi.c:2):
without a launcher environment (no WORLD_SIZE) bench.py starts N rank
processes through torch.distributed.run before it touches torch or the GPU,
relays rank 0's JSON line and exits with the launcher's status.  Under a
launcher, WORLD_SIZE must equal --gpus (else it exits non-zero).  Each rank
needs a GPU of its own; --share-gpus lets ranks share devices (RCCL then runs
them as separate "nodes" over its socket transport: a correctness rehearsal
of the multi-rank path on a one-GPU box, not a performance number).

After the timed steps (outside the timed region) the same engine runs one
more step with per-phase device timing (kernels / halos / fills / flag
reductions, --no-phase-step to skip), and then --verify G generations
that are checked bit for bit against an fp32 PyTorch oracle (rolled-copy
neighbour sums, ops/life_ops.py life_step_torch_roll) and the
byte-per-cell layout, started from the engine's state at that point:
`verified` in the JSON line says whether the credited schedule is exact.

Data: synthetic - counter-based RNG random init at density 0.5 (the same
distribution as generate.sh's $((RANDOM % 2))), generated on the device.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "cell-updates/sec (whole node), 32768^2 x 1000 gens; scaling at 1/2/4/8 GPUs"
HEADLINE = (32768, 32768, 1000)  # BASELINE.json's grid and GEN_LIMIT
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



def _launch_ranks(ngpus: int, argv: list[str], out_fd: int) -> int:
    """`mpiexec -n N` for bench.py: N rank processes on this node, one per
    GPU, through torch.distributed.run.  Nothing here touches torch or the
    GPU; rank 0's JSON line is relayed to stdout, everything else to stderr."""
    # --standalone: the launcher's rendezvous store binds 127.0.0.1:0 itself
    # (a port probed free and then bound by the launcher could be taken in
    # between: EADDRINUSE seen once on a busy box).
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
           f"--nproc-per-node={ngpus}", os.path.abspath(__file__), *argv]
    log(f"bench.py: launching {ngpus} rank processes: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE)
    assert proc.stdout is not None
    lines = 0
    for raw in proc.stdout:
        if raw.lstrip().startswith(b"{") and b'"metric"' in raw:
            os.write(out_fd, raw)
            lines += 1
        else:
            sys.stderr.buffer.write(raw)
            sys.stderr.flush()
    rc = proc.wait()
    if rc == 0 and lines != 1:
        log(f"bench.py: the rank processes printed {lines} result lines, expected 1")
        return 1
    return rc


def metric_label(S: int, Hg: int, gps: int, rehearsal: str | None = None) -> tuple[str, bool, int | None]:
    """(metric, headline, config_id) of a run.  Only the BASELINE.json grid and
    generation count carry the headline metric string; any other grid names
    itself.  config_id is the BASELINE.json config the grid belongs to (1-5:
    256^2 CPU plumbing, 8192^2 byte tile, 32768^2 node, 65536^2 bits,
    1048576^2 bytes), None for an experiment's grid.  A rehearsal (ranks
    sharing GPUs, or one rank exchanging with itself through RCCL) is never a
    headline or a BASELINE config, whatever its grid: its metric names it,
    e.g. "(rehearsal: 8 ranks on 1 GPU)"."""
    grid = f"{S}^2" if S == Hg else f"{S}x{Hg}"
    if rehearsal:
        return f"cell-updates/sec, {grid} x {gps} gens (rehearsal: {rehearsal})", False, None
    headline = (S, Hg, gps) == HEADLINE
    metric = METRIC if headline else f"cell-updates/sec (whole node), {grid} x {gps} gens"
    ids = {256: 1, 8192: 2, 32768: 3, 65536: 4, 1048576: 5}
    return metric, headline, (ids.get(S) if S == Hg else None)


def rehearsal_label(world: int, shared: bool, self_rccl: bool, infos: list[dict]) -> str | None:
    """What a rehearsal ran on, or None for a real run: ranks that share GPUs
    (--share-gpus), or the one-rank RCCL self-exchange (--rehearse-rccl)."""
    gpus = len({(i.get("host"), i.get("uuid") or i.get("pci_bus_id")) for i in infos}) or 1
    if shared:
        return f"{world} ranks on {gpus} GPU{'s' if gpus > 1 else ''}"
    if self_rccl:
        return "1 rank exchanging with itself through RCCL"
    return None


# The fp32 oracle runs on the whole grid up to 2^30 cells (the headline
# grid); larger grids are checked on row bands with their light cones.
ORACLE_WHOLE_CELLS = 1 << 30
ORACLE_BAND_ROWS = 128
# Several ranks gather the whole grid for the check up to this size (2^34
# cells = 16 GiB per byte copy); one rank checks any size on bands read
# straight from the device (Engine.store_rows), with no whole-grid host copy.
VERIFY_MAX_CELLS = 1 << 34


def band_starts(H: int) -> list[int]:
    """First rows of the oracle bands: top, middle and bottom of the torus."""
    b = min(ORACLE_BAND_ROWS, H)
    return sorted({0, max(0, H // 2 - b // 2), max(0, H - b)})


def wrapped_rows(eng, H: int, r0: int, n: int):
    """Rows r0 .. r0 + n - 1 of the torus (indices mod H) from the device, in
    contiguous pieces (Engine.store_rows)."""
    import numpy as np  # noqa: PLC0415

    parts, r, left = [], r0 % H, n
    while left > 0:
        k = min(left, H - r)
        parts.append(eng.store_rows(r, k))
        r, left = 0, left - k
    return np.concatenate(parts, axis=0)


def band_oracle(snap, r0: int, gens: int, device: str):
    """Rows [r0, r0 + ORACLE_BAND_ROWS) of the grid `gens` generations after
    `snap`, from the fp32 oracle on the band plus `gens` rows of light cone on
    each side (rows wrap around the torus; the band's own wrap only corrupts
    the cone rows, which are dropped)."""
    import numpy as np  # noqa: PLC0415

    from gol_amd.ops.life_ops import life_step_torch_roll  # noqa: PLC0415

    H = snap.shape[0]
    b = min(ORACLE_BAND_ROWS, H)
    rows = np.arange(r0 - gens, r0 + b + gens) % H
    return life_step_torch_roll(snap[rows], gens, device=device)[gens:gens + b]


def dtype_label(layout: str, u8_compute, kernel: str) -> str:
    """What the cells are stored as and what the timed loop computes on.  A
    byte grid whose epochs run on its bit image (u8_compute "bits", the GPU
    default) says so: the timed loop never touches the bytes, which are
    unpacked only when read (VERDICT r05 "Weak 5")."""
    if layout == "bits":
        return "u1 bit-packed cells (exact boolean B3/S23; reference stores u8 chars)"
    if u8_compute == "bits":
        return "u8 storage, computed on a live bit image (packed once, unpacked on read; exact)"
    if "LDS-tiled" in kernel:
        return "u8 byte-per-cell, LDS-tiled byte kernel (exact)"
    return "u8 byte-per-cell, computed on the bytes (exact)"


def grid_digest(parts) -> str:
    """sha256 of the verified final cells (0/1 bytes, row-major): the same seed
    and step count must give the same digest on any schedule or build, so two
    trees can be compared bit for bit (e.g. before and after a refactor)."""
    import hashlib  # noqa: PLC0415

    import numpy as np  # noqa: PLC0415

    h = hashlib.sha256()
    for p in parts:
        h.update(np.ascontiguousarray(p, dtype=np.uint8).tobytes())
    return h.hexdigest()


def check_ranks(world: int, shared: bool, comm_count: int, infos: list[dict]) -> str | None:
    """What RCCL saw must be what the bench reports (the reference's
    MPI_Comm_size, src/game_mpi.c:159): the communicator holds `world` ranks,
    every rank reported in, and without --share-gpus no two ranks ran on the
    same physical GPU (PCI bus id).  Returns the reason to refuse, or None."""
    if comm_count != world:
        return f"the halo communicator has {comm_count} ranks, but {world} rank processes were launched"
    if len(infos) != world or sorted(i["rank"] for i in infos) != list(range(world)):
        return f"{len(infos)} of {world} ranks reported their device"
    if not shared:
        # One physical device (or partition) per rank, named by (host, device
        # UUID, PCI bus id) - never the process-local ordinal, which differs
        # between ranks that see one GPU under different HIP_VISIBLE_DEVICES.
        keys = [(i.get("host"), i.get("uuid"), i["pci_bus_id"]) for i in infos if i.get("pci_bus_id")]
        dup = sorted({k[2] for k in keys if keys.count(k) > 1})
        if dup:
            return f"ranks share GPU(s) {dup} without --share-gpus: n_gpus would overstate the GPUs used"
    return None


def parse_tune(pairs: list[str]) -> dict:
    """--tune key=value (repeatable) -> dict; keys and values are validated
    by the native Tuning when the backend is made."""
    out = {}
    for kv in pairs:
        k, eq, v = kv.partition("=")
        if not eq or not k:
            raise SystemExit(f"bench.py: --tune {kv!r}: expected key=value")
        out[k] = v
    return out


def parse_args(argv=None):
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
    ap.add_argument("--u8-compute", default="auto", choices=["auto", "bits", "bytes"],
                    help="byte layout: epochs on bit words (auto on the GPU) or on the bytes themselves")
    ap.add_argument("--engine", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--comm", default="auto", choices=["auto", "rccl", "torch"],
                    help="halo transport between rank processes (auto: rccl on GPU, torch/gloo on CPU)")
    ap.add_argument("--decomp", default="auto")
    ap.add_argument("--tmax", type=int, default=0)
    ap.add_argument("--epoch", type=int, default=0)
    ap.add_argument("--poll", type=int, default=0)
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off", "trigger"])
    ap.add_argument("--graphs", default="off", choices=["auto", "on", "off"])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--repeats", type=int, default=1, help="timed repetitions (best is reported)")
    ap.add_argument("--rehearse-rccl", action="store_true",
                    help="one GPU: run the multi-rank row-strip schedule (epoch depth, boundary-trigger overlap, "
                         "RCCL send/recv + all-reduce) against a 1-rank RCCL communicator that exchanges with "
                         "itself; use with --height H/N to rehearse one rank of an N-GPU run")
    ap.add_argument("--share-gpus", action="store_true",
                    help="let ranks share GPUs (rehearsal of the multi-rank path on fewer GPUs than ranks)")
    ap.add_argument("--verify", type=int, default=240,
                    help="after the timed steps, run G more generations and check them against the fp32 "
                         "PyTorch oracle and the u8 layout (0: skip)")
    ap.add_argument("--verify-bands", action="store_true",
                    help="check on row bands read from the device even below the whole-grid limits "
                         "(one rank: torus bands; several: each rank's own bands, cones from its neighbours)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="runtime tuning (repeatable; python -m gol_amd.cli --tune help lists the keys)")
    ap.add_argument("--no-phase-step", action="store_true",
                    help="skip the extra per-phase-timed step after the timed ones")
    return ap.parse_args(argv)


def main() -> int:
    out_fd = _claim_stdout()
    a = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if a.gpus > 1:
            return _launch_ranks(a.gpus, sys.argv[1:], out_fd)
    elif int(env_world) != a.gpus:
        log(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={env_world} ranks; refusing to "
            "report a number for a different GPU count")
        return 2

    from gol_amd.parallel.dist import env_rank  # noqa: PLC0415

    rank, world, local = env_rank()
    on_gpu = a.engine == "hip"
    shared = False
    tune = parse_tune(a.tune)
    if on_gpu and world > 1:
        import torch  # noqa: PLC0415

        ndev = torch.cuda.device_count()  # does not initialise the GPU
        if ndev < world:
            if not a.share_gpus:
                log(f"bench.py: {world} ranks but {ndev} GPU(s) visible; every rank needs a GPU of its own "
                    "(--share-gpus for a shared-device rehearsal)")
                return 2
            # RCCL refuses two ranks of one communicator on one device when
            # they share a host hash; distinct host ids make every rank its
            # own "node" (socket transport over loopback).
            shared = True
            os.environ["NCCL_HOSTID"] = f"gol-bench-rank{rank}"
            # Each rank of a shared GPU runs on a disjoint slice of its CUs
            # (tuning cu_partition: CU-masked streams, its RCCL kernels
            # included), as on a node where every rank owns a GPU.  The GPU
            # still time-slices the processes' queues, so the backend leaves
            # out the schedules whose waves wait on other workgroups (chained
            # groups, linked launches); everything else runs unchanged.
            per = -(-world // ndev)
            tune.setdefault("cu_partition", f"{local // ndev}/{per}")
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        local = local % max(1, ndev)

    import numpy as np  # noqa: PLC0415
    import torch  # noqa: PLC0415

    from gol_amd import LifeConfig, Simulation, make_backend, native  # noqa: PLC0415
    from gol_amd.models.life import make_tuning  # noqa: PLC0415
    from gol_amd.parallel.dist import allreduce_max_float  # noqa: PLC0415

    if on_gpu:
        if not torch.cuda.is_available():
            raise SystemExit("bench.py: no GPU visible (use --engine cpu for a CPU dry run)")
        torch.cuda.set_device(local)
    backend = make_backend(a.engine, local, tune=tune)
    dist = None
    if world > 1:
        from gol_amd.parallel.dist import init_process_group, make_transport  # noqa: PLC0415

        # torch.distributed over RCCL on the GPU, shared-device rehearsals
        # included: every rank has its own NCCL_HOSTID, so torch's own RCCL
        # communicator (gather_grid, the MAX of the rank timings) runs the
        # same code path as on the node.
        dist = init_process_group("nccl" if on_gpu else "gloo", device=local if on_gpu else None)
        transport = make_transport(a.comm, backend, local, tune=tune)
    elif a.rehearse_rccl and on_gpu:
        C = native()
        transport = C.rccl_transport(C.rccl_unique_id(), 0, 1, local, tune=make_tuning(tune))
    else:
        transport = native().self_transport()

    # Which communicator size and which physical GPU every rank saw.
    comm_count = transport.comm_count()
    me = {"rank": rank, "local_rank": local, "host": socket.gethostname(),
          "device": (int(backend.device()) if on_gpu else "cpu"),
          "pci_bus_id": (native().hip_pci_bus_id(int(backend.device())) if on_gpu else None),
          "uuid": (native().hip_uuid(int(backend.device())) if on_gpu else None),
          "comm_device": transport.comm_device()}
    if dist is not None:
        infos = [None] * world
        dist.all_gather_object(infos, me)
    else:
        infos = [me]
    why = check_ranks(world, shared, comm_count, infos)
    if why:
        log(f"bench.py: {why}; refusing to report a number")
        return 2

    S = a.size
    Hg = a.height or S
    gps = max(1, a.gens_per_step)
    extra = (0 if a.no_phase_step else gps) + max(0, a.verify)
    trial_cap = 16384  # prewarm generations allowed beyond --prewarm for the placement trials
    total = a.prewarm + trial_cap + (a.warmup + a.steps * a.repeats) * gps + extra
    cfg = LifeConfig(S, Hg, gen_limit=total, layout=a.layout, decomp=a.decomp, tmax=a.tmax, epoch=a.epoch,
                     poll_gens=a.poll, overlap=a.overlap, graphs=a.graphs, timing_barriers=False,
                     self_exchange=bool(a.rehearse_rccl and world == 1), u8_compute=a.u8_compute,
                     watchdog_s=300.0,  # a stuck rank or kernel fails the run instead of hanging it
                     tune=tune)
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

    trial_gens = 0
    if a.prewarm > 0:
        eng.run_until(sim.generation + a.prewarm)
        # The overlap and poll-placement trials decide on the ranks over the first epochs and poll
        # windows (the same generation on every rank); keep them out of the timed region.
        while "trial" in eng.overlap_mode() + eng.poll_mode() and trial_gens < trial_cap:
            eng.run_until(sim.generation + 1024)
            trial_gens += 1024
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

    # One more step with per-phase device timing (outside the timed region:
    # the event pairs around every operation add a little launch overhead).
    phases = None
    if not a.no_phase_step:
        sync()
        eng.phase_timing = True
        r = step()
        eng.phase_timing = False
        sync()
        phases = {k: allreduce_max_float(float(getattr(r, k))) for k in
                  ("loop_ms", "compute_ms", "halo_ms", "fill_ms", "allreduce_ms")}
        phases["generations"] = int(r.executed)
        phases["rank"] = "max over ranks"

    # Correctness gate at the credited configuration: the same engine (same
    # kernel choice, epoch, wrap + fold, autotuned chain picks, drift state)
    # continues from its current state; the oracle restarts from a snapshot.
    verify = None
    verified = None
    if a.verify > 0 and (S * Hg > ORACLE_WHOLE_CELLS or a.verify_bands) and world == 1:
        # One rank, a grid beyond the whole-grid oracle (up to 1048576^2 on one
        # GPU): top, middle and bottom row bands with their light cones are read
        # from the device before and after G generations - no whole-grid host
        # copy, so no size limit - and checked against the fp32 oracle.
        from gol_amd.ops.life_ops import life_step_torch_roll  # noqa: PLC0415

        t_v = time.perf_counter()
        g_snap = sim.generation
        G, b = a.verify, min(ORACLE_BAND_ROWS, Hg)
        starts = band_starts(Hg)
        snaps = [wrapped_rows(eng, Hg, r0 - G, b + 2 * G) for r0 in starts]
        rv = eng.run_until(g_snap + G)
        done = sim.generation - g_snap
        dev = "cuda" if on_gpu else "cpu"
        ok_torch = True
        for r0, snap in zip(starts, snaps):
            # A run that stopped early ran `done` generations; its cone is the
            # middle b + 2 done rows of the snapshot.
            cone = snap[G - done:G + b + done]
            want = life_step_torch_roll(cone, done, device=dev)[done:done + b]
            ok_torch = ok_torch and bool(np.array_equal(eng.store_rows(r0, b), want))
            del want, cone
        del snaps
        verified = ok_torch
        digest = grid_digest([eng.store_rows(r0, b) for r0 in starts])
        verify = {"generations": int(done), "from_generation": int(g_snap), "stop_reason": rv.stop_reason,
                  "oracle": f"{len(starts)} row bands of {b} read from the device (light cones of {done} rows)",
                  "final_sha256": digest, "digest_of": "the checked row bands",
                  "vs_torch_fp32_oracle": ok_torch, "vs_u8_layout": None,
                  "seconds": round(time.perf_counter() - t_v, 2)}
    elif a.verify > 0 and (S * Hg > VERIFY_MAX_CELLS or a.verify_bands) and eng.decomp.Px == 1:
        # Several ranks, a grid no host holds whole (BASELINE config 5): every
        # rank checks row bands of its own tile, the light-cone rows beyond it
        # sent by its neighbours - no gather (parallel/dist.py verify_row_bands).
        from gol_amd.parallel.dist import verify_row_bands  # noqa: PLC0415

        t_v = time.perf_counter()
        g_snap = sim.generation
        vb = verify_row_bands(sim, a.verify, ORACLE_BAND_ROWS, device="cuda" if on_gpu else "cpu")
        verified = vb["ok"]
        verify = {"generations": vb["generations"], "from_generation": int(g_snap), "stop_reason": vb["stop_reason"],
                  "oracle": f"{vb['bands_per_rank']} row bands of {vb['band_rows']} per rank (top, middle, bottom "
                            f"of each tile), light cones of {vb['cone_rows']} rows from the neighbours; no gather",
                  "vs_torch_fp32_oracle": vb["ok"], "vs_u8_layout": None,
                  "seconds": round(time.perf_counter() - t_v, 2)}
    elif a.verify > 0 and S * Hg > VERIFY_MAX_CELLS:
        # Several ranks in a 2-D decomposition: gathering the grid would not fit.
        log(f"bench.py: --verify skipped: {S}x{Hg} on {world} ranks exceeds {VERIFY_MAX_CELLS} cells (2-D tiles)")
        verify = {"skipped": f"grid beyond {VERIFY_MAX_CELLS} cells on a 2-D decomposition"}
    elif a.verify > 0:
        from gol_amd.ops.life_ops import life_step_torch_roll  # noqa: PLC0415
        from gol_amd.parallel.dist import gather_grid  # noqa: PLC0415

        t_v = time.perf_counter()
        g_snap = sim.generation
        snap = gather_grid(sim)
        rv = eng.run_until(g_snap + a.verify)
        done = sim.generation - g_snap
        final = gather_grid(sim)
        ok_torch = ok_u8 = True
        oracle = "whole grid"
        if rank == 0:
            dev = "cuda" if on_gpu else "cpu"
            if S * Hg <= ORACLE_WHOLE_CELLS:
                want = life_step_torch_roll(snap, done, device=dev)
                ok_torch = bool(np.array_equal(final, want))
            else:
                # Grids beyond 2^30 cells: the fp32 oracle on row bands with
                # their light cones (`done` rows per side, wrapped), top,
                # middle and bottom, instead of one 2^32-element tensor.
                oracle = f"{len(band_starts(Hg))} row bands of {ORACLE_BAND_ROWS} (light cones of {done} rows)"
                ok_torch = all(np.array_equal(final[r0:r0 + ORACLE_BAND_ROWS], band_oracle(snap, r0, done, dev))
                               for r0 in band_starts(Hg))
                want = final  # the byte kernels are checked against the bit engine, whole grid
            # The byte kernels themselves: an engine path independent of the
            # bit kernels (whatever layout the timed run used).
            u8 = Simulation(LifeConfig(S, Hg, gen_limit=done, layout="u8", u8_compute="bytes",
                                       check_similarity=False),
                            transport=native().self_transport(), backend=backend)
            u8.load(snap)
            u8.advance(done)
            ok_u8 = bool(np.array_equal(u8.tile(), want))
            del u8
        verified = bool(ok_torch and ok_u8)
        verify = {"generations": int(done), "from_generation": int(g_snap), "stop_reason": rv.stop_reason,
                  "oracle": oracle,
                  "final_sha256": grid_digest([final]) if rank == 0 else None, "digest_of": "the whole grid",
                  "vs_torch_fp32_oracle": ok_torch, "vs_u8_layout": ok_u8,
                  "seconds": round(time.perf_counter() - t_v, 2)}
        if dist is not None:
            dist.barrier()

    desc = sim.describe()
    if desc["row_ring_fallback"]:
        log(f"bench.py: WARNING: the row ring fell back to periodic fills ({desc['row_ring_fallback']}); "
            "the number below is not the ring schedule's")
    rehearsal = rehearsal_label(world, shared, bool(a.rehearse_rccl and world == 1 and on_gpu), infos)
    metric, headline, config_id = metric_label(S, Hg, gps, rehearsal)
    if rank == 0:
        rec = {
            "metric": metric,
            "value": value,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3 / max(1, a.steps),
            "higher_is_better": True,
            "scaling": "strong",
            "verified": verified,
            "vs_baseline": value / BASELINE_VALUE,
            "dtype": dtype_label(a.layout, desc["u8_compute"], desc["kernel"]),
            "data": "synthetic: on-device counter-based RNG random grid, density 0.5 (generate.sh distribution)",
            "headline": headline,
            "config_id": config_id,
            "rccl_nranks": comm_count,
            "devices": infos,
            "config": {
                "model": f"Game of Life B3/S23 torus {S}x{Hg}",
                "global_batch": 1,
                "seq_len": S * Hg,
                "parallelism": f"{desc['decomp']} row/col tiles, {desc['transport'] if world > 1 else 'rccl-self (rehearsal)' if a.rehearse_rccl else 'single'} halos",
                "grid": f"{S}x{Hg}",
                "layout": a.layout,
                "u8_compute": desc["u8_compute"],
                "engine": backend.name(),
                "kernel": desc["kernel"],
                "tmax": desc["tmax"],
                "epoch": desc["epoch"],
                "gens_per_step": gps,
                "generations_timed": gens,
                "step_stop_reasons": stops,
                "prewarm_generations": a.prewarm,
                "prewarm_trial_generations": trial_gens,
                "warmup_generations": a.warmup * gps,
                "loop_ms_engine_per_step": sum(r.loop_ms for r in rs) / max(1, len(rs)),
                "exchanges_per_step": rs[-1].exchanges if rs else 0,
                "polls_per_step": rs[-1].polls if rs else 0,
                "kernel_launches_per_step": rs[-1].kernel_launches if rs else 0,
                "linked_launches_per_step": rs[-1].linked_launches if rs else 0,
                "row_ring": desc["row_ring"],
                # A ring the tile should have had but the backend could not
                # map (its error): the run used periodic row fills instead.
                "row_ring_fallback": desc["row_ring_fallback"],
                # Knobs set by hand: GOL_* variables, and every tuning key off
                # its default with its source (bench.py's own rehearsal
                # partition aside); the effective values of the tune class.
                "env_knobs": {k: v for k, v in sorted(os.environ.items()) if k.startswith("GOL_")},
                "tuning_changed": {k: v for k, v in desc["tuning_changed"].items()
                                   if not (shared and k == "cu_partition")},
                "tuning": desc["tuning"],
                "cu_partition": desc["tuning"]["cu_partition"] if shared else None,
                "halo_bytes_per_step": rs[-1].halo_bytes if rs else 0,
                "overlapped_halo_exchange": bool(rs and rs[-1].overlapped),
                "overlap_mode": desc["overlap_mode"],
                "overlap_trial_ms_per_epoch": {"plain": desc["overlap_trial_ms_plain"],
                                               "trigger": desc["overlap_trial_ms_trigger"]},
                "triggered_sends": desc["triggered_sends"],
                "poll_mode": desc["poll_mode"],
                "poll_trial_ms_per_window": desc["poll_trial_ms_per_window"],
                "graph_epochs": sum(r.graph_launches for r in rs),
                "phase_ms_one_step": phases,
                "verify": verify,
                "shared_gpus": shared,
                "rehearsal": rehearsal,
                "baseline": "8.9e8 cell-updates/s (best reference run in BASELINE.md: MPI, 4 ranks, 2048^2, CPU)",
            },
        }
        os.write(out_fd, (json.dumps(rec) + "\n").encode())
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 1 if verified is False else 0


if __name__ == "__main__":
    raise SystemExit(main())
