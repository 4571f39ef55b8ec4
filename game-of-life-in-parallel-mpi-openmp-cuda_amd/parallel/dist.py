"""Multi-process runs: one process per GPU, torch.distributed bootstrap.

Reference: ``MPI_Init`` inside ``game()`` (src/game_mpi.c:158-160), one
MPICH rank per core, persistent point-to-point halos and Allreduce flags.
Here every process owns one MI355X (``LOCAL_RANK``), the process group is
``torch.distributed`` (``nccl`` = RCCL on ROCm, ``gloo`` on CPU) and the halo
transport is one of:

* ``rccl``  - native RCCL communicator inside the C++ engine; its
  ``ncclUniqueId`` is created by rank 0 and broadcast through the torch
  process group.  Halos and flag reductions are enqueued on the engine's
  HIP stream with no Python on the hot path (default on GPU).
* ``torch`` - the engine calls back into Python, which runs
  ``torch.distributed.batch_isend_irecv`` / ``all_reduce`` on zero-copy tensor
  views of the engine's buffers (works with ``nccl`` and ``gloo``; default
  on CPU, used by the multi-process CPU tests).
"""
from __future__ import annotations

import contextlib
import ctypes
import datetime
import os
import sys
from typing import Optional

import numpy as np

from .._native import native


def env_rank() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


@contextlib.contextmanager
def stdout_to_stderr():
    """fd 1 -> stderr inside the block.  RCCL prints a version banner to stdout
    when a communicator is created; stdout carries the program's own output
    (the reference's stdout lines, bench.py's JSON line)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def init_process_group(backend: Optional[str] = None, timeout_s: int = 600, device: Optional[int] = None):
    """Initialise torch.distributed from the torchrun environment (idempotent).
    ``device``: this rank's GPU for the ``nccl`` backend (default LOCAL_RANK;
    ranks sharing GPUs pass LOCAL_RANK modulo the device count)."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    if dist.is_available() and dist.is_initialized():
        return dist
    rank, world, local = env_rank()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        dev = local if device is None else int(device)
        torch.cuda.set_device(dev)
        kw["device_id"] = torch.device("cuda", dev)
    with stdout_to_stderr():
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        if backend == "nccl":
            dist.barrier()  # creates torch's communicator now, while stdout is diverted
    return dist


# ---------------------------------------------------------------------------
# Zero-copy tensor views of engine buffers
# ---------------------------------------------------------------------------
class _DeviceBuf:
    """Minimal ``__cuda_array_interface__`` provider for a raw device pointer."""

    def __init__(self, ptr: int, nbytes: int, typestr: str = "|u1", itemsize: int = 1):
        self.__cuda_array_interface__ = {
            "shape": (nbytes // itemsize,), "typestr": typestr, "data": (int(ptr), False),
            "version": 2, "strides": None,
        }


def _host_view(ptr: int, nbytes: int, dtype=np.uint8):
    buf = (ctypes.c_uint8 * nbytes).from_address(int(ptr))
    return np.frombuffer(buf, dtype=dtype)


def tensor_view(ptr: int, nbytes: int, on_device: bool, dtype: str = "u1"):
    import torch  # noqa: PLC0415

    if on_device:
        typestr, item = ("|u1", 1) if dtype == "u1" else ("<i4", 4)
        return torch.as_tensor(_DeviceBuf(ptr, nbytes, typestr, item), device="cuda")
    arr = _host_view(ptr, nbytes, np.uint8 if dtype == "u1" else np.int32)
    return torch.from_numpy(arr)


def torch_transport(backend_obj, group=None):
    """Engine transport implemented with torch.distributed collectives."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    on_dev = bool(backend_obj.is_device())
    rank, world = dist.get_rank(group), dist.get_world_size(group)

    def _stream_ctx(stream_ptr: int):
        if on_dev and stream_ptr:
            return torch.cuda.stream(torch.cuda.ExternalStream(int(stream_ptr)))
        import contextlib  # noqa: PLC0415
        return contextlib.nullcontext()

    def exchange(ops, stream_ptr):
        with _stream_ctx(stream_ptr):
            p2p = []
            for send, peer, addr, nbytes in ops:
                t = tensor_view(addr, nbytes, on_dev)
                p2p.append(dist.P2POp(dist.isend if send else dist.irecv, t, int(peer), group))
            if p2p:
                for w in dist.batch_isend_irecv(p2p):
                    w.wait()

    def allreduce(addr, n, stream_ptr):
        with _stream_ctx(stream_ptr):
            t = tensor_view(addr, 4 * n, on_dev, dtype="i4")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            if not on_dev:
                return

    def barrier():
        dist.barrier(group=group)

    return native().callback_transport(rank, world, exchange, allreduce, barrier)


def rccl_transport(device: int, group=None, tune=None):
    """Native RCCL communicator, uid broadcast over the torch process group
    (``tune``: side_poll / cu_partition, see models.life.make_tuning)."""
    from ..models.life import make_tuning  # noqa: PLC0415

    import torch.distributed as dist  # noqa: PLC0415

    C = native()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [C.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return C.rccl_transport(obj[0], rank, world, int(device), tune=make_tuning(tune))


def make_transport(kind: str, backend_obj, device: int = 0, tune=None):
    """``self`` (1 rank) | ``rccl`` | ``torch``; ``auto`` -> rccl on GPU, torch on CPU."""
    import torch.distributed as dist  # noqa: PLC0415

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return native().self_transport()
    if kind == "auto":
        kind = "rccl" if backend_obj.is_device() else "torch"
    if kind == "rccl":
        return rccl_transport(device, tune=tune)
    if kind == "torch":
        return torch_transport(backend_obj)
    raise ValueError(f"unknown transport {kind!r}")


def allreduce_max_float(x: float) -> float:
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    if not (dist.is_available() and dist.is_initialized()):
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_grid(sim, group=None):
    """Whole grid assembled on every rank from the ranks' tiles (the
    reference's rank-0 gather, src/game_mpi.c:429-458, as one all_gather of
    padded tiles over the process group: RCCL on GPU, gloo on CPU).  Used
    for verification and the --show viewer, not on the hot path."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    tile = np.ascontiguousarray(sim.tile(), dtype=np.uint8)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return tile
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    world = dist.get_world_size(group)
    (r0, r1), (c0, c1) = sim.rows, sim.cols
    ext = torch.tensor([r0, r1, c0, c1], dtype=torch.int64, device=dev)
    exts = [torch.zeros_like(ext) for _ in range(world)]
    dist.all_gather(exts, ext, group=group)
    exts = [tuple(int(v) for v in e.cpu()) for e in exts]
    mh = max(e[1] - e[0] for e in exts)
    mw = max(e[3] - e[2] for e in exts)
    pad = torch.zeros((mh, mw), dtype=torch.uint8, device=dev)
    pad[: r1 - r0, : c1 - c0] = torch.from_numpy(tile).to(dev)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    H, W = sim.config.height, sim.config.width
    out = np.zeros((H, W), dtype=np.uint8)
    for (a, b, c, d), t in zip(exts, parts):
        out[a:b, c:d] = t[: b - a, : d - c].cpu().numpy()
    return out


def band_starts_local(rows: int, band_rows: int) -> list[int]:
    """First local rows of a rank's check bands: its top, middle and bottom
    rows (the top and bottom bands sit on the rows the halo exchange feeds)."""
    b = min(band_rows, rows)
    return sorted({0, max(0, rows // 2 - b // 2), rows - b})


def verify_row_bands(sim, gens: int, band_rows: int = 128, device: str = "cpu", group=None,
                     after_snapshot=None) -> dict:
    """Check the next `gens` generations of a multi-rank run on row bands of
    every rank's own tile, with no gather: the multi-rank counterpart of
    bench.py's single-rank band check, for grids no host can hold whole
    (BASELINE config 5: 2^40 cells over 8 ranks).

    Row strips (Px == 1, the default decomposition): each rank snapshots, for
    each of its bands (top, middle, bottom rows of its tile), the band plus
    `gens` rows of light cone on each side.  Cone rows beyond its tile come
    from its neighbours: before the run every rank sends its top `gens` rows
    north and its bottom `gens` rows south (one batched send/recv pair each
    way over the process group, RCCL on GPU, gloo on CPU).  After the
    collective run of `gens` generations each rank compares its bands, read
    straight from the device (Engine.store_rows), with the fp32 oracle on the
    cone (ops.life_ops.life_step_torch_roll; columns wrap, the cone's own row
    wrap only corrupts rows that are dropped), and the verdict is the AND
    over ranks.  Nothing larger than (band + 2 gens) rows of one rank's
    width is ever copied to a host.  The reference checks nothing of the
    kind; its collective variants gather the whole grid to write it
    (src/game_mpi_collective.c:331-361).  `after_snapshot(sim)` (tests) runs
    between the snapshots and the run: a corrupted cell there must fail."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    from ..ops.life_ops import life_step_torch_roll  # noqa: PLC0415

    eng = sim.native_engine
    dec = eng.decomp
    rank = sim.rank
    if dec.Px != 1:
        raise ValueError("verify_row_bands: row strips only (Px == 1)")
    r0, r1 = sim.rows
    ht = r1 - r0
    G = int(gens)
    comm_dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    # The shortest tile bounds the cone: a neighbour must hold G rows.
    hmin = torch.tensor([ht], dtype=torch.int64, device=comm_dev)
    dist.all_reduce(hmin, op=dist.ReduceOp.MIN, group=group)
    if G > int(hmin.item()):
        raise ValueError(f"verify_row_bands: {G} generations of light cone exceed a {int(hmin.item())}-row tile")
    b = min(band_rows, ht)
    starts = band_starts_local(ht, band_rows)
    nb = dec.neighbors(rank)
    north, south = int(nb[0]), int(nb[1])
    W = sim.config.width

    def rows(lo: int, n: int) -> np.ndarray:
        return eng.store_rows(lo, n) if n > 0 else np.zeros((0, W), np.uint8)

    # Cone rows of the neighbours, in issue order on every rank: sends top ->
    # north, bottom -> south; receives from south (its top rows, below mine),
    # then from north (its bottom rows) - so two ranks that are each other's
    # north and south (Py == 2) still pair the right messages.
    send_top = torch.from_numpy(np.ascontiguousarray(rows(0, G))).to(comm_dev)
    send_bot = torch.from_numpy(np.ascontiguousarray(rows(ht - G, G))).to(comm_dev)
    from_south = torch.empty((G, W), dtype=torch.uint8, device=comm_dev)
    from_north = torch.empty((G, W), dtype=torch.uint8, device=comm_dev)
    ops = [dist.P2POp(dist.isend, send_top, north, group), dist.P2POp(dist.isend, send_bot, south, group),
           dist.P2POp(dist.irecv, from_south, south, group), dist.P2POp(dist.irecv, from_north, north, group)]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    above, below = from_north.cpu().numpy(), from_south.cpu().numpy()
    del send_top, send_bot, from_south, from_north

    def cone(s: int) -> np.ndarray:
        """Snapshot of local rows [s - G, s + b + G), neighbours' rows where
        they fall outside the tile."""
        lo, hi = s - G, s + b + G
        parts = []
        if lo < 0:
            parts.append(above[G + lo:])
        parts.append(rows(max(lo, 0), min(hi, ht) - max(lo, 0)))
        if hi > ht:
            parts.append(below[:hi - ht])
        return np.concatenate(parts, axis=0)

    snaps = [cone(s) for s in starts]
    if after_snapshot is not None:
        after_snapshot(sim)
    g0 = sim.generation
    rv = eng.run_until(g0 + G)
    done = sim.generation - g0
    ok = True
    for s, snap in zip(starts, snaps):
        c = snap[G - done:G + b + done]  # a run that stopped early ran `done` generations
        want = life_step_torch_roll(c, done, device=device)[done:done + b]
        ok = ok and bool(np.array_equal(rows(s, b), want))
        del want, c
    del snaps
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=comm_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return {"ok": bool(flag.item()), "generations": int(done), "stop_reason": rv.stop_reason,
            "bands_per_rank": len(starts), "band_rows": b, "cone_rows": G}
