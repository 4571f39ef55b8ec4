"""Rank process of the multi-rank RCCL tests (tests/test_rccl_multirank.py).

Started by torch.distributed.run, N processes on ONE GPU: every rank claims
its own NCCL_HOSTID, so RCCL treats the ranks as separate nodes (socket
transport over loopback) instead of refusing the duplicate device.  The
native RcclTransport (ncclSend/ncclRecv halos, ncclAllReduce MAX flags) then
runs with N real ranks - the path a multi-GPU node runs - and every case is
checked against the fp32 PyTorch conv2d oracle and the exact serial loop.

    argv: CASES   comma-separated decomp:layout:overlap, e.g. 1x2:bits:auto
"""
import os
import sys

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
os.environ["NCCL_HOSTID"] = f"gol-test-rank{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import gol_amd  # noqa: E402
from gol_amd.ops.life_ops import life_step_torch  # noqa: E402
from gol_amd.parallel.dist import gather_grid  # noqa: E402


def log(*a):
    print(f"[rank {rank}]", *a, file=sys.stderr, flush=True)


def main() -> int:
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    C = gol_amd.native()
    obj = [C.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    tr = C.rccl_transport(obj[0], rank, world, 0)
    be = C.hip_backend(0)
    failures = []
    for case in sys.argv[1].split(","):
        decomp, layout, overlap = case.split(":")
        px, py = (int(v) for v in decomp.split("x"))
        # Tall enough for an interior at the multi-rank epoch depth, wide
        # enough for column halos; odd sizes for uneven splits.
        W = 32 * 24 * px if layout == "bits" else 32 * 24 * px + 7
        H = 420 * py + 13
        gens = 500
        g = gol_amd.random_grid(W, H, 17 + px * 10 + py)
        cfg = gol_amd.LifeConfig(W, H, gen_limit=gens, decomp=decomp, layout=layout, overlap=overlap,
                                 tmax=12 if layout == "bits" else 16, epoch=48)
        sim = gol_amd.Simulation(cfg, transport=tr, backend=be)
        sim.load(g)
        sim.phase_timing = True
        rep = sim.advance(gens)
        full = gather_grid(sim)
        want = life_step_torch(g, gens, device="cuda")
        ok = bool(np.array_equal(full, want))
        mode = sim.describe()["overlap_mode"]
        log(case, "exact" if ok else "MISMATCH", "mode", mode, "exchanges", rep.exchanges,
            "phases", round(rep.compute_ms, 2), round(rep.halo_ms, 2), round(rep.allreduce_ms, 2))
        if not ok:
            failures.append(case)
        if rep.exchanges < gens // 48 or not rep.phase_timed or rep.halo_ms <= 0:
            failures.append(case + ":counters")
        if overlap == "auto" and py > 1 and px == 1 and not mode.startswith("auto:"):
            failures.append(case + ":auto-undecided")
        del sim
    # Termination through the RCCL flag all-reduce: exact Generations line.
    from golden import CONVERGING  # noqa: PLC0415

    for W, H, seed, density in [c for c in CONVERGING if c[0] % 32 == 0 and c[1] >= 2 * world][:3]:
        g = gol_amd.random_grid(W, H, seed, density)
        ref, rgens, _ = gol_amd.reference_run(g)
        sim = gol_amd.Simulation(gol_amd.LifeConfig(W, H, decomp=f"1x{world}", tmax=4, epoch=8, poll_gens=16),
                                 transport=tr, backend=be)
        sim.load(g)
        rep = sim.run()
        full = gather_grid(sim)
        ok = rep.generations == rgens and bool(np.array_equal(full, ref))
        log("terminating", (W, H, seed), rep.generations, rgens, "exact" if ok else "MISMATCH")
        if not ok:
            failures.append(f"terminating{(W, H, seed)}")
        del sim
    res = torch.tensor([len(failures)])
    dist.all_reduce(res, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(f"MULTIRANK {'PASS' if res.item() == 0 else 'FAIL'} world={world}", flush=True)
    if failures:
        log("failures:", failures)
    del tr
    dist.destroy_process_group()
    return 0 if res.item() == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
