#!/usr/bin/env python3
"""Probe: can N RCCL ranks share one GPU when each claims its own host id?

RCCL refuses two ranks of one communicator on the same device ("Duplicate GPU
detected") only when their host hashes match; NCCL_HOSTID overrides the hash,
so every rank looks like a separate node and the ranks talk through the
network (socket) transport over loopback.  Run under torchrun:

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        scripts/rccl_shared_gpu_probe.py
"""
import os
import sys

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
os.environ["NCCL_HOSTID"] = f"gol-shared-gpu-rank{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import gol_amd  # noqa: E402
from gol_amd.ops.life_ops import life_step_torch  # noqa: E402

dist.init_process_group("gloo", rank=rank, world_size=world)
C = gol_amd.native()
torch.cuda.set_device(0)
obj = [C.rccl_unique_id() if rank == 0 else None]
dist.broadcast_object_list(obj, src=0)
tr = C.rccl_transport(obj[0], rank, world, 0)
print(f"rank {rank}: communicator up", file=sys.stderr, flush=True)

n = 4096
src = torch.full((n,), rank + 1, dtype=torch.uint8, device="cuda")
dst = torch.zeros_like(src)
s = torch.cuda.current_stream().cuda_stream
nxt, prv = (rank + 1) % world, (rank - 1) % world
tr.exchange([(True, nxt, src.data_ptr(), n), (False, prv, dst.data_ptr(), n)], s)
flags = torch.tensor([rank, 0, 7 * (rank == 0)], dtype=torch.int32, device="cuda")
tr.allreduce_max_u32(flags.data_ptr(), 3, s)
torch.cuda.synchronize()
ok_ring = bool((dst == prv + 1).all())
ok_red = flags.tolist() == [world - 1, 0, 7]
print(f"rank {rank}: ring {ok_ring} allreduce {ok_red}", file=sys.stderr, flush=True)

W, H, gens = 32 * 40, 64 * world + 37, 200
g = gol_amd.random_grid(W, H, 5)
sim = gol_amd.Simulation(gol_amd.LifeConfig(W, H, gen_limit=gens, decomp=f"1x{world}", tmax=12, epoch=24),
                         transport=tr, backend=C.hip_backend(0))
sim.load(g)
rep = sim.advance(gens)
want = life_step_torch(g, gens, device="cuda")
(r0, r1), (c0, c1) = sim.rows, sim.cols
ok_sim = bool(np.array_equal(sim.tile(), want[r0:r1, c0:c1]))
print(f"rank {rank}: engine 1x{world} exact {ok_sim} exchanges {rep.exchanges} ms {rep.loop_ms:.1f}",
      file=sys.stderr, flush=True)
res = torch.tensor([int(ok_ring and ok_red and ok_sim)])
dist.all_reduce(res, op=dist.ReduceOp.MIN)
if rank == 0:
    print(f"PROBE {'PASS' if res.item() else 'FAIL'} world={world}", flush=True)
del sim, tr
dist.destroy_process_group()
sys.exit(0 if res.item() else 1)
