#!/usr/bin/env python3
"""Fixed per-operation cost of the engine's RCCL calls on one MI355X.

A 1-rank communicator (RCCL refuses two ranks on one GPU) runs the engine's
halo-row group (send N, recv S, send S, recv N of one epoch's D = 256 rows of a
32768-cell bit tile, every peer = self) and the termination-flag MAX
all-reduce of one 256-generation poll window, back to back on one stream.
What it measures is the launch + protocol floor of each call; the xGMI
transfer time of a real multi-GPU exchange comes on top.
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import gol_amd  # noqa: E402

C = gol_amd.native()
torch.cuda.set_device(0)
tr = C.rccl_transport(C.rccl_unique_id(), 0, 1, 0)
s = torch.cuda.current_stream()
n = 256 * 4352
bufs = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(4)]
flags = torch.zeros(256, dtype=torch.int32, device="cuda")
ops = [(True, 0, bufs[0].data_ptr(), n), (False, 0, bufs[1].data_ptr(), n),
       (True, 0, bufs[2].data_ptr(), n), (False, 0, bufs[3].data_ptr(), n)]


def timed(fn, iters=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


res = {
    "exchange_4x%dB_us" % n: timed(lambda: tr.exchange(ops, s.cuda_stream)),
    "allreduce_256xu32_us": timed(lambda: tr.allreduce_max_u32(flags.data_ptr(), 256, s.cuda_stream)),
    "exchange_plus_allreduce_us": timed(lambda: (tr.exchange(ops, s.cuda_stream),
                                                 tr.allreduce_max_u32(flags.data_ptr(), 256, s.cuda_stream))),
}
barrier_t = timed(tr.barrier, 100)
res["barrier_host_paired_us"] = barrier_t
print(json.dumps(res))
