#!/usr/bin/env python3
"""Host NUMA layout as seen by this process (round 6, 8192^2 spread probe):
prints the GPU's PCI bus id and NUMA node, then one line per NUMA node with
the CPUs of that node this process may run on, in taskset -c form:

    gpu <bus id> node <n>
    node <n> <cpu list>

    python scripts/numa_cpus.py [--no-gpu]
"""
import ctypes
import glob
import os
import sys


def cpulist(s):
    out = set()
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


allowed = os.sched_getaffinity(0)
if "--no-gpu" not in sys.argv:
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, 0) == 0:
        bus = buf.value.decode().lower()
        try:
            with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
                print(f"gpu {bus} node {f.read().strip()}")
        except OSError:
            print(f"gpu {bus} node ?")
for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*"), key=lambda p: int(p.rsplit("node", 1)[1])):
    with open(os.path.join(d, "cpulist")) as f:
        cpus = sorted(cpulist(f.read()) & allowed)
    if cpus:
        print(f"node {d.rsplit('node', 1)[1]} {','.join(map(str, cpus))}")
