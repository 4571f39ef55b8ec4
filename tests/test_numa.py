"""Host NUMA placement (csrc/include/gol/numa.hpp, tuning numa_pin): a device
backend pins its process's host threads to the CPUs of its GPU's NUMA node
(numa_pin = 1) or of one L3 cache there (2).  The reference leaves placement
to the MPI launcher (`mpiexec -n [x] -f machines`, src/game_mpi.c:2), so
there is nothing of its to pin against: these tests pin the contract."""
import os

import pytest

from gol_amd import LifeConfig, Simulation


def test_parse_cpulist(native):
    assert native.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert native.parse_cpulist("") == []
    assert native.parse_cpulist("5") == [5]


def test_unknown_pci_device_has_no_node(native):
    assert native.pci_numa_node("0000:ff:1f.7") == -1


def test_cpu_backend_leaves_placement_alone(native):
    if native.pinned_numa_node() >= 0:
        pytest.skip("a device backend already pinned this process")
    before = os.sched_getaffinity(0)
    sim = Simulation(LifeConfig(64, 64, gen_limit=3), engine="cpu")
    sim.init_random(1, 0.5)
    sim.run()
    assert os.sched_getaffinity(0) == before and native.pinned_numa_node() == -1


@pytest.mark.gpu
def test_hip_backend_pins_to_its_gpus_node(native):
    b = native.hip_backend(0)
    node = native.pci_numa_node(native.hip_pci_bus_id(0))
    if node < 0:
        assert "numa=" not in b.name()
        pytest.skip("sysfs names no NUMA node for this GPU")
    assert native.pinned_numa_node() == node and f"numa={node}:" in b.name()
    with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
        node_cpus = set(native.parse_cpulist(f.read()))
    mine = os.sched_getaffinity(0)
    assert mine and mine <= node_cpus
    assert f":{len(mine)}cpus" in b.name()
