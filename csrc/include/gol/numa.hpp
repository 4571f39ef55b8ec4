// Host NUMA placement of a GPU process (tuning numa_pin).
//
// A process that drives one MI355X from the other socket pays a longer hop for
// every doorbell, AQL packet and completion signal; on the 8192^2 grid, whose
// linked launches take 14 us of device time each, that shows in the step time:
// 8 CPUs of the GPU's node 1.43-1.44 ms, of the other node 1.47-1.48, unpinned
// 1.48-1.69; alternating processes, medians 1.50-1.53 pinned to the node vs
// 1.55-1.56 unpinned (profiles/r06/numa/numa.md).  The reference leaves
// placement to the MPI launcher (`mpiexec -n [x] -f machines`,
// src/game_mpi.c:2); here a device backend pins its process itself, once, to
// the CPUs of its GPU's node.
#pragma once

#include <string>
#include <vector>

namespace gol {

// "0-3,8,10-11" -> {0, 1, 2, 3, 8, 10, 11} (sysfs cpulist syntax).
std::vector<int> parse_cpulist(const std::string& s);
// NUMA node of a PCI device ("0000:5d:00.0"), -1 when sysfs does not say.
int pci_numa_node(const std::string& bus_id);
// Restrict every thread of this process to the CPUs of PCI device `bus_id`'s
// NUMA node that its original affinity allowed - with `one_l3`, to those of
// them that share one L3 cache, the GPU's ordinal on its node choosing which.
// Once per process: a later call for the same node is a no-op, a call for
// another node (devices on both sockets in one process) restores the original
// affinity and pins nothing again.  Returns the node the process is pinned
// to, or -1.
int pin_process_to_numa(const std::string& bus_id, bool one_l3);
// The node pin_process_to_numa left the process on (-1: none).
int pinned_numa_node();

}  // namespace gol
