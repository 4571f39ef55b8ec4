// Host NUMA placement of a GPU process (gol/numa.hpp).
#include "gol/numa.hpp"

#include <dirent.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <mutex>
#include <sstream>

namespace gol {

std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    while (!part.empty() && std::isspace(static_cast<unsigned char>(part.back()))) part.pop_back();
    if (part.empty()) continue;
    const size_t dash = part.find('-');
    const int a = std::atoi(part.substr(0, dash).c_str());
    const int b = dash == std::string::npos ? a : std::atoi(part.substr(dash + 1).c_str());
    for (int c = a; c <= b; ++c) out.push_back(c);
  }
  return out;
}

int pci_numa_node(const std::string& bus_id) {
  std::string id = bus_id;
  for (char& c : id) c = char(std::tolower(static_cast<unsigned char>(c)));
  std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
  int n = -1;
  if (!(f >> n)) return -1;
  return n;
}

namespace {

std::mutex g_mu;
bool g_saved = false;
cpu_set_t g_orig;
int g_node = -1;
bool g_mixed = false;

// Every thread of the process (the runtime's helper threads included) gets
// `set`; threads created later inherit it from their creator.
void set_all_threads(const cpu_set_t& set) {
  DIR* d = opendir("/proc/self/task");
  if (!d) {
    sched_setaffinity(0, sizeof(set), &set);
    return;
  }
  while (dirent* e = readdir(d)) {
    const int tid = std::atoi(e->d_name);
    if (tid > 0) sched_setaffinity(pid_t(tid), sizeof(set), &set);
  }
  closedir(d);
}

// Ordinal of GPU `bus_id` among the AMD accelerators on `node` (PCI order).
int gpu_ordinal_on_node(const std::string& bus_id, int node) {
  std::string id = bus_id;
  for (char& c : id) c = char(std::tolower(static_cast<unsigned char>(c)));
  std::vector<std::string> gpus;
  if (DIR* d = opendir("/sys/bus/pci/devices")) {
    while (dirent* e = readdir(d)) {
      const std::string dev = e->d_name;
      if (dev[0] == '.') continue;
      const std::string base = "/sys/bus/pci/devices/" + dev + "/";
      std::ifstream v(base + "vendor"), c(base + "class");
      std::string vendor, cls;
      if (!(v >> vendor) || !(c >> cls) || vendor != "0x1002") continue;
      if (cls.compare(0, 4, "0x12") != 0 && cls.compare(0, 6, "0x0380") != 0) continue;
      if (pci_numa_node(dev) == node) gpus.push_back(dev);
    }
    closedir(d);
  }
  std::sort(gpus.begin(), gpus.end());
  for (size_t i = 0; i < gpus.size(); ++i)
    if (gpus[i] == id) return int(i);
  return 0;
}

// The CPUs of `cpus` that share one last-level (L3) cache, group `ordinal`
// (mod the number of groups), groups ordered by their first CPU.
std::vector<int> l3_group(const std::vector<int>& cpus, int ordinal) {
  std::vector<std::vector<int>> groups;
  for (int c : cpus) {
    std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/shared_cpu_list");
    std::string list;
    if (!std::getline(f, list)) return cpus;
    std::vector<int> g;
    for (int x : parse_cpulist(list))
      if (std::find(cpus.begin(), cpus.end(), x) != cpus.end()) g.push_back(x);
    if (std::find(groups.begin(), groups.end(), g) == groups.end()) groups.push_back(g);
  }
  if (groups.empty()) return cpus;
  std::sort(groups.begin(), groups.end());
  return groups[size_t(ordinal) % groups.size()];
}

}  // namespace

int pin_process_to_numa(const std::string& bus_id, bool one_l3) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int node = pci_numa_node(bus_id);
  if (node < 0 || g_mixed) return -1;
  if (g_node == node) return node;
  if (!g_saved) {
    CPU_ZERO(&g_orig);
    if (sched_getaffinity(0, sizeof(g_orig), &g_orig) != 0) return -1;
    g_saved = true;
  }
  if (g_node >= 0) {  // devices on two nodes: back to the original placement
    set_all_threads(g_orig);
    g_node = -1;
    g_mixed = true;
    return -1;
  }
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(f, list)) return -1;
  std::vector<int> cpus;
  for (int c : parse_cpulist(list))
    if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &g_orig)) cpus.push_back(c);
  if (cpus.empty()) return -1;
  if (one_l3) cpus = l3_group(cpus, gpu_ordinal_on_node(bus_id, node));
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  set_all_threads(set);
  g_node = node;
  return node;
}

int pinned_numa_node() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_node;
}

}  // namespace gol
