// Inter-rank transport for halo exchange and termination-flag reduction.
//
// Reference: 16 persistent MPI requests per buffer (8 Recv_init + 8
// Send_init, rows / strided columns / corner cells), Startall+Waitall every
// generation (src/game_mpi.c:340-401), plus two MPI_Allreduce(SUM) of 4-byte
// flags (empty_all every generation, similarity_all every 3rd:
// src/game_mpi.c:104-143).  Here a halo exchange happens once per epoch of
// Dv generations, as one group of 2 sends + 2 receives per phase, and the
// termination flags of many generations travel in one MAX all-reduce.
//
// Implementations:
//   RcclTransport     - RCCL ncclSend/ncclRecv/ncclAllReduce over xGMI, one
//                       process per GPU, communicator bootstrapped through
//                       torch.distributed (transport_rccl.cpp).
//   ThreadTransport   - in-process ranks (one host thread per rank); used for
//                       multi-subdomain runs on one device and CPU tests.
//   CallbackTransport - delegates to Python (torch.distributed: gloo on CPU,
//                       nccl=RCCL on GPU); defined in bindings.cpp.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gol/tuning.hpp"

namespace gol {

class Backend;

struct P2POp {
  bool send = false;
  int peer = 0;
  void* buf = nullptr;  // backend address space (device memory for HIP)
  size_t bytes = 0;
};

class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual const char* name() const = 0;
  // Executes a group of point-to-point operations.  Messages between a pair
  // of ranks are matched in issue order.  Enqueued on `stream` (HIP) or
  // completed before return (host transports).
  virtual void exchange(const std::vector<P2POp>& ops, void* stream) = 0;
  // In-place element-wise MAX over ranks of n uint32 values.
  virtual void allreduce_max_u32(uint32_t* buf, size_t n, void* stream) = 0;
  virtual void barrier() = 0;
  // exchange()/allreduce enqueue device work only (no host waits), so they
  // can be captured into a HIP graph.
  virtual bool capturable() const { return false; }
  // Throws if the communicator has failed asynchronously (RCCL async error);
  // called by the engine while it waits on the device.
  virtual void check_health() {}
  // allreduce_max_u32 runs on a communicator of its own, so it may be
  // enqueued on another stream than exchange() and run concurrently with it
  // (the engine then reduces termination flags beside the compute stream).
  virtual bool side_reduce() const { return false; }
  // Ranks the underlying communicator reports (RCCL: ncclCommCount; the
  // reference's MPI_Comm_size, src/game_mpi.c:159) and the device it is
  // bound to (ncclCommCuDevice; -1 for host transports).  bench.py checks
  // them against WORLD_SIZE and the rank's own device.
  virtual int comm_count() const { return size(); }
  virtual int comm_device() const { return -1; }
};

// Single rank: nothing to exchange with.
class SelfTransport final : public Transport {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  const char* name() const override { return "self"; }
  void exchange(const std::vector<P2POp>& ops, void* stream) override;
  void allreduce_max_u32(uint32_t*, size_t, void*) override {}
  void barrier() override {}
  bool capturable() const override { return true; }
};

// Shared state of a group of in-process ranks.
class ThreadHub {
 public:
  explicit ThreadHub(int nranks);
  int size() const { return n_; }

  struct Msg {
    const void* buf;
    size_t bytes;
    int device = -1;  // sender's device (-1: host memory)
    bool consumed = false;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> queues;  // (src,dst)
  // barrier / reduction state
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<uint32_t> red;

 private:
  int n_;
};

class ThreadTransport final : public Transport {
 public:
  ThreadTransport(std::shared_ptr<ThreadHub> hub, int rank, Backend* backend,
                  const Tuning& tune = Tuning::from_env());
  int rank() const override { return rank_; }
  int size() const override { return hub_->size(); }
  const char* name() const override { return "thread"; }
  void exchange(const std::vector<P2POp>& ops, void* stream) override;
  void allreduce_max_u32(uint32_t* buf, size_t n, void* stream) override;
  void barrier() override;
  // Tuning cpu_side_poll=1 (tests): claims a flag reduction of its own, so the
  // engine's poll placement trial runs on CPU ranks (both placements reduce
  // through the hub in program order there).
  bool side_reduce() const override { return side_; }

 private:
  bool side_ = false;
  std::shared_ptr<ThreadHub> hub_;
  int rank_;
  Backend* backend_;
  // Fault injection for tests: tuning fault_delay_us =
  // random delay (0..N us) before publishing and before consuming each
  // message, to shake out ordering bugs; fault_garble = corrupt the N-th
  // message this rank receives (1-based; low bit of every 8th byte), which
  // the golden comparison must catch.
  int delay_us_ = 0;
  int64_t garble_at_ = 0, received_ = 0;
  uint64_t rng_ = 0;
  std::vector<int> peers_enabled_;  // devices this rank's device may read directly
  void fault_delay();
};

// RCCL transport (one process per GPU).  `unique_id` is the 128-byte
// ncclUniqueId created on rank 0 and broadcast by the caller.  From `tune`:
// side_poll (a second communicator for the flag reductions) and
// cu_partition (its barrier stream's CUs).
std::unique_ptr<Transport> make_rccl_transport(const std::vector<uint8_t>& unique_id, int rank,
                                               int nranks, int device, const Tuning& tune = Tuning::from_env());
std::vector<uint8_t> rccl_unique_id();
bool rccl_available();
// PCI bus id ("0000:05:00.0") of a HIP device: which physical GPU a rank ran on.
std::string hip_pci_bus_id(int device);
// HIP errors the release paths ignored and reported (hip_util.hpp clear_release_error).
int64_t hip_release_errors();
std::string hip_uuid(int device);

}  // namespace gol
