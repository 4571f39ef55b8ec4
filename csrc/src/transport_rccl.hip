// RCCL transport: halo exchange with grouped ncclSend/ncclRecv and the
// termination-flag MAX all-reduce, enqueued on the engine's HIP stream.
//
// Replaces the reference's MPI layer (src/game_mpi.c:340-401 persistent
// Send_init/Recv_init + Startall/Waitall every generation, and
// MPI_Allreduce in empty_all/similarity_all, src/game_mpi.c:104-143).  On an
// MI355X node every GPU pair has a direct xGMI link, so a 1 x P row-strip
// exchange is 2 sends + 2 receives per epoch, one hop each; halo messages
// are a few hundred KB, i.e. latency-bound, which is why the engine
// exchanges Dv rows once per Dv generations instead of 1 row per generation.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "gol/common.hpp"
#include "gol/hip_util.hpp"
#include "gol/transport.hpp"

#define NCCL_CHECK(expr)                                                                      \
  do {                                                                                        \
    ncclResult_t r_ = (expr);                                                                 \
    if (r_ != ncclSuccess)                                                                    \
      ::gol::fail(std::string("RCCL error in ") + __FILE__ + ":" + std::to_string(__LINE__) + \
                  " (" #expr "): " + ncclGetErrorString(r_));                                 \
    ::gol::clear_release_error("RCCL", true); /* RCCL's probes' HIP errors are not ours */    \
  } while (0)

namespace gol {
namespace {

// RCCL prints a version banner ("RCCL version : ...", HIP/ROCm versions,
// hostname, library path) to stdout when the library initialises.  Stdout
// belongs to the program: the reference's "Generations:" lines, bench.py's
// one JSON line.  Library initialisation runs with fd 1 pointed at stderr.
// The P transports of an in-process run are built on P threads at once
// (ncclCommInitRank blocks until every rank has joined), so the redirect is
// process-wide and reference-counted: the first scope saves fd 1, the last
// one restores it, whatever the order the threads leave in.
class StdoutToStderr {
 public:
  StdoutToStderr() {
    std::lock_guard<std::mutex> lk(mu());
    if (depth()++ == 0) {
      std::fflush(stdout);
      saved() = dup(1);
      if (saved() >= 0) dup2(2, 1);
    }
  }
  ~StdoutToStderr() {
    std::lock_guard<std::mutex> lk(mu());
    if (--depth() == 0) {
      std::fflush(stdout);
      if (saved() >= 0) {
        dup2(saved(), 1);
        close(saved());
        saved() = -1;
      }
    }
  }
  StdoutToStderr(const StdoutToStderr&) = delete;
  StdoutToStderr& operator=(const StdoutToStderr&) = delete;

 private:
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static int& depth() {
    static int d = 0;
    return d;
  }
  static int& saved() {
    static int fd = -1;
    return fd;
  }
};

class RcclTransport final : public Transport {
 public:
  RcclTransport(const std::vector<uint8_t>& uid, int rank, int nranks, int device, const Tuning& tune)
      : rank_(rank), size_(nranks), dev_(device) {
    GOL_REQUIRE(uid.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    DeviceScope on(dev_);
    {
      StdoutToStderr quiet;
      NCCL_CHECK(ncclCommInitRank(&comm_, nranks, id, rank));
      // Side-stream polls (tuning side_poll on or auto, the same on every
      // rank): the termination-flag reductions get their own communicator.
      // RCCL orders the operations of one communicator by issue, and two
      // streams on one communicator could interleave differently on
      // different ranks.
      if (tune.i("side_poll") != 0) NCCL_CHECK(ncclCommSplit(comm_, 0, rank, &flags_comm_, nullptr));
    }
    barrier_stream_ = make_stream(dev_, tune.s("cu_partition"));
    HIP_CHECK(hipMalloc(&barrier_buf_, 64));
    HIP_CHECK(hipMemsetAsync(barrier_buf_, 0, 64, barrier_stream_));  // HIP's hipMemset may return before it ran
    HIP_CHECK(hipStreamSynchronize(barrier_stream_));
  }
  ~RcclTransport() override {
    DeviceScope on(dev_);
    if (barrier_buf_) hipFree(barrier_buf_);
    if (barrier_stream_) hipStreamDestroy(barrier_stream_);
    clear_release_error("~RcclTransport");
    if (flags_comm_) ncclCommDestroy(flags_comm_);
    if (comm_) ncclCommDestroy(comm_);
    clear_release_error("~RcclTransport (RCCL)", true);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* name() const override { return "rccl"; }

  void exchange(const std::vector<P2POp>& ops, void* stream) override {
    DeviceScope on(dev_);
    auto s = static_cast<hipStream_t>(stream);
    NCCL_CHECK(ncclGroupStart());
    for (const auto& op : ops) {
      if (op.send)
        NCCL_CHECK(ncclSend(op.buf, op.bytes, ncclUint8, op.peer, comm_, s));
      else
        NCCL_CHECK(ncclRecv(op.buf, op.bytes, ncclUint8, op.peer, comm_, s));
    }
    NCCL_CHECK(ncclGroupEnd());
  }
  void allreduce_max_u32(uint32_t* buf, size_t n, void* stream) override {
    DeviceScope on(dev_);
    NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclUint32, ncclMax, flags_comm_ ? flags_comm_ : comm_,
                             static_cast<hipStream_t>(stream)));
  }
  bool side_reduce() const override { return flags_comm_ != nullptr; }
  int comm_count() const override {
    int n = 0;
    NCCL_CHECK(ncclCommCount(comm_, &n));
    return n;
  }
  int comm_device() const override {
    int d = -1;
    NCCL_CHECK(ncclCommCuDevice(comm_, &d));
    return d;
  }
  void barrier() override {
    DeviceScope on(dev_);
    NCCL_CHECK(ncclAllReduce(barrier_buf_, barrier_buf_, 1, ncclUint32, ncclMax, comm_, barrier_stream_));
    if (hipStreamSynchronize(barrier_stream_) != hipSuccess) fail("RCCL barrier failed");
  }
  bool capturable() const override { return true; }  // grouped send/recv are stream-ordered
  void check_health() override {
    ncclResult_t r = ncclSuccess;
    for (ncclComm_t c : {comm_, flags_comm_}) {
      if (!c) continue;
      NCCL_CHECK(ncclCommGetAsyncError(c, &r));
      if (r != ncclSuccess && r != ncclInProgress)
        fail(std::string("RCCL communicator failed asynchronously: ") + ncclGetErrorString(r));
    }
  }

 private:
  int rank_, size_, dev_;
  ncclComm_t comm_ = nullptr;
  ncclComm_t flags_comm_ = nullptr;  // allreduce_max_u32 (side_reduce)
  hipStream_t barrier_stream_ = nullptr;
  void* barrier_buf_ = nullptr;
};

}  // namespace

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  {
    StdoutToStderr quiet;
    NCCL_CHECK(ncclGetUniqueId(&id));
  }
  std::vector<uint8_t> v(sizeof(id));
  std::memcpy(v.data(), &id, sizeof(id));
  return v;
}

bool rccl_available() { return true; }

int64_t hip_release_errors() { return release_error_count().load(); }

std::string hip_pci_bus_id(int device) {
  char id[64] = {0};
  HIP_CHECK(hipDeviceGetPCIBusId(id, int(sizeof(id)), device));
  return id;
}

// Device UUID (hipDeviceGetUuid) as 32 hex digits: names one physical GPU or
// partition across processes, whatever HIP_VISIBLE_DEVICES / the process-
// local ordinal make of it.
std::string hip_uuid(int device) {
  hipUUID u{};
  HIP_CHECK(hipDeviceGetUuid(&u, device));
  static const char* hex = "0123456789abcdef";
  std::string s;
  for (unsigned char c : u.bytes) {
    s.push_back(hex[c >> 4]);
    s.push_back(hex[c & 15]);
  }
  return s;
}

std::unique_ptr<Transport> make_rccl_transport(const std::vector<uint8_t>& uid, int rank, int nranks,
                                               int device, const Tuning& tune) {
  return std::make_unique<RcclTransport>(uid, rank, nranks, device, tune);
}

}  // namespace gol
