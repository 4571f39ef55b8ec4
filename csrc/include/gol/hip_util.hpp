// HIP-side helpers shared by the HIP translation units (backend, RCCL
// transport): the error check and the device scope.  Reference: the
// cudaSafeCall macro (src/game_cuda.cu:18-27) prints the error and exits;
// here a failing call throws gol::Error with file, line, call and HIP's
// error string.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "gol/common.hpp"

#define HIP_CHECK(expr)                                                                     \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      ::gol::fail(std::string("HIP error in ") + __FILE__ + ":" + std::to_string(__LINE__) + \
                  " (" #expr "): " + hipGetErrorString(e_));                                \
  } while (0)

namespace gol {

// `dev` is the current device for the extent of the scope; the caller's
// device is restored after it.  Every entry point of a per-device object
// (HipBackend, RcclTransport) that allocates, creates streams or events,
// enqueues work or waits opens one: the rank threads of a single-process
// multi-GPU run (bin/gol --gpus N, InProcessGroup(devices=...)) start on
// device 0, and Python threads on whatever torch selected last.  The
// reference owns its buffers one process per rank (src/game_mpi.c:192-197);
// here any thread may drive any rank's objects.
class DeviceScope {
 public:
  explicit DeviceScope(int dev) : dev_(dev) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    if (prev_ != dev_) HIP_CHECK(hipSetDevice(dev_));
  }
  ~DeviceScope() {
    if (prev_ >= 0 && prev_ != dev_) (void)hipSetDevice(prev_);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;

 private:
  int dev_, prev_ = -1;
};

// Release paths (destructors, frees) cannot throw, so they ignore their calls'
// results - but HIP keeps a failed call's error as the thread's last error,
// and the next launch check (HIP_CHECK(hipGetLastError()) after a kernel
// launch), in another object and much later, would report it as its own
// (with Python's garbage collector deciding when a release runs, at a
// different place on every run).  Release paths end with this: a failure is
// reported on stderr under the release's name and cleared.  `quiet` clears
// without a report: third-party setup and teardown (RCCL's), whose own
// results are checked, may leave errors of internal probes behind.
// The reported ones are counted (hip_release_errors(), tests/conftest.py
// prints the count of a GPU test session).
inline std::atomic<int64_t>& release_error_count() {
  static std::atomic<int64_t> n{0};
  return n;
}
inline void clear_release_error(const char* where, bool quiet = false) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess && !quiet) {
    ++release_error_count();
    std::fprintf(stderr, "gol: %s: ignored HIP error: %s\n", where, hipGetErrorString(e));
  }
}

// CU partition of this process on its device (tuning cu_partition = "k/n":
// the k-th of n equal, disjoint slices of the CUs).  Ranks that share one GPU
// in a rehearsal (bench.py --share-gpus) each take a slice, so each rank's
// kernels - its own and the RCCL kernels it enqueues on its streams - run on
// CUs of their own, as on a node where every rank owns a GPU, and the
// backend plans its launches for the slice.  Empty mask: the whole device.
inline std::vector<uint32_t> cu_partition_mask(const std::string& spec, int cus) {
  if (spec.empty()) return {};
  int k = -1, n = 0;
  if (std::sscanf(spec.c_str(), "%d/%d", &k, &n) != 2 || n < 1 || k < 0 || k >= n || n > cus)
    fail("tuning cu_partition=" + spec + ": expected k/n with 0 <= k < n <= " + std::to_string(cus));
  std::vector<uint32_t> m(size_t((cus + 31) / 32), 0u);
  for (int c = int(int64_t(k) * cus / n); c < int(int64_t(k + 1) * cus / n); ++c) m[size_t(c / 32)] |= 1u << (c % 32);
  return m;
}
inline int mask_cus(const std::vector<uint32_t>& m) {
  int c = 0;
  for (uint32_t w : m) c += __builtin_popcount(w);
  return c;
}
// A stream for `dev`'s work: non-blocking, or restricted to the CU partition
// `cu_partition` when it names one (HIP's CU-masked streams).  `own_queue`:
// CU-masked to the whole device when no partition is named - HIP gives a
// CU-masked stream a hardware queue of its own instead of one from the
// process's shared pool.
inline hipStream_t make_stream(int dev, const std::string& cu_partition, bool own_queue = false) {
  hipDeviceProp_t prop;
  HIP_CHECK(hipGetDeviceProperties(&prop, dev));
  std::vector<uint32_t> m = cu_partition_mask(cu_partition, prop.multiProcessorCount);
  if (m.empty() && own_queue) m = cu_partition_mask("0/1", prop.multiProcessorCount);
  hipStream_t s = nullptr;
  if (m.empty())
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  else
    HIP_CHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(m.size()), m.data()));
  return s;
}

}  // namespace gol
