// HIP-side helpers shared by the HIP translation units (backend, RCCL
// transport): the error check and the device scope.  Reference: the
// cudaSafeCall macro (src/game_cuda.cu:18-27) prints the error and exits;
// here a failing call throws gol::Error with file, line, call and HIP's
// error string.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

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

}  // namespace gol
