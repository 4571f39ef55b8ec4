// Host cost of the launch patterns the engine uses, on MI355X: a ~256-byte
// kernel argument block (like LifeBlockParams), launched back to back
//   A  on one stream;
//   B  alternating two non-blocking streams, each launch preceded by an event
//      recorded on the other stream and a stream wait on it (linked launches,
//      life_block_launch.hpp launch_linked);
//   C  alternating two streams without events;
//   D  like B but the event recorded on the launch's own stream after it.
// For each: host microseconds per launch (enqueue loop only) and device
// microseconds per launch (loop + drain), for an empty kernel and a ~10 us one.
//   hipcc --offload-arch=gfx950 -O3 csrc/tools/ubench_launch.hip -o bin/ubench_launch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP %s at line %d\n", hipGetErrorString(e_), __LINE__);    \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

struct Params {
  uint64_t v[32];  // 256 bytes of kernel arguments
};

__global__ void busy(Params p, uint32_t* out, int spins) {
  uint32_t x = uint32_t(p.v[threadIdx.x & 31]) + threadIdx.x;
  for (int i = 0; i < spins; ++i) x = x * 1664525u + 1013904223u;
  if (x == 0x12345678u) out[blockIdx.x] = x;  // keeps the loop
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  hipStream_t s[2];
  hipEvent_t ev[2];
  for (int i = 0; i < 2; ++i) {
    CHK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
    CHK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  }
  uint32_t* out;
  CHK(hipMalloc(&out, 1 << 20));
  Params p{};
  for (int i = 0; i < 32; ++i) p.v[i] = i;
  const char* names[] = {"A one stream", "B two streams + record/wait", "C two streams, no events",
                         "D two streams + record after"};
  for (int spins : {0, 4000}) {
    for (int pat = 0; pat < 4; ++pat) {
      for (int rep = 0; rep < 2; ++rep) {  // first pass warms up
        CHK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; ++i) {
          const int w = pat == 0 ? 0 : (i & 1);
          if (pat == 1) {
            CHK(hipEventRecord(ev[1 - w], s[1 - w]));
            CHK(hipStreamWaitEvent(s[w], ev[1 - w], 0));
          }
          hipLaunchKernelGGL(busy, dim3(512), dim3(256), 0, s[w], p, out, spins);
          if (pat == 3) {
            CHK(hipEventRecord(ev[w], s[w]));
            CHK(hipStreamWaitEvent(s[1 - w], ev[w], 0));
          }
        }
        const auto t1 = std::chrono::steady_clock::now();
        CHK(hipDeviceSynchronize());
        const auto t2 = std::chrono::steady_clock::now();
        if (rep == 1)
          std::printf("%-30s spins %5d: host %6.2f us/launch, device %6.2f us/launch\n", names[pat], spins,
                      std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                      std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
      }
    }
  }
  CHK(hipFree(out));
  return 0;
}
