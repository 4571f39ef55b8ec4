// Microbenchmark: can a HIP graph carry the linked-launch pattern of the
// small tiles (consecutive launches alternating between two streams, each
// ordered after an event recorded just before the previous launch, the data
// order kept by completion counters), and what does the host pay per launch?
//
//   ubench_graph_link [K launches] [workgroups] [spin us] [replays]
//
// Each launch has G workgroups of 512 threads; every workgroup of launch b
// first waits until all G workgroups of launch b-1 have bumped counter[b-1]
// (bounded: a timeout sets an error word instead of hanging), spins for the
// given time on s_memrealtime, then bumps counter[b].  Two fit on the GPU at
// once (G <= 256 on 256 CUs), as the engine's fit rule demands.
//   streams: K launches enqueued per run (hipEventRecord + hipStreamWaitEvent
//            + launch), the engine's pattern;
//   graph:   the same sequence captured once from the two streams (cross-
//            stream capture through the events), replayed; a memset node
//            resets the counters at the start of each replay.
// Reported: host microseconds per launch to enqueue, device microseconds per
// launch (events around the whole run), and the device time of K launches
// on one stream with no overlap at all, for reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ void __launch_bounds__(512) linked_spin(unsigned* counters, int b, unsigned G, unsigned spin_ticks,
                                                   unsigned* err) {
  if (b > 0) {
    if (threadIdx.x == 0) {
      unsigned seen = 0;
      for (int i = 0; i < (1 << 15); ++i) {  // bounded: ~30-60 ms
        seen = __hip_atomic_load(counters + b - 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (seen >= G) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if (seen < G) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
  }
  // s_memrealtime ticks at 100 MHz.
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(counters + b, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

struct Run {
  double host_us, dev_us;
};

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 32;
  const unsigned G = argc > 2 ? unsigned(std::atoi(argv[2])) : 255;
  const double spin_us = argc > 3 ? std::atof(argv[3]) : 8.0;
  const int R = argc > 4 ? std::atoi(argv[4]) : 20;
  const unsigned ticks = unsigned(spin_us * 100.0);
  if (K < 2 || K > 1024 || G < 1 || G > 256 || R < 1) {
    std::fprintf(stderr, "bad arguments\n");
    return 2;
  }
  unsigned *counters = nullptr, *err = nullptr;
  CK(hipMalloc(&counters, size_t(K) * sizeof(unsigned)));
  CK(hipHostMalloc(reinterpret_cast<void**>(&err), sizeof(unsigned), hipHostMallocMapped));
  *err = 0;
  unsigned* err_dev = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev), err, 0));
  hipStream_t s[2];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t before[2], t0, t1, joinev;
  for (auto& e : before) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&joinev, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));

  // The engine's enqueue pattern (lb::launch_linked with events).
  auto enqueue = [&]() {
    CK(hipMemsetAsync(counters, 0, size_t(K) * sizeof(unsigned), s[0]));
    int cur = 0;
    for (int b = 0; b < K; ++b) {
      const int which = b == 0 ? 0 : 1 - cur;
      if (b > 0) CK(hipStreamWaitEvent(s[which], before[cur], 0));
      CK(hipEventRecord(before[which], s[which]));
      hipLaunchKernelGGL(linked_spin, dim3(G), dim3(512), 0, s[which], counters, b, G, ticks, err_dev);
      cur = which;
    }
    CK(hipEventRecord(joinev, s[1]));  // join: s[0] after s[1]
    CK(hipStreamWaitEvent(s[0], joinev, 0));
  };
  auto timed = [&](auto&& body) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(t0, s[0]));
    const auto h0 = std::chrono::steady_clock::now();
    body();
    const auto h1 = std::chrono::steady_clock::now();
    CK(hipEventRecord(t1, s[0]));
    CK(hipEventSynchronize(t1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t0, t1));
    return Run{std::chrono::duration<double, std::micro>(h1 - h0).count(), ms * 1e3};
  };

  // Reference: one stream, every launch after the previous one's end.
  auto serial = [&]() {
    CK(hipMemsetAsync(counters, 0, size_t(K) * sizeof(unsigned), s[0]));
    for (int b = 0; b < K; ++b)
      hipLaunchKernelGGL(linked_spin, dim3(G), dim3(512), 0, s[0], counters, b, G, ticks, err_dev);
  };
  auto say = [&](const char* what) {
    std::fprintf(stderr, "[ubench_graph_link] %s (error word %u)\n", what, *err);
    std::fflush(stderr);
  };
  say("start");
  timed(serial);
  say("serial warm-up done");
  timed(enqueue);  // warm up
  say("two-stream warm-up done");
  std::vector<Run> rs, rl, rg;
  for (int r = 0; r < R; ++r) rs.push_back(timed(serial));
  for (int r = 0; r < R; ++r) rl.push_back(timed(enqueue));

  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
  enqueue();
  CK(hipStreamEndCapture(s[0], &g));
  size_t nodes = 0;
  CK(hipGraphGetNodes(g, nullptr, &nodes));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  say("graph instantiated");
  timed([&]() { CK(hipGraphLaunch(ge, s[0])); });  // warm up
  say("graph warm-up done");
  for (int r = 0; r < R; ++r) rg.push_back(timed([&]() { CK(hipGraphLaunch(ge, s[0])); }));

  auto med = [](std::vector<Run> v, bool host) {
    std::vector<double> x;
    for (auto& r : v) x.push_back(host ? r.host_us : r.dev_us);
    std::sort(x.begin(), x.end());
    return x[x.size() / 2];
  };
  std::printf("K=%d launches, %u workgroups x 512 threads, %.1f us spin each, %d runs (medians); graph nodes %zu\n",
              K, G, spin_us, R, nodes);
  std::printf("  one stream, serial      : host %6.2f us/launch, device %7.2f us/launch\n", med(rs, true) / K,
              med(rs, false) / K);
  std::printf("  two streams + events    : host %6.2f us/launch, device %7.2f us/launch\n", med(rl, true) / K,
              med(rl, false) / K);
  std::printf("  graph of the same       : host %6.2f us/launch, device %7.2f us/launch\n", med(rg, true) / K,
              med(rg, false) / K);
  std::printf("  error word %u (1: a launch waited too long for its predecessor)\n", *err);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return *err ? 3 : 0;
}
