// HIP backend: device memory, one non-blocking stream, CDNA4 kernels.
//
// Reference runtime pattern (src/game_cuda.cu:185-276): cudaMalloc of
// (W+2)(H+2) bytes computed in int, cudaMemcpy of the whole grid, and a
// cudaDeviceSynchronize after every kernel.  Here every call is enqueued on
// the backend's stream and only the engine's periodic flag poll and the
// final copy-out block the host.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../kernels/life_kernels.hpp"
#include "gol/backend.hpp"
#include "gol/hip_util.hpp"
#include "gol/numa.hpp"
#include "gol/trace.hpp"

namespace gol {
namespace {

// Tuning check_device=1 (GOL_CHECK_DEVICE): every entry point asserts that its device is current,
// and every buffer the backend allocates or a launch touches is checked to
// live on that device (hipPointerGetAttributes).
#define GOL_ON_DEVICE()              \
  DeviceScope device_scope_(dev_);   \
  if (check_dev_) assert_current(__func__)

class HipBackend final : public Backend {
 public:
  HipBackend(int device, const Tuning& t) : Backend(t), dev_(device) {
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    GOL_REQUIRE(n > 0, "no HIP device available");
    GOL_REQUIRE(device >= 0 && device < n, "HIP device index out of range");
    check_dev_ = t.on("check_device");
    ring_on_ = t.on("row_ring");
    GOL_ON_DEVICE();
    // Tuning link_queue: -1 (default) the second linked stream gets a
    // hardware queue of its own when another backend already lives on this
    // device in this process, 1 always, 2 both linked streams, 0 never.
    const int lq = t.i("link_queue");
    GOL_REQUIRE(lq >= -1 && lq <= 2, "tuning link_queue: -1, 0, 1 or 2");
    const bool shared_dev = live_backends(dev_).fetch_add(1) > 0;
    stream_ = make_stream(dev_, tuning_.s("cu_partition"), lq >= 2);
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, dev_));
    arch_ = prop.gcnArchName;
    cus_ = prop.multiProcessorCount;
    // The process's host threads on this GPU's NUMA node (gol/numa.hpp).
    if (t.i("numa_pin") > 0) {
      char bus[64] = {0};
      if (hipDeviceGetPCIBusId(bus, int(sizeof(bus)), dev_) == hipSuccess)
        numa_ = pin_process_to_numa(bus, t.i("numa_pin") == 2 && t.s("cu_partition").empty());
      cpu_set_t s;
      if (numa_ >= 0 && sched_getaffinity(0, sizeof(s), &s) == 0) numa_cpus_ = CPU_COUNT(&s);
    }
    // A CU partition (tuning cu_partition, ranks sharing a GPU): every stream
    // of this backend runs on the slice, and launches are planned for it.
    if (const int part = mask_cus(cu_partition_mask(t.s("cu_partition"), cus_))) {
      cu_part_ = " cu-partition=" + t.s("cu_partition") + ":" + std::to_string(part) + "CUs";
      cus_ = part;
    }
    tune_.cus = cus_;
    tune_.target_waves = t.i("target_waves");
    tune_.min_seg_rows = t.i("min_seg_rows");
    tune_.xlane = t.i("xlane");
    GOL_REQUIRE(tune_.xlane == hipk::kXlaneAuto || tune_.xlane == hipk::kXlaneDpp || tune_.xlane == hipk::kXlaneAdd,
                "tuning xlane: -1 (auto), 0 (DPP window) or 3 (adder window)");
    tune_.u8_lds = t.s("u8_kernel") == "lds";
    GOL_REQUIRE(tune_.u8_lds || t.s("u8_kernel") == "auto", "tuning u8_kernel: auto or lds");
    tune_.lds_rows = t.i("lds_rows");
    tune_.lds_pack = t.on("lds_pack");
    tune_.lds_xcd = t.on("lds_xcd");
    tune_.lds_waves = t.i("lds_waves");
    GOL_REQUIRE(tune_.lds_waves == 0 || tune_.lds_waves == 8 || tune_.lds_waves == 16, "tuning lds_waves: 0, 8 or 16");
    // 8192^2 per generation: bytes T = 1 26.6, 2 24.9, 4 20.4, 8 17.9 us; packed T = 8 6.5, 16 4.9, 32 4.7
    tune_.lds_T = t.i("lds_t") > 0 ? t.i("lds_t") : tune_.lds_pack ? 32 : 8;
    GOL_REQUIRE(tune_.lds_T == 1 || tune_.lds_T == 2 || tune_.lds_T == 4 || tune_.lds_T == 8 ||
                    (tune_.lds_pack && (tune_.lds_T == 16 || tune_.lds_T == 32)),
                "tuning lds_t must be 1, 2, 4 or 8 (16 or 32 with the packed tile, lds_pack=1)");
    tune_.group = t.i("group");  // grouped schedule (life_group_impl.hpp)
    tune_.group_small = !t.is_default("group") && t.is_default("group_small") ? tune_.group : t.i("group_small");
    tune_.wrap = t.on("wrap");
    tune_.fold = t.on("fold");
    chain_mode_ = t.i("chain");
    GOL_REQUIRE(chain_mode_ >= -1 && chain_mode_ <= 1, "tuning chain: -1, 0 or 1");
    // Linked launches: consecutive grouped launches of an epoch overlap on
    // two streams, ordered by per-group completion words (LifeBlockParams::
    // link_*): small tiles whose launches alone hold only 2 waves per SIMD.
    // Tuning link: 1 every eligible launch, 0 never, -1 (default) where the
    // engine passes KernelChoice::link (small single-rank ring tiles).
    link_mode_ = t.i("link");
    link_on_ = link_mode_ > 0;
    if (link_mode_ != 0) {
      link_.stream[0] = stream_;
      // A queue of its own (tuning link_queue): from HIP's pool of
      // GPU_MAX_HW_QUEUES queues a later backend's second stream can share one
      // with its first, and linked launches on one queue serialise (8192^2
      // 2.68 vs 1.47 ms).  Not for a process's only backend: there the
      // CU-masked queue measured the same on single-rank tiles but made the
      // rehearsed rank tile's side-stream polls 2x slower
      // (profiles/r06/link_queue/).
      link_.stream[1] = make_stream(dev_, tuning_.s("cu_partition"), lq >= 1 || (lq < 0 && shared_dev));
      for (auto& e : link_.before) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // A GPU shared by several processes (a CU partition) time-slices their
    // queues, so a producer workgroup can be switched out for longer than a
    // bounded cross-workgroup wait: no chained groups or linked launches there
    // (a rank tile's launch does not fit its slice twice anyway).
    if (!cu_part_.empty()) {
      chain_mode_ = 0;
      link_mode_ = 0;
      link_on_ = false;
    }
    tune_.chain = chain_mode_ < 0 ? 0 : chain_mode_;
    tune_.fault_delay = std::max(0, std::min(4096, t.i("fault_delay_spins")));
    tune_log_ = t.on("tune_log");
    trigger_ok_ = link_mode_ != 0;  // armed only on linked launches
    tune_.chain_seq = &chain_seq_;
    // which: 0 chain flags, 1 chain slots, 2..4 linked-launch completion words
    // (zeroed when allocated: flags and words are compared with sequence
    // numbers).
    tune_.chain_mem = [this](int which, size_t n) -> uint32_t* {
      void*& buf = chain_[which];
      size_t& cap = chain_bytes_[which];
      if (n > cap) {
        GOL_ON_DEVICE();
        HIP_CHECK(hipStreamSynchronize(stream_));  // earlier launches may still use it
        if (link_.stream[1]) HIP_CHECK(hipStreamSynchronize(link_.stream[1]));
        if (buf) HIP_CHECK(hipFree(buf));
        HIP_CHECK(hipMalloc(&buf, n));
        if (which != 1) HIP_CHECK(hipMemsetAsync(buf, 0, n, stream_));  // ordered before the launch on stream_
        cap = n;
      }
      if (check_dev_) check_ptr(buf, which == 0 ? "chain flags" : which == 1 ? "chain slots" : "link words");
      return static_cast<uint32_t*>(buf);
    };
    if (split_trace(t.s("wg_trace"), &trace_at_, &trace_path_)) {
      // "N:path:pair": launches N and N + 1, left linked (overlap evidence).
      const size_t c2 = trace_path_.rfind(":pair");
      if (c2 != std::string::npos && c2 + 5 == trace_path_.size()) {
        trace_pair_ = true;
        trace_path_ = trace_path_.substr(0, c2);
      }
    }
    // Kernel error word: fine-grained pinned host memory the kernels write
    // through its device alias and the host reads without a copy.
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_host_), 4 * sizeof(uint32_t), hipHostMallocMapped));
    for (int i = 0; i < 4; ++i) err_host_[i] = 0;
    tune_.chain_spin_log2 = std::min(24, std::max(4, t.i("chain_spin")));
    HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&tune_.err), err_host_, 0));
  }
  static std::atomic<int>& live_backends(int dev) {
    static std::atomic<int> n[64];
    return n[dev & 63];
  }
  ~HipBackend() override {
    live_backends(dev_).fetch_sub(1);
    if (prof_on_ && prof_n_ > 0)
      std::fprintf(stderr, "gol host profile: %lld blocks; per block: engine between blocks %.2f us, run_block %.2f us "
                   "(launch call %.2f us)\n", (long long)prof_n_, prof_gap_ / double(std::max<int64_t>(1, prof_n_ - 1)),
                   prof_in_ / double(prof_n_), prof_launch_ / double(prof_n_));
    DeviceScope device_scope(dev_);
    // Every stream drains before any ring is unmapped: linked launches on
    // link_.stream[1] and transport work on comm_ may still use the rings.
    if (stream_) hipStreamSynchronize(stream_);
    if (link_.stream[1]) hipStreamSynchronize(link_.stream[1]);
    if (comm_) hipStreamSynchronize(comm_);
    for (auto& kv : rings_) release_ring(kv.second);
    if (stage_) hipFree(stage_);
    if (trigger_mem_) hipFree(trigger_mem_);
    for (void* c : chain_)
      if (c) hipFree(c);
    for (auto& p : pending_) {
      hipEventDestroy(p.e0);
      hipEventDestroy(p.e1);
    }
    for (hipEvent_t e : free_events_) hipEventDestroy(e);
    for (hipEvent_t e : timing_pool_) hipEventDestroy(e);
    if (err_host_) hipHostFree(err_host_);
    for (auto& e : tail_)
      if (e) hipEventDestroy(e);
    if (comm_) hipStreamDestroy(comm_);
    for (auto& e : link_.before)
      if (e) hipEventDestroy(e);
    if (link_.stream[1]) hipStreamDestroy(link_.stream[1]);
    if (stream_) hipStreamDestroy(stream_);
    clear_release_error("~HipBackend");
  }

  // Linked launches: everything on the second stream precedes what comes
  // next on the compute stream (every entry point but a linkable run_block).
  void join_streams() override {
    if (link_.stream[1]) {
      DeviceScope device_scope(dev_);
      hipk::link_join(link_);
    }
  }
  int64_t linked_launches() const override { return link_.linked; }
  std::string name() const override {
    hipk::LifeTuning t = tune_;
    t.chain = chain_mode_;
    const std::string numa = numa_ >= 0 ? " numa=" + std::to_string(numa_) + ":" + std::to_string(numa_cpus_) + "cpus" : "";
    return "hip:" + std::to_string(dev_) + ":" + arch_ + cu_part_ + numa + " [" + hipk::life_block_variant(Layout::Bits, t) +
           "; " + hipk::life_block_variant(Layout::U8, t) + "]";
  }
  int preferred_tmax(Layout l) const override { return hipk::life_block_max_T(l, tune_); }
  bool is_device() const override { return true; }
  int device() const override { return dev_; }
  void* stream() const override { return stream_; }

  void* alloc(size_t bytes) override {
    join_streams();
    GOL_ON_DEVICE();
    void* p = nullptr;
    HIP_CHECK(hipMalloc(&p, bytes ? bytes : 1));
    HIP_CHECK(hipMemsetAsync(p, 0, bytes ? bytes : 1, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    if (check_dev_) check_ptr(p, "alloc");
    return p;
  }
  void release(void* p) override {
    if (!p) return;
    join_streams();
    DeviceScope device_scope(dev_);
    hipStreamSynchronize(stream_);
    auto it = rings_.find(p);
    if (it != rings_.end()) {
      release_ring(it->second);
      rings_.erase(it);
    } else {
      hipFree(p);
    }
    clear_release_error("HipBackend::release");
  }
  // Row ring (Backend::row_ring_halo): three physical allocations A (first
  // Dv owned rows), B (the rest but the last Dv), C (last Dv), mapped as
  //   [C | A B C | A]
  // into one reserved virtual range (hipMemMap takes offset 0 only, so every
  // piece is a handle of its own).  The top halo is then the last owned rows
  // and the bottom halo the first ones: the single-rank torus never fills its
  // periodic row halos, and every temporal block runs over exactly the owned
  // rows (no trapezoid).  A kernel reads one buffer and writes the other, so
  // no launch reads an alias of what it writes.  GOL_ROW_RING=0: off.
  size_t ring_granularity() const {
    if (ring_gran_ == 0) {
      hipMemAllocationProp prop{};
      prop.type = hipMemAllocationTypePinned;
      prop.location.type = hipMemLocationTypeDevice;
      prop.location.id = dev_;
      size_t g = 0;
      if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityMinimum) != hipSuccess || g == 0) {
        (void)hipGetLastError();
        g = size_t(-1);  // unsupported
      }
      ring_gran_ = g;
    }
    return ring_gran_;
  }
  int row_ring_halo(int64_t H, int64_t pitch, int min_halo) const override {
    if (!ring_on_) return 0;
    const size_t gran = ring_granularity();
    if (gran == size_t(-1) || pitch <= 0) return 0;
    int64_t dv = std::max<int64_t>(1, min_halo);
    while ((dv * pitch) % int64_t(gran) != 0) {
      if (++dv > H) return 0;
    }
    if ((H * pitch) % int64_t(gran) != 0 || H < 2 * dv) return 0;
    return int(dv);
  }
  size_t mem_free() const override {
    DeviceScope device_scope(dev_);
    size_t fr = 0, total = 0;
    if (hipMemGetInfo(&fr, &total) != hipSuccess) {
      (void)hipGetLastError();
      return ~size_t(0);
    }
    return fr;
  }
  struct Ring {
    void* va = nullptr;
    size_t bytes = 0;
    hipMemGenericAllocationHandle_t h[3] = {};
    std::vector<std::pair<void*, size_t>> mapped;
  };
  // One attempt at a ring's mappings [C | A B C | A] (alloc_row_ring).
  uint8_t* map_ring(Ring& r, size_t halo, size_t owned, size_t gran) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev_;
    const size_t sizes[3] = {halo, owned - 2 * halo, halo};
    for (int i = 0; i < 3; ++i)
      if (sizes[i]) HIP_CHECK(hipMemCreate(&r.h[i], sizes[i], &prop, 0));
    HIP_CHECK(hipMemAddressReserve(&r.va, r.bytes, gran, nullptr, 0));
    auto* b = static_cast<uint8_t*>(r.va);
    const struct {
      size_t at;
      int piece;
    } maps[5] = {{0, 2}, {halo, 0}, {2 * halo, 1}, {owned, 2}, {owned + halo, 0}};
    for (const auto& m : maps) {
      if (!sizes[m.piece]) continue;
      HIP_CHECK(hipMemMap(b + m.at, sizes[m.piece], 0, r.h[m.piece], 0));
      r.mapped.push_back({b + m.at, sizes[m.piece]});
    }
    hipMemAccessDesc acc{};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = dev_;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    const hipError_t e = hipMemSetAccess(r.va, r.bytes, &acc, 1);
    if (e != hipSuccess)
      fail(std::string("row ring: hipMemSetAccess(") + std::to_string(r.bytes) + " bytes, granularity " +
           std::to_string(gran) + "): " + hipGetErrorString(e));
    HIP_CHECK(hipMemsetAsync(b + halo, 0, owned, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    return b;
  }
  void* alloc_row_ring(const TileGeom& g) override {
    if (!ring_on_) return nullptr;
    join_streams();
    GOL_ON_DEVICE();
    const size_t halo = size_t(g.Dv) * size_t(g.pitch), owned = size_t(g.H) * size_t(g.pitch);
    const size_t gran = ring_granularity();
    GOL_REQUIRE(gran != size_t(-1) && halo % gran == 0 && owned % gran == 0 && owned >= 2 * halo && halo > 0,
                "row ring: geometry does not fit the mapping granularity (Backend::row_ring_halo)");
    // A ring's address range is never mapped twice: bin/ring_stress (round
    // 6, profiles/r06/ring_stress.txt) maps 300 rings of mixed geometry with
    // allocation churn in between, and when an unmapped range is freed and
    // reserved again (hipMemAddressFree) or reused for the next ring, reads
    // through the new halo alias return the old pages' contents or zeros in
    // 210 resp. 224 of 300 rings - translations of the reused range are not
    // the new mapping - while with every range kept reserved all 300 alias
    // correctly.  So release_ring frees the memory and keeps the reservation
    // (address space only, 2 x (owned + 2 halo) bytes per engine), bounded
    // by kRingVaBudget: past it rings are refused and the engine falls back
    // to periodic fills, loudly (Engine::row_ring_fallback).  Setting access
    // mapping by mapping also fails on the first mapping of a doubly mapped
    // handle, hence one whole-range hipMemSetAccess; a failed attempt is
    // retried once on a new range.
    if (ring_va_held().load() + owned + 2 * halo > kRingVaBudget)
      fail("row ring: address space held by released rings (" + std::to_string(ring_va_held().load() >> 30) +
           " GiB) would pass the " + std::to_string(kRingVaBudget >> 40) + " TiB budget");
    Ring r;
    uint8_t* b = nullptr;
    for (int attempt = 0;; ++attempt) {
      r = Ring{};
      r.bytes = owned + 2 * halo;
      try {
        b = map_ring(r, halo, owned, gran);
        break;
      } catch (const std::exception& ex) {
        // A partial ring (out of memory or address space, or the above) gives
        // back its memory, so the engine's fallback to plain buffers has it.
        release_ring(r);
        (void)hipGetLastError();
        if (attempt > 0) throw;
        std::fprintf(stderr, "gol: row ring: %s; retrying on a new address range\n", ex.what());
      }
    }
    if (check_dev_) check_ptr(b + halo, "row ring");
    rings_[r.va] = r;
    return r.va;
  }
  void* alloc_host(size_t bytes) override {
    GOL_ON_DEVICE();
    void* p = nullptr;
    HIP_CHECK(hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault));
    return p;
  }
  void release_host(void* p) override {
    DeviceScope device_scope(dev_);
    if (p) hipHostFree(p);
    clear_release_error("HipBackend::release_host");
  }
  void memset_async(void* p, int v, size_t bytes) override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipMemsetAsync(p, v, bytes, stream_));
  }
  void copy_h2d(void* d, const void* s, size_t n) override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void copy_d2h(void* d, const void* s, size_t n) override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void copy_d2h_async_on(void* d, const void* s, size_t n, void* stream) override {
    if (!stream) join_streams();  // a side stream was ordered by its caller (poll_side)
    GOL_ON_DEVICE();
    HIP_CHECK(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, stream ? static_cast<hipStream_t>(stream) : stream_));
  }
  void copy_2d_async(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                     int64_t rows) override {
    if (rows <= 0 || width <= 0) return;
    GOL_ON_DEVICE();
    HIP_CHECK(hipMemcpy2DAsync(dst, size_t(dpitch), src, size_t(spitch), size_t(width), size_t(rows),
                               hipMemcpyDefault, stream_));
  }
  void synchronize() override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void synchronize_stream(void* s) override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipStreamSynchronize(s ? static_cast<hipStream_t>(s) : stream_));
  }
  void* event_record_on(void* stream) override {
    if (!stream) join_streams();
    GOL_ON_DEVICE();
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(e, stream ? static_cast<hipStream_t>(stream) : stream_));
    return e;
  }
  void event_wait(void* ev) override {
    GOL_ON_DEVICE();
    HIP_CHECK(hipEventSynchronize(static_cast<hipEvent_t>(ev)));
  }
  void event_destroy(void* ev) override {
    DeviceScope device_scope(dev_);
    hipEventDestroy(static_cast<hipEvent_t>(ev));
    clear_release_error("HipBackend::event_destroy");
  }
  bool event_query(void* ev) override {
    GOL_ON_DEVICE();
    const hipError_t e = hipEventQuery(static_cast<hipEvent_t>(ev));
    if (e == hipErrorNotReady) return false;
    HIP_CHECK(e);
    return true;
  }
  // Phase timing: timing-enabled events from a pool.
  void* timing_mark(void* stream) override {
    join_streams();
    GOL_ON_DEVICE();
    hipEvent_t e;
    if (timing_pool_.empty()) {
      HIP_CHECK(hipEventCreate(&e));
    } else {
      e = timing_pool_.back();
      timing_pool_.pop_back();
    }
    HIP_CHECK(hipEventRecord(e, stream ? static_cast<hipStream_t>(stream) : stream_));
    return e;
  }
  double timing_ms(void* a, void* b) override {
    GOL_ON_DEVICE();
    HIP_CHECK(hipEventSynchronize(static_cast<hipEvent_t>(b)));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, static_cast<hipEvent_t>(a), static_cast<hipEvent_t>(b)));
    return double(ms);
  }
  void timing_release(void* m) override {
    if (m) timing_pool_.push_back(static_cast<hipEvent_t>(m));
  }
  void bind_thread() override {
    HIP_CHECK(hipSetDevice(dev_));
    if (check_dev_) assert_current(__func__);
  }
  // Direct reads of another device's buffers (ThreadTransport across GPUs).
  void enable_peer(int peer) override {
    if (peer == dev_ || peer < 0) return;
    GOL_ON_DEVICE();
    int can = 0;
    HIP_CHECK(hipDeviceCanAccessPeer(&can, dev_, peer));
    GOL_REQUIRE(can, "device " + std::to_string(dev_) + " cannot access device " + std::to_string(peer) +
                         " (no peer access): the thread transport cannot copy between them; use --comm rccl");
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
      (void)hipGetLastError();
      return;
    }
    HIP_CHECK(e);
  }
  bool supports_graphs() const override { return true; }
  void capture_begin() override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    capturing_ = true;
  }
  void* capture_end() override {
    GOL_ON_DEVICE();
    hipGraph_t g = nullptr;
    capturing_ = false;
    HIP_CHECK(hipStreamEndCapture(stream_, &g));
    hipGraphExec_t exec = nullptr;
    HIP_CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
    return exec;
  }
  void graph_launch(void* g) override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipGraphLaunch(static_cast<hipGraphExec_t>(g), stream_));
  }
  void graph_destroy(void* g) override {
    DeviceScope device_scope(dev_);
    if (g) hipGraphExecDestroy(static_cast<hipGraphExec_t>(g));
    clear_release_error("HipBackend::graph_destroy");
  }
  void i64_async(int64_t* dev, int64_t v, bool add) override {
    join_streams();
    GOL_ON_DEVICE();
    hipk::launch_i64(dev, v, add, stream_);
    HIP_CHECK(hipGetLastError());
  }
  // Default priority: a high-priority stream (hipStreamCreateWithPriority)
  // made every epoch ~0.9 ms slower in the one-GPU RCCL rehearsal
  // (profiles/r02/rehearsal_overlap.jsonl).
  void* comm_stream() override {
    if (!comm_) {
      GOL_ON_DEVICE();
      comm_ = make_stream(dev_, tuning_.s("cu_partition"));
      if (check_dev_) {
        int d = -1;
        HIP_CHECK(hipStreamGetDevice(comm_, &d));
        GOL_REQUIRE(d == dev_, "GOL_CHECK_DEVICE: comm stream created on device " + std::to_string(d));
      }
    }
    return comm_;
  }
  // The comm stream, after the tails of both compute streams (no join: the
  // linked chain keeps its state).  Not inside a capture: polls are issued
  // between captured epochs.
  void* poll_side() override {
    hipStream_t side = static_cast<hipStream_t>(comm_stream());
    GOL_ON_DEVICE();
    const hipStream_t tails[2] = {stream_, link_.stream[1]};
    for (int i = 0; i < 2; ++i) {
      if (!tails[i]) continue;
      if (!tail_[i]) HIP_CHECK(hipEventCreateWithFlags(&tail_[i], hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(tail_[i], tails[i]));
      HIP_CHECK(hipStreamWaitEvent(side, tail_[i], 0));
    }
    return side;
  }
  // Boundary trigger (Backend::trigger_stream).  Armed when the trigger
  // launch ran linked on the second compute stream: the compute stream, whose
  // last work is the launch before it, waits for the boundary groups' count
  // (one sleeping wave, hipk::launch_wait_counter) and the link chain is left
  // intact, so the next launch on it - the next epoch's first
  // block, after the exchange - still links to the trigger launch.  Else a
  // join: the exchange follows the whole launch.
  void* trigger_stream(bool* armed) override {
    *armed = false;
    if (trigger_target_ && link_.stream[1] && link_.cur == 1 && link_.prev_valid) {
      GOL_ON_DEVICE();
      hipk::launch_wait_counter(trigger_counter(), trigger_target_, tune_.err, stream_);
      HIP_CHECK(hipGetLastError());
      link_.started = true;  // the next launch on this stream follows the trigger launch's start
      *armed = true;
    } else {
      join_streams();
    }
    trigger_target_ = 0;
    return stream_;
  }
  bool supports_trigger() const override { return trigger_ok_; }

  // GOL_HOST_PROFILE=1: host time per block, printed when the backend goes:
  // the engine between blocks, run_block itself, and its launch call.
  int run_block(const BlockArgs& a) override {
    if (!prof_on_) return run_block_impl(a);
    const auto t0 = std::chrono::steady_clock::now();
    if (prof_n_ > 0) prof_gap_ += std::chrono::duration<double, std::micro>(t0 - prof_exit_).count();
    const int r = run_block_impl(a);
    prof_exit_ = std::chrono::steady_clock::now();
    prof_in_ += std::chrono::duration<double, std::micro>(prof_exit_ - t0).count();
    ++prof_n_;
    return r;
  }
  int run_block_impl(const BlockArgs& a) {
    GOL_ON_DEVICE();
    if (check_dev_) {
      check_ptr(a.in, "run_block input");
      check_ptr(a.out, "run_block output");
    }
    const bool capturing = capturing_;  // capture_begin / capture_end (no query per launch)
    // A launch may join a linked chain only outside a capture, for the bit
    // layout; anything else first joins.
    const bool linkable =
        (link_on_ || (a.link && link_mode_ < 0)) && link_.stream[1] && !capturing && a.g.layout == Layout::Bits;
    if (!linkable) join_streams();
    tune_.link = linkable ? &link_ : nullptr;
    if (chain_mode_) {  // chained groups: own stream only, never inside a graph capture
      tune_.chain_ok = !capturing && !linkable;
    }
    if (trace_at_ >= 0 && trace_pair_ && (launches_ == trace_at_ || launches_ == trace_at_ + 1))
      return run_block_traced_pair(a, linkable);
    if (trace_at_ >= 0 && launches_ == trace_at_) {
      join_streams();
      tune_.link = nullptr;
      return run_block_traced(a);
    }
    ++launches_;
    hipStream_t s = stream_;
    // Boundary trigger: armed only if the launch runs linked (the grouped
    // kernel's publish path counts the boundary groups).
    trigger_target_ = 0;
    link_.bnd_n = 0;
    link_.bnd_req = (a.trigger || a.hot) && linkable && trigger_counter();
    link_.bnd_count_req = a.trigger;
    if (link_.bnd_req) {
      for (int i = 0; i < 4; ++i) link_.bnd_r[i] = a.trigger_rows[i];
      link_.bnd_count = trigger_counter();
    }
    Pending* timed = nullptr;
    if (chain_mode_ < 0 && !linkable) timed = autotune_chain(a);
    if (linkable) tune_.chain = 0;
    if (timed) HIP_CHECK(hipEventRecord(timed->e0, s));
    const auto l0 = prof_on_ ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
    const int drift = hipk::launch_life_block(a, tune_, s);
    if (prof_on_) prof_launch_ += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - l0).count();
    HIP_CHECK(hipGetLastError());
    if (timed) HIP_CHECK(hipEventRecord(timed->e1, s));
    if (a.trigger && link_.bnd_n > 0) {  // the linked kernel carries the counter
      trigger_total_ += uint64_t(link_.bnd_n);
      trigger_target_ = trigger_total_;
    }
    link_.bnd_req = false;
    return drift;
  }

  // Launch-shape autotuning of the chained groups (GOL_CHAIN=-1).  Chaining
  // changes nothing but the inside of a launch (same rows, same flags), so
  // every rank may decide for itself.  Per launch shape (layout, T, rows / 256,
  // row width, drift, whole width) the first kTrials launches of each
  // option are timed with events, alternating; the completed timings are
  // collected without blocking at later launches, and the shape keeps the
  // option whose median is >= 1 % faster (else the plain grouped kernel).
  // Measured: +2 % on the 8-GPU rank tile, -1...-12 % on other tiles
  // (docs/PERFORMANCE.md), so no static rule picks it well.
  static constexpr int kTrials = 3;
  using TuneKey = std::array<int64_t, 6>;
  struct TuneStats {
    std::vector<float> ms[2];
    int issued[2] = {0, 0};
    int pick = -1;
  };
  struct Pending {
    TuneKey key;
    int opt;
    hipEvent_t e0, e1;
  };
  Pending* autotune_chain(const BlockArgs& a) {
    collect_tuning();
    tune_.chain = 0;
    if (!tune_.chain_ok) return nullptr;
    const TuneKey key{int64_t(a.g.layout), a.T, (a.row_hi - a.row_lo) >> 8, a.g.Wp(), a.allow_drift,
                      a.full_width};
    TuneStats& st = tuned_[key];
    if (st.pick >= 0) {
      tune_.chain = st.pick;
      return nullptr;
    }
    const int opt = st.issued[0] <= st.issued[1] ? 0 : 1;
    if (st.issued[opt] >= kTrials) return nullptr;  // trials in flight: plain kernel, untimed
    ++st.issued[opt];
    tune_.chain = opt;
    Pending p{key, opt, event_take(), event_take()};
    pending_.push_back(p);
    return &pending_.back();
  }
  void collect_tuning() {
    while (!pending_.empty()) {
      Pending& p = pending_.front();
      const hipError_t q = hipEventQuery(p.e1);
      if (q == hipErrorNotReady) break;
      HIP_CHECK(q);
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, p.e0, p.e1));
      TuneStats& st = tuned_[p.key];
      st.ms[p.opt].push_back(ms);
      if (st.pick < 0 && int(st.ms[0].size()) >= kTrials && int(st.ms[1].size()) >= kTrials) {
        const auto median = [](std::vector<float> v) {
          std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
          return v[v.size() / 2];
        };
        const float m0 = median(st.ms[0]), m1 = median(st.ms[1]);
        st.pick = m1 < 0.99f * m0 ? 1 : 0;
        if (tune_log_)
          std::fprintf(stderr, "gol autotune: layout %d T %d rows~%lld x %lld words: plain %.1f us, chained %.1f us -> %s\n",
                       int(p.key[0]), int(p.key[1]), (long long)(p.key[2] << 8), (long long)p.key[3], 1e3 * m0,
                       1e3 * m1, st.pick ? "chained" : "plain");
      }
      free_events_.push_back(p.e0);
      free_events_.push_back(p.e1);
      pending_.pop_front();
    }
  }
  hipEvent_t event_take() {
    if (free_events_.empty()) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreate(&e));
      return e;
    }
    hipEvent_t e = free_events_.back();
    free_events_.pop_back();
    return e;
  }
  bool drifts(Layout l) const override {
    if (l == Layout::U8 && tune_.u8_lds) return false;  // the LDS-tiled byte kernels run the DPP window
    return tune_.xlane == hipk::kXlaneAdd;
  }
  // The adder window (kXlaneAdd) beats the DPP window only at four resident
  // waves per SIMD; its grouped kernel fits that at T = 12 (120 VGPRs) with
  // segments of at least 2T = 24 rows.  Measured (profiles/r02/adder_ab.jsonl),
  // per 1000 generations on one MI355X: 32768^2 12.8 -> 11.3 ms, 32768 x 16384
  // 6.9 -> 5.9 ms, 32768 x 8192 3.9 -> 3.4 ms; the 32768 x 4096 tile (8-GPU
  // split) cannot fill four waves per SIMD and stays on the DPP window
  // (2.40 ms vs 2.47 ms at T = 8).
  //
  // The byte layout is HBM-bound on large tiles (every T-generation pass
  // reads and writes the whole byte grid once: ~500 us per pass at 32768^2,
  // any T), so there it runs T = 32 (245 VGPRs) or 24 (210), still 2 waves
  // per SIMD: 32768^2 31.3 (T = 16) -> 21.4 (24) -> 17.7 (32) us per
  // generation, 65536^2 128 -> 83 -> 64, 32768 x 16384 16.0 -> 11.4 -> 10.4,
  // 32768 x 8192 8.1 -> 6.6 -> 6.3.  The deepest T whose 4T-row segments
  // give every SIMD one is taken; below that T = 16 (8192^2: 2.83 vs 3.03 at
  // 24; 32768 x 4096: 3.7-3.9 vs 4.4 at 24 and 4.9 at 32;
  // profiles/r02/u8_t24*.jsonl, u8_t32.jsonl).
  // (A T = 48 pass as level-pipelined wave pairs ran no faster than T = 32,
  // the byte kernels being VALU-bound: removed in round 6, HISTORY.md.)
  KernelChoice choose_kernel(Layout l, int64_t rows, int64_t cols, int tmax_req) const override {
    KernelChoice k{tmax_req > 0 ? tmax_req : preferred_tmax(l), false};
    if (l == Layout::U8 && tmax_req <= 0 && !tune_.u8_lds) {
      const int64_t strips = ceil_div(cols + 32 * 16, 62 * 32);
      k.tmax = 16;
      for (int64_t kT : {32, 24})
        if (strips * (rows / (4 * kT)) >= int64_t(4) * cus_) {
          k.tmax = int(kT);
          break;
        }
    }
    if (tune_.xlane == hipk::kXlaneAdd && !(l == Layout::U8 && tune_.u8_lds)) {
      k.drift = true;
      if (tmax_req <= 0) k.tmax = 12;
    } else if (tune_.xlane == hipk::kXlaneAuto && l == Layout::Bits && tune_.group != 0 &&
               (tmax_req <= 0 || tmax_req == 12)) {
      constexpr int64_t kT = 12;
      const int64_t strips = ceil_div(ceil_div(cols, 32) + 16, 63);  // + a deep halo's words
      if (strips * (rows / (2 * kT)) >= int64_t(16) * cus_) k = {int(kT), true};
    }
    // DPP window on a small tile: the deepest T whose 2T-row segments still
    // give every SIMD two waves; below two waves per SIMD a wave's level chain
    // runs exposed (8192^2: T = 16 2.39-2.41 ms per 1000 generations, 1 wave
    // per SIMD; T = 12 2.48-2.50; T = 8 2.05-2.08, 2 waves; T = 4 2.97 (twice
    // the launches); the 8-GPU rank tile 32768 x 4096 keeps T = 16 at 2 waves;
    // profiles/r04/small_grid_T_sweep.jsonl).
    if (!k.drift && tmax_req <= 0 && l == Layout::Bits && tune_.group != 0 && k.tmax == 16) {
      const int64_t strips = ceil_div(ceil_div(cols, 32) + 16, 63);
      for (int t : {16, 12, 8}) {
        k.tmax = t;
        if (strips * (rows / (2 * t)) >= int64_t(8) * cus_) break;
      }
      // Such tiles also link consecutive launches where each holds at least
      // 1.5 waves per SIMD: two launches then fill the SIMDs together (8192^2
      // 1.93 -> 1.60 ms per 1000 generations with the folded strip; the 8-GPU
      // rank tile 2.26 -> 2.24 single-rank, 2.44 -> 2.40 in the multi-rank
      // schedule; 4096^2, with 0.75 waves per SIMD, measured slower linked;
      // profiles/r04/linked_*.jsonl).  Launches too large to run two at once
      // are never linked (launch_linked).
      k.link = strips * (rows / (2 * k.tmax)) >= int64_t(6) * cus_;
    }
    return k;
  }
  bool wraps_columns(Layout l) const override { return tune_.wrap; }
  // The LDS-tiled byte kernels read rows modulo the torus too.
  bool wraps_rows(Layout l) const override { return tune_.wrap && l == Layout::U8 && tune_.u8_lds; }
  void rotate_cols(const void* src, void* dst, const TileGeom& g, int64_t shift) override {
    join_streams();
    GOL_ON_DEVICE();
    hipk::launch_rotate_cols(static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), g, shift, stream_);
    HIP_CHECK(hipGetLastError());
  }
  void convert_rows(const void* src, const TileGeom& gs, void* dst, const TileGeom& gd, int64_t i0,
                    int64_t n) override {
    join_streams();
    GOL_ON_DEVICE();
    hipk::launch_convert_rows(static_cast<const uint8_t*>(src), gs, static_cast<uint8_t*>(dst), gd, i0, n,
                              stream_);
    HIP_CHECK(hipGetLastError());
  }
  // GOL_WG_TRACE=<launch index>:<csv path>: one life_block launch records
  // where and when each of its waves ran (grouped kernel, LifeBlockParams::
  // wg_trace); scripts/wg_trace.py turns the CSV into a per-CU makespan view.
  int run_block_traced(const BlockArgs& a) {
    ++launches_;
    const size_t bytes = size_t(hipk::kWgTraceWaves) * 4 * sizeof(uint64_t);
    uint64_t* d = nullptr;
    HIP_CHECK(hipStreamSynchronize(stream_));
    HIP_CHECK(hipMalloc(&d, bytes));
    HIP_CHECK(hipMemsetAsync(d, 0, bytes, stream_));
    tune_.wg_trace = d;
    const int drift = hipk::launch_life_block(a, tune_, stream_);
    tune_.wg_trace = nullptr;
    HIP_CHECK(hipGetLastError());
    std::vector<uint64_t> h(size_t(hipk::kWgTraceWaves) * 4);
    HIP_CHECK(hipMemcpyAsync(h.data(), d, bytes, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    HIP_CHECK(hipFree(d));
    std::FILE* f = std::fopen(trace_path_.c_str(), "w");
    GOL_REQUIRE(f != nullptr, "GOL_WG_TRACE: cannot open " + trace_path_);
    std::fprintf(f, "block,wave,xcc_id,hw_id,t_start,t_end,T,rows\n");
    for (int64_t i = 0; i < hipk::kWgTraceWaves; ++i) {
      const uint64_t* r = &h[size_t(4 * i)];
      if (!(r[0] >> 63)) continue;
      std::fprintf(f, "%llu,%llu,%llu,%llu,%llu,%llu,%d,%lld\n", (unsigned long long)((r[0] & ~(1ull << 63)) >> 8),
                   (unsigned long long)(r[0] & 255), (unsigned long long)(r[1] >> 32),
                   (unsigned long long)(r[1] & 0xFFFFFFFFull), (unsigned long long)r[2], (unsigned long long)r[3],
                   a.T, (long long)(a.row_hi - a.row_lo));
    }
    std::fclose(f);
    return drift;
  }
  // GOL_WG_TRACE=N:path:pair: per-wave records of launches N and N + 1 with
  // the second one left linked to the first (scripts/wg_trace.py --pair
  // reports how far they overlapped).  Buffers are set up before launch N.
  int run_block_traced_pair(const BlockArgs& a, bool linkable) {
    const size_t bytes = size_t(hipk::kWgTraceWaves) * 4 * sizeof(uint64_t);
    const int which = int(launches_ - trace_at_);
    if (which == 0) {
      join_streams();
      HIP_CHECK(hipStreamSynchronize(stream_));
      for (auto& d : pair_trace_) {
        HIP_CHECK(hipMalloc(&d, bytes));
        HIP_CHECK(hipMemsetAsync(d, 0, bytes, stream_));
      }
      HIP_CHECK(hipStreamSynchronize(stream_));
      pair_T_ = a.T;
    }
    ++launches_;
    hipStream_t s = stream_;
    if (linkable) tune_.chain = 0;
    tune_.wg_trace = pair_trace_[which];
    const int drift = hipk::launch_life_block(a, tune_, s);
    tune_.wg_trace = nullptr;
    HIP_CHECK(hipGetLastError());
    if (which == 1) {
      join_streams();
      HIP_CHECK(hipStreamSynchronize(stream_));
      std::FILE* f = std::fopen(trace_path_.c_str(), "w");
      GOL_REQUIRE(f != nullptr, "GOL_WG_TRACE: cannot open " + trace_path_);
      std::fprintf(f, "launch,block,wave,xcc_id,hw_id,t_start,t_end,T,linked\n");
      std::vector<uint64_t> h(size_t(hipk::kWgTraceWaves) * 4);
      for (int l = 0; l < 2; ++l) {
        HIP_CHECK(hipMemcpy(h.data(), pair_trace_[l], bytes, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < hipk::kWgTraceWaves; ++i) {
          const uint64_t* r = &h[size_t(4 * i)];
          if (!(r[0] >> 63)) continue;
          std::fprintf(f, "%d,%llu,%llu,%llu,%llu,%llu,%llu,%d,%d\n", l,
                       (unsigned long long)((r[0] & ~(1ull << 63)) >> 8), (unsigned long long)(r[0] & 255),
                       (unsigned long long)(r[1] >> 32), (unsigned long long)(r[1] & 0xFFFFFFFFull),
                       (unsigned long long)r[2], (unsigned long long)r[3], l ? a.T : pair_T_, int(linkable));
        }
        HIP_CHECK(hipFree(pair_trace_[l]));
        pair_trace_[l] = nullptr;
      }
      std::fclose(f);
    }
    return drift;
  }
  void check_device_errors() override {
    const uint32_t e = __atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
    if (e != 0) {
      *err_host_ = 0;
      const std::string diag = e == 2 ? " [flag " + std::to_string(err_host_[3]) + " read " +
                                            std::to_string(err_host_[1]) + ", expected " +
                                            std::to_string(err_host_[2]) + "]"
                                      : "";
      fail(std::string(e == 2   ? "life_group kernel (chained groups): a wave gave up waiting for the group below" + diag
                       : e == 3 ? "life_group kernel (linked launches): a group gave up waiting for the previous "
                                  "launch's rows"
                       : e == 7 ? "boundary trigger: the exchange's wait gave up on the boundary groups' count"
                                : "life_block kernel: unknown device error") +
           " (device error word " + std::to_string(e) + "); the rows of that launch are invalid");
    }
  }
  void fill_periodic(void* buf, const TileGeom& g, bool cols, bool rows) override {
    join_streams();
    GOL_ON_DEVICE();
    auto* p = static_cast<uint8_t*>(buf);
    if (!(cols && rows && hipk::launch_fill_all(p, g, stream_))) {
      if (cols) hipk::launch_fill_cols(p, g, stream_);
      if (rows) hipk::launch_fill_rows(p, g, stream_);
    }
    HIP_CHECK(hipGetLastError());
  }
  void fill_cols_rows(void* buf, const TileGeom& g, int64_t r0, int64_t n, void* stream) override {
    join_streams();
    GOL_ON_DEVICE();
    hipk::launch_fill_cols_rows(static_cast<uint8_t*>(buf), g, r0, n, stream ? static_cast<hipStream_t>(stream) : stream_);
    HIP_CHECK(hipGetLastError());
  }
  void alive_any(const void* buf, const TileGeom& g, uint32_t* flag) override {
    join_streams();
    GOL_ON_DEVICE();
    HIP_CHECK(hipMemsetAsync(flag, 0, 4, stream_));
    hipk::launch_alive(static_cast<const uint8_t*>(buf), g, flag, nullptr, stream_);
    HIP_CHECK(hipGetLastError());
  }
  int64_t alive_count(const void* buf, const TileGeom& g) override {
    join_streams();
    GOL_ON_DEVICE();
    unsigned long long* d = nullptr;
    HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&d), 8, stream_));
    HIP_CHECK(hipMemsetAsync(d, 0, 8, stream_));
    hipk::launch_alive(static_cast<const uint8_t*>(buf), g, nullptr, d, stream_);
    HIP_CHECK(hipGetLastError());
    unsigned long long h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipFreeAsync(d, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    return int64_t(h);
  }

  // Host <-> tile transfers go through a bounded device staging buffer so a
  // 32768^2 (1 GiB) or larger grid never needs a second full-size copy.
  void load_owned(void* buf, const TileGeom& g, const uint8_t* cells, int64_t ld) override {
    join_streams();
    GOL_ON_DEVICE();
    const int64_t chunk = rows_per_chunk(g);
    uint8_t* stage = static_cast<uint8_t*>(stage_buf(chunk * g.W));
    for (int64_t r = 0; r < g.H; r += chunk) {
      const int64_t n = std::min(chunk, g.H - r);
      HIP_CHECK(hipMemcpy2DAsync(stage, size_t(g.W), cells + r * ld, size_t(ld), size_t(g.W), size_t(n),
                                 hipMemcpyHostToDevice, stream_));
      hipk::launch_load_rows(static_cast<uint8_t*>(buf), g, stage, g.W, r, n, stream_);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
  }
  void store_owned(const void* buf, const TileGeom& g, uint8_t* cells, int64_t ld, bool ascii) override {
    join_streams();
    GOL_ON_DEVICE();
    const int64_t chunk = rows_per_chunk(g);
    uint8_t* stage = static_cast<uint8_t*>(stage_buf(chunk * g.W));
    for (int64_t r = 0; r < g.H; r += chunk) {
      const int64_t n = std::min(chunk, g.H - r);
      hipk::launch_store_rows(static_cast<const uint8_t*>(buf), g, stage, g.W, r, n, ascii, stream_);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpy2DAsync(cells + r * ld, size_t(ld), stage, size_t(g.W), size_t(g.W), size_t(n),
                                 hipMemcpyDeviceToHost, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
  }
  void init_random(void* buf, const TileGeom& g, uint64_t seed, double density, int64_t grow0,
                   int64_t gcol0) override {
    join_streams();
    GOL_ON_DEVICE();
    hipk::launch_init_random(static_cast<uint8_t*>(buf), g, seed, density_thresh(density), grow0, gcol0,
                             stream_);
    HIP_CHECK(hipGetLastError());
  }

 private:
  void release_ring(Ring& r) {
    for (auto& m : r.mapped)
      if (hipMemUnmap(m.first, m.second) != hipSuccess) clear_release_error("row ring: hipMemUnmap");
    r.mapped.clear();
    if (r.va) ring_va_held() += r.bytes;
    r.va = nullptr;  // the reservation is kept (alloc_row_ring): address space only
    for (auto& h : r.h) {
      if (h && hipMemRelease(h) != hipSuccess) clear_release_error("row ring: hipMemRelease");
      h = {};
    }
  }
  // Trace settings "N:path": launch N's trace goes to path.
  static bool split_trace(const std::string& v, int64_t* at, std::string* path) {
    const size_t c = v.find(':');
    if (c == std::string::npos) return false;
    *at = std::atoll(v.substr(0, c).c_str());
    *path = v.substr(c + 1);
    return true;
  }
  int64_t rows_per_chunk(const TileGeom& g) const {
    const int64_t budget = int64_t(256) << 20;
    return std::max<int64_t>(1, std::min<int64_t>(g.H, budget / std::max<int64_t>(1, g.W)));
  }
  void* stage_buf(int64_t bytes) {
    if (bytes > stage_bytes_) {
      if (stage_) {
        HIP_CHECK(hipStreamSynchronize(stream_));
        HIP_CHECK(hipFree(stage_));
      }
      HIP_CHECK(hipMalloc(&stage_, size_t(bytes)));
      stage_bytes_ = bytes;
    }
    if (check_dev_) check_ptr(stage_, "staging buffer");
    return stage_;
  }
  void assert_current(const char* where) const {
    int d = -1;
    HIP_CHECK(hipGetDevice(&d));
    GOL_REQUIRE(d == dev_, std::string("GOL_CHECK_DEVICE: ") + where + " runs on device " + std::to_string(d) +
                               ", backend owns device " + std::to_string(dev_));
  }
  void check_ptr(const void* p, const char* what) const {
    if (!p) return;
    hipPointerAttribute_t at{};
    HIP_CHECK(hipPointerGetAttributes(&at, p));
    GOL_REQUIRE(at.device == dev_, std::string("GOL_CHECK_DEVICE: ") + what + " lives on device " +
                                       std::to_string(at.device) + ", backend owns device " + std::to_string(dev_));
  }

  int dev_;
  bool check_dev_ = false;  // GOL_CHECK_DEVICE
  bool ring_on_ = true;     // GOL_ROW_RING
  mutable size_t ring_gran_ = 0;
  // Address space of released rings in this process, never reserved again
  // (alloc_row_ring), and its bound: a quarter of the 2^47-byte user range.
  static std::atomic<size_t>& ring_va_held() {
    static std::atomic<size_t> held{0};
    return held;
  }
  static constexpr size_t kRingVaBudget = size_t(32) << 40;
  std::map<void*, Ring> rings_;
  std::vector<hipEvent_t> timing_pool_;  // timing_mark() events
  hipStream_t stream_ = nullptr;
  std::string arch_;
  int cus_ = 256;          // CUs this backend's launches may use (its partition, if any)
  std::string cu_part_;    // GOL_CU_PARTITION, for name()
  int numa_ = -1;          // NUMA node the process was pinned to (tuning numa_pin), for name()
  int numa_cpus_ = 0;      // CPUs it may run on there
  hipk::LifeTuning tune_;
  hipStream_t comm_ = nullptr;
  // chain_mem: chained groups' flags, slots; linked launches' 3 x completion words.
  void* chain_[5] = {};
  size_t chain_bytes_[5] = {};
  hipk::LinkState link_;  // linked launches (GOL_LINK)
  bool link_on_ = false;  // every eligible launch (GOL_LINK=1)
  int link_mode_ = -1;
  uint32_t chain_seq_ = 0;
  // Boundary trigger: cumulative device counter, increments expected so
  // far, and the target of the last armed launch (0: none pending).
  unsigned long long* trigger_counter() {
    if (!trigger_ok_) return nullptr;
    if (!trigger_mem_) {
      GOL_ON_DEVICE();
      HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&trigger_mem_), 256));
      HIP_CHECK(hipMemsetAsync(trigger_mem_, 0, 256, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
      trigger_total_ = 0;
    }
    return trigger_mem_;
  }
  unsigned long long* trigger_mem_ = nullptr;
  uint64_t trigger_total_ = 0, trigger_target_ = 0;
  bool trigger_ok_ = false;
  int chain_mode_ = 0;  // GOL_CHAIN: 0 off, 1 on, -1 autotuned per launch shape
  bool tune_log_ = false;
  std::map<TuneKey, TuneStats> tuned_;
  std::deque<Pending> pending_;  // timed trial launches not collected yet
  std::vector<hipEvent_t> free_events_;
  int64_t launches_ = 0;
  bool prof_on_ = tuning_.on("host_profile");
  int64_t prof_n_ = 0;
  double prof_gap_ = 0, prof_in_ = 0, prof_launch_ = 0;
  std::chrono::steady_clock::time_point prof_exit_{};
  int64_t trace_at_ = -1;
  std::string trace_path_;
  bool trace_pair_ = false;
  uint64_t* pair_trace_[2] = {nullptr, nullptr};
  int pair_T_ = 0;
  hipEvent_t tail_[2] = {nullptr, nullptr};  // poll_side(): the compute streams' tails
  bool capturing_ = false;                    // between capture_begin and capture_end
  void* stage_ = nullptr;
  int64_t stage_bytes_ = 0;
  uint32_t* err_host_ = nullptr;
};

}  // namespace

bool hip_available() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return false;
  return n > 0;
}

std::unique_ptr<Backend> make_hip_backend(int device, const Tuning& tune) {
  GOL_REQUIRE(hip_available(), "no HIP device available (HIP backend requested)");
  // Engine trace ranges -> roctx (visible with rocprofv3 --marker-trace).
  trace::set_hooks([](const char* m) { roctxRangePushA(m); }, [] { roctxRangePop(); });
  return std::make_unique<HipBackend>(device, tune);
}

}  // namespace gol
