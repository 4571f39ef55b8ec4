// Compute backends.  The engine (engine.hpp) is written once against this
// interface; two implementations exist:
//   * HipBackend  - MI355X: hand-written CDNA4 kernels, one HIP stream,
//                   everything asynchronous (backend_hip.hip, kernels/*.hip).
//   * CpuBackend  - bit-exact C++ emulation of the same kernels on host
//                   threads; it replaces the reference's OpenMP loops
//                   (src/game_openmp.c:34,63,97) and lets the whole engine
//                   (epochs, halos, lazy termination) be tested without a GPU.
#pragma once

#include <memory>
#include <string>

#include "gol/tile.hpp"
#include "gol/tuning.hpp"

namespace gol {

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  virtual bool is_device() const = 0;
  virtual int device() const { return -1; }
  virtual void* stream() const { return nullptr; }  // hipStream_t for HIP

  // Memory.  alloc() returns zeroed memory in the backend's address space.
  virtual void* alloc(size_t bytes) = 0;
  virtual void release(void* p) = 0;
  virtual void* alloc_host(size_t bytes) = 0;  // pinned host staging for HIP
  virtual void release_host(void* p) = 0;
  virtual void memset_async(void* p, int v, size_t bytes) = 0;
  virtual void copy_h2d(void* dst, const void* src, size_t bytes) = 0;        // synchronous
  virtual void copy_d2h(void* dst, const void* src, size_t bytes) = 0;        // synchronous
  // Into pinned memory, on `stream` (nullptr = the compute stream).
  virtual void copy_d2h_async_on(void* dst, const void* src, size_t bytes, void* stream) = 0;
  virtual void copy_2d_async(void* dst, int64_t dpitch, const void* src, int64_t spitch,
                             int64_t width_bytes, int64_t rows) = 0;
  virtual void synchronize() = 0;
  // Host waits for `stream` (nullptr = the compute stream) to drain.
  virtual void synchronize_stream(void* stream) {
    (void)stream;
    synchronize();
  }
  // Events: an opaque handle recorded on `stream` (nullptr = the compute
  // stream).
  virtual void* event_record_on(void* stream) = 0;
  virtual void event_wait(void* ev) = 0;  // host blocks until the event completes
  virtual void event_destroy(void* ev) = 0;
  // Non-blocking: has the event completed?  (Synchronous backends: always.)
  virtual bool event_query(void* /*ev*/) { return true; }
  // Second queue for communication that overlaps compute (HIP: a separate
  // non-blocking stream, poll_side's; synchronous backends return nullptr and
  // run everything in program order).
  virtual void* comm_stream() { return nullptr; }
  // Stream capture into replayable graphs (HIP graphs).  capture_end()
  // returns an executable graph handle; graph_launch() enqueues it.
  virtual bool supports_graphs() const { return false; }
  virtual void capture_begin() {}
  virtual void* capture_end() { return nullptr; }
  virtual void graph_launch(void* /*graph*/) {}
  virtual void graph_destroy(void* /*graph*/) {}
  // Stream-ordered update of a device int64 (set, or add).
  virtual void i64_async(int64_t* dev, int64_t v, bool add) {
    if (add)
      *dev += v;
    else
      *dev = v;
  }
  // Boundary trigger (BlockArgs::trigger).  trigger_stream() returns the
  // compute stream, ordered so that work enqueued on it next starts once the
  // groups of the last run_block that met the trigger rows have written them
  // - not after the whole launch: with linked launches that block runs on
  // the second compute stream, and the first one waits on the device counter
  // instead - and *armed says whether that happened.  Not armed, it orders
  // the stream after the whole launch (a join).  Either way the next
  // run_block on the stream is ordered after what was enqueued in between,
  // and, armed, may still link to the trigger launch.  Synchronous backends:
  // nullptr (program order).
  virtual bool supports_trigger() const { return false; }
  virtual void* trigger_stream(bool* armed) {
    *armed = false;
    join_streams();
    return stream();
  }
  // A side stream for a termination poll that does not join the compute
  // streams: returned after it has been made to wait for everything enqueued
  // so far on every compute stream (a linked chain's second stream
  // included), so the change flags of the generations computed so far are
  // final on it, while a linked chain continues across the poll.  The poll's
  // reduction, copy and event go on it (copy_d2h_async_on / event_record_on
  // with a side stream do not join the compute streams).  nullptr: none (the
  // engine joins and polls on the compute stream).
  virtual void* poll_side() { return nullptr; }

  // Phase timing: timing_mark() records a timestamp on
  // `stream` (nullptr = the compute stream); timing_ms(a, b) is the time
  // between two marks of one stream (blocks until b has completed);
  // timing_release() recycles a mark.  Device backends use timing events,
  // synchronous backends the host clock (their operations complete in
  // program order).
  virtual void* timing_mark(void* stream) = 0;
  virtual double timing_ms(void* a, void* b) = 0;
  virtual void timing_release(void* mark) = 0;
  // Linked launches (HIP, GOL_LINK): work on the backend's second compute
  // stream precedes what comes next on its compute stream.  The engine calls
  // it before enqueueing transport operations on stream() itself.
  virtual void join_streams() {}
  virtual int64_t linked_launches() const { return 0; }
  // Makes this backend's device current for the calling thread (rank
  // threads of single-process multi-GPU runs call it first).
  virtual void bind_thread() {}
  // Lets this backend's device read memory of `device` directly (peer
  // access); throws if the hardware cannot.  No-op for host backends.
  virtual void enable_peer(int /*device*/) {}

  // Kernels.  run_block returns the drift of the stored frame in cells
  // (BlockArgs::allow_drift): the output's column x holds the cell the input
  // frame had at x - drift.
  virtual int run_block(const BlockArgs& a) = 0;
  // Whether run_block may drift the frame for this layout when allowed
  // (the engine then sizes the left halo for the one-sided light cone).
  virtual bool drifts(Layout) const { return false; }
  // Whether run_block honours BlockArgs::full_width for this layout (wraps
  // column reads within the owned words): the engine then skips the periodic
  // column fills of whole-width tiles.
  virtual bool wraps_columns(Layout) const { return false; }
  // Whether run_block also honours BlockArgs::wrap_rows for this layout (a
  // single-rank whole-torus tile read modulo its owned rows at T = 1): the
  // engine then runs one-generation epochs with no periodic fill at all.
  virtual bool wraps_rows(Layout) const { return false; }
  // Owned rows of src rotated left by `shift` cells (0 < shift < W) into dst:
  // dst cell x = src cell (x + shift) mod W.  Halos of dst are not written.
  virtual void rotate_cols(const void* src, void* dst, const TileGeom& g, int64_t shift) = 0;
  // Owned rows [i0, i0 + n) of src (geometry gs) converted into dst
  // (geometry gd: the same owned tile in the other layout, halos and pitch
  // may differ), owned cells only: byte cells -> bit words or back.
  // Enqueued on the compute stream.
  virtual void convert_rows(const void* src, const TileGeom& gs, void* dst, const TileGeom& gd, int64_t i0,
                            int64_t n) = 0;
  // Throws if a kernel enqueued so far reported an error through the
  // backend's device-visible error word (call after the work completed).
  virtual void check_device_errors() {}
  // Largest temporal block size (generations per run_block) the backend runs
  // at full occupancy for this layout; the engine's default tmax.
  virtual int preferred_tmax(Layout) const { return 16; }
  // Kernel family for a rows x cols tile: the temporal block size (tmax_req
  // > 0: the caller's) and whether blocks may drift the frame (drifts()).
  struct KernelChoice {
    int tmax = 16;
    bool drift = false;
    bool link = false;  // consecutive blocks may run linked (BlockArgs::link)
  };
  virtual KernelChoice choose_kernel(Layout l, int64_t /*rows*/, int64_t /*cols*/, int tmax_req) const {
    return {tmax_req > 0 ? tmax_req : preferred_tmax(l), drifts(l)};
  }
  // Row ring (single-rank torus): a tile whose top Dv halo rows are a second
  // virtual mapping of its last Dv owned rows and whose bottom halo rows map
  // its first ones, so the periodic row halos are always valid and never
  // filled.  row_ring_halo() returns the halo rows per side (>= min_halo) a
  // ring of H rows of `pitch` bytes needs for the mapping granularity, or 0
  // when the backend cannot build one for that geometry; alloc_row_ring()
  // returns such a tile (zeroed) for a geometry with that Dv, or nullptr.
  // release() frees rings too.
  virtual int row_ring_halo(int64_t /*H*/, int64_t /*pitch*/, int /*min_halo*/) const { return 0; }
  // Bytes the backend can still allocate (device memory free; host backends:
  // unlimited).  The engine leaves the ring out when it would not fit beside
  // the rest of the tile's buffers.
  virtual size_t mem_free() const { return ~size_t(0); }
  virtual void* alloc_row_ring(const TileGeom& /*g*/) { return nullptr; }
  // Periodic self-fill of halo regions of a single tile (any tile size):
  // columns (left/right halo words of owned rows) and/or rows (full padded
  // rows of the top/bottom halo, which also fills the corners).
  virtual void fill_periodic(void* buf, const TileGeom& g, bool cols, bool rows) = 0;
  // Periodic column halos of padded rows [r0, r0 + n) only (whole-width
  // tiles), on `stream` (nullptr = the compute stream).
  virtual void fill_cols_rows(void* buf, const TileGeom& g, int64_t r0, int64_t n, void* stream = nullptr) = 0;
  // OR of all owned cells -> *flag (device) = 1 if any cell is alive.
  virtual void alive_any(const void* buf, const TileGeom& g, uint32_t* flag) = 0;
  // Count of live owned cells (synchronous, for diagnostics/tests).
  virtual int64_t alive_count(const void* buf, const TileGeom& g) = 0;
  // Host <-> tile conversion: `cells` is an H x W array of bytes (ld = row
  // stride); load treats byte == '1' or byte == 1 as alive; store writes
  // '0'/'1' when ascii else 0/1.
  virtual void load_owned(void* buf, const TileGeom& g, const uint8_t* cells, int64_t ld) = 0;
  virtual void store_owned(const void* buf, const TileGeom& g, uint8_t* cells, int64_t ld,
                           bool ascii) = 0;
  // Counter-based random init of owned cells from global coordinates, so the
  // grid is identical for every decomposition and layout.
  virtual void init_random(void* buf, const TileGeom& g, uint64_t seed, double density,
                           int64_t grow0, int64_t gcol0) = 0;

  // The tuning the backend was constructed with (gol/tuning.hpp): its knobs
  // are read from it once, at construction.
  const Tuning& tuning() const { return tuning_; }

 protected:
  explicit Backend(const Tuning& t) : tuning_(t) {}
  Tuning tuning_;
};

// drift: emulate the drifting frame of the HIP adder window (each block's
// output shifted right by T cells), so the engine's drift bookkeeping is
// testable on the CPU; -1: the tuning's cpu_drift.
std::unique_ptr<Backend> make_cpu_backend(int threads, int drift = -1, const Tuning& tune = Tuning::from_env());
// Defined in backend_hip.hip; throws if no device or the kernels are missing,
// or if `tune` selects a kernel that does not exist.
std::unique_ptr<Backend> make_hip_backend(int device, const Tuning& tune = Tuning::from_env());
bool hip_available();

// Counter-based RNG used by init_random (host and device agree bit-for-bit).
GOL_HD inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
GOL_HD inline bool rng_cell(uint64_t seed, int64_t row, int64_t col, uint32_t thresh24) {
  uint64_t k = seed ^ (uint64_t(row) * 0xD1B54A32D192ED03ull) ^ (uint64_t(col) * 0xABC98388FB8FAC03ull);
  return uint32_t(splitmix64(k) >> 40) < thresh24;
}
inline uint32_t density_thresh(double d) {
  if (d <= 0) return 0;
  if (d >= 1) return 1u << 24;
  return uint32_t(d * double(1u << 24) + 0.5);
}

}  // namespace gol
