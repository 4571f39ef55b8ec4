// The generation engine: one rank's tile, its double buffer, the epoch /
// temporal-block schedule, halo exchange and lazy exact termination.
//
// Reference loops: serial src/game.c:169-196, MPI src/game_mpi.c:385-422,
// CUDA src/game_cuda.cu:213-276.  All of them test termination every
// generation (a full scan + MPI_Allreduce, or a kernel + 4-byte D2H copy).
// Both stop conditions are absorbing: an empty grid stays
// empty and G_t == G_{t-1} implies G_{t+k} == G_t.  So the kernels record
// one "changed" flag per generation, the engine polls them every few hundred
// generations, and the reference's reported generation count is rebuilt
// exactly from the first unchanged generation g_f:
//   * grid at g_f empty   -> extinction, reports g_f - 1 (src/game.c:177)
//   * otherwise, with similarity checks every F gens -> the first check
//     t >= g_f reports t - 1 (the break skips generation++, src/game.c:186)
//   * otherwise -> GEN_LIMIT.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "gol/backend.hpp"
#include "gol/decomp.hpp"
#include "gol/tile.hpp"
#include "gol/transport.hpp"

namespace gol {

struct EngineConfig {
  int64_t W = 0, H = 0;            // global grid (cells)
  Layout layout = Layout::Bits;
  std::string decomp = "auto";     // "auto" or "PxQ"
  int64_t gen_limit = 1000;        // GEN_LIMIT (src/game.c:6)
  bool check_similarity = true;    // CHECK_SIMILARITY (src/game.c:8)
  int sim_freq = 3;                // SIMILARITY_FREQUENCY (src/game.c:9)
  int64_t start_gen = 0;           // generation number of the loaded state (resume)
  int sim_phase = 0;               // similarity counter value at start_gen (resume)
  int tmax = 0;                    // max generations per kernel launch (0 = backend default)
  int epoch = 0;                   // generations per halo exchange (0 = auto)
  int poll_gens = 0;               // generations between termination polls (0 = auto)
  // Overlap the epoch's halo exchange with compute (row strips, Px == 1):
  //    3 trigger (1 on is the same): the last temporal block of a full epoch runs as usual, but
  //      its boundary groups count themselves done on a device counter; with
  //      linked launches that block runs on the second compute stream, and
  //      the first one - idle once the block before it is done - waits on the
  //      counter (Backend::trigger_stream) and sends the new boundary rows
  //      while the block's interior groups still run; the next epoch's first
  //      block follows the exchange on that stream and still links to the
  //      last block, so the chain runs through the epoch boundary.  No dual
  //      launch, no spinning consumer, no comm-stream hop; byte tiles on bit
  //      words included.  (Rounds 1-5 also had an early-boundary schedule - a
  //      dual launch of the boundary strips on the comm stream - and an edge-
  //      strip schedule; both measured slower and were removed, docs/HISTORY.md);
  //    0 off: everything on the compute stream;
  //   -1 auto: where the trigger schedule applies (row strips on a backend
  //      that supports it), the first epochs alternate it with the plain
  //      schedule, every rank times them with events, the per-epoch medians
  //      are MAX-reduced over ranks, and all ranks keep the faster one
  //      (GOL_OVERLAP_AUTO=plain|trigger forces the outcome after the trial,
  //      for tests); elsewhere as off.
  int overlap = -1;
  // Check each termination poll one poll window later, so the host never
  // drains the device queue (stops are absorbing, so running past is exact).
  bool lagged_poll = true;
  // Replay full epochs as captured HIP graphs (one per buffer parity):
  // -1 auto (single rank on a graph-capable backend), 0 off, 1 whenever the
  // backend and transport allow it.  Off by default: on ROCm 7 / MI355X the
  // replayed epochs measured 2-50% slower than stream launches
  // (profiles/sweep_graphs.jsonl); the host is never the bottleneck here.
  int graphs = 0;
  // Watchdog: fail (instead of hanging) when a termination poll waits on the
  // device longer than this many seconds (0: GOL_WATCHDOG_S or 900 s).
  double watchdog_s = 0;
  // Bracket each run's generation loop with a transport barrier (plus a
  // device sync) so loop_ms covers every rank's loop - the reference times
  // rank 0 only, with no barrier (src/game_mpi.c:385-424).  A caller that
  // brackets the run itself (bench.py) turns them off.
  bool timing_barriers = true;
  // Rehearsal of a multi-rank row-strip schedule on one rank: the north /
  // south halos go through the transport (a 1-rank RCCL communicator sending
  // to itself) instead of the local periodic fill, with the multi-rank epoch
  // depth and overlap.  Results are identical (the torus wraps to self).
  bool self_exchange = false;
  // Compute representation of the byte layout (width % 32 == 0):
  //    1 bits: the byte-per-cell grid stays the storage (load / store / read-
  //      out / drift rotation / alive count / checkpoints), but each run packs
  //      the owned rows into bit words inside the spare byte buffer, its
  //      epochs exchange or fill the halos there (8x fewer bytes) and run the
  //      bit-sliced temporal blocks, and the run ends by unpacking the owned
  //      rows back: two byte passes per run instead of one per temporal block
  //      (docs/PERFORMANCE.md);
  //    0 bytes: temporal blocks on the byte grid itself (the byte kernels);
  //   -1 auto: bits on a device backend (GOL_U8_VIA_BITS=0|1 overrides),
  //      else bytes.
  int u8_compute = -1;
  // Runtime tuning (gol/tuning.hpp): the engine's own knobs (u8_via_bits,
  // side_poll, cpu_side_poll, poll_copy_side, watchdog_s, overlap_auto) come from here; the
  // backend's from the Tuning it was constructed with.  Default: the table's
  // defaults under the GOL_* environment overrides.
  Tuning tune = Tuning::from_env();
};

struct RunResult {
  int64_t generations = 0;       // the reference's "Generations:" value
  int64_t executed = 0;          // generations actually evaluated in this run
  int64_t first_unchanged = -1;  // g_f, or -1 if no fixed point was seen
  bool extinct = false;
  std::string stop_reason = "limit";  // limit | extinction | similarity | fixed_point
  double loop_ms = 0;            // wall time of the generation loop (incl. final sync)
  int64_t exchanges = 0;         // halo exchanges performed
  int64_t polls = 0;             // termination polls performed
  int64_t kernel_launches = 0;
  bool overlapped = false;       // epochs ran with the overlapped halo exchange
  int64_t graph_launches = 0;    // epochs replayed from a captured HIP graph
  int64_t halo_bytes = 0;        // bytes this rank sent in halo exchanges
  int64_t linked_launches = 0;   // launches that overlapped the previous one (GOL_LINK)
  // Per-phase device time of this run (Engine::set_phase_timing; SURVEY
  // 5.1/5.5): temporal-block kernels, halo exchanges (pack / send / recv /
  // unpack), periodic halo fills, termination-flag reductions (all-reduce +
  // copy to the host).  Phases on different streams may overlap, so the sum
  // can exceed loop_ms; the rest of loop_ms is host gaps and idle device.
  bool phase_timed = false;
  double compute_ms = 0, halo_ms = 0, fill_ms = 0, allreduce_ms = 0;
};

// The reference's "Generations:" value of a run over (start_gen, limit] whose
// first unchanged generation is g_f = first_unchanged (-1: none), given
// whether the grid at g_f is empty; *reason (optional) receives limit |
// extinction | similarity | fixed_point.  Mirrored by utils/termination.py.
int64_t reported_generations(int64_t first_unchanged, bool extinct, int64_t limit, int64_t start_gen,
                             bool check_similarity, int sim_freq, int sim_phase, std::string* reason = nullptr);

class Engine {
 public:
  Engine(const EngineConfig& cfg, Backend* backend, Transport* transport);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  const EngineConfig& config() const { return cfg_; }
  const Decomposition& decomp() const { return dec_; }
  const TileGeom& geom() const { return g_; }
  // The tile the temporal blocks run on: geom(), or its bit-word image when
  // the byte layout computes on bit words (via_bits(); the byte tile then has
  // no halos).
  const TileGeom& compute_geom() const { return via_bits_ ? gb_ : g_; }
  int rank() const { return rank_; }
  Extent rows() const { return dec_.rows(rank_); }
  Extent cols() const { return dec_.cols(rank_); }
  int epoch_depth() const { return D_; }
  int tmax() const { return tmax_; }
  bool overlap() const { return trigger_; }
  // "off" | "trigger" | "auto:trial" | "auto:plain" | "auto:trigger".
  std::string overlap_mode() const;
  // Median epoch time (ms, MAX over ranks) of the plain and the trigger
  // schedule in the auto trial (-1: not measured).
  double trial_ms_plain() const { return auto_ms_[0]; }
  double trial_ms_trigger() const { return auto_ms_[1]; }
  // Termination polls: "joined" (the flag all-reduce on the compute stream),
  // "side" (a side stream, tuning side_poll=1), "auto:trial", "auto:side" or
  // "auto:joined" (side_poll = -1, decided on the ranks), and the trial's
  // per-window medians (ms, MAX over ranks; -1: not measured).
  std::string poll_mode() const;
  double poll_trial_ms_joined() const { return poll_ms_[0]; }
  double poll_trial_ms_side() const { return poll_ms_[1]; }
  // Median of the run of side windows that checked a side decision (-1: none).
  double poll_trial_ms_side_steady() const { return poll_side_steady_ms_; }
  // Epoch exchanges started by the boundary trigger so far (diagnostics).
  int64_t triggered_sends() const { return triggered_sends_; }
  // Sample per-phase device times into RunResult (event pairs around every
  // kernel, exchange, fill and reduction; adds a little launch overhead).
  void set_phase_timing(bool on) { phase_timing_ = on; }
  bool phase_timing() const { return phase_timing_; }
  bool graphs() const { return use_graphs_; }
  int64_t generation() const { return gen_; }
  void set_generation(int64_t g) { gen_ = g; }
  Backend* backend() const { return be_; }
  // The byte (or bit) tile's current buffer, brought up to date first.
  void* current_buffer() {
    sync_bytes();
    return buf_[cur_];
  }
  // Storage-frame drift (cells, mod W) left by drifting kernels
  // (Backend::drifts): stored column x holds true column x - drift.
  int64_t drift() const { return drift_; }
  // Whether temporal blocks may run the drifting (adder-window) kernel.
  bool drifting() const { return drift_ok_; }
  // Whether byte-layout epochs compute on bit words (EngineConfig::u8_compute).
  bool via_bits() const { return via_bits_; }
  // Whether the tile is a row ring (Backend::row_ring_halo): no row fills,
  // one temporal block per epoch over the owned rows.
  bool row_ring() const { return rows_ring_; }
  // Why a row ring this tile should have had could not be built (the
  // backend's error; the tile then runs with periodic row fills), or "".
  const std::string& row_ring_fallback() const { return ring_fallback_; }
  // Rotates the drift out of the current buffer (owned rows); every
  // read-out (store_cells) does this first.
  void normalize();

  // State I/O.  `cells` is this rank's owned tile (rows() x cols()).
  void load_cells(const uint8_t* cells, int64_t ld);
  // `grid` is the full global grid; this rank copies out its subarray.
  void load_global(const uint8_t* grid, int64_t ld);
  void store_cells(uint8_t* cells, int64_t ld, bool ascii);
  // Owned rows [r0, r0 + n) of the tile only (0 <= r0, r0 + n <= rows()):
  // checks a band of a grid whose whole-tile host copy would not fit.
  void store_rows(uint8_t* cells, int64_t ld, int64_t r0, int64_t n, bool ascii);
  void init_random(uint64_t seed, double density);
  int64_t alive_count();  // local owned cells

  // Runs from the current generation up to config().gen_limit with the
  // reference's termination semantics.
  RunResult run();
  // Same, but stops at `limit` (<= gen_limit) - used for chunked runs with
  // checkpoints; the result's generation count is relative to `limit`.
  RunResult run_until(int64_t limit);
  // Runs exactly n more generations (termination flags still recorded, but
  // no early stop): the bench path.
  RunResult advance(int64_t n);

  // Exchange halos of the current buffer (exposed for tests).
  void halo_exchange();
  // Performs one temporal block from the current buffer (tests).
  void step_block(int T, int64_t row_lo, int64_t row_hi);

 private:
  struct Poll {
    int64_t from = 0, to = 0;
    void* ev = nullptr;
  };
  RunResult run_impl(int64_t limit, bool stop_early);
  Poll poll_issue(int64_t from, int64_t to);
  bool poll_check(Poll& p, int64_t* first_unchanged);
  int pick_T(int64_t remaining) const;
  // One temporal block in <in> -> <out> for generations (gen_base, gen_base+T];
  // returns the frame drift of the launch (cells).
  int launch(void* in, void* out, const TileGeom& g, int T, int64_t row_lo, int64_t row_hi, int64_t gen_base,
             const int64_t* trigger_rows = nullptr, bool hot_only = false);
  // A block of a trigger epoch before its last: the boundary rows' light
  // cone at top issue priority (engine.cpp).
  void hot_block(void* in, void* out, const TileGeom& g, int T, int64_t row_lo, int64_t row_hi, int64_t d);
  void add_drift(int64_t cells);
  void exchange_columns(void* buf, const TileGeom& g);
  std::vector<P2POp> row_ops(void* buf, const TileGeom& g) const;
  void halo_exchange_on(void* buf, const TileGeom& g);
  // Byte layout on bit words (EngineConfig::u8_compute = 1): one epoch on
  // the bit tile, and the per-run pack / unpack of the byte tile.
  void epoch_via_bits(int64_t d, bool sent_ahead);
  void pack_bits();
  void unpack_bits();
  void sync_bytes();  // unpack a live bit image into the byte tile (pack_bits in engine.cpp)
  void* bit_scratch(int i) const;
  // Last block of a full epoch in the trigger schedule, in -> out on tile g
  // (the byte tile or its bit image); the caller flips its buffer parity.
  void last_block_trigger(void* in, void* out, const TileGeom& g, int T);
  // Waits for a triggered exchange still in flight; `invalidate` when the
  // buffers are about to change outside the schedule.
  void settle_pending(bool invalidate);
  void run_epoch(int64_t d);
  void release_graphs();
  int graph_key() const { return via_bits_ ? 2 * cur_ + bpar_ : cur_; }
  // Overlap auto trial (EngineConfig::overlap == -1): picks the schedule of
  // the next full epoch, records its start, and decides once enough epochs
  // of both schedules have been timed (at the same epoch on every rank).
  void auto_choose(bool full_epoch);
  void auto_mark();
  void auto_decide();
  void poll_trial_step();
  // Phase timing: a mark on `stream` (nullptr when off or capturing), and
  // the span [a, now] of `phase` on that stream.
  void* phase_begin(void* stream);
  void phase_end(int phase, void* a, void* stream);
  void collect_phases(RunResult& res);

  EngineConfig cfg_;
  Backend* be_;
  Transport* tr_;
  Decomposition dec_;
  int rank_ = 0;
  TileGeom g_;
  int D_ = 0, tmax_ = 0, poll_gens_ = 0;
  void* buf_[2] = {nullptr, nullptr};
  int cur_ = 0;
  uint32_t* flags_ = nullptr;      // device: changed[t - flags_base_]
  uint32_t* flags_host_ = nullptr; // pinned mirror
  int64_t flags_base_ = 0, flags_len_ = 0;
  uint32_t* alive_dev_ = nullptr;
  void* colbuf_[4] = {nullptr, nullptr, nullptr, nullptr};  // send W, send E, recv W, recv E
  bool trigger_ = false;             // boundary-triggered sends (overlap = 3)
  int64_t triggered_sends_ = 0;
  bool send_next_ = false;           // the current epoch is followed by another one in this run
  bool rows_pending_ = false;        // halo rows of buf_[cur_] were sent by the last block
  int64_t boundary_sends_ = 0;      // exchanges sent from an epoch's last block (RunResult::overlapped)
  bool use_graphs_ = false, capturing_ = false;
  int64_t* gen_dev_ = nullptr;        // device: (epoch start - flags_base_) for graph replays
  int64_t epoch_start_ = 0;
  // Captured epochs, keyed by graph_key(): the parity of the buffer pair the
  // epochs alternate over and, for the byte layout on bit words, the byte
  // buffer the bit scratch lives in (bit_scratch depends on cur_, which
  // normalize() flips between runs).
  void* graph_[4] = {nullptr, nullptr, nullptr, nullptr};
  int graph_flip_[4] = {0, 0, 0, 0};
  int64_t graph_kernels_[4] = {0, 0, 0, 0};
  uint32_t* graph_flags_ = nullptr;   // flags buffer the graphs were captured with
  int64_t graph_runs_ = 0;
  int64_t halo_bytes_ = 0;
  double watchdog_s_ = 900;
  int64_t gen_ = 0;
  int64_t exchanges_ = 0, polls_ = 0, launches_ = 0;
  bool drift_ok_ = false;   // whole-width tile of 32-cell words on a drifting backend
  bool cols_filled_ = true; // column halos kept valid by fills (false: the backend wraps column reads)
  bool rows_wrapped_ = false; // single-rank torus read modulo its rows (no fills at all)
  bool rows_ring_ = false;    // row halos are second mappings of the owned rows (Backend::row_ring_halo)
  std::string ring_fallback_;  // alloc_row_ring's error when the ring fell back to fills
  bool link_ = false;         // blocks may run linked (Backend::KernelChoice::link; ring tiles only)
  bool via_bits_ = false;    // byte layout computed on bit words (epoch_via_bits)
  TileGeom gb_;              // the tile in the bit layout (same rows, halos, words)
  void* bitbuf_[2] = {nullptr, nullptr};  // own bit scratch when the spare byte buffer cannot hold it
  int bpar_ = 0;             // bit_scratch(bpar_) holds the current generation during a run
  bool bits_live_ = false;   // ... and after it, until the byte tile is read (sync_bytes)
  bool poll_side_ = false;   // termination polls reduce on the comm stream (Transport::side_reduce)
  bool polled_side_ = false;  // a poll of this run went to Backend::poll_side()
  bool poll_copy_side_ = true;  // tuning poll_copy_side: single-rank polls on Backend::poll_side()
  int64_t drift_ = 0;
  int64_t graph_drift_[4] = {0, 0, 0, 0};
  // Overlap auto trial.
  bool auto_overlap_ = false;       // trial still running
  bool auto_decided_ = false;
  int auto_sched_ = 0;              // trial slot of the current epoch: 0 plain, 1 trigger
  int64_t auto_full_epochs_ = 0;    // full epochs seen so far
  void* auto_open_ = nullptr;       // start mark of the current epoch
  int auto_open_sched_ = -1;        // its schedule (-1: not a trial epoch)
  struct AutoSpan {
    int sched;
    void* a;
    void* b;
  };
  std::vector<AutoSpan> auto_spans_;
  int auto_counts_[2] = {0, 0};
  double auto_ms_[2] = {-1, -1};
  void trial_medians(std::vector<AutoSpan>& spans, double out[2]);
  // Poll placement trial (tuning side_poll = -1, poll_trial_step).
  bool poll_trial_ = false, poll_decided_ = false;
  int64_t ptrial_polls_ = 0;
  int ptrial_mode_ = -1;            // placement of the open window: 0 joined, 1 side, -1 warm-up
  void* ptrial_open_ = nullptr;
  std::vector<AutoSpan> ptrial_spans_;
  int ptrial_counts_[2] = {0, 0};
  double poll_ms_[2] = {-1, -1};
  bool ptrial_verify_ = false;      // checking a side decision on consecutive side windows
  double poll_side_steady_ms_ = -1;
  // Phase timing.
  bool phase_timing_ = false;
  struct PhaseSpan {
    int phase;
    void* a;
    void* b;
  };
  std::vector<PhaseSpan> phase_spans_;
};

}  // namespace gol
