#include "gol/engine.hpp"

#include <algorithm>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "gol/trace.hpp"

namespace gol {

namespace {
// Temporal block sizes built for every backend; 32 and 24 for the byte
// layout only (one grid read + write per pass, docs/PERFORMANCE.md).
constexpr int kTSizes[] = {32, 24, 16, 12, 8, 4, 2, 1};

// Phases of RunResult's device-time split.
enum Phase { kCompute = 0, kHalo = 1, kFill = 2, kReduce = 3, kPhases = 4 };
constexpr size_t kMaxPhaseSpans = size_t(1) << 16;  // per run; later spans go unmeasured

// Overlap auto trial: warm-up epochs (first launches autotune the chained
// groups), then kAutoTrials timed epochs of each schedule, alternating.
constexpr int64_t kAutoWarm = 2;
constexpr int kAutoTrials = 4;

int64_t min_tile_rows(const Decomposition& d) { return d.H / d.Py; }
int64_t min_tile_cols(const Decomposition& d) { return (d.W / d.col_unit / d.Px) * d.col_unit; }
}  // namespace

Engine::Engine(const EngineConfig& cfg, Backend* backend, Transport* transport)
    : cfg_(cfg), be_(backend), tr_(transport) {
  GOL_REQUIRE(be_ && tr_, "engine needs a backend and a transport");
  GOL_REQUIRE(cfg_.W > 0 && cfg_.H > 0, "grid dimensions must be positive");
  GOL_REQUIRE(cfg_.sim_freq > 0, "similarity frequency must be positive");
  GOL_REQUIRE(cfg_.gen_limit >= 0, "generation limit must be >= 0");
  rank_ = tr_->rank();
  if (cfg_.overlap == 1) cfg_.overlap = 3;  // "on" is the trigger schedule
  int64_t unit = (cfg_.layout == Layout::Bits || cfg_.W % 32 == 0) ? 32 : 1;
  if (cfg_.layout == Layout::Bits)
    GOL_REQUIRE(cfg_.W % 32 == 0, "bit-packed layout needs width % 32 == 0 (use the u8 layout)");
  dec_ = Decomposition::make(cfg_.W, cfg_.H, tr_->size(), cfg_.decomp, unit);

  // Byte layout computed on bit words (EngineConfig::u8_compute): the same
  // decision on every rank (configuration, backend kind and environment).
  if (cfg_.layout == Layout::U8 && cfg_.W % 32 == 0) {
    int mode = cfg_.u8_compute;
    if (mode < 0) mode = cfg_.tune.i("u8_via_bits");
    if (mode < 0) mode = be_->is_device();
    else mode = mode != 0;
    via_bits_ = mode == 1;
  }
  // Layout the temporal blocks run on.
  const Layout cl = via_bits_ ? Layout::Bits : cfg_.layout;
  // Every rank must take the same decision (a drifting frame or a schedule
  // that moves a halo exchange is only consistent in lockstep), so it is
  // made for the smallest tile of the decomposition, not this rank's.
  const Backend::KernelChoice kc =
      be_->choose_kernel(cl, min_tile_rows(dec_), std::max<int64_t>(1, min_tile_cols(dec_)), cfg_.tmax);
  tmax_ = std::min(kc.tmax, cl == Layout::U8 ? 32 : 16);
  // Epoch depth: a deeper halo means fewer latency-bound exchanges (or local
  // periodic fills: two ~5 us launches each) but ~D redundant rows per epoch.
  // With the grouped kernel the per-rank tile costs the same from 8T to 24T
  // (profiles/sweep_epoch_group.jsonl; 4T is 4 % slower), so one rank uses 8T
  // and several ranks 16T: half the RCCL exchanges (4 per 1000 generations),
  // each one latency-bound.
  const bool row_exchange = dec_.Py > 1 || cfg_.self_exchange;
  int D = cfg_.epoch > 0 ? cfg_.epoch : (tr_->size() > 1 || cfg_.self_exchange ? 16 : 8) * tmax_;
  if (dec_.Py > 1) D = int(std::min<int64_t>(D, min_tile_rows(dec_)));
  if (dec_.Px > 1) {
    int64_t cap = 32 * (min_tile_cols(dec_) / 32);
    GOL_REQUIRE(cap >= 1, "tiles narrower than 32 cells cannot exchange column halos");
    D = int(std::min<int64_t>(D, cap));
  }
  D_ = std::max(1, D);
  tmax_ = std::min(tmax_, D_);
  // A drifting kernel (one-sided window, Backend::drifts) consumes 2 cells of
  // left halo per generation and none on the right; it needs the tile to be
  // the whole torus width so that the drift is a relabeling of columns.
  drift_ok_ = kc.drift && dec_.Px == 1 && cfg_.W % 32 == 0;
  // Whole-width tiles on a backend that wraps column reads (lane_cols in the
  // HIP kernels) never read their halo columns: no column fills.
  cols_filled_ = !(dec_.Px == 1 && cfg_.W % 32 == 0 && be_->wraps_columns(cl));
  // A single-rank torus on a backend that also wraps row reads (the LDS-tiled
  // byte kernels): one block per epoch over the owned rows, no fills at all.
  rows_wrapped_ = !cols_filled_ && dec_.Px == 1 && dec_.Py == 1 && !cfg_.self_exchange && be_->wraps_rows(cl);
  if (rows_wrapped_) D_ = tmax_;  // one block per epoch; nothing to fill or exchange
  // Halo columns: none when the kernels wrap (smaller rows to exchange and
  // fill); else D cells per side, 2D on the left for the drifting window.
  int hw = cols_filled_ ? int(ceil_div(drift_ok_ ? 2 * int64_t(D_) : int64_t(D_), 32)) : 0;
  Extent r = rows(), c = cols();
  // Row ring (Backend::row_ring_halo): a single-rank torus whose row halos
  // are second mappings of its own owned rows.  Nothing is ever filled, and
  // every temporal block runs over exactly the owned rows, so an epoch is one
  // block (D = tmax, unless the configuration sets the epoch).
  // The rings are allocated here, before any geometry is committed: if the
  // backend cannot build them after all (address space, driver), the tile
  // falls back to plain buffers with periodic fills.
  int ring_dv = 0;
  void* ring_bufs[2] = {nullptr, nullptr};
  if (dec_.Px == 1 && dec_.Py == 1 && !cfg_.self_exchange && !rows_wrapped_) {
    const TileGeom probe = TileGeom::make(cl, r.size(), c.size(), 0, hw);
    ring_dv = be_->row_ring_halo(probe.H, probe.pitch, tmax_);
    // The byte layout on bit words keeps its byte tiles too: the rings must
    // fit beside them (BASELINE config 5's share, 2 x 137 GB of bytes, has no
    // room for 2 x 17 GB of bit rings on a 288 GB GPU; its bit words then
    // live in the spare byte buffer with periodic fills).
    if (ring_dv > 0 && via_bits_) {
      const double bytes = 2.0 * double(TileGeom::make(cfg_.layout, r.size(), c.size(), 0, 0).bytes()) +
                           2.0 * double(TileGeom::make(cl, r.size(), c.size(), ring_dv, hw).bytes());
      if (bytes + double(size_t(1) << 31) > double(be_->mem_free())) ring_dv = 0;
    }
    if (ring_dv > 0) {
      const TileGeom gr = TileGeom::make(cl, r.size(), c.size(), ring_dv, hw);
      try {
        for (auto& b : ring_bufs) {
          b = be_->alloc_row_ring(gr);
          GOL_REQUIRE(b, "the backend returned no ring");
        }
      } catch (const std::exception& e) {
        for (auto& b : ring_bufs)
          if (b) be_->release(b);
        ring_bufs[0] = ring_bufs[1] = nullptr;
        ring_dv = 0;
        ring_fallback_ = e.what();
        std::fprintf(stderr, "gol: WARNING: row ring unavailable (%s); periodic row fills instead\n", e.what());
      }
    }
  }
  if (via_bits_) {
    // The byte tile is storage only (owned cells, no halos); the epochs run
    // on its bit-word image, which carries the halos.
    g_ = TileGeom::make(cfg_.layout, r.size(), c.size(), 0, 0);
    gb_ = TileGeom::make(Layout::Bits, r.size(), c.size(), ring_dv > 0 ? ring_dv : D_, hw);
  } else {
    g_ = TileGeom::make(cfg_.layout, r.size(), c.size(), ring_dv > 0 ? ring_dv : D_, hw);
  }
  if (ring_dv > 0) {
    rows_ring_ = true;
    if (cfg_.epoch <= 0) D_ = tmax_;  // an epoch only paces the polls (and column fills) now
  }
  // Linked launches (Backend::KernelChoice::link): consecutive blocks of an
  // epoch overlap; anything else on the stream (fills, exchanges, polls)
  // joins the streams first.  Not with column fills between blocks.
  link_ = kc.link && !cols_filled_;
  // Several ranks: every poll is a flag all-reduce on the compute stream
  // (latency-bound), so poll half as often; a stop is still exact and at most
  // two windows late.
  poll_gens_ = cfg_.poll_gens > 0 ? cfg_.poll_gens : (tr_->size() > 1 || cfg_.self_exchange) ? 512 : 256;
  if (rows_ring_ && !via_bits_) {
    for (int i = 0; i < 2; ++i) buf_[i] = ring_bufs[i];
  } else {
    for (auto& b : buf_) b = be_->alloc(size_t(g_.bytes()));
  }
  if (via_bits_) {
    // The bit words live in the spare byte buffer (about an eighth of its
    // size per parity) unless a small tile's halo rows or pitch rounding do
    // not leave room, or they form a row ring.
    if (rows_ring_) {
      for (int i = 0; i < 2; ++i) bitbuf_[i] = ring_bufs[i];
    } else if (2 * gb_.bytes() > g_.bytes()) {
      for (auto& b : bitbuf_) b = be_->alloc(size_t(gb_.bytes()));
    }
  }
  alive_dev_ = static_cast<uint32_t*>(be_->alloc(64));
  if (dec_.Px > 1) {
    const TileGeom& gc = via_bits_ ? gb_ : g_;  // the tile whose halos are exchanged
    size_t n = size_t(gc.span_bytes(32 * int64_t(gc.hw)) * gc.H);
    for (auto& b : colbuf_) b = be_->alloc(n);
  }
  // Boundary-triggered sends (overlap = 3; last_block_trigger): row strips
  // on a backend that can count boundary groups done.  Byte tiles on bit
  // words too: the trigger runs on the bit image.
  const bool trigger_ok = row_exchange && dec_.Px == 1 && be_->supports_trigger();
  trigger_ = trigger_ok && cfg_.overlap == 3;
  watchdog_s_ = cfg_.watchdog_s > 0 ? cfg_.watchdog_s : cfg_.tune.f("watchdog_s") > 0 ? cfg_.tune.f("watchdog_s") : 900.0;
  use_graphs_ = cfg_.graphs != 0 && be_->supports_graphs() && tr_->capturable() &&
                (cfg_.graphs > 0 || tr_->size() == 1);
  if (use_graphs_) gen_dev_ = static_cast<int64_t*>(be_->alloc(sizeof(int64_t)));
  if (use_graphs_) trigger_ = false;  // captured epochs stay on one stream
  // Overlap auto: measure both schedules on the real ranks (see auto_choose);
  // the one-GPU rehearsal has no xGMI latency in it, so on a multi-GPU node
  // the decision is taken from the node itself.
  auto_overlap_ = cfg_.overlap == -1 && trigger_ok && !use_graphs_;
  // Side polls: with a transport whose flag reduction has its own
  // communicator (RCCL), a poll's all-reduce and D2H copy run on the comm
  // stream after a mark on the compute stream, which never waits for them:
  // the reduction's latency leaves the critical path.  The halo exchanges
  // stay on the compute stream.
  // Opt-in (tuning side_poll=1): in the one-GPU RCCL rehearsal the cross-stream
  // hop cost ~10 us per poll, more than the 1-rank reduction it hides
  // (profiles/r02/side_poll_ab.jsonl); with 8 ranks the reduction is longer.
  // Single-rank poll copies on a side stream (poll_issue): a linked chain
  // continues across the poll (the rank tile's ring: 2.24 -> 2.17 ms per 1000
  // generations, 32768^2 -0.5 %), but with blocks of T <= 8 (8192^2, ~13 us
  // per linked block) it measured 5-10 % slower (profiles/r05/poll_side.jsonl).
  // Auto: deeper blocks only.
  const int pcs = cfg_.tune.i("poll_copy_side");
  poll_copy_side_ = pcs > 0 || (pcs < 0 && tmax_ > 8);
  // A single-rank device tile whose polls join the compute streams (T <= 8:
  // each join restarts the linked chain) polls every 1024 generations: 8192^2
  // 1.52 vs 1.62 ms per 1000 generations, 4096^2 1.20 vs 1.22 (medians of 8,
  // profiles/r06/poll_interval.jsonl).  A stop is still exact, and at most two
  // windows late.
  if (cfg_.poll_gens <= 0 && be_->is_device() && tr_->size() == 1 && !cfg_.self_exchange && !poll_copy_side_)
    poll_gens_ = 1024;
  // side_poll = -1 (default): after the overlap trial the ranks time both
  // poll placements (poll_trial_step) and keep the faster, as for overlap.
  const int sp = cfg_.tune.i("side_poll");
  const bool side_ok = tr_->side_reduce() && (be_->is_device() || cfg_.tune.on("cpu_side_poll")) && !use_graphs_ &&
                       (tr_->size() > 1 || cfg_.self_exchange);
  poll_side_ = side_ok && sp > 0 && !auto_overlap_;
  poll_trial_ = side_ok && sp < 0;
  gen_ = cfg_.start_gen;
}

void Engine::release_graphs() {
  for (auto& g : graph_) {
    if (g) be_->graph_destroy(g);
    g = nullptr;
  }
}

Engine::~Engine() {
  release_graphs();
  for (auto* spans : {&auto_spans_, &ptrial_spans_})
    for (auto& sp : *spans) {
      be_->timing_release(sp.a);
      be_->timing_release(sp.b);
    }
  if (ptrial_open_) be_->timing_release(ptrial_open_);
  if (auto_open_) be_->timing_release(auto_open_);
  for (auto& sp : phase_spans_) {
    be_->timing_release(sp.a);
    be_->timing_release(sp.b);
  }
  if (gen_dev_) be_->release(gen_dev_);
  for (auto& b : buf_)
    if (b) be_->release(b);
  for (auto& b : colbuf_)
    if (b) be_->release(b);
  for (auto& b : bitbuf_)
    if (b) be_->release(b);
  if (flags_) be_->release(flags_);
  if (flags_host_) be_->release_host(flags_host_);
  if (alive_dev_) be_->release(alive_dev_);
}

void Engine::load_cells(const uint8_t* cells, int64_t ld) {
  settle_pending(true);
  bits_live_ = false;  // the byte tile is the state again
  be_->load_owned(buf_[cur_], g_, cells, ld);
  be_->synchronize();
  drift_ = 0;
}

void Engine::load_global(const uint8_t* grid, int64_t ld) {
  Extent r = rows(), c = cols();
  load_cells(grid + r.begin * ld + c.begin, ld);
}

void Engine::store_cells(uint8_t* cells, int64_t ld, bool ascii) {
  settle_pending(false);
  sync_bytes();
  normalize();
  be_->synchronize();
  be_->store_owned(buf_[cur_], g_, cells, ld, ascii);
}

void Engine::store_rows(uint8_t* cells, int64_t ld, int64_t r0, int64_t n, bool ascii) {
  GOL_REQUIRE(r0 >= 0 && n >= 0 && r0 + n <= g_.H, "store_rows: rows outside the tile");
  if (n == 0) return;
  settle_pending(false);
  sync_bytes();
  normalize();
  be_->synchronize();
  // A view of the band: the same pitch and halos, its first owned row at r0.
  TileGeom v = g_;
  v.H = n;
  be_->store_owned(static_cast<uint8_t*>(buf_[cur_]) + r0 * g_.pitch, v, cells, ld, ascii);
}

void Engine::init_random(uint64_t seed, double density) {
  settle_pending(true);
  bits_live_ = false;
  be_->init_random(buf_[cur_], g_, seed, density, rows().begin, cols().begin);
  be_->synchronize();
  drift_ = 0;
}

void Engine::add_drift(int64_t cells) { drift_ = (drift_ + cells) % cfg_.W; }

void Engine::normalize() {
  sync_bytes();  // the rotation's target is the spare byte buffer, which holds the bit image
  if (drift_ == 0) return;
  settle_pending(true);  // the rotated copy has no halo rows
  be_->rotate_cols(buf_[cur_], buf_[cur_ ^ 1], g_, drift_);
  cur_ ^= 1;
  drift_ = 0;
}

int64_t Engine::alive_count() {
  be_->synchronize();
  if (bits_live_) return be_->alive_count(bit_scratch(bpar_), gb_);
  return be_->alive_count(buf_[cur_], g_);
}

int Engine::pick_T(int64_t remaining) const {
  if (rows_wrapped_) {  // the LDS-tiled byte kernels: T = 1, 2, 4, ... (powers of two)
    int t = 1;
    while (2 * t <= tmax_ && 2 * t <= remaining) t *= 2;
    return t;
  }
  for (int t : kTSizes)
    if (t <= tmax_ && t <= remaining) return t;
  return 1;
}

// Phase A of the halo exchange (halo_exchange_on): west / east halo columns
// of the owned rows, packed into contiguous buffers (RCCL has no strided
// datatype, unlike the reference's MPI_Type_vector column).
void Engine::exchange_columns(void* buf, const TileGeom& g) {
  auto* base = static_cast<uint8_t*>(buf);
  auto nb = dec_.neighbors(rank_);
  const int64_t H = g.H, pitch = g.pitch;
  if (dec_.Px == 1) {
    if (cols_filled_) {
      void* t = phase_begin(nullptr);
      be_->fill_periodic(buf, g, /*cols=*/true, /*rows=*/false);
      phase_end(kFill, t, nullptr);
    }
    return;
  }
  void* t = phase_begin(nullptr);
  const int64_t halo = 32 * int64_t(g.hw);
  const int64_t span = g.span_bytes(halo);
  const int64_t r0 = g.row0();
  be_->copy_2d_async(colbuf_[0], span, base + g.offset(r0, g.cell0()), pitch, span, H);
  be_->copy_2d_async(colbuf_[1], span, base + g.offset(r0, g.cell0() + g.W - halo), pitch, span, H);
  std::vector<P2POp> ops = {
      {true, nb[kWest], colbuf_[0], size_t(span * H)},
      {false, nb[kEast], colbuf_[3], size_t(span * H)},
      {true, nb[kEast], colbuf_[1], size_t(span * H)},
      {false, nb[kWest], colbuf_[2], size_t(span * H)},
  };
  tr_->exchange(ops, be_->stream());
  halo_bytes_ += 2 * span * H;
  be_->copy_2d_async(base + g.offset(r0, 0), pitch, colbuf_[2], span, span, H);
  be_->copy_2d_async(base + g.offset(r0, g.cell0() + g.W), pitch, colbuf_[3], span, span, H);
  phase_end(kHalo, t, nullptr);
}

// Two-phase halo exchange (columns, then full-width rows so the corner
// cells travel with the rows): 4 messages instead of the reference's 8
// per-generation messages with a strided MPI_Type_vector column
// (src/game_mpi.c:335-383).
void Engine::halo_exchange() { halo_exchange_on(buf_[cur_], g_); }

void Engine::halo_exchange_on(void* buf, const TileGeom& g) {
  trace::Range tr("gol.halo_exchange");
  if (rows_wrapped_ || (rows_ring_ && !cols_filled_)) {
    // Nothing to move: the kernels read the torus modulo its rows, or the
    // row halos alias the owned rows.  No stream join either, so linked
    // launches (GOL_LINK) chain across such epochs.
    ++exchanges_;
    return;
  }
  be_->join_streams();  // transports enqueue on the compute stream directly
  if (rows_ring_) {  // the row halos alias the owned rows; only column halos need a fill
    if (cols_filled_) {
      void* t = phase_begin(nullptr);
      be_->fill_periodic(buf, g, /*cols=*/true, /*rows=*/false);
      phase_end(kFill, t, nullptr);
    }
    ++exchanges_;
    return;
  }
  if (dec_.Px == 1 && dec_.Py == 1 && !cfg_.self_exchange) {  // one rank: both periodic fills, one launch
    void* t = phase_begin(nullptr);
    be_->fill_periodic(buf, g, /*cols=*/cols_filled_, /*rows=*/true);
    phase_end(kFill, t, nullptr);
    ++exchanges_;
    return;
  }
  // Phase A: west/east halo columns of the owned rows.
  exchange_columns(buf, g);
  // Phase B: north/south halo rows over the full padded width.
  if (dec_.Py == 1 && !cfg_.self_exchange) {
    void* t = phase_begin(nullptr);
    be_->fill_periodic(buf, g, /*cols=*/false, /*rows=*/true);
    phase_end(kFill, t, nullptr);
  } else {
    void* t = phase_begin(nullptr);
    tr_->exchange(row_ops(buf, g), be_->stream());
    phase_end(kHalo, t, nullptr);
    halo_bytes_ += 2 * g.Dv * g.pitch;
  }
  ++exchanges_;
}

// North / south halo rows over the full padded width, Dv rows each way.
std::vector<P2POp> Engine::row_ops(void* buf, const TileGeom& g) const {
  auto* base = static_cast<uint8_t*>(buf);
  const auto nb = dec_.neighbors(rank_);
  const int64_t Dv = g.Dv, H = g.H, pitch = g.pitch;
  const size_t bytes = size_t(Dv * pitch);
  return {
      {true, nb[kNorth], base + Dv * pitch, bytes},        // my top rows -> north's bottom halo
      {false, nb[kSouth], base + (Dv + H) * pitch, bytes},  // south's top rows -> my bottom halo
      {true, nb[kSouth], base + H * pitch, bytes},          // my bottom rows -> south's top halo
      {false, nb[kNorth], base, bytes},                     // north's bottom rows -> my top halo
  };
}

void* Engine::bit_scratch(int i) const {
  if (bitbuf_[i]) return bitbuf_[i];
  return static_cast<uint8_t*>(buf_[cur_ ^ 1]) + i * gb_.bytes();
}

// Byte-layout epoch on bit words (run_impl packs the byte tile into
// bit_scratch(bpar_) when a run starts and unpacks it when the run ends): the
// halo exchange or fill and every temporal block run on the bit tile, whose
// per-generation flags are those of the same cells.
void Engine::epoch_via_bits(int64_t d, bool sent_ahead) {
  trace::Range tr("gol.epoch_via_bits");
  if (!sent_ahead) halo_exchange_on(bit_scratch(bpar_), gb_);
  // A partial epoch's trapezoid starts d rows outside the owned rows; a row
  // ring's blocks all cover exactly the owned rows (a = Dv - T).
  const bool full = d == D_;
  int64_t a = D_ - d;
  while (d > 0) {
    const int T = pick_T(d);
    if (rows_ring_) a = gb_.Dv - T;
    if (d == T && trigger_ && send_next_ && full)
      last_block_trigger(bit_scratch(bpar_), bit_scratch(bpar_ ^ 1), gb_, T);
    else if (trigger_ && send_next_ && full)
      hot_block(bit_scratch(bpar_), bit_scratch(bpar_ ^ 1), gb_, T, a + T, gb_.R() - a - T, d);
    else
      add_drift(launch(bit_scratch(bpar_), bit_scratch(bpar_ ^ 1), gb_, T, a + T, gb_.R() - a - T, gen_));
    bpar_ ^= 1;
    gen_ += T;
    a += T;
    d -= T;
  }
}

// The byte grid <-> its bit-word image in the spare byte buffer: a run packs
// the byte grid unless the image is already the state (bits_live_: the
// previous run's result, not unpacked since), and leaves its result in the
// image; the byte tile is brought up to date (sync_bytes) only when someone
// reads it or its buffers (read-out, bands, drift rotation, checkpoints, raw
// views), so back-to-back runs - bench.py's steps - pack and unpack once, not
// per run.  Loading or initialising the byte tile makes it the state again.
// A drifting bit kernel leaves the byte grid drifted by the same amount (a
// relabeling of columns, rotated out by normalize() like the bit layout's).
void Engine::sync_bytes() {
  if (!bits_live_) return;
  unpack_bits();
  bits_live_ = false;
}

void Engine::pack_bits() {
  bpar_ = 0;
  void* t = phase_begin(nullptr);
  be_->convert_rows(buf_[cur_], g_, bit_scratch(0), gb_, 0, g_.H);
  phase_end(kCompute, t, nullptr);
}

void Engine::unpack_bits() {
  void* t = phase_begin(nullptr);
  be_->convert_rows(bit_scratch(bpar_), gb_, buf_[cur_], g_, 0, g_.H);
  phase_end(kCompute, t, nullptr);
}

void Engine::run_epoch(int64_t d) {
  const bool sent_ahead = rows_pending_;
  // The previous epoch's last block sent this buffer's boundary rows
  // (stream-ordered before this epoch's first block).
  rows_pending_ = false;
  // The previous epoch ends here.
  if (auto_overlap_) auto_mark();
  if (via_bits_) {
    epoch_via_bits(d, sent_ahead);
    return;
  }
  if (!sent_ahead) halo_exchange();
  // A partial epoch (d < D) needs only d halo rows: its trapezoid starts d
  // rows outside the owned rows, not D.
  const bool full = d == D_;
  int64_t a = D_ - d;
  while (d > 0) {
    const int T = pick_T(d);
    if (rows_ring_) a = g_.Dv - T;  // every block covers exactly the owned rows
    if (d == T && trigger_ && send_next_ && full) {
      last_block_trigger(buf_[cur_], buf_[cur_ ^ 1], g_, T);
      cur_ ^= 1;
      gen_ += T;
    } else if (trigger_ && send_next_ && full) {
      hot_block(buf_[cur_], buf_[cur_ ^ 1], g_, T, a + T, g_.R() - a - T, d);
      cur_ ^= 1;
      gen_ += T;
    } else {
      step_block(T, a + T, g_.R() - a - T);
    }
    a += T;
    d -= T;
  }
}

void Engine::settle_pending(bool invalidate) {
  if (!rows_pending_) return;
  be_->synchronize();
  if (invalidate) rows_pending_ = false;
}

// Trigger schedule (overlap = 3; Py > 1 or the one-rank RCCL rehearsal, Px
// == 1).  The reference exchanges halos and then waits (MPI_Startall +
// MPI_Waitall before evolve, src/game_mpi.c:392-403).  Here the last temporal
// block of a full epoch writes exactly the owned rows, and the next epoch's
// halos are the first and last Dv of them.  That block runs as one ordinary
// launch whose groups meeting those rows count themselves done on a device
// counter once their rows are written through.  With linked launches it runs
// on the second compute stream, and the first one - whose last work, the
// block before, is done - waits on the counter (Backend::trigger_stream) and
// sends the rows while the block's interior groups still run.  The next
// epoch's first block follows the exchange on that stream and links to the
// last block, so the chain is not restarted at the epoch boundary.  Nothing
// spins on the exchange: it is stream-ordered before the launch that reads
// the halo rows, and it waits only on work already running.  Measured on the
// one-GPU rehearsal: docs/PERFORMANCE.md.
void Engine::last_block_trigger(void* in, void* out, const TileGeom& g, int T) {
  trace::Range tr("gol.last_block_trigger");
  const int64_t Dv = g.Dv, H = g.H, pitch = g.pitch;
  const int64_t rows[4] = {Dv, 2 * Dv, H, H + Dv};
  add_drift(launch(in, out, g, T, Dv, Dv + H, gen_, rows));
  bool armed = false;
  void* s = be_->trigger_stream(&armed);  // not armed: after the whole block (a join)
  if (armed) ++triggered_sends_;
  if (cols_filled_) {  // column halos of the new rows (armed launches wrap their columns: never here)
    void* t = phase_begin(nullptr);
    be_->fill_cols_rows(out, g, Dv, H);
    phase_end(kFill, t, nullptr);
  }
  // Phase timing would join the streams (timing_mark): only when it is on.
  void* tx = phase_begin(s);
  tr_->exchange(row_ops(out, g), s ? s : be_->stream());
  phase_end(kHalo, tx, s);
  rows_pending_ = true;  // stream-ordered before the next block on the compute stream
  halo_bytes_ += 2 * Dv * pitch;
  ++exchanges_;
  ++boundary_sends_;
}

// An earlier block of a trigger epoch (d generations left before it): the
// groups in the light cone of the rows the epoch will send - the first and
// last Dv owned rows widened by the d - T generations still to come - run at
// top issue priority, so that region leads the interior and the last block's
// boundary groups finish ahead of the rest (last_block_trigger).
void Engine::hot_block(void* in, void* out, const TileGeom& g, int T, int64_t row_lo, int64_t row_hi, int64_t d) {
  const int64_t Dv = g.Dv, H = g.H, w = d - T;
  const int64_t rows[4] = {row_lo, 2 * Dv + w, H - w, row_hi};
  add_drift(launch(in, out, g, T, row_lo, row_hi, gen_, rows, /*hot_only=*/true));
}

int Engine::launch(void* in, void* out, const TileGeom& g, int T, int64_t row_lo, int64_t row_hi,
                   int64_t gen_base, const int64_t* trigger_rows, bool hot_only) {
  BlockArgs a;
  a.in = in;
  a.out = out;
  a.g = g;
  a.row_lo = row_lo;
  a.row_hi = row_hi;
  a.T = T;
  a.gen_base = gen_base;
  if (capturing_) {
    // Replayable: the flags offset comes from gen_dev_ at run time.
    a.changed = flags_;
    a.gen_dev = gen_dev_;
    a.gen_rel = gen_base - epoch_start_ + 1;
  } else {
    a.changed =
        (flags_ && gen_base + T < flags_base_ + flags_len_ && gen_base >= flags_base_) ? flags_ : nullptr;
  }
  a.flags_base = flags_base_;
  a.allow_drift = drift_ok_;
  a.full_width = dec_.Px == 1 && cfg_.W % 32 == 0;
  a.wrap_rows = rows_wrapped_;
  // Linked launches assume the device to themselves: not while transport
  // work may run beside them on the comm stream (side polls).  The trigger
  // schedule links: its sends start only once the boundary groups are done,
  // and the next epoch's first block follows them on the same stream.
  a.link = link_ && !poll_side_;
  if (trigger_rows) {
    a.trigger = !hot_only;
    a.hot = hot_only;
    for (int i = 0; i < 4; ++i) a.trigger_rows[i] = trigger_rows[i];
  }
  a.ring = rows_ring_;
  void* t = phase_begin(nullptr);
  const int drift = be_->run_block(a);
  phase_end(kCompute, t, nullptr);
  ++launches_;
  return drift;
}

void Engine::step_block(int T, int64_t row_lo, int64_t row_hi) {
  GOL_REQUIRE(!via_bits_, "step_block: the byte tile has no halos when it computes on bit words (u8_compute)");
  add_drift(launch(buf_[cur_], buf_[cur_ ^ 1], g_, T, row_lo, row_hi, gen_));
  cur_ ^= 1;
  gen_ += T;
}

// Termination polls.  poll_issue() reduces the flags of generations
// (from, to] over ranks (MAX == logical OR) and starts their copy to the
// pinned mirror; poll_check() waits for that copy and scans it.  With lagged
// polling a window is checked only when the next one has been issued, by
// which time the device has long passed it, so the host never drains the
// queue; stopping up to one window late is exact because both stop
// conditions are absorbing.
Engine::Poll Engine::poll_issue(int64_t from, int64_t to) {
  Poll p;
  p.from = from;
  p.to = to;
  const int64_t n = to - from;
  if (n <= 0) return p;
  uint32_t* dev = flags_ + (from + 1 - flags_base_);
  // A side stream that waits for the compute streams' tails without joining
  // them: side polls (the reduction on the flags communicator), and on one
  // rank the copy alone (nothing to reduce, poll_copy_side_) - a linked chain
  // then continues across the poll instead of restarting behind a join (a
  // join, the copy and the restart left the GPU idle ~20 us per poll).
  // Phase timing keeps the compute-stream path (it times the reduction there).
  void* side = nullptr;
  if (poll_side_ || (tr_->size() == 1 && !cfg_.self_exchange && !phase_timing_ && poll_copy_side_))
    side = be_->poll_side();
  if (side) {
    polled_side_ = true;
    void* t = phase_begin(side);
    // The one-rank RCCL rehearsal reduces too, through its 1-rank communicator.
    if (tr_->size() > 1 || cfg_.self_exchange) tr_->allreduce_max_u32(dev, size_t(n), side);
    be_->copy_d2h_async_on(flags_host_ + (from + 1 - flags_base_), dev, size_t(n) * sizeof(uint32_t), side);
    phase_end(kReduce, t, side);
    p.ev = be_->event_record_on(side);
    ++polls_;
    return p;
  }
  be_->join_streams();  // transports enqueue on the compute stream directly
  void* t = phase_begin(nullptr);
  if (tr_->size() > 1) tr_->allreduce_max_u32(dev, size_t(n), be_->stream());
  be_->copy_d2h_async_on(flags_host_ + (from + 1 - flags_base_), dev, size_t(n) * sizeof(uint32_t), nullptr);
  phase_end(kReduce, t, nullptr);
  p.ev = be_->event_record_on(nullptr);
  ++polls_;
  return p;
}

bool Engine::poll_check(Poll& p, int64_t* first_unchanged) {
  if (p.to <= p.from) return false;
  if (!be_->event_query(p.ev)) {
    // Watchdog: poll instead of blocking, check the communicator, and fail
    // with a message rather than hang forever on a dead peer or kernel.
    trace::Range tr("gol.poll_wait");
    const auto t0 = std::chrono::steady_clock::now();
    while (!be_->event_query(p.ev)) {
      tr_->check_health();
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (s > watchdog_s_)
        fail("watchdog: generation " + std::to_string(p.to) + " not reached after " + std::to_string(s) +
             " s (GOL_WATCHDOG_S); a rank or kernel is stuck");
      // Fine-grained while the wait is short (the last poll of a run waits
      // for the run's last blocks: a coarse sleep there idles the GPU before
      // the next run), coarser later.
      // Spin (yield) for the first 2 ms: a sleep overshoots by the kernel's
      // timer slack (~50 us), which idled the GPU at every run boundary.
      if (s < 0.002)
        std::this_thread::yield();
      else
        std::this_thread::sleep_for(std::chrono::microseconds(s < 0.05 ? 20 : 500));
    }
  }
  be_->event_wait(p.ev);
  be_->event_destroy(p.ev);
  p.ev = nullptr;
  be_->check_device_errors();
  const uint32_t* h = flags_host_ + (p.from + 1 - flags_base_);
  for (int64_t i = 0; i < p.to - p.from; ++i)
    if (h[i] == 0) {
      *first_unchanged = p.from + 1 + i;
      return true;
    }
  return false;
}

int64_t reported_generations(int64_t first_unchanged, bool extinct, int64_t limit, int64_t start_gen,
                             bool check_similarity, int sim_freq, int sim_phase, std::string* reason) {
  std::string why = "limit";
  int64_t gens = limit;
  if (first_unchanged >= 0 && first_unchanged <= limit) {
    why = "fixed_point";
    if (extinct) {
      // G_{g_f - 1} is the first empty grid: the loop's emptiness test stops
      // at the next iteration and reports g_f - 1 (src/game.c:177).
      gens = first_unchanged - 1;
      why = "extinction";
    } else if (check_similarity) {
      // Similarity checks happen at generations t > start_gen with
      // (t - start_gen + sim_phase) % F == 0 (counter reset only on a failed
      // check, src/game.c:181-189); the first one at or after g_f fires and
      // reports t - 1 (the break skips generation++).  The phase is anchored
      // at the configured start generation, so an earlier advance() or
      // run_until() on the same engine does not shift it.
      const int64_t F = sim_freq;
      const int64_t k = first_unchanged - start_gen + sim_phase;
      const int64_t tsim = first_unchanged + ((F - (k % F)) % F);
      if (tsim <= limit) {
        gens = tsim - 1;
        why = "similarity";
      }
    }
  }
  if (reason) *reason = why;
  return gens;
}

RunResult Engine::run() { return run_impl(cfg_.gen_limit, /*stop_early=*/true); }

RunResult Engine::run_until(int64_t limit) {
  return run_impl(std::min(limit, cfg_.gen_limit), /*stop_early=*/true);
}

RunResult Engine::advance(int64_t n) { return run_impl(gen_ + n, /*stop_early=*/false); }

RunResult Engine::run_impl(int64_t limit, bool stop_early) {
  RunResult res;
  const int64_t start = gen_;
  if (limit < start) limit = start;
  // (Re)allocate per-generation flags for (start, limit].
  const int64_t need = limit - start + 2;
  if (!flags_ || flags_len_ < need) {
    if (flags_) be_->release(flags_);
    if (flags_host_) be_->release_host(flags_host_);
    flags_len_ = std::max<int64_t>(need, 64);
    flags_ = static_cast<uint32_t*>(be_->alloc(size_t(flags_len_) * 4));
    flags_host_ = static_cast<uint32_t*>(be_->alloc_host(size_t(flags_len_) * 4));
  }
  flags_base_ = start;
  be_->memset_async(flags_, 0, size_t(flags_len_) * 4);
  if (use_graphs_) {
    if (graph_flags_ != flags_) release_graphs();  // kernel arguments point at the flags
    graph_flags_ = flags_;
    be_->i64_async(gen_dev_, 0, /*add=*/false);  // first epoch starts at flags_base_
  }
  const int64_t g0 = graph_runs_;
  const int64_t e0 = exchanges_, p0 = polls_, l0 = launches_, hb0 = halo_bytes_, es0 = boundary_sends_;
  const int64_t lk0 = be_->linked_launches();
  trace::Range trace_run("gol.run");
  if (cfg_.timing_barriers) {
    settle_pending(false);  // one stream at a time on the communicator
    tr_->barrier();
    be_->synchronize();
  }
  // Without timing barriers (a caller that brackets the run itself, bench.py)
  // the flag reset stays queued ahead of the first block: no host round trip
  // between two runs (8192^2: ~2 % of a 1000-generation run).
  auto t0 = std::chrono::steady_clock::now();
  if (via_bits_ && !bits_live_) pack_bits();

  int64_t checked = start, found = -1;
  const int64_t poll_epochs = std::max<int64_t>(1, poll_gens_ / D_);
  int64_t epoch = 0;
  Poll pending;
  bool have_pending = false;
  while (gen_ < limit) {
    const int64_t d = std::min<int64_t>(D_, limit - gen_);
    send_next_ = gen_ + d < limit;
    if (use_graphs_ && d == D_) {
      // Full epochs replay a captured graph; the only per-epoch input is the
      // device generation offset, advanced by the graph itself.  Graphs are
      // keyed by the parity of the buffer pair the epochs alternate over and
      // by the addresses baked into them (graph_key).
      int& cur = via_bits_ ? bpar_ : cur_;
      const int par = graph_key();
      if (!graph_[par]) {
        const int64_t k0 = launches_;
        const int64_t dr0 = drift_;
        capturing_ = true;
        epoch_start_ = gen_;
        be_->capture_begin();
        run_epoch(d);
        be_->i64_async(gen_dev_, D_, /*add=*/true);
        graph_[par] = be_->capture_end();
        capturing_ = false;
        graph_flip_[par] = cur ^ (par & 1);
        graph_kernels_[par] = launches_ - k0;
        graph_drift_[par] = ((drift_ - dr0) % cfg_.W + cfg_.W) % cfg_.W;
        be_->graph_launch(graph_[par]);  // capture only recorded it
      } else {
        be_->graph_launch(graph_[par]);
        cur ^= graph_flip_[par];
        add_drift(graph_drift_[par]);
        gen_ += D_;
        ++exchanges_;
        launches_ += graph_kernels_[par];
      }
      ++graph_runs_;
    } else {
      if (use_graphs_) be_->i64_async(gen_dev_, d, /*add=*/true);  // keep the offset in step
      if (auto_overlap_) auto_choose(d == D_ && send_next_);
      run_epoch(d);
    }
    ++epoch;
    if (stop_early && (epoch % poll_epochs == 0 || gen_ == limit)) {
      if (poll_trial_) poll_trial_step();
      Poll p = poll_issue(checked, gen_);
      checked = gen_;
      if (have_pending && poll_check(pending, &found)) {
        have_pending = false;
        if (p.ev) be_->event_destroy(p.ev);
        break;
      }
      pending = p;
      have_pending = true;
      if (!cfg_.lagged_poll || gen_ == limit) {
        have_pending = false;
        if (poll_check(pending, &found)) break;
      }
    }
  }
  if (have_pending) poll_check(pending, &found);
  if (via_bits_) bits_live_ = true;  // unpacked when the byte tile is next read (sync_bytes)
  // A poll issued just before an early stop may still run on the side stream
  // (the final alive reduction below uses the same communicator, and the
  // next run may reallocate the flags it reads).
  if (polled_side_) be_->synchronize_stream(be_->comm_stream());
  polled_side_ = false;
  be_->synchronize();
  be_->check_device_errors();
  if (auto_open_) {  // an auto-trial epoch span does not continue into the next run
    be_->timing_release(auto_open_);
    auto_open_ = nullptr;
  }
  if (ptrial_open_) {  // nor does a poll-trial window
    be_->timing_release(ptrial_open_);
    ptrial_open_ = nullptr;
  }
  if (cfg_.timing_barriers) {
    settle_pending(false);
    tr_->barrier();
  }
  auto t1 = std::chrono::steady_clock::now();
  res.loop_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  res.executed = gen_ - start;
  res.exchanges = exchanges_ - e0;
  res.polls = polls_ - p0;
  res.kernel_launches = launches_ - l0;
  res.overlapped = boundary_sends_ > es0;
  res.graph_launches = graph_runs_ - g0;
  res.halo_bytes = halo_bytes_ - hb0;
  res.linked_launches = be_->linked_launches() - lk0;
  res.generations = limit;
  collect_phases(res);
  if (found >= 0) {
    res.first_unchanged = found;
    if (bits_live_)
      be_->alive_any(bit_scratch(bpar_), gb_, alive_dev_);
    else
      be_->alive_any(buf_[cur_], g_, alive_dev_);
    if (tr_->size() > 1) tr_->allreduce_max_u32(alive_dev_, 1, be_->stream());
    uint32_t alive = 0;
    be_->copy_d2h(&alive, alive_dev_, 4);
    res.extinct = !alive;
    res.generations = reported_generations(found, res.extinct, limit, cfg_.start_gen, cfg_.check_similarity,
                                           cfg_.sim_freq, cfg_.sim_phase, &res.stop_reason);
  }
  return res;
}

// ---- overlap auto trial ---------------------------------------------------
// The schedule of each full epoch is a function of the epoch count only, so
// every rank runs the same sequence, reaches the decision at the same epoch
// and issues the decision's all-reduce at the same point of its operation
// stream (RCCL matches operations by issue order).
void Engine::auto_choose(bool full_epoch) {
  int sched = 0;
  int trial = -1;
  if (full_epoch) {
    const int64_t i = auto_full_epochs_++;
    if (i >= kAutoWarm) {
      sched = ((i - kAutoWarm) % 2 == 0) ? 1 : 0;
      trial = sched;
    }
  }
  trigger_ = sched == 1;
  auto_sched_ = trial;
}

void Engine::auto_mark() {
  if (auto_open_) {
    void* end = be_->timing_mark(nullptr);
    if (auto_open_sched_ >= 0) {
      auto_spans_.push_back({auto_open_sched_, auto_open_, end});
      ++auto_counts_[auto_open_sched_];
    } else {
      be_->timing_release(auto_open_);
      be_->timing_release(end);
    }
    auto_open_ = nullptr;
  }
  if (auto_counts_[0] >= kAutoTrials && auto_counts_[1] >= kAutoTrials) {
    auto_decide();
    return;
  }
  auto_open_ = be_->timing_mark(nullptr);
  auto_open_sched_ = auto_sched_;
}

// Medians of two schedules' timed spans, MAX over ranks (the slowest rank
// decides; every rank gets the same values), in ms; releases the spans.
void Engine::trial_medians(std::vector<AutoSpan>& spans, double out[2]) {
  std::vector<double> ms[2];
  for (auto& sp : spans) {
    ms[sp.sched].push_back(be_->timing_ms(sp.a, sp.b));
    be_->timing_release(sp.a);
    be_->timing_release(sp.b);
  }
  spans.clear();
  uint32_t v[2];
  for (int k = 0; k < 2; ++k) {
    std::sort(ms[k].begin(), ms[k].end());
    const double med = ms[k].empty() ? 0.0 : ms[k][ms[k].size() / 2];
    v[k] = uint32_t(std::min(4.0e9, std::max(0.0, med * 1e4)));  // 0.1 us units
  }
  uint32_t* dev = alive_dev_ + 4;
  be_->copy_h2d(dev, v, sizeof(v));
  if (tr_->size() > 1) tr_->allreduce_max_u32(dev, 2, be_->stream());
  be_->copy_d2h(v, dev, sizeof(v));
  out[0] = v[0] * 1e-4;
  out[1] = v[1] * 1e-4;
}

// Poll placement trial (tuning side_poll = -1).  Once the overlap trial has
// decided (and where polls do not ride the comm stream with the exchanges),
// the poll windows - from one termination poll to the next - alternate a
// poll whose flag all-reduce joins the compute stream and one that runs on a
// side stream through the transport's flags communicator (poll_side_, which
// also leaves linked launches off for that window: transport work may run
// beside them), after two warm-up windows; each window is timed from its
// poll's issue to the next's on the compute stream, and when kAutoTrials of
// each are in, at the same poll on every rank, the medians are MAX-reduced
// and every rank keeps the faster placement.  A side decision is then
// checked on kAutoTrials consecutive side windows (after one warm-up) and
// kept only if their median still beats the joined median: windows that
// alternate with joined ones can time faster than a run of side windows (the
// rehearsed rank tiles with the second linked stream on its own queue: side
// chosen, then 2x slower).  The reference all-reduces every generation on
// the critical path (src/game_mpi_collective.c:70-109).
void Engine::poll_trial_step() {
  if (auto_overlap_) return;  // the overlap trial runs first
  if (ptrial_open_) {
    void* end = be_->timing_mark(nullptr);
    if (ptrial_mode_ >= 0) {
      ptrial_spans_.push_back({ptrial_mode_, ptrial_open_, end});
      ++ptrial_counts_[ptrial_mode_];
    } else {
      be_->timing_release(ptrial_open_);
      be_->timing_release(end);
    }
    ptrial_open_ = nullptr;
  }
  if (!ptrial_verify_ && ptrial_counts_[0] >= kAutoTrials && ptrial_counts_[1] >= kAutoTrials) {
    trial_medians(ptrial_spans_, poll_ms_);
    if (poll_ms_[1] < 0.98 * poll_ms_[0]) {  // side wins the alternation: check a run of side windows
      ptrial_verify_ = true;
      ptrial_counts_[0] = ptrial_counts_[1] = 0;
      ptrial_polls_ = 0;
    } else {
      poll_side_ = false;
      poll_trial_ = false;
      poll_decided_ = true;
      return;
    }
  } else if (ptrial_verify_ && ptrial_counts_[1] >= kAutoTrials) {
    double v[2];
    trial_medians(ptrial_spans_, v);
    poll_side_steady_ms_ = v[1];
    poll_side_ = v[1] < poll_ms_[0];
    poll_trial_ = false;
    poll_decided_ = true;
    return;
  }
  const int64_t i = ptrial_polls_++;
  if (ptrial_verify_)
    ptrial_mode_ = i < 1 ? -1 : 1;
  else
    ptrial_mode_ = i < kAutoWarm ? -1 : int((i - kAutoWarm) % 2);
  poll_side_ = ptrial_verify_ || ptrial_mode_ == 1;
  ptrial_open_ = be_->timing_mark(nullptr);
}

std::string Engine::poll_mode() const {
  if (poll_trial_) return "auto:trial";
  if (poll_decided_) return poll_side_ ? "auto:side" : "auto:joined";
  return poll_side_ ? "side" : "joined";
}

void Engine::auto_decide() {
  // Slowest rank decides: every rank ends up with the same MAX values.
  trial_medians(auto_spans_, auto_ms_);
  const double v[2] = {auto_ms_[0], auto_ms_[1]};
  bool alt = v[1] < 0.98 * v[0];
  const std::string& forced = cfg_.tune.s("overlap_auto");  // fault injection (tests)
  GOL_REQUIRE(forced.empty() || forced == "plain" || forced == "trigger",
              "tuning overlap_auto=" + forced + ": plain or trigger");
  if (!forced.empty()) alt = forced == "trigger";
  trigger_ = alt;
  auto_overlap_ = false;
  auto_decided_ = true;
}

std::string Engine::overlap_mode() const {
  if (cfg_.overlap == 3) return trigger_ ? "trigger" : "off";
  if (cfg_.overlap == -1) {
    if (auto_overlap_) return "auto:trial";
    if (auto_decided_) return trigger_ ? "auto:trigger" : "auto:plain";
  }
  return "off";
}

// ---- phase timing -----------------------------------------------------------
void* Engine::phase_begin(void* stream) {
  if (!phase_timing_ || capturing_ || phase_spans_.size() >= kMaxPhaseSpans) return nullptr;
  return be_->timing_mark(stream);
}

void Engine::phase_end(int phase, void* a, void* stream) {
  if (!a) return;
  phase_spans_.push_back({phase, a, be_->timing_mark(stream)});
}

void Engine::collect_phases(RunResult& res) {
  if (!phase_timing_) return;
  double ms[kPhases] = {0, 0, 0, 0};
  for (auto& sp : phase_spans_) {
    ms[sp.phase] += be_->timing_ms(sp.a, sp.b);
    be_->timing_release(sp.a);
    be_->timing_release(sp.b);
  }
  phase_spans_.clear();
  res.phase_timed = true;
  res.compute_ms = ms[kCompute];
  res.halo_ms = ms[kHalo];
  res.fill_ms = ms[kFill];
  res.allreduce_ms = ms[kReduce];
}

}  // namespace gol
