// gol: command-line front end, contract-compatible with the reference's
// `./a.out <width> <height> <input_file>` (README.md:50-57, src/game.c:224-245).
//
//   gol 1024 1024 input.txt                 # like the serial build
//   gol 32768 32768 --random 7 --gpus 8     # 8 GPUs in one process
//   gol 96 96 in.txt --engine ref           # exact serial src/game.c loop
//
// Width/height default to 30 when <= 0 (src/game.c:233-236); without an
// input file (and no --random) nothing runs and only "Finished" is printed
// (src/game.c:238-241).  The compile-time knobs of the reference
// (GEN_LIMIT, CHECK_SIMILARITY, SIMILARITY_FREQUENCY: README.md:65) are
// runtime flags with the same defaults.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "gol/backend.hpp"
#include "gol/checkpoint.hpp"
#include "gol/cpu_ref.hpp"
#include "gol/engine.hpp"
#include "gol/io.hpp"
#include "gol/transport.hpp"

using namespace gol;

namespace {

// A JSON string literal of s (quotes, backslashes and control bytes escaped):
// tuning values such as trace paths are arbitrary text.
std::string jstr(const std::string& s) {
  std::string o = "\"";
  for (const unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += char(c);
    } else if (c < 0x20) {
      char b[8];
      std::snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else {
      o += char(c);
    }
  }
  return o + "\"";
}

struct Options {
  int64_t W = 0, H = 0;
  std::string input;
  std::string engine = "auto";  // auto | hip | cpu | ref
  std::string layout = "auto";  // auto | bits | u8
  std::string decomp = "auto";
  std::string comm = "auto";  // auto | thread | rccl (in-process ranks)
  std::string output;  // default: the matching reference build's file (see default_output)
  std::string style = "serial";  // serial | mpi | async | collective | openmp | cuda
  std::string metrics;
  int64_t gens = 1000;
  int sim_freq = 3;
  bool similarity = true;
  bool random = false;
  uint64_t seed = 1;
  double density = 0.5;
  int ranks = 1, gpus = 0, threads = 0, tmax = 0, epoch = 0, poll = 0, overlap = -1, graphs = 0;
  int u8_compute = -1;  // auto | bytes (0) | bits (1)
  bool show = false;
  bool phase_timing = false;  // per-phase device times in --metrics-json
  int64_t checkpoint_every = 0;     // generations between checkpoints (0: none)
  int64_t start_gen = 0;            // resume: generation of the loaded grid
  int sim_phase = 0;                // resume: similarity counter at start_gen
  std::string checkpoint_dir;       // where they go
  std::string resume;               // checkpoint directory to resume from
  bool gens_set = false, sim_set = false;
  Tuning tune = Tuning::from_env();  // --tune key=value over the GOL_* environment
};

[[noreturn]] void usage(int code) {
  std::fprintf(code ? stderr : stdout,
               "usage: gol [width] [height] [input_file] [options]\n"
               "  --engine auto|hip|cpu|ref   compute engine (ref = exact serial game.c loop)\n"
               "  --layout auto|bits|u8       cell storage (bits needs width %% 32 == 0)\n"
               "  --u8-compute auto|bits|bytes  byte-layout epochs on bit words (packed once per\n"
               "                              epoch; auto: on the GPU) or on the bytes themselves\n"
               "  --gens N                    GEN_LIMIT (default 1000)\n"
               "  --sim-freq F                SIMILARITY_FREQUENCY (default 3)\n"
               "  --no-similarity             disable the similarity check\n"
               "  --random SEED[:DENSITY]     random initial grid instead of an input file\n"
               "  --output PATH|none          output file (default: the reference build's name for\n"
               "                              --style: ./game_output.out, ./mpi_output.out, ...)\n"
               "  --gpus N                    run on N GPUs in this process (one rank each)\n"
               "  --ranks N                   in-process ranks (subdomains; share devices)\n"
               "  --comm auto|thread|rccl     in-process halo transport (auto: rccl when every rank\n"
               "                              has a GPU of its own, else thread)\n"
               "  --decomp auto|PxQ           process grid (Px columns x Py rows)\n"
               "  --tmax T --epoch D --poll N temporal block, halo depth, poll interval\n"
               "  --overlap auto|on|off|trigger\n"
               "                              trigger = an epoch's new boundary rows are sent as soon\n"
               "                              as the groups writing them finish (on = trigger);\n"
               "                              off = no overlap; auto = time plain against trigger\n"
               "                              epochs on the ranks, keep the faster\n"
               "  --graphs auto|on|off        replay full epochs as captured HIP graphs\n"
               "  --threads N                 host threads for the cpu engine\n"
               "  --tune KEY=VALUE            runtime tuning (repeatable; --tune help lists the keys,\n"
               "                              their GOL_* overrides and defaults)\n"
               "  --style serial|mpi|async|collective|openmp|cuda\n"
               "                              stdout format and output name of that reference build\n"
               "  --metrics-json PATH         write run metrics as JSON\n"
               "  --phase-timing              time kernels / halos / fills / reductions (per-phase\n"
               "                              device times in --metrics-json; adds events to the loop)\n"
               "  --checkpoint-every K        write a checkpoint every K generations ...\n"
               "  --checkpoint-dir DIR        ... into DIR (grid-<gen>.txt + meta.json; crash-safe)\n"
               "  --resume DIR                continue from a checkpoint: same final grid and\n"
               "                              Generations line as the uninterrupted run\n"
               "  --show                      print the final grid with VT100 escapes\n");
  std::exit(code);
}

Options parse(int argc, char** argv) {
  Options o;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) usage(2);
      return argv[++i];
    };
    if (a == "-h" || a == "--help") usage(0);
    else if (a == "--engine") o.engine = next();
    else if (a == "--layout") o.layout = next();
    else if (a == "--u8-compute") {
      std::string v = next();
      if (v != "auto" && v != "bits" && v != "bytes") usage(2);
      o.u8_compute = v == "bits" ? 1 : v == "bytes" ? 0 : -1;
    }
    else if (a == "--decomp") o.decomp = next();
    else if (a == "--comm") o.comm = next();
    else if (a == "--gens") o.gens = std::atoll(next().c_str()), o.gens_set = true;
    else if (a == "--sim-freq") o.sim_freq = std::atoi(next().c_str()), o.sim_set = true;
    else if (a == "--no-similarity") o.similarity = false, o.sim_set = true;
    else if (a == "--checkpoint-every") o.checkpoint_every = std::atoll(next().c_str());
    else if (a == "--checkpoint-dir") o.checkpoint_dir = next();
    else if (a == "--resume") o.resume = next();
    else if (a == "--output") o.output = next();
    else if (a == "--style") o.style = next();
    else if (a == "--metrics-json") o.metrics = next();
    else if (a == "--gpus") o.gpus = std::atoi(next().c_str());
    else if (a == "--ranks") o.ranks = std::atoi(next().c_str());
    else if (a == "--threads") o.threads = std::atoi(next().c_str());
    else if (a == "--tune") {
      const std::string kv = next();
      if (kv == "help") {
        for (const TuningKey& k : tuning_keys())
          std::printf("%-22s %-13s %-27s default %-6s %s\n", k.key, k.cls, k.env, *k.dflt ? k.dflt : "''", k.doc);
        std::exit(0);
      }
      o.tune.set(kv);
    }
    else if (a == "--tmax") o.tmax = std::atoi(next().c_str());
    else if (a == "--epoch" || a == "--halo-depth") o.epoch = std::atoi(next().c_str());
    else if (a == "--poll" || a == "--poll-every") o.poll = std::atoi(next().c_str());
    else if (a == "--overlap") {
      std::string v = next();
      GOL_REQUIRE(v == "auto" || v == "on" || v == "off" || v == "trigger", "--overlap: auto, on, off or trigger");
      o.overlap = v == "on" ? 3 : v == "off" ? 0 : v == "trigger" ? 3 : -1;
    } else if (a == "--graphs") {
      std::string v = next();
      o.graphs = v == "on" ? 1 : v == "off" ? 0 : -1;
    }
    else if (a == "--show") o.show = true;
    else if (a == "--phase-timing") o.phase_timing = true;
    else if (a == "--random") {
      std::string v = next();
      o.random = true;
      auto c = v.find(':');
      o.seed = std::strtoull(v.substr(0, c).c_str(), nullptr, 10);
      if (c != std::string::npos) o.density = std::atof(v.substr(c + 1).c_str());
    } else if (!a.empty() && a[0] == '-' && a.size() > 1) {
      std::fprintf(stderr, "unknown option %s\n", a.c_str());
      usage(2);
    } else pos.push_back(a);
  }
  if (pos.size() > 0) o.W = std::atoll(pos[0].c_str());
  if (pos.size() > 1) o.H = std::atoll(pos[1].c_str());
  if (pos.size() > 2) o.input = pos[2];
  if (!o.resume.empty()) {
    // The checkpoint fixes the grid and the counters; --gens / --sim-freq /
    // --no-similarity given on the command line still win.
    const CheckpointMeta m = checkpoint_load(o.resume);
    if ((o.W > 0 && o.W != m.W) || (o.H > 0 && o.H != m.H))
      throw Error("--resume: checkpoint is " + std::to_string(m.W) + "x" + std::to_string(m.H) +
                  ", not the requested " + std::to_string(o.W) + "x" + std::to_string(o.H));
    o.W = m.W;
    o.H = m.H;
    o.input = checkpoint_grid_path(o.resume);
    if (!o.gens_set) o.gens = m.gen_limit;
    // The checkpoint's similarity phase counts modulo its own frequency; a
    // different one would match neither the original run nor a fresh run
    // at the new frequency.
    if (o.sim_set && o.similarity && o.sim_freq != m.sim_freq)
      throw Error("--resume: checkpoint was taken with --sim-freq " + std::to_string(m.sim_freq) +
                  "; resuming with --sim-freq " + std::to_string(o.sim_freq) + " would shift the similarity checks");
    if (!o.sim_set) o.similarity = m.check_similarity;
    o.sim_freq = m.sim_freq;
    o.start_gen = m.generation;
    o.sim_phase = m.sim_phase;
    if (o.layout == "auto" && (m.layout == "bits" || m.layout == "u8")) o.layout = m.layout;
  }
  if (o.W <= 0) o.W = 30;
  if (o.H <= 0) o.H = 30;
  if (o.gpus > 0) o.ranks = o.gpus;
  // --metrics-json does not imply --phase-timing: the event pairs around
  // every kernel, exchange, fill and reduction would sit inside the timed
  // loop that loop_ms and cell_updates_per_s report.
  static const char* kStyles[] = {"serial", "mpi", "async", "collective", "openmp", "cuda"};
  if (std::find(std::begin(kStyles), std::end(kStyles), o.style) == std::end(kStyles)) usage(2);
  // Output file of the matching reference build: src/game.c:27,
  // src/game_mpi.c:29, src/game_mpi_async.c:432, src/game_mpi_collective.c:429,
  // src/game_openmp.c:445, src/game_cuda.cu:37.
  if (o.output.empty()) o.output = "./" + std::string(o.style == "serial" ? "game" : o.style) + "_output.out";
  return o;
}

void show(const std::vector<uint8_t>& g, int64_t W, int64_t H) {
  // VT100 viewer (src/game.c:42-58): reverse video for live cells.
  std::printf("\033[H");
  for (int64_t y = 0; y < H; ++y) {
    for (int64_t x = 0; x < W; ++x) std::printf(g[size_t(y * W + x)] ? "\033[07m  \033[m" : "  ");
    std::printf("\033[E");
  }
  std::fflush(stdout);
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int run(const Options& o) {
  const bool have_input = o.random || !o.input.empty();
  if (!have_input) {
    std::printf("Finished\n");
    return 0;
  }
  std::string engine = o.engine;
  if (engine == "auto") engine = hip_available() ? "hip" : "cpu";
  Layout layout = Layout::Bits;
  if (o.layout == "u8" || (o.layout == "auto" && o.W % 32 != 0)) layout = Layout::U8;
  else if (o.layout != "auto" && o.layout != "bits") throw Error("unknown layout " + o.layout);

  double read_ms = 0, write_ms = 0;
  RunResult res;
  std::vector<uint8_t> final_grid;
  const bool want_grid = o.output != "none" || o.show;

  if (engine == "ref" && (!o.resume.empty() || o.checkpoint_every > 0))
    throw Error("--engine ref is the plain serial loop from generation 0: no checkpoint / resume");
  if (engine == "ref") {
    // Exact serial semantics (src/game.c), every generation evaluated eagerly.
    auto t0 = std::chrono::steady_clock::now();
    std::vector<uint8_t> grid;
    if (o.random) {
      grid.resize(size_t(o.W * o.H));
      uint32_t th = density_thresh(o.density);
      for (int64_t r = 0; r < o.H; ++r)
        for (int64_t x = 0; x < o.W; ++x) grid[size_t(r * o.W + x)] = rng_cell(o.seed, r, x, th);
    } else {
      read_text_grid(o.input, o.W, o.H, grid);
    }
    read_ms = ms_since(t0);
    RefResult rr = cpu_reference_run(grid, o.W, o.H, o.gens, o.similarity, o.sim_freq, o.threads);
    res.generations = rr.generations;
    res.loop_ms = rr.loop_ms;
    res.executed = rr.generations;
    final_grid = std::move(grid);
    if (o.output != "none") {
      auto t1 = std::chrono::steady_clock::now();
      write_text_grid(o.output, o.W, o.H, final_grid.data());
      write_ms = ms_since(t1);
    }
  } else {
    const int P = std::max(1, o.ranks);
    EngineConfig cfg;
    cfg.W = o.W;
    cfg.H = o.H;
    cfg.layout = layout;
    cfg.decomp = o.decomp;
    cfg.gen_limit = o.gens;
    cfg.check_similarity = o.similarity;
    cfg.sim_freq = o.sim_freq;
    cfg.tmax = o.tmax;
    cfg.epoch = o.epoch;
    cfg.poll_gens = o.poll;
    cfg.overlap = o.overlap;
    cfg.graphs = o.graphs;
    cfg.u8_compute = o.u8_compute;
    cfg.start_gen = o.start_gen;
    cfg.sim_phase = o.sim_phase;
    cfg.tune = o.tune;
    int ndev = 1;
    if (engine == "hip") {
      GOL_REQUIRE(hip_available(), "--engine hip: no HIP device available");
      ndev = o.gpus > 0 ? o.gpus : 1;
    }
    std::vector<std::unique_ptr<Backend>> backends(P);
    std::vector<std::unique_ptr<Transport>> transports(P);
    std::vector<std::unique_ptr<Engine>> engines(P);
    auto hub = std::make_shared<ThreadHub>(P);
    // One process, P rank threads.  RCCL needs every rank on a GPU of its
    // own (it refuses duplicate devices in one communicator); ranks that
    // share devices, and CPU ranks, use the thread transport.
    std::string comm = o.comm;
    if (comm == "auto") comm = (engine == "hip" && P > 1 && P <= ndev) ? "rccl" : "thread";
    if (comm == "rccl" && P > 1) {
      GOL_REQUIRE(engine == "hip", "--comm rccl needs --engine hip");
      GOL_REQUIRE(P <= ndev, "--comm rccl needs one GPU per rank (--gpus N, not --ranks)");
    }
    std::vector<uint8_t> uid;
    if (comm == "rccl" && P > 1) uid = rccl_unique_id();
    for (int r = 0; r < P; ++r)
      backends[r] = engine == "hip" ? make_hip_backend(r % ndev, o.tune)
                                    : make_cpu_backend(o.threads > 0 ? o.threads : 0, -1, o.tune);
    if (P == 1) {
      transports[0] = std::make_unique<SelfTransport>();
    } else if (comm == "rccl") {
      std::vector<std::thread> th;
      std::vector<std::string> errs(P);
      for (int r = 0; r < P; ++r)
        th.emplace_back([&, r] {
          try {
            backends[r]->bind_thread();
            transports[r] = make_rccl_transport(uid, r, P, r % ndev, o.tune);
          } catch (const std::exception& e) {
            errs[r] = e.what();
          }
        });
      for (auto& t : th) t.join();
      for (auto& e : errs)
        if (!e.empty()) throw Error(e);
    } else {
      for (int r = 0; r < P; ++r) transports[r] = std::make_unique<ThreadTransport>(hub, r, backends[r].get(), o.tune);
    }
    for (int r = 0; r < P; ++r) {
      engines[r] = std::make_unique<Engine>(cfg, backends[r].get(), transports[r].get());
      engines[r]->set_phase_timing(o.phase_timing);
    }

    auto par = [&](const std::function<void(int)>& fn) {
      std::vector<std::thread> th;
      std::vector<std::string> errs(P);
      for (int r = 0; r < P; ++r)
        th.emplace_back([&, r] {
          try {
            backends[r]->bind_thread();  // a new thread starts on device 0
            fn(r);
          } catch (const std::exception& e) {
            errs[r] = e.what();
          }
        });
      for (auto& t : th) t.join();
      for (auto& e : errs)
        if (!e.empty()) throw Error(e);
    };

    auto t0 = std::chrono::steady_clock::now();
    std::vector<double> parse_ms(P, 0.0), load_ms(P, 0.0);
    par([&](int r) {
      Engine& e = *engines[r];
      if (o.random) {
        e.init_random(o.seed, o.density);
      } else {
        // Uninitialised host tile (a multi-GB zero fill would cost more than
        // the parallel read that overwrites it).
        const auto a = std::chrono::steady_clock::now();
        std::unique_ptr<uint8_t[]> tile(new uint8_t[size_t(e.rows().size() * e.cols().size())]);
        read_text_tile_into(o.input, o.W, o.H, e.rows(), e.cols(), tile.get(), e.cols().size());
        parse_ms[r] = ms_since(a);
        const auto b = std::chrono::steady_clock::now();
        e.load_cells(tile.get(), e.cols().size());
        load_ms[r] = ms_since(b);
      }
    });
    read_ms = ms_since(t0);
    const double read_parse_ms = *std::max_element(parse_ms.begin(), parse_ms.end());
    const double read_load_ms = *std::max_element(load_ms.begin(), load_ms.end());
    // Generation loop, in chunks of --checkpoint-every generations when
    // checkpointing (each chunk ends with every rank's tile on disk).
    std::vector<RunResult> results(P);
    RunResult total;
    const int64_t limit = o.gens;
    int64_t checkpoints_written = 0;
    for (;;) {
      const int64_t gen = engines[0]->generation();
      const int64_t target = o.checkpoint_every > 0 ? std::min(limit, gen + o.checkpoint_every) : limit;
      par([&](int r) { results[r] = engines[r]->run_until(target); });
      double ms = 0;
      for (auto& rr : results) ms = std::max(ms, rr.loop_ms);
      total.loop_ms += ms;
      total.executed += results[0].executed;
      total.exchanges += results[0].exchanges;
      total.polls += results[0].polls;
      total.kernel_launches += results[0].kernel_launches;
      // Per-phase device times: the slowest rank's, like loop_ms.
      for (auto& rr : results) {
        total.phase_timed = total.phase_timed || rr.phase_timed;
      }
      const RunResult* slow = &results[0];
      for (auto& rr : results)
        if (rr.loop_ms > slow->loop_ms) slow = &rr;
      total.compute_ms += slow->compute_ms;
      total.halo_ms += slow->halo_ms;
      total.fill_ms += slow->fill_ms;
      total.allreduce_ms += slow->allreduce_ms;
      const RunResult& last = results[0];
      if (last.first_unchanged >= 0 || engines[0]->generation() >= limit) {
        total.first_unchanged = last.first_unchanged;
        total.extinct = last.extinct;
        total.generations = reported_generations(last.first_unchanged, last.extinct, limit, o.start_gen,
                                                 o.similarity, o.sim_freq, o.sim_phase, &total.stop_reason);
        break;
      }
      if (!o.checkpoint_dir.empty()) {
        const int64_t g = engines[0]->generation();
        const std::string grid_path = checkpoint_begin(o.checkpoint_dir, o.W, o.H, g);
        par([&](int r) {
          Engine& e = *engines[r];
          std::vector<uint8_t> tile(size_t(e.rows().size() * e.cols().size()));
          e.store_cells(tile.data(), e.cols().size(), false);
          write_text_tile(grid_path, o.W, o.H, e.rows(), e.cols(), tile.data(),
                          e.cols().size());
        });
        CheckpointMeta m;
        m.W = o.W;
        m.H = o.H;
        m.generation = g;
        m.sim_phase = sim_phase_at(g, o.start_gen, o.sim_phase, o.sim_freq);
        m.gen_limit = limit;
        m.check_similarity = o.similarity;
        m.sim_freq = o.sim_freq;
        m.layout = layout_name(layout);
        // Fault injection (tests): die after the N-th checkpoint's tiles are
        // written, before it is committed.
        if (const int c = o.tune.i("fault_checkpoint_crash"))
          if (++checkpoints_written == c) std::_Exit(86);
        checkpoint_commit(o.checkpoint_dir, grid_path, m);
      }
    }
    res = total;

    std::vector<double> store_ms(P, 0.0), format_ms(P, 0.0);
    if (want_grid) {
      auto t1 = std::chrono::steady_clock::now();
      if (o.output != "none") create_text_file(o.output, o.W, o.H);
      if (o.show) final_grid.assign(size_t(o.W * o.H), 0);
      par([&](int r) {
        Engine& e = *engines[r];
        const auto a = std::chrono::steady_clock::now();
        std::unique_ptr<uint8_t[]> tile(new uint8_t[size_t(e.rows().size() * e.cols().size())]);
        e.store_cells(tile.get(), e.cols().size(), false);
        store_ms[r] = ms_since(a);
        const auto b = std::chrono::steady_clock::now();
        if (o.output != "none")
          write_text_tile(o.output, o.W, o.H, e.rows(), e.cols(), tile.get(), e.cols().size());
        format_ms[r] = ms_since(b);
        if (o.show)
          for (int64_t i = 0; i < e.rows().size(); ++i)
            std::memcpy(&final_grid[size_t((e.rows().begin + i) * o.W + e.cols().begin)],
                        &tile[size_t(i * e.cols().size())], size_t(e.cols().size()));
      });
      write_ms = ms_since(t1);
    }
    if (!o.metrics.empty()) {
      std::ofstream f(o.metrics);
      double cups = res.loop_ms > 0 ? double(o.W) * double(o.H) * double(res.executed) / (res.loop_ms * 1e-3) : 0;
      std::string tuning_changed = "{";
      for (const auto& kv : o.tune.changed())
        tuning_changed += (tuning_changed.size() > 1 ? ", " : "") + jstr(kv.first) + ": " + jstr(kv.second);
      tuning_changed += "}";
      f << "{\"engine\": " << jstr(engine) << ", \"backend\": " << jstr(backends[0]->name())
        << ", \"layout\": " << jstr(layout_name(layout)) << ", \"ranks\": " << P
        << ", \"decomp\": " << jstr(engines[0]->decomp().describe()) << ", \"tuning\": " << jstr(o.tune.summary())
        << ", \"tuning_changed\": " << tuning_changed << ", \"W\": " << o.W
        << ", \"H\": " << o.H << ", \"generations\": " << res.generations
        << ", \"executed\": " << res.executed << ", \"stop_reason\": " << jstr(res.stop_reason)
        << ", \"loop_ms\": " << res.loop_ms << ", \"read_ms\": " << read_ms
        << ", \"read_parse_ms\": " << read_parse_ms << ", \"read_load_ms\": " << read_load_ms
        << ", \"write_ms\": " << write_ms
        << ", \"write_store_ms\": " << *std::max_element(store_ms.begin(), store_ms.end())
        << ", \"write_format_ms\": " << *std::max_element(format_ms.begin(), format_ms.end())
        << ", \"file_bytes\": " << o.H * (o.W + 1) << ", \"cell_updates_per_s\": " << cups
        << ", \"epoch\": " << engines[0]->epoch_depth() << ", \"tmax\": " << engines[0]->tmax()
        << ", \"exchanges\": " << res.exchanges << ", \"polls\": " << res.polls
        << ", \"kernel_launches\": " << res.kernel_launches << ", \"comm\": " << jstr(P > 1 ? comm : "self")
        << ", \"overlap_mode\": " << jstr(engines[0]->overlap_mode())
        << ", \"overlap_trial_ms_plain\": " << engines[0]->trial_ms_plain()
        << ", \"overlap_trial_ms_trigger\": " << engines[0]->trial_ms_trigger()
        << ", \"phase_timed\": " << (res.phase_timed ? "true" : "false") << ", \"compute_ms\": " << res.compute_ms
        << ", \"halo_ms\": " << res.halo_ms << ", \"fill_ms\": " << res.fill_ms
        << ", \"allreduce_ms\": " << res.allreduce_ms << "}\n";
    }
  }

  // stdout contract of the matching reference build.
  if (o.style == "mpi" || o.style == "async" || o.style == "collective" || o.style == "openmp") {
    std::printf("Reading file:\t%.2lf msecs\n", read_ms);
    std::printf("Generations:\t%d\n", int(res.generations));
    std::printf("Execution time:\t%.2lf msecs\n", res.loop_ms);
    std::printf("Writing file:\t%.2lf msecs\n", write_ms);
    if (o.style != "openmp")  // every MPI process prints it (src/game_mpi.c:514)
      for (int r = 0; r < std::max(1, o.ranks); ++r) std::printf("Finished\n");
  } else if (o.style == "cuda") {
    std::printf("Generations:\t%d\n", int(res.generations));
    std::printf("Execution time:\t%.2f msecs\n", res.loop_ms);
    std::printf("Finished\n");
  } else {
    std::printf("Finished.\n\n");
    std::printf("Generations:\t%d\n", int(res.generations));
    std::printf("Execution time:\t%.2f msecs\n", res.loop_ms);
    std::printf("Finished\n");
  }
  std::fflush(stdout);
  if (o.show && !final_grid.empty()) show(final_grid, o.W, o.H);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  try {
    return run(parse(argc, argv));
  } catch (const std::exception& e) {
    std::fprintf(stderr, "gol: error: %s\n", e.what());
    return 1;
  }
}
