// Host-only self test of the runtime (engine, CPU backend, in-process thread
// transport, decomposition, text I/O) against the exact serial oracle.
// Built without HIP so it can run under AddressSanitizer / UBSan and
// ThreadSanitizer (the reference has no sanitizer coverage and
// its hybrid build relies on unchecked thread/MPI assumptions):
//
//   python gol_amd/native_build.py --selftest address   -> bin/gol_selftest_address
//   python gol_amd/native_build.py --selftest thread    -> bin/gol_selftest_thread
//
// T0 unit checks (decomposition math, text-format edge cases) come first.
// Every configuration runs P ranks as threads (ThreadHub/ThreadTransport),
// each with its own CPU backend, and compares the gathered grid and the
// "Generations" value with cpu_reference_run.
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "gol/backend.hpp"
#include "gol/cpu_ref.hpp"
#include "gol/decomp.hpp"
#include "gol/engine.hpp"
#include "gol/io.hpp"
#include "gol/transport.hpp"

using namespace gol;

namespace {

struct Case {
  int64_t W, H;
  std::string decomp;
  int P;
  Layout layout;
  int tmax, epoch, overlap;
  int64_t gens;
  uint64_t seed;
  double density;
};

std::vector<uint8_t> random_cells(int64_t W, int64_t H, uint64_t seed, double density) {
  std::vector<uint8_t> g(size_t(W * H));
  const uint32_t th = density_thresh(density);
  for (int64_t r = 0; r < H; ++r)
    for (int64_t c = 0; c < W; ++c) g[size_t(r * W + c)] = rng_cell(seed, r, c, th) ? 1 : 0;
  return g;
}

bool run_case(const Case& k) {
  std::vector<uint8_t> grid = random_cells(k.W, k.H, k.seed, k.density);
  std::vector<uint8_t> ref = grid;
  const RefResult rr = cpu_reference_run(ref, k.W, k.H, k.gens, true, 3, 1);

  auto hub = std::make_shared<ThreadHub>(k.P);
  std::vector<uint8_t> out(grid.size(), 0);
  std::vector<int64_t> gens(size_t(k.P), -1);
  std::vector<std::string> errs(size_t(k.P));
  std::vector<std::thread> ts;
  for (int r = 0; r < k.P; ++r) {
    ts.emplace_back([&, r] {
      try {
        auto be = make_cpu_backend(k.P == 1 ? 4 : 2);  // exercises the thread pool too
        ThreadTransport tr(hub, r, be.get());
        EngineConfig cfg;
        cfg.W = k.W;
        cfg.H = k.H;
        cfg.layout = k.layout;
        cfg.decomp = k.decomp;
        cfg.gen_limit = k.gens;
        cfg.tmax = k.tmax;
        cfg.epoch = k.epoch;
        cfg.overlap = k.overlap;
        cfg.poll_gens = 5;
        Engine eng(cfg, be.get(), &tr);
        eng.load_global(grid.data(), k.W);
        const RunResult res = eng.run();
        gens[size_t(r)] = res.generations;
        const Extent rows = eng.rows(), cols = eng.cols();
        std::vector<uint8_t> tile(size_t(rows.size() * cols.size()));
        eng.store_cells(tile.data(), cols.size(), false);
        for (int64_t i = 0; i < rows.size(); ++i)
          for (int64_t j = 0; j < cols.size(); ++j)
            out[size_t((rows.begin + i) * k.W + cols.begin + j)] = tile[size_t(i * cols.size() + j)];
      } catch (const std::exception& e) {
        errs[size_t(r)] = e.what();
      }
    });
  }
  for (auto& t : ts) t.join();
  bool ok = out == ref;
  for (int r = 0; r < k.P; ++r) {
    if (!errs[size_t(r)].empty()) {
      std::printf("  rank %d error: %s\n", r, errs[size_t(r)].c_str());
      ok = false;
    }
    if (gens[size_t(r)] != rr.generations) ok = false;
  }
  std::printf("%-4s %4lldx%-4lld %-4s P=%d T=%d D=%d overlap=%d gens=%lld ref=%lld -> %s\n",
              k.layout == Layout::Bits ? "bits" : "u8", (long long)k.W, (long long)k.H, k.decomp.c_str(), k.P,
              k.tmax, k.epoch, k.overlap, (long long)gens[0], (long long)rr.generations, ok ? "ok" : "MISMATCH");
  return ok;
}

bool text_roundtrip() {
  const int64_t W = 77, H = 31;
  std::vector<uint8_t> g = random_cells(W, H, 5, 0.4);
  const std::string path = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") +
                           "/gol_selftest_" + std::to_string(::getpid()) + ".txt";
  write_text_grid(path, W, H, g.data());
  std::vector<uint8_t> back;
  read_text_grid(path, W, H, back);
  std::remove(path.c_str());
  const bool ok = back == g;
  std::printf("text round trip %lldx%lld -> %s\n", (long long)W, (long long)H, ok ? "ok" : "MISMATCH");
  return ok;
}

// T0 unit checks: decomposition math and text-format edge cases.
bool unit_checks() {
  bool ok = true;
  auto check = [&](bool c, const char* what) {
    if (!c) std::printf("  unit check failed: %s\n", what);
    ok = ok && c;
  };
  // split_range: balanced, contiguous, covering
  for (int64_t n : {1, 7, 64, 1000, 32768})
    for (int p : {1, 2, 3, 8}) {
      int64_t next = 0;
      for (int i = 0; i < p; ++i) {
        const Extent e = split_range(n, p, i);
        check(e.begin == next && e.size() >= n / p && e.size() <= n / p + 1, "split_range");
        next = e.end;
      }
      check(next == n, "split_range covers");
    }
  // neighbours on a periodic Px x Py torus; north = previous rows (the
  // reference inverts N/S, src/game_mpi.c:293-294)
  for (int Px : {1, 2, 3, 4})
    for (int Py : {1, 2, 3}) {
      const Decomposition d(96 * Px, 10 * Py, Px, Py, 32);
      for (int r = 0; r < d.nranks(); ++r) {
        const auto nb = d.neighbors(r);
        const int px = d.px_of(r), py = d.py_of(r);
        check(nb[kNorth] == d.rank_of(px, py - 1) && nb[kSouth] == d.rank_of(px, py + 1), "N/S");
        check(nb[kWest] == d.rank_of(px - 1, py) && nb[kEast] == d.rank_of(px + 1, py), "W/E");
        check(nb[kNW] == d.rank_of(px - 1, py - 1) && nb[kSE] == d.rank_of(px + 1, py + 1), "corners");
        check(d.rows(nb[kNorth]).end % d.H == d.rows(r).begin, "north tile ends where mine starts");
        check(d.cols(r).begin % 32 == 0, "column splits word aligned");
      }
    }
  // short input file: an error, not a hang (the reference loops forever,
  // src/game.c:149-167)
  const std::string dir = std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp";
  const std::string path = dir + "/gol_selftest_short_" + std::to_string(::getpid()) + ".txt";
  if (FILE* f = std::fopen(path.c_str(), "w")) {
    std::fputs("0101\n1010\n", f);
    std::fclose(f);
  }
  bool threw = false;
  std::vector<uint8_t> g;
  try {
    read_text_grid(path, 4, 3, g);
  } catch (const std::exception&) {
    threw = true;
  }
  check(threw, "short file raises");
  // CRLF line ends are accepted like '\n' (fgetc semantics skip both)
  if (FILE* f = std::fopen(path.c_str(), "w")) {
    std::fputs("0101\r\n1010\r\n0011\r\n", f);
    std::fclose(f);
  }
  g.clear();
  read_text_grid(path, 4, 3, g);
  const std::vector<uint8_t> want = {0, 1, 0, 1, 1, 0, 1, 0, 0, 0, 1, 1};
  check(g == want, "CRLF input");
  std::remove(path.c_str());
  std::printf("unit checks -> %s\n", ok ? "ok" : "FAILED");
  return ok;
}

}  // namespace

int main() {
  std::setvbuf(stdout, nullptr, _IOLBF, 0);  // progress survives a timeout kill
  const Case cases[] = {
      {96, 64, "1x2", 2, Layout::U8, 4, 8, 0, 40, 1, 0.5},
      {96, 64, "1x2", 2, Layout::U8, 4, 8, 1, 40, 1, 0.5},
      {128, 96, "2x2", 4, Layout::Bits, 8, 8, 1, 33, 2, 0.5},
      {100, 37, "1x3", 3, Layout::U8, 2, 6, -1, 50, 3, 0.5},
      {160, 90, "2x3", 6, Layout::U8, 4, 12, 1, 30, 4, 0.5},
      {64, 32, "2x1", 2, Layout::Bits, 16, 16, 0, 1000, 11, 0.2},  // terminates early
      {33, 17, "1x1", 1, Layout::U8, 16, 0, -1, 1000, 4, 0.35},
  };
  bool ok = unit_checks();
  for (const Case& k : cases) ok = run_case(k) && ok;
  ok = text_roundtrip() && ok;
  std::printf(ok ? "SELFTEST OK\n" : "SELFTEST FAILED\n");
  return ok ? 0 : 1;
}
