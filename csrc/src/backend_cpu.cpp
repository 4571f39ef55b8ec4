// CPU backend: bit-exact host emulation of the HIP kernels.
//
// Serves three purposes: (1) the engine's logic (epochs, deep halos, lazy
// termination, decomposition) is testable without a GPU; (2) it is the
// multi-threaded CPU engine that replaces the reference's OpenMP variant
// (src/game_openmp.c:29-112); (3) it is an independent oracle for the HIP
// kernels (the bit-sliced rule written as plain boolean word expressions, not
// the kernels' v_bitop3 truth tables).  run_block sweeps per-thread row bands
// with a 3-row window per level, like the GPU kernel's register schedule.
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gol/backend.hpp"
#include "gol/parallel.hpp"

namespace gol {
namespace {

inline uint32_t pack32(const uint8_t* p) {
  uint32_t w = 0;
  for (int j = 0; j < 32; ++j) w |= uint32_t(p[j] != 0) << j;
  return w;
}
inline void unpack32(uint32_t w, uint8_t* p) {
  for (int j = 0; j < 32; ++j) p[j] = uint8_t((w >> j) & 1u);
}

// ifunc resolvers run before the ThreadSanitizer runtime is up and crash it,
// so sanitizer builds of the host self test use the default clone only.
#if defined(__SANITIZE_THREAD__)
#define GOL_ROW_CLONES
#else
#define GOL_ROW_CLONES __attribute__((target_clones("avx2", "default")))
#endif

// Horizontal 3-sums of one row of Wp words; w[-1] and w[Wp] are zero pads.
// Plain word loops the compiler vectorises (no cross-iteration state); an
// AVX2 clone is picked at load time where the CPU has it.
GOL_ROW_CLONES void hsum_row(const uint32_t* w, int64_t Wp, uint32_t* h0,
                                                                uint32_t* h1) {
  for (int64_t c = 0; c < Wp; ++c) {
    const uint32_t x = w[c];
    const uint32_t l = (x << 1) | (w[c - 1] >> 31);  // cell x-1 at bit of x
    const uint32_t r = (x >> 1) | (w[c + 1] << 31);  // cell x+1
    h0[c] = l ^ x ^ r;
    h1[c] = (l & x) | (r & (l ^ x));
  }
}

// B3/S23 of a row from the horizontal sums (a, b, c = rows above / at /
// below; suffix 0 / 1 = sum bits) and the centre cells; returns
// the OR of (new ^ old) over the owned cells.  S = x0 + 2 (x1 + y0) + 4 y1:
// born / survives at S == 3, survives at S == 4.
GOL_ROW_CLONES uint32_t rule_row(const uint32_t* a0, const uint32_t* a1, const uint32_t* b0, const uint32_t* b1,
                         const uint32_t* c0, const uint32_t* c1, const uint32_t* mid, int64_t Wp,
                         const uint32_t* owned, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t c = 0; c < Wp; ++c) {
    const uint32_t p0 = a0[c] ^ b0[c], p1 = a1[c] ^ b1[c];
    const uint32_t x0 = p0 ^ c0[c], x1 = (a0[c] & b0[c]) | (c0[c] & p0);
    const uint32_t y0 = p1 ^ c1[c], y1 = (a1[c] & b1[c]) | (c1[c] & p1);
    const uint32_t s3 = ~y1 & (x1 ^ y0);
    const uint32_t s4 = ~(x1 ^ y0) & (x1 ^ y1);
    const uint32_t nw = (x0 & s3) | (~x0 & mid[c] & s4);
    out[c] = nw;
    acc |= (nw ^ mid[c]) & owned[c];
  }
  return acc;
}

// Mask of owned cells inside padded word c.
inline uint32_t owned_mask(const TileGeom& g, int64_t c) {
  int64_t lo = g.cell0(), hi = g.cell0() + g.W;
  int64_t b = 32 * c;
  if (b + 32 <= lo || b >= hi) return 0;
  uint32_t m = 0xFFFFFFFFu;
  if (b < lo) m &= 0xFFFFFFFFu << (lo - b);
  if (b + 32 > hi) m &= 0xFFFFFFFFu >> (b + 32 - hi);
  return m;
}

class CpuBackend final : public Backend {
 public:
  CpuBackend(int threads, bool drift, const Tuning& t)
      : Backend(t),
        pool_(threads > 0 ? threads : t.i("host_threads") > 0 ? t.i("host_threads") : default_host_threads()),
        drift_(drift) {
    const std::string& ring = t.s("cpu_ring");
    ring_ = !ring.empty() && ring != "0";
    ring_fail_ = ring == "fail";  // tests: the mapping fails after the size check
    trigger_ = t.on("cpu_trigger");
  }
  // GOL_CPU_TRIGGER=1: the engine's boundary-trigger schedule (overlap =
  // trigger) on the host.  Every operation completes in program order, so the
  // boundary rows of a trigger launch are written when run_block returns and
  // the wait is armed at once; the engine's bookkeeping (triggered sends, the
  // arrival before the next epoch, the auto trial) is what this tests.
  bool supports_trigger() const override { return trigger_; }
  void* trigger_stream(bool* armed) override {
    *armed = armed_;
    armed_ = false;
    return nullptr;
  }
  ~CpuBackend() override {
    for (auto& kv : rings_) ::munmap(kv.first, kv.second);
  }
  // GOL_CPU_RING=1: the HIP backend's row ring, emulated with a memfd mapped
  // three times (last owned rows, the owned rows, first owned rows), so the
  // engine's ring schedule is testable on the CPU.
  int row_ring_halo(int64_t H, int64_t pitch, int min_halo) const override {
    if (!ring_) return 0;
    const int64_t page = ::sysconf(_SC_PAGESIZE);
    int64_t dv = std::max<int64_t>(1, min_halo);
    while ((dv * pitch) % page != 0) ++dv;  // pitch is a multiple of 256
    if ((H * pitch) % page != 0 || H < dv) return 0;
    return int(dv);
  }
  void* alloc_row_ring(const TileGeom& g) override {
    if (!ring_ || ring_fail_) return nullptr;
    const size_t halo = size_t(g.Dv) * size_t(g.pitch), owned = size_t(g.H) * size_t(g.pitch);
    const int fd = ::memfd_create("gol_row_ring", 0);
    GOL_REQUIRE(fd >= 0, std::string("row ring: memfd_create failed: ") + std::strerror(errno));
    void* va = MAP_FAILED;
    try {
      GOL_REQUIRE(::ftruncate(fd, off_t(owned)) == 0, "row ring: ftruncate failed");
      va = ::mmap(nullptr, owned + 2 * halo, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      GOL_REQUIRE(va != MAP_FAILED, "row ring: address reservation failed");
      auto* b = static_cast<uint8_t*>(va);
      const auto map = [&](uint8_t* at, size_t len, off_t off) {
        void* r = ::mmap(at, len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, off);
        GOL_REQUIRE(r == at, "row ring: mmap failed");
      };
      map(b, halo, off_t(owned - halo));  // top halo  = last owned rows
      map(b + halo, owned, 0);            // owned rows
      map(b + halo + owned, halo, 0);     // bottom halo = first owned rows
    } catch (...) {
      if (va != MAP_FAILED) ::munmap(va, owned + 2 * halo);  // the whole range, mapped pieces included
      ::close(fd);
      throw;
    }
    ::close(fd);  // the mappings keep the memory
    std::lock_guard<std::mutex> lk(ring_mu_);
    rings_[va] = owned + 2 * halo;
    return va;  // memfd pages start zeroed
  }
  std::string name() const override {
    return drift_ ? "cpu [drift]" : "cpu";
  }
  bool drifts(Layout) const override { return drift_; }
  void rotate_cols(const void* src, void* dst, const TileGeom& g, int64_t shift) override;
  void convert_rows(const void* src, const TileGeom& gs, void* dst, const TileGeom& gd, int64_t r0,
                    int64_t n) override;
  bool is_device() const override { return false; }

  void* alloc(size_t bytes) override {
    void* p = std::calloc(bytes ? bytes : 1, 1);
    GOL_REQUIRE(p, "host allocation of " + std::to_string(bytes) + " bytes failed");
    return p;
  }
  void release(void* p) override {
    {
      std::lock_guard<std::mutex> lk(ring_mu_);
      auto it = rings_.find(p);
      if (it != rings_.end()) {
        ::munmap(it->first, it->second);
        rings_.erase(it);
        return;
      }
    }
    std::free(p);
  }
  void* alloc_host(size_t bytes) override { return std::calloc(bytes ? bytes : 1, 1); }
  void release_host(void* p) override { std::free(p); }
  void memset_async(void* p, int v, size_t bytes) override { std::memset(p, v, bytes); }
  void copy_h2d(void* d, const void* s, size_t n) override { std::memcpy(d, s, n); }
  void copy_d2h(void* d, const void* s, size_t n) override { std::memcpy(d, s, n); }
  void copy_d2h_async_on(void* d, const void* s, size_t n, void*) override { std::memcpy(d, s, n); }
  void copy_2d_async(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                     int64_t rows) override {
    auto* d = static_cast<uint8_t*>(dst);
    auto* s = static_cast<const uint8_t*>(src);
    for (int64_t r = 0; r < rows; ++r) std::memmove(d + r * dpitch, s + r * spitch, size_t(width));
  }
  void synchronize() override {}
  void* event_record_on(void*) override { return nullptr; }
  void event_wait(void*) override {}
  void event_destroy(void*) override {}
  // Every operation completes before it returns: a mark is the host clock.
  void* timing_mark(void*) override {
    return new std::chrono::steady_clock::time_point(std::chrono::steady_clock::now());
  }
  double timing_ms(void* a, void* b) override {
    const auto* ta = static_cast<std::chrono::steady_clock::time_point*>(a);
    const auto* tb = static_cast<std::chrono::steady_clock::time_point*>(b);
    return std::chrono::duration<double, std::milli>(*tb - *ta).count();
  }
  void timing_release(void* m) override { delete static_cast<std::chrono::steady_clock::time_point*>(m); }

  int run_block(const BlockArgs& a) override;
  void fill_periodic(void* buf, const TileGeom& g, bool cols, bool rows) override;
  void fill_cols_rows(void* buf, const TileGeom& g, int64_t r0, int64_t n, void* stream = nullptr) override;
  void alive_any(const void* buf, const TileGeom& g, uint32_t* flag) override {
    *flag = alive_count(buf, g) > 0 ? 1u : 0u;
  }
  int64_t alive_count(const void* buf, const TileGeom& g) override;
  void load_owned(void* buf, const TileGeom& g, const uint8_t* cells, int64_t ld) override;
  void store_owned(const void* buf, const TileGeom& g, uint8_t* cells, int64_t ld,
                   bool ascii) override;
  void init_random(void* buf, const TileGeom& g, uint64_t seed, double density, int64_t grow0,
                   int64_t gcol0) override;

 private:
  // Word c of padded row r as a 32-cell bit word (0 outside [0, Wp)).
  uint32_t read_word(const uint8_t* base, const TileGeom& g, int64_t r, int64_t c) const {
    if (c < 0 || c >= g.Wp()) return 0;
    const uint8_t* row = base + r * g.pitch;
    if (g.layout == Layout::Bits) {
      uint32_t w;
      std::memcpy(&w, row + 4 * c, 4);
      return w;
    }
    return pack32(row + 32 * c);
  }
  ThreadPool pool_;
  bool drift_ = false;
  bool ring_ = false;      // GOL_CPU_RING
  bool ring_fail_ = false;  // GOL_CPU_RING=fail
  bool trigger_ = false;    // GOL_CPU_TRIGGER
  bool armed_ = false;      // the last run_block carried BlockArgs::trigger
  std::mutex ring_mu_;
  std::map<void*, size_t> rings_;  // row rings: base -> mapped bytes
};

int CpuBackend::run_block(const BlockArgs& a) {
  armed_ = a.trigger && trigger_;
  const TileGeom& g = a.g;
  const int T = a.T;
  const int64_t Wp = g.Wp();
  const int64_t r0 = a.row_lo - T, r1 = a.row_hi + T;  // input rows
  GOL_REQUIRE(r0 >= 0 && r1 <= g.R() && a.row_lo < a.row_hi && T >= 1, "run_block: bad row range");
  std::vector<uint32_t> owned(static_cast<size_t>(Wp));
  for (int64_t c = 0; c < Wp; ++c) owned[size_t(c)] = owned_mask(g, c);
  // Drift emulation: the HIP adder window stores generation t+1's cell x-1 at
  // column x, so after T levels the row sits T cells to the right with zeros
  // (junk on the GPU) entering at the left edge of the padded row.
  const int drift = (drift_ && a.allow_drift && T < 32 && 32 * g.hw >= 2 * T) ? T : 0;

  // Row bands: each task runs all T levels of its output rows [lo, hi) on the
  // trapezoid [lo - T + L, hi + T - L) of level L, in private buffers (the
  // host counterpart of the GPU's temporal blocking: no barrier per level).
  // Level rows outside the band are recomputed by both neighbours; every
  // computed row is a valid row, so the per-band change flags OR together
  // into the block's per-generation flags exactly.
  const int64_t out_rows = a.row_hi - a.row_lo;
  const int64_t bs = std::max<int64_t>(4 * int64_t(T), ceil_div(out_rows, 2 * int64_t(pool_.size())));
  const int64_t nb = ceil_div(out_rows, bs);
  std::vector<uint8_t> any(size_t(nb * T), 0);
  auto* in = static_cast<const uint8_t*>(a.in);
  auto* out = static_cast<uint8_t*>(a.out);
  const int64_t P = Wp + 2;  // row stride of the level buffers: a zero word either side
  pool_.parallel_for(nb, [&](int64_t b0, int64_t b1) {
    // Row sweep with a 3-row window per level (the GPU kernel's schedule on
    // the host): input row k enters level 0, level L's window yields level
    // L+1's row k - L - 1, so a band's working set is T x 3 rows, cache-
    // resident, instead of whole level planes.  Per-thread scratch is kept
    // across blocks (fresh large vectors were mmap'd and page-faulted every
    // block, which serialised the threads).
    const int64_t S = P + 2 * Wp;  // one window slot: padded cells, h0, h1
    thread_local std::vector<uint32_t> win, outrow;
    thread_local std::vector<int64_t> cnt;
    if (win.size() < size_t(int64_t(T) * 3 * S)) win.resize(size_t(int64_t(T) * 3 * S));
    if (outrow.size() < size_t(P)) outrow.resize(size_t(P));
    cnt.assign(size_t(T), 0);
    auto cells = [&](int L, int64_t slot) { return &win[size_t((L * 3 + slot) * S + 1)]; };
    auto hs0 = [&](int L, int64_t slot) { return &win[size_t((L * 3 + slot) * S + P)]; };
    auto hs1 = [&](int L, int64_t slot) { return &win[size_t((L * 3 + slot) * S + P + Wp)]; };
    for (int L = 0; L < T; ++L)
      for (int64_t sl = 0; sl < 3; ++sl) cells(L, sl)[-1] = cells(L, sl)[Wp] = 0u;  // zero pads
    outrow[0] = outrow[size_t(P - 1)] = 0u;
    for (int64_t band = b0; band < b1; ++band) {
      const int64_t lo = a.row_lo + band * bs, hi = std::min(lo + bs, a.row_hi);
      std::fill(cnt.begin(), cnt.end(), 0);
      std::vector<uint32_t> acc(size_t(T), 0u);
      for (int64_t r = lo - T; r < hi + T; ++r) {
        const int64_t s0 = cnt[0] % 3;
        uint32_t* w = cells(0, s0);
        if (g.layout == Layout::Bits)
          std::memcpy(w, in + r * g.pitch, size_t(4 * Wp));
        else
          for (int64_t c = 0; c < Wp; ++c) w[c] = read_word(in, g, r, c);
        hsum_row(w, Wp, hs0(0, s0), hs1(0, s0));
        ++cnt[0];
        for (int L = 0; L < T && cnt[size_t(L)] >= 3; ++L) {
          const int64_t n = cnt[size_t(L)];
          const int64_t sa = (n - 3) % 3, sb = (n - 2) % 3, sc = (n - 1) % 3;
          const bool last = L + 1 == T;
          const int64_t sd = last ? 0 : cnt[size_t(L + 1)] % 3;
          uint32_t* dst = last ? &outrow[1] : cells(L + 1, sd);
          acc[size_t(L)] |= rule_row(hs0(L, sa), hs1(L, sa), hs0(L, sb), hs1(L, sb), hs0(L, sc), hs1(L, sc),
                                     cells(L, sb), Wp, owned.data(), dst);
          if (!last) {
            hsum_row(dst, Wp, hs0(L + 1, sd), hs1(L + 1, sd));
            ++cnt[size_t(L + 1)];
            continue;
          }
          // Level-T row lo + n - 3 (n rows received by level T-1 so far).
          if (drift)
            for (int64_t c = Wp - 1; c >= 0; --c)
              dst[c] = (dst[c] << drift) | (c > 0 ? dst[c - 1] >> (32 - drift) : 0u);
          uint8_t* row = out + (lo + n - 3) * g.pitch;
          if (g.layout == Layout::Bits)
            std::memcpy(row, dst, size_t(4 * Wp));
          else
            for (int64_t c = 0; c < Wp; ++c) unpack32(dst[c], row + 32 * c);
        }
      }
      for (int L = 0; L < T; ++L) any[size_t(band * T + L)] = acc[size_t(L)] != 0;
    }
  });
  if (a.changed)
    for (int L = 1; L <= T; ++L) {
      bool ch = false;
      for (int64_t b = 0; b < nb && !ch; ++b) ch = any[size_t(b * T + L - 1)] != 0;
      const int64_t idx = a.gen_dev ? *a.gen_dev + a.gen_rel + (L - 1) : a.gen_base + L - a.flags_base;
      if (ch) a.changed[idx] = 1u;
    }
  return drift;
}

void CpuBackend::rotate_cols(const void* src, void* dst, const TileGeom& g, int64_t shift) {
  auto* s = static_cast<const uint8_t*>(src);
  auto* d = static_cast<uint8_t*>(dst);
  const int64_t W = g.W;
  shift = ((shift % W) + W) % W;
  pool_.parallel_for(g.H, [&](int64_t b, int64_t e) {
    std::vector<uint8_t> cells(static_cast<size_t>(W));
    for (int64_t i = b; i < e; ++i) {
      const uint8_t* row = s + (g.row0() + i) * g.pitch;
      uint8_t* out = d + (g.row0() + i) * g.pitch;
      for (int64_t x = 0; x < W; ++x) {
        const int64_t c = g.cell0() + x;
        cells[size_t(x)] = g.layout == Layout::Bits ? uint8_t((row[4 * (c / 32) + (c % 32) / 8] >> (c % 8)) & 1u)
                                                     : uint8_t(row[c] != 0);
      }
      for (int64_t x = 0; x < W; ++x) {
        const int64_t c = g.cell0() + x;
        const uint8_t v = cells[size_t((x + shift) % W)];
        if (g.layout == Layout::Bits) {
          uint8_t& byte = out[4 * (c / 32) + (c % 32) / 8];
          byte = uint8_t((byte & ~(1u << (c % 8))) | (unsigned(v) << (c % 8)));
        } else {
          out[c] = v;
        }
      }
    }
  });
}

void CpuBackend::convert_rows(const void* src, const TileGeom& gs, void* dst, const TileGeom& gd, int64_t i0,
                              int64_t n) {
  GOL_REQUIRE(gs.layout != gd.layout, "convert_rows: layouts must differ");
  GOL_REQUIRE(gs.H == gd.H && gs.W == gd.W && gs.W % 32 == 0, "convert_rows: geometries differ");
  GOL_REQUIRE(i0 >= 0 && n >= 0 && i0 + n <= gs.H, "convert_rows: rows out of range");
  auto* s = static_cast<const uint8_t*>(src);
  auto* d = static_cast<uint8_t*>(dst);
  const int64_t ow = gs.W / 32;
  const bool to_bits = gs.layout == Layout::U8;
  pool_.parallel_for(n, [&](int64_t b, int64_t e) {
    for (int64_t i = i0 + b; i < i0 + e; ++i) {
      const uint8_t* in = s + gs.offset(gs.row0() + i, gs.cell0());
      uint8_t* out = d + gd.offset(gd.row0() + i, gd.cell0());
      for (int64_t k = 0; k < ow; ++k) {
        if (to_bits) {
          uint32_t w = 0;
          for (int j = 0; j < 32; ++j) w |= uint32_t(in[32 * k + j] != 0) << j;
          std::memcpy(out + 4 * k, &w, 4);
        } else {
          uint32_t w;
          std::memcpy(&w, in + 4 * k, 4);
          for (int j = 0; j < 32; ++j) out[32 * k + j] = uint8_t((w >> j) & 1u);
        }
      }
    }
  });
}

void CpuBackend::fill_periodic(void* buf, const TileGeom& g, bool cols, bool rows) {
  auto* p = static_cast<uint8_t*>(buf);
  const int64_t H = g.H;
  if (cols) fill_cols_rows(buf, g, g.row0(), H);
  if (rows) {
    for (int64_t r = 0; r < g.R(); ++r) {
      if (r >= g.row0() && r < g.row0() + H) continue;
      int64_t src = g.row0() + (((r - g.row0()) % H) + H) % H;
      std::memcpy(p + r * g.pitch, p + src * g.pitch, size_t(g.pitch));
    }
  }
}

void CpuBackend::fill_cols_rows(void* buf, const TileGeom& g, int64_t r0, int64_t n, void*) {
  auto* p = static_cast<uint8_t*>(buf);
  const int64_t W = g.W, c0 = g.cell0();
  {
    pool_.parallel_for(n, [&](int64_t b, int64_t e) {
      for (int64_t r = r0 + b; r < r0 + e; ++r) {
        uint8_t* row = p + r * g.pitch;
        if (g.layout == Layout::Bits) {
          auto* w = reinterpret_cast<uint32_t*>(row);
          const int64_t ow = W / 32, h = g.hw;
          for (int64_t c = 0; c < g.Wp(); ++c) {
            if (c >= h && c < h + ow) continue;
            w[c] = w[h + (((c - h) % ow) + ow) % ow];
          }
        } else {
          for (int64_t x = 0; x < 32 * g.Wp(); ++x) {
            if (x >= c0 && x < c0 + W) continue;
            if (x >= g.Wc()) break;
            row[x] = row[c0 + (((x - c0) % W) + W) % W];
          }
        }
      }
    });
  }
}

int64_t CpuBackend::alive_count(const void* buf, const TileGeom& g) {
  auto* p = static_cast<const uint8_t*>(buf);
  std::vector<int64_t> part(size_t(g.H), 0);
  pool_.parallel_for(g.H, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      const uint8_t* row = p + (g.row0() + i) * g.pitch;
      int64_t n = 0;
      if (g.layout == Layout::Bits) {
        const auto* w = reinterpret_cast<const uint32_t*>(row) + g.hw;
        for (int64_t c = 0; c < g.W / 32; ++c) n += __builtin_popcount(w[c]);
      } else {
        for (int64_t x = 0; x < g.W; ++x) n += row[g.cell0() + x] != 0;
      }
      part[size_t(i)] = n;
    }
  });
  int64_t s = 0;
  for (auto v : part) s += v;
  return s;
}

void CpuBackend::load_owned(void* buf, const TileGeom& g, const uint8_t* cells, int64_t ld) {
  auto* p = static_cast<uint8_t*>(buf);
  pool_.parallel_for(g.H, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      uint8_t* row = p + (g.row0() + i) * g.pitch;
      const uint8_t* src = cells + i * ld;
      if (g.layout == Layout::Bits) {
        auto* w = reinterpret_cast<uint32_t*>(row) + g.hw;
        for (int64_t c = 0; c < g.W / 32; ++c) {
          uint32_t v = 0;
          for (int j = 0; j < 32; ++j) {
            uint8_t ch = src[32 * c + j];
            v |= uint32_t(ch == '1' || ch == 1) << j;
          }
          w[c] = v;
        }
      } else {
        for (int64_t x = 0; x < g.W; ++x) {
          uint8_t ch = src[x];
          row[g.cell0() + x] = uint8_t(ch == '1' || ch == 1);
        }
      }
    }
  });
}

void CpuBackend::store_owned(const void* buf, const TileGeom& g, uint8_t* cells, int64_t ld,
                             bool ascii) {
  auto* p = static_cast<const uint8_t*>(buf);
  const uint8_t base = ascii ? '0' : 0;
  pool_.parallel_for(g.H, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      const uint8_t* row = p + (g.row0() + i) * g.pitch;
      uint8_t* dst = cells + i * ld;
      if (g.layout == Layout::Bits) {
        const auto* w = reinterpret_cast<const uint32_t*>(row) + g.hw;
        for (int64_t x = 0; x < g.W; ++x) dst[x] = uint8_t(base + ((w[x / 32] >> (x % 32)) & 1u));
      } else {
        for (int64_t x = 0; x < g.W; ++x) dst[x] = uint8_t(base + (row[g.cell0() + x] != 0));
      }
    }
  });
}

void CpuBackend::init_random(void* buf, const TileGeom& g, uint64_t seed, double density,
                             int64_t grow0, int64_t gcol0) {
  auto* p = static_cast<uint8_t*>(buf);
  const uint32_t th = density_thresh(density);
  pool_.parallel_for(g.H, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      uint8_t* row = p + (g.row0() + i) * g.pitch;
      if (g.layout == Layout::Bits) {
        auto* w = reinterpret_cast<uint32_t*>(row) + g.hw;
        for (int64_t c = 0; c < g.W / 32; ++c) {
          uint32_t v = 0;
          for (int j = 0; j < 32; ++j) v |= uint32_t(rng_cell(seed, grow0 + i, gcol0 + 32 * c + j, th)) << j;
          w[c] = v;
        }
      } else {
        for (int64_t x = 0; x < g.W; ++x) row[g.cell0() + x] = uint8_t(rng_cell(seed, grow0 + i, gcol0 + x, th));
      }
    }
  });
}

}  // namespace

std::unique_ptr<Backend> make_cpu_backend(int threads, int drift, const Tuning& tune) {
  if (drift < 0) drift = tune.on("cpu_drift");
  return std::make_unique<CpuBackend>(threads, drift != 0, tune);
}

}  // namespace gol
