#include "gol/cpu_ref.hpp"

#include <chrono>
#include <memory>

#include "gol/common.hpp"
#include "gol/parallel.hpp"

namespace gol {

RefResult cpu_reference_run(std::vector<uint8_t>& grid, int64_t W, int64_t H, int64_t gen_limit,
                            bool check_similarity, int sim_freq, int threads) {
  GOL_REQUIRE(int64_t(grid.size()) == W * H, "grid size mismatch");
  GOL_REQUIRE(sim_freq > 0, "similarity frequency must be positive");
  std::vector<uint8_t> a(grid.size()), b(grid.size());
  for (size_t i = 0; i < grid.size(); ++i) a[i] = uint8_t(grid[i] == 1 || grid[i] == '1');
  std::unique_ptr<ThreadPool> pool;
  if (threads > 1) pool = std::make_unique<ThreadPool>(threads);
  auto rows = [&](const std::function<void(int64_t, int64_t)>& fn) {
    if (pool)
      pool->parallel_for(H, fn, 4);
    else
      fn(0, H);
  };
  uint8_t* univ = a.data();
  uint8_t* next = b.data();
  auto empty = [&]() {
    for (int64_t i = 0; i < W * H; ++i)
      if (univ[i]) return false;
    return true;
  };
  auto similar = [&]() {
    for (int64_t i = 0; i < W * H; ++i)
      if (univ[i] != next[i]) return false;
    return true;
  };

  int64_t generation = 1;
  int counter = 0;
  auto t0 = std::chrono::steady_clock::now();
  while (!empty() && generation <= gen_limit) {
    const uint8_t* u = univ;
    uint8_t* n = next;
    rows([&](int64_t rb, int64_t re) {
      for (int64_t y = rb; y < re; ++y) {
        const uint8_t* up = u + ((y + H - 1) % H) * W;
        const uint8_t* mid = u + y * W;
        const uint8_t* dn = u + ((y + 1) % H) * W;
        for (int64_t x = 0; x < W; ++x) {
          int64_t xl = x == 0 ? W - 1 : x - 1, xr = x == W - 1 ? 0 : x + 1;
          int s = up[xl] + up[x] + up[xr] + mid[xl] + mid[xr] + dn[xl] + dn[x] + dn[xr];
          n[y * W + x] = uint8_t(s == 3 || (s == 2 && mid[x]));
        }
      }
    });
    if (check_similarity && ++counter == sim_freq) {
      if (similar()) break;
      counter = 0;
    }
    std::swap(univ, next);
    ++generation;
  }
  auto t1 = std::chrono::steady_clock::now();
  RefResult r;
  r.generations = generation - 1;
  r.loop_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  std::copy(univ, univ + W * H, grid.begin());
  return r;
}

}  // namespace gol
