// Row-ring stress test (VERDICT r05 "Weak 6"): creates and destroys hundreds
// of row rings of mixed geometry in one process, exactly as
// HipBackend::alloc_row_ring maps them - three physical pieces A (first Dv
// owned rows), B (the middle), C (last Dv rows) mapped as [C | A B C | A] in
// one reserved range, access set on the whole range - with ordinary
// hipMalloc / hipFree churn in between, and checks every ring's aliasing
// (a halo row reads back the owned row it maps).  Three policies for a
// released ring's address range:
//   keep   never give it back (the round-5 backend)
//   free   hipMemAddressFree it, so later reservations may land on it
//   reuse  keep it on a free list and map the next ring of equal or smaller
//          size into it (the round-6 backend)
// For every failed hipMemSetAccess the tool prints the iteration, the
// range, the sizes, and whether the range overlaps one an earlier ring used.
//   ring_stress [iterations] [keep|free|reuse|all]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#define CHK(x)                                                                              \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                         \
    }                                                                                       \
  } while (0)

namespace {

struct Range {
  uintptr_t lo, hi;
};

struct Ring {
  void* va = nullptr;
  size_t bytes = 0, reserved = 0;
  hipMemGenericAllocationHandle_t h[3] = {};
  std::vector<std::pair<void*, size_t>> mapped;
};

// Every byte of row r of the owned rows holds (r & 0xFF) ^ seed.
__global__ void fill_rows(uint8_t* owned, size_t pitch, size_t rows, uint8_t seed) {
  const size_t n = pitch * rows;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    owned[i] = uint8_t((i / pitch) & 0xFF) ^ seed;
}

struct Stats {
  int rings = 0, access_fail = 0, access_fail_reused_va = 0, alias_fail = 0, reserve_fail = 0;
};

size_t g_gran = 0;
int g_dev = 0;
std::vector<Range> g_used;  // ranges earlier rings occupied

bool overlaps_used(uintptr_t lo, uintptr_t hi) {
  for (const Range& r : g_used)
    if (lo < r.hi && hi > r.lo) return true;
  return false;
}

void release(Ring& r) {
  for (auto& m : r.mapped) CHK(hipMemUnmap(m.first, m.second));
  r.mapped.clear();
  for (auto& h : r.h)
    if (h) {
      CHK(hipMemRelease(h));
      h = {};
    }
}

// One ring of `owned` bytes with `halo`-byte halos; false when access could
// not be set (the failure under study).
bool make_ring(Ring& r, size_t halo, size_t owned, size_t pitch, std::vector<Ring>& free_list, const char* policy,
               Stats& st, int it) {
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = g_dev;
  const size_t sizes[3] = {halo, owned - 2 * halo, halo};
  for (int i = 0; i < 3; ++i)
    if (sizes[i]) CHK(hipMemCreate(&r.h[i], sizes[i], &prop, 0));
  r.bytes = owned + 2 * halo;
  bool reused = false;
  if (!std::strcmp(policy, "reuse")) {
    // Smallest free reservation that holds the ring.
    int best = -1;
    for (int i = 0; i < int(free_list.size()); ++i)
      if (free_list[i].reserved >= r.bytes && (best < 0 || free_list[i].reserved < free_list[best].reserved)) best = i;
    if (best >= 0) {
      r.va = free_list[best].va;
      r.reserved = free_list[best].reserved;
      free_list.erase(free_list.begin() + best);
      reused = true;
    }
  }
  if (!reused) {
    if (hipMemAddressReserve(&r.va, r.bytes, g_gran, nullptr, 0) != hipSuccess) {
      (void)hipGetLastError();
      ++st.reserve_fail;
      release(r);
      return false;
    }
    r.reserved = r.bytes;
  }
  auto* b = static_cast<uint8_t*>(r.va);
  const struct {
    size_t at;
    int piece;
  } maps[5] = {{0, 2}, {halo, 0}, {2 * halo, 1}, {owned, 2}, {owned + halo, 0}};
  for (const auto& m : maps) {
    if (!sizes[m.piece]) continue;
    CHK(hipMemMap(b + m.at, sizes[m.piece], 0, r.h[m.piece], 0));
    r.mapped.push_back({b + m.at, sizes[m.piece]});
  }
  hipMemAccessDesc acc{};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = g_dev;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  const uintptr_t lo = uintptr_t(r.va), hi = lo + r.bytes;
  const bool seen = overlaps_used(lo, hi);
  const hipError_t e = hipMemSetAccess(r.va, r.bytes, &acc, 1);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    ++st.access_fail;
    st.access_fail_reused_va += seen ? 1 : 0;
    std::printf("  [%s] iteration %d: hipMemSetAccess(%p, %zu bytes; halo %zu, owned %zu) failed: %s; range %s\n",
                policy, it, r.va, r.bytes, halo, owned, hipGetErrorString(e),
                reused ? "reused from the free list" : seen ? "overlaps an earlier ring's range" : "fresh");
    return false;
  }
  g_used.push_back({lo, hi});
  // Aliasing: the top halo row 0 is the last owned row, the bottom halo's
  // first row the first owned row.
  const size_t rows = owned / pitch, hrows = halo / pitch;
  const uint8_t seed = uint8_t(it * 37);
  fill_rows<<<256, 256>>>(b + halo, pitch, rows, seed);
  CHK(hipGetLastError());
  CHK(hipDeviceSynchronize());
  uint8_t top = 0, bot = 0;
  CHK(hipMemcpy(&top, b, 1, hipMemcpyDeviceToHost));                  // halo row 0 = owned row rows - hrows
  CHK(hipMemcpy(&bot, b + halo + owned, 1, hipMemcpyDeviceToHost));  // = owned row 0
  if (top != (uint8_t(((rows - hrows) & 0xFF)) ^ seed) || bot != seed) {
    ++st.alias_fail;
    std::printf("  [%s] iteration %d: aliasing wrong (top %u, bottom %u)\n", policy, it, top, bot);
  }
  return true;
}

Stats run(const char* policy, int iters) {
  Stats st;
  std::vector<Ring> live, free_list;
  std::vector<void*> churn;
  g_used.clear();
  std::srand(12345);
  const size_t pitches[] = {4096, 8192, 4096 * 3, 131072};
  for (int it = 0; it < iters; ++it) {
    // Mixed geometry: halos of 1-4 granules, 3-64 granules owned, rounded to
    // whole rows of the pitch as the backend does (row_ring_halo).
    const size_t pitch = pitches[std::rand() % 4];
    size_t halo = g_gran * (1 + std::rand() % 4);
    while (halo % pitch) halo += g_gran;
    size_t owned = g_gran * (3 + std::rand() % 62);
    while (owned % pitch || owned < 2 * halo) owned += g_gran;
    Ring r;
    if (make_ring(r, halo, owned, pitch, free_list, policy, st, it)) {
      ++st.rings;
      live.push_back(r);
    } else {
      release(r);
      if (r.va) {
        if (!std::strcmp(policy, "free")) CHK(hipMemAddressFree(r.va, r.reserved));
        else if (!std::strcmp(policy, "reuse")) free_list.push_back(r);
      }
    }
    // Churn: ordinary allocations come and go between rings.
    if (std::rand() % 2) {
      void* p = nullptr;
      CHK(hipMalloc(&p, g_gran * (1 + std::rand() % 32)));
      churn.push_back(p);
    }
    if (churn.size() > 4) {
      CHK(hipFree(churn.front()));
      churn.erase(churn.begin());
    }
    // Rings live one to three iterations (engines of a test session).
    while (live.size() > size_t(1 + std::rand() % 3)) {
      Ring& o = live.front();
      release(o);
      if (!std::strcmp(policy, "free")) CHK(hipMemAddressFree(o.va, o.reserved));
      else if (!std::strcmp(policy, "reuse")) free_list.push_back(o);
      live.erase(live.begin());
    }
  }
  for (Ring& o : live) {
    release(o);
    if (!std::strcmp(policy, "free")) CHK(hipMemAddressFree(o.va, o.reserved));
    else if (!std::strcmp(policy, "reuse")) free_list.push_back(o);
  }
  for (Ring& o : free_list) CHK(hipMemAddressFree(o.va, o.reserved));
  for (void* p : churn) CHK(hipFree(p));
  return st;
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 300;
  const std::string which = argc > 2 ? argv[2] : "all";
  CHK(hipSetDevice(g_dev));
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = g_dev;
  CHK(hipMemGetAllocationGranularity(&g_gran, &prop, hipMemAllocationGranularityMinimum));
  std::printf("granularity %zu bytes, %d rings per policy\n", g_gran, iters);
  int bad = 0;
  for (const char* policy : {"keep", "free", "reuse"}) {
    if (which != "all" && which != policy) continue;
    const Stats st = run(policy, iters);
    std::printf("%-5s rings %d  setaccess failures %d (%d on a range an earlier ring used)  alias failures %d  "
                "reserve failures %d\n",
                policy, st.rings, st.access_fail, st.access_fail_reused_va, st.alias_fail, st.reserve_fail);
    bad += st.alias_fail;
  }
  return bad ? 1 : 0;
}
