// Resident epoch kernel: plan and launch (the kernel is in
// life_resident_impl.hpp; its RW instantiations build in parallel in
// life_resident_rw*.hip).
#include <algorithm>
#include <string>

#include "gol/common.hpp"
#include "life_kernels.hpp"

namespace gol {
namespace hipk {
namespace lr {
template <int RW>
void launch_resident(const ResidentParams& p, hipStream_t s);
}  // namespace lr

// Rows per wave in VGPRs: every count up to 48 so the bands' slack rows stay
// few (the slack goes into deeper halos, see plan_resident); <= 88 keeps a
// wave under 128 VGPRs (four waves per SIMD).
#define GOL_RESIDENT_RW_LIST(X) \
  X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) \
      X(26) X(27) X(28) X(29) X(30) X(31) X(32) X(33) X(34) X(35) X(36) X(37) X(38) X(39) X(40) X(41) X(42) \
      X(43) X(44) X(45) X(46) X(47) X(48) X(52) X(56) X(60) X(64) X(72) X(80) X(88)

#define GOL_RW_VALUE(n) n,
const int kResidentRW[] = {GOL_RESIDENT_RW_LIST(GOL_RW_VALUE)};
const int kResidentRWCount = int(sizeof(kResidentRW) / sizeof(kResidentRW[0]));
#undef GOL_RW_VALUE

#define GOL_RW_EXTERN(n) extern template void lr::launch_resident<n>(const ResidentParams&, hipStream_t);
GOL_RESIDENT_RW_LIST(GOL_RW_EXTERN)
#undef GOL_RW_EXTERN

void launch_resident_rw(int rw, const ResidentParams& p, hipStream_t s) {
  switch (rw) {
#define GOL_RW_CASE(n) \
  case n:              \
    lr::launch_resident<n>(p, s); \
    return;
    GOL_RESIDENT_RW_LIST(GOL_RW_CASE)
#undef GOL_RW_CASE
    default:
      fail("resident kernel: no instantiation for " + std::to_string(rw) + " rows per wave");
  }
}

bool plan_resident(const BlockArgs& a, int cus, int k_req, ResidentPlan* pl) {
  const TileGeom& g = a.g;
  if (g.layout != Layout::Bits || !a.full_width || !a.allow_drift || a.dual_offset != 0 || g.W % 32 != 0)
    return false;
  // k_req <= 0: plan with 8 halo rows per side, then deepen the halos into
  // the band's slack rows (up to the halo lane's 16 generations): fewer
  // refreshes at no cost.
  const int k = k_req > 0 ? k_req : 8;
  if (k < 1 || k > 16 || a.T < 1 || a.row_lo >= a.row_hi) return false;
  const int64_t ww = g.W / 32;
  const int64_t ns = ceil_div(ww, int64_t(63));
  const int64_t ext = a.row_hi - a.row_lo + 2 * int64_t(a.T);
  if (a.row_lo - a.T < 0 || a.row_hi + a.T > g.R()) return false;
  if ((a.row_lo - a.T + ext) * g.pitch >= (int64_t(1) << 31)) return false;  // 32-bit buffer offsets
  int64_t nb = std::min<int64_t>(cus / ns, ext / k);                        // bands of >= k rows
  if (nb < 1) return false;
  const int64_t band_rows = ext / nb, band_rem = ext % nb;
  const int64_t need = band_rows + (band_rem ? 1 : 0) + 2 * int64_t(k);
  int rw = 0;
  for (int i = 0; i < kResidentRWCount; ++i)
    if (int64_t(kResidentWaves) * kResidentRW[i] >= need) {
      rw = kResidentRW[i];
      break;
    }
  if (rw == 0) return false;
  pl->ns = int(ns);
  pl->sw = int(ceil_div(ww, ns));
  pl->nb = int(nb);
  pl->band_rows = int(band_rows);
  pl->band_rem = int(band_rem);
  pl->rw = rw;
  pl->k = k_req > 0 ? k
                    : int(std::min<int64_t>(16, (int64_t(kResidentWaves) * rw - band_rows - (band_rem ? 1 : 0)) / 2));
  pl->ext_rows = ext;
  return true;
}

int launch_life_resident(const BlockArgs& a, const ResidentPlan& pl, const LifeTuning& tune, uint8_t* mirror0,
                         uint8_t* mirror1, uint32_t* flags, int probe, hipStream_t s, uint64_t* trace) {
  const TileGeom& g = a.g;
  ResidentParams p{};
  p.in = static_cast<const uint8_t*>(a.in);
  p.out = static_cast<uint8_t*>(a.out);
  p.mirror[0] = mirror0;
  p.mirror[1] = mirror1;
  p.flags = flags;
  if (a.gen_dev) {
    p.changed = a.changed;  // resolved on the device: changed + *gen_dev + gen_rel
    p.gen_dev = a.changed ? a.gen_dev : nullptr;
    p.gen_rel = a.gen_rel;
  } else {
    p.changed = a.changed ? a.changed + (a.gen_base + 1 - a.flags_base) : nullptr;
  }
  p.err = tune.err;
  p.pitch = g.pitch;
  p.row0 = a.row_lo - a.T;
  p.ext_rows = int(pl.ext_rows);
  p.T = a.T;
  p.k = pl.k;
  p.ww = int(g.W / 32);
  p.own_w0 = int(g.cell0() / 32);
  p.ns = pl.ns;
  p.sw = pl.sw;
  p.nb = pl.nb;
  p.band_rows = pl.band_rows;
  p.band_rem = pl.band_rem;
  p.nreg = pl.ns * pl.nb;
  p.spin_log2 = std::min(24, std::max(4, tune.chain_spin_log2 + 4));
  p.probe = probe;
  p.trace = trace;
  GOL_REQUIRE(p.nreg <= tune.cus, "resident kernel: more workgroups than CUs");
  (void)hipMemsetAsync(flags, 0, size_t(p.nreg) * 4, s);
  launch_resident_rw(pl.rw, p, s);
  return a.T;
}

}  // namespace hipk
}  // namespace gol
