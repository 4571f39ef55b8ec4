#include "gol/decomp.hpp"

#include <cstdio>
#include <cstdlib>

namespace gol {

void fail(const std::string& msg) { throw Error(msg); }

Extent split_range(int64_t n, int p, int i) {
  GOL_REQUIRE(p > 0 && i >= 0 && i < p, "split_range: bad part index");
  int64_t base = n / p, rem = n % p;
  int64_t b = i * base + (i < rem ? i : rem);
  int64_t e = b + base + (i < rem ? 1 : 0);
  return {b, e};
}

Decomposition::Decomposition(int64_t W_, int64_t H_, int Px_, int Py_, int64_t unit)
    : W(W_), H(H_), Px(Px_), Py(Py_), col_unit(unit) {
  GOL_REQUIRE(W > 0 && H > 0, "grid dimensions must be positive");
  GOL_REQUIRE(Px > 0 && Py > 0, "process grid dimensions must be positive");
  GOL_REQUIRE(col_unit > 0 && W % col_unit == 0, "width must be a multiple of the column unit");
  GOL_REQUIRE(W / col_unit >= Px, "more process columns than column units");
  GOL_REQUIRE(H >= Py, "more process rows than grid rows");
}

int Decomposition::rank_of(int px, int py) const {
  px = ((px % Px) + Px) % Px;
  py = ((py % Py) + Py) % Py;
  return py * Px + px;
}

Extent Decomposition::rows(int rank) const { return split_range(H, Py, py_of(rank)); }

Extent Decomposition::cols(int rank) const {
  Extent u = split_range(W / col_unit, Px, px_of(rank));
  return {u.begin * col_unit, u.end * col_unit};
}

std::array<int, 8> Decomposition::neighbors(int rank) const {
  int px = px_of(rank), py = py_of(rank);
  std::array<int, 8> n{};
  n[kNorth] = rank_of(px, py - 1);
  n[kSouth] = rank_of(px, py + 1);
  n[kWest] = rank_of(px - 1, py);
  n[kEast] = rank_of(px + 1, py);
  n[kNW] = rank_of(px - 1, py - 1);
  n[kNE] = rank_of(px + 1, py - 1);
  n[kSW] = rank_of(px - 1, py + 1);
  n[kSE] = rank_of(px + 1, py + 1);
  return n;
}

Decomposition Decomposition::make(int64_t W, int64_t H, int nranks, const std::string& spec,
                                  int64_t col_unit) {
  GOL_REQUIRE(nranks > 0, "nranks must be positive");
  int Px = 1, Py = nranks;
  if (!spec.empty() && spec != "auto") {
    int a = 0, b = 0;
    if (std::sscanf(spec.c_str(), "%dx%d", &a, &b) != 2 || a <= 0 || b <= 0)
      fail("bad decomposition spec '" + spec + "' (want auto or PxQ)");
    Px = a;
    Py = b;
    GOL_REQUIRE(Px * Py == nranks, "decomposition " + spec + " does not match " +
                                       std::to_string(nranks) + " ranks");
  } else if (H < nranks) {
    // Too few rows for row strips: fall back to column strips.
    Px = nranks;
    Py = 1;
  }
  return Decomposition(W, H, Px, Py, col_unit);
}

std::string Decomposition::describe() const {
  return std::to_string(Px) + "x" + std::to_string(Py);
}

}  // namespace gol
