// Domain decomposition of the periodic W x H torus over Px x Py ranks.
//
// Reference: MPI_Cart_create with dims {q,q}, q = (int)sqrt(P), periods {1,1}
// (src/game_mpi.c:162-185) and width_local = height_local = N / q
// (src/game_mpi.c:172).  That only works for perfect-square P with N divisible
// by q and its 8-neighbour table swaps north and
// south (src/game_mpi.c:293-294, quirk Q1).  Here any Px x Py works (1x8 row
// strips, 2x4 blocks, ...), splits are balanced with remainders, and "north"
// is always the tile holding the previous rows.
#pragma once

#include <array>
#include <string>
#include <vector>

#include "gol/common.hpp"

namespace gol {

struct Extent {
  int64_t begin = 0, end = 0;
  int64_t size() const { return end - begin; }
};

// Balanced split of n units into p parts; part i gets floor(n/p) (+1 for the
// first n%p parts).
Extent split_range(int64_t n, int p, int i);

enum Dir : int { kNorth = 0, kSouth = 1, kWest = 2, kEast = 3, kNW = 4, kNE = 5, kSW = 6, kSE = 7 };

struct Decomposition {
  int64_t W = 0, H = 0;  // global grid (cells)
  int Px = 1, Py = 1;    // process grid: Px columns x Py rows; rank = py*Px + px
  int64_t col_unit = 1;  // column splits happen in multiples of this many cells

  Decomposition() = default;
  Decomposition(int64_t W, int64_t H, int Px, int Py, int64_t col_unit);

  int nranks() const { return Px * Py; }
  int px_of(int rank) const { return rank % Px; }
  int py_of(int rank) const { return rank / Px; }
  int rank_of(int px, int py) const;  // periodic wrap of coordinates
  Extent rows(int rank) const;        // global row range of a rank's tile
  Extent cols(int rank) const;        // global column (cell) range
  std::array<int, 8> neighbors(int rank) const;  // indexed by Dir

  // "auto" -> 1 x P row strips (contiguous halos); "PxQ" -> Px=P, Py=Q.
  static Decomposition make(int64_t W, int64_t H, int nranks, const std::string& spec,
                            int64_t col_unit);
  std::string describe() const;
};

}  // namespace gol
