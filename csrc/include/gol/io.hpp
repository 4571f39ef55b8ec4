// Text-grid I/O, byte-compatible with the reference.
//
// Format (README.md:61): H lines of W characters '0'/'1', each
// terminated by '\n'; file size H*(W+1).  The reference has three readers:
//   * sequential fgetc loops that skip '\n' and accept any other byte as a
//     cell, and spin forever on a short file (src/game.c:149-167, quirk Q8);
//   * rank-0 read + MPI_Send scatter (src/game_mpi.c:201-260);
//   * MPI-IO subarray views {H, W+1} / {h_l, w_l} / {r*h_l, c*w_l} with
//     File_iread or File_read_all (src/game_mpi_async.c:168-221,
//     src/game_mpi_collective.c:168-218).
// Here: a parallel exact-layout reader (each rank / worker preads its
// subarray at offset row*(W+1)+col - the same offset math as the MPI-IO
// view) with a sequential fgetc-compatible fallback for files that do not
// have the exact layout.  A short file is an error, never a hang.  Output
// mirrors the MPI-IO writers (src/game_mpi_async.c:382-455): every rank
// pwrites its rows, the rightmost tile writes the '\n' column.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "gol/decomp.hpp"

namespace gol {

// Reads rows [rows.begin, rows.end) x cells [cols.begin, cols.end) of a
// W x H text grid into `out` (0/1 bytes, row stride cols.size()).
void read_text_tile(const std::string& path, int64_t W, int64_t H, Extent rows, Extent cols,
                    std::vector<uint8_t>& out);
// The same into caller memory (row stride ld), which it fully overwrites:
// no zero-fill of a multi-GB host buffer before the parallel read.
void read_text_tile_into(const std::string& path, int64_t W, int64_t H, Extent rows, Extent cols, uint8_t* dst,
                         int64_t ld);
inline void read_text_grid(const std::string& path, int64_t W, int64_t H,
                           std::vector<uint8_t>& out) {
  read_text_tile(path, W, H, {0, H}, {0, W}, out);
}

// Creates (or truncates) `path` sized for a W x H grid.  Call once (rank 0)
// before any rank calls write_text_tile.
void create_text_file(const std::string& path, int64_t W, int64_t H);
// Writes a tile (0/1 bytes or ASCII, row stride ld) at its subarray offsets.
void write_text_tile(const std::string& path, int64_t W, int64_t H, Extent rows, Extent cols,
                     const uint8_t* cells, int64_t ld);
inline void write_text_grid(const std::string& path, int64_t W, int64_t H, const uint8_t* cells) {
  create_text_file(path, W, H);
  write_text_tile(path, W, H, {0, H}, {0, W}, cells, W);
}

// Random grid in the same text format (replaces generate.sh, which takes
// ~2.2 us/cell: SURVEY 6.2).  Cells come from the same counter-based RNG as
// the device init, so `--random SEED` and a generated file agree.
void generate_text_file(const std::string& path, int64_t W, int64_t H, uint64_t seed,
                        double density);

}  // namespace gol
