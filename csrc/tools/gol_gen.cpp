// gol_gen: random input generator (replacement for generate.sh).
//
// generate.sh (generate.sh:1-13) emits `width` lines of `height` chars of
// $((RANDOM % 2)) at ~2.2 us/cell with no seed.  This writes the
// same text format (H lines of W chars, README.md:61) with a seeded
// counter-based RNG, in parallel with pwrite, and to a file rather than
// stdout so multi-GB grids are practical.
//
//   gol_gen <width> <height> <output_file> [seed] [density]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "gol/io.hpp"

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: gol_gen <width> <height> <output_file> [seed] [density]\n");
    return 2;
  }
  try {
    int64_t W = std::atoll(argv[1]), H = std::atoll(argv[2]);
    uint64_t seed = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 1;
    double density = argc > 5 ? std::atof(argv[5]) : 0.5;
    if (W <= 0 || H <= 0) throw gol::Error("width and height must be positive");
    gol::generate_text_file(argv[3], W, H, seed, density);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "gol_gen: error: %s\n", e.what());
    return 1;
  }
  return 0;
}
