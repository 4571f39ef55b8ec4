// Serial reference engine with exactly the semantics of src/game.c (the
// canonical variant): toroidal B3/S23, an extinction test before
// every generation, a similarity test every SIMILARITY_FREQUENCY generations,
// "Generations" = generation - 1.  It evaluates every generation eagerly, so
// it is the oracle for the lazy termination logic of the engine, and the
// 256^2 CPU plumbing configuration of BASELINE.json.
#pragma once

#include <cstdint>
#include <vector>

namespace gol {

struct RefResult {
  int64_t generations = 0;
  double loop_ms = 0;
};

// `grid` holds H*W cells (0/1 or ASCII) and is overwritten with the final
// generation as 0/1 bytes.  threads > 1 splits the rows like the
// reference's OpenMP build (src/game_openmp.c:34).
RefResult cpu_reference_run(std::vector<uint8_t>& grid, int64_t W, int64_t H, int64_t gen_limit,
                            bool check_similarity, int sim_freq, int threads);

}  // namespace gol
