// Checkpoint / resume for the native CLI.
//
// Reference: no checkpointing, but its output file is in exactly the input
// format, so `./a.out N N game_output.out` resumes from the last generation -
// losing the generation counter and the similarity-counter phase
// (src/game.c:171, the counter restarts at 0).  A checkpoint here is a
// directory holding
//   grid.txt  - the text grid, written by every rank at its subarray offsets
//               (the output writer's path, so it stays a valid input), and
//   meta.json - generation, similarity phase and run config,
// so a resumed run reproduces an uninterrupted one exactly: same final grid,
// same "Generations" line.  The format is shared with the Python package
// (gol_amd/utils/checkpoint.py): either side resumes the other's checkpoints.
#pragma once

#include <cstdint>
#include <string>

namespace gol {

struct CheckpointMeta {
  int64_t W = 0, H = 0;
  int64_t generation = 0;   // generation number of the saved grid
  int sim_phase = 0;        // similarity counter after `generation` (no check fired)
  int64_t gen_limit = 1000;
  bool check_similarity = true;
  int sim_freq = 3;
  std::string layout = "auto";
};

constexpr const char* kCheckpointFormat = "gol-mi355x-checkpoint-v1";

// Similarity counter after generation `gen` of a run that started at
// `start_gen` with counter `phase` (utils/termination.py:sim_phase_at).
inline int sim_phase_at(int64_t gen, int64_t start_gen, int phase, int freq) {
  return int(((gen - start_gen + phase) % freq + freq) % freq);
}

std::string checkpoint_grid_path(const std::string& dir);
// Creates the directory (if needed) and the sized grid file; call once, before
// any rank writes its tile with write_text_tile(checkpoint_grid_path(dir), ...).
void checkpoint_begin(const std::string& dir, int64_t W, int64_t H);
// Publishes meta.json atomically (write + rename): call after every rank's
// tile is on disk, so a checkpoint with a meta.json is always complete.
void checkpoint_commit(const std::string& dir, const CheckpointMeta& m);
// Reads meta.json (throws on a missing file, a different format or missing keys).
CheckpointMeta checkpoint_load(const std::string& dir);

}  // namespace gol
