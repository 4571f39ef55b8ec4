// Checkpoint / resume for the native CLI.
//
// Reference: no checkpointing, but its output file is in exactly the input
// format, so `./a.out N N game_output.out` resumes from the last generation -
// losing the generation counter and the similarity-counter phase
// (src/game.c:171, the counter restarts at 0).  A checkpoint here is a
// directory holding
//   grid-<gen>[b].txt - the text grid, written by every rank at its subarray
//               offsets (the output writer's path, so it stays a valid
//               input), and
//   meta.json - generation, similarity phase, run config and the name of
//               the grid file it belongs to,
// so a resumed run reproduces an uninterrupted one exactly: same final grid,
// same "Generations" line.  The format is shared with the Python package
// (gol_amd/utils/checkpoint.py): either side resumes the other's checkpoints.
//
// Crash safety: a new checkpoint never touches the files of the committed
// one.  Its grid goes to a fresh file name, is fsync'ed, and only then is
// meta.json replaced (write + fsync + rename + directory fsync); the old grid
// file is deleted after that, with any orphan of an interrupted checkpoint.  A crash at any point leaves either the old
// checkpoint or the new one, complete.  (Format v1 checkpoints without a
// "grid" key use grid.txt.)
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
  std::string grid = "grid.txt";  // grid file name inside the checkpoint directory
};

constexpr const char* kCheckpointFormat = "gol-mi355x-checkpoint-v1";

// Similarity counter after generation `gen` of a run that started at
// `start_gen` with counter `phase` (utils/termination.py:sim_phase_at).
inline int sim_phase_at(int64_t gen, int64_t start_gen, int phase, int freq) {
  return int(((gen - start_gen + phase) % freq + freq) % freq);
}

// Whether `name` may be a checkpoint's grid file: the plain basename
// grid-<digits>[b].txt or the legacy grid.txt - never a path, "..", or
// meta.json (a tampered meta.json must not make --resume read, or a commit
// delete, anything else).  Mirrored by utils/checkpoint.py:grid_name_ok.
bool checkpoint_grid_name_ok(const std::string& name);
// Grid file of the committed checkpoint in `dir` (reads meta.json).
std::string checkpoint_grid_path(const std::string& dir);
// Creates the directory (if needed) and a sized grid file for generation
// `generation` under a name the committed checkpoint does not use; returns
// its path.  Call once, before every rank writes its tile there with
// write_text_tile(path, ...).
std::string checkpoint_begin(const std::string& dir, int64_t W, int64_t H, int64_t generation);
// After every rank's tile is on disk: fsyncs the grid file `grid_path`
// (from checkpoint_begin), publishes meta.json for it atomically, then
// removes the previous checkpoint's grid file and any grid file an
// interrupted checkpoint left behind.
void checkpoint_commit(const std::string& dir, const std::string& grid_path, CheckpointMeta m);
// Reads meta.json (throws on a missing file, a different format or missing keys).
CheckpointMeta checkpoint_load(const std::string& dir);

}  // namespace gol
