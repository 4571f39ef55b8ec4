#include "gol/checkpoint.hpp"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

#include "gol/common.hpp"
#include "gol/io.hpp"

namespace gol {
namespace {

// Grids checkpoint_begin created that no commit has taken over yet, one name
// per line (the orphan sweep's only source of names).
constexpr const char* kInflightName = ".gol-inflight";

void mkdirs(const std::string& dir) {
  std::string cur;
  for (size_t i = 0; i <= dir.size(); ++i) {
    if (i == dir.size() || dir[i] == '/') {
      if (!cur.empty() && ::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
        fail("cannot create checkpoint directory '" + cur + "': " + std::strerror(errno));
    }
    if (i < dir.size()) cur += dir[i];
  }
}

// Value text of "key": <value> in a flat JSON object (numbers, booleans,
// strings); empty if the key is absent.
std::string json_field(const std::string& js, const std::string& key) {
  const std::string k = "\"" + key + "\"";
  size_t p = js.find(k);
  if (p == std::string::npos) return {};
  p = js.find(':', p + k.size());
  if (p == std::string::npos) return {};
  ++p;
  while (p < js.size() && (js[p] == ' ' || js[p] == '\n' || js[p] == '\t' || js[p] == '\r')) ++p;
  if (p < js.size() && js[p] == '"') {
    const size_t e = js.find('"', p + 1);
    return e == std::string::npos ? std::string() : js.substr(p + 1, e - p - 1);
  }
  size_t e = p;
  while (e < js.size() && js[e] != ',' && js[e] != '}' && js[e] != '\n') ++e;
  std::string v = js.substr(p, e - p);
  while (!v.empty() && (v.back() == ' ' || v.back() == '\r')) v.pop_back();
  return v;
}

int64_t need_int(const std::string& js, const std::string& key, const std::string& dir) {
  const std::string v = json_field(js, key);
  char* end = nullptr;
  const long long x = std::strtoll(v.c_str(), &end, 10);
  if (v.empty() || end == v.c_str() || *end != '\0')
    fail("checkpoint '" + dir + "': meta.json has no integer '" + key + "'");
  return int64_t(x);
}

}  // namespace

bool checkpoint_grid_name_ok(const std::string& name) {
  if (name == "grid.txt") return true;  // legacy single-file checkpoints
  // grid-<digits>[b].txt: a plain basename, never meta.json or a path.
  const std::string pre = "grid-", suf = ".txt";
  if (name.size() <= pre.size() + suf.size() || name.compare(0, pre.size(), pre) != 0 ||
      name.compare(name.size() - suf.size(), suf.size(), suf) != 0)
    return false;
  std::string mid = name.substr(pre.size(), name.size() - pre.size() - suf.size());
  if (!mid.empty() && mid.back() == 'b') mid.pop_back();
  if (mid.empty()) return false;
  for (char c : mid)
    if (c < '0' || c > '9') return false;
  return true;
}

std::string checkpoint_grid_path(const std::string& dir) { return dir + "/" + checkpoint_load(dir).grid; }

namespace {

bool file_exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0;
}

void fsync_path(const std::string& path, bool directory) {
  const int fd = ::open(path.c_str(), directory ? (O_RDONLY | O_DIRECTORY) : O_RDONLY);
  if (fd < 0) fail("checkpoint: cannot open '" + path + "' to sync it: " + std::strerror(errno));
  const int rc = ::fsync(fd);
  const int err = errno;
  ::close(fd);
  if (rc != 0 && !(directory && (err == EINVAL || err == EROFS)))
    fail("checkpoint: fsync of '" + path + "' failed: " + std::strerror(err));
}

}  // namespace

std::string checkpoint_begin(const std::string& dir, int64_t W, int64_t H, int64_t generation) {
  mkdirs(dir);
  std::string committed;
  if (file_exists(dir + "/meta.json")) committed = checkpoint_load(dir).grid;
  std::string name = "grid-" + std::to_string(generation) + ".txt";
  if (name == committed) name = "grid-" + std::to_string(generation) + "b.txt";
  const std::string path = dir + "/" + name;
  // Record the grid as this run's before creating it: a commit only ever
  // sweeps grids a checkpoint of ours created (an interrupted one's), never
  // a user's file that happens to be named like one.
  {
    std::ofstream in(dir + "/" + kInflightName, std::ios::app);
    if (!in || !(in << name << "\n") || !in.flush())
      fail("checkpoint: cannot record the in-flight grid in '" + dir + "/" + kInflightName + "'");
  }
  create_text_file(path, W, H);
  return path;
}

void checkpoint_commit(const std::string& dir, const std::string& grid_path, CheckpointMeta m) {
  const size_t slash = grid_path.find_last_of('/');
  m.grid = slash == std::string::npos ? grid_path : grid_path.substr(slash + 1);
  std::string previous;
  if (file_exists(dir + "/meta.json")) previous = checkpoint_load(dir).grid;
  fsync_path(grid_path, false);  // the tiles are on disk before meta.json names them
  std::ostringstream o;
  o << "{\n \"format\": \"" << kCheckpointFormat << "\",\n \"width\": " << m.W << ",\n \"height\": " << m.H
    << ",\n \"generation\": " << m.generation << ",\n \"sim_phase\": " << m.sim_phase
    << ",\n \"gen_limit\": " << m.gen_limit << ",\n \"check_similarity\": "
    << (m.check_similarity ? "true" : "false") << ",\n \"sim_freq\": " << m.sim_freq << ",\n \"layout\": \""
    << m.layout << "\",\n \"grid\": \"" << m.grid << "\"\n}";
  const std::string tmp = dir + "/meta.json.tmp", fin = dir + "/meta.json";
  {
    std::ofstream f(tmp, std::ios::trunc);
    if (!f) fail("cannot write checkpoint metadata '" + tmp + "'");
    f << o.str();
    if (!f.flush()) fail("cannot write checkpoint metadata '" + tmp + "'");
  }
  fsync_path(tmp, false);
  if (std::rename(tmp.c_str(), fin.c_str()) != 0)
    fail("cannot publish checkpoint metadata '" + fin + "': " + std::strerror(errno));
  fsync_path(dir, true);
  // The committed checkpoint no longer needs the previous grid, nor any grid
  // an interrupted checkpoint of ours left behind (crash between begin and
  // commit): exactly the names checkpoint_begin recorded in the in-flight
  // list, which is then cleared.
  if (!previous.empty() && previous != m.grid) std::remove((dir + "/" + previous).c_str());
  const std::string inflight = dir + "/" + kInflightName;
  {
    std::ifstream in(inflight);
    std::string n;
    while (std::getline(in, n))
      if (n != m.grid && checkpoint_grid_name_ok(n)) std::remove((dir + "/" + n).c_str());
  }
  std::remove(inflight.c_str());
}

CheckpointMeta checkpoint_load(const std::string& dir) {
  std::ifstream f(dir + "/meta.json");
  if (!f) fail("checkpoint '" + dir + "': no meta.json (incomplete or not a checkpoint)");
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string js = ss.str();
  const std::string fmt = json_field(js, "format");
  if (fmt != kCheckpointFormat)
    fail("checkpoint '" + dir + "': format '" + fmt + "', expected '" + kCheckpointFormat + "'");
  CheckpointMeta m;
  m.W = need_int(js, "width", dir);
  m.H = need_int(js, "height", dir);
  m.generation = need_int(js, "generation", dir);
  m.sim_phase = int(need_int(js, "sim_phase", dir));
  m.gen_limit = need_int(js, "gen_limit", dir);
  m.sim_freq = int(need_int(js, "sim_freq", dir));
  const std::string cs = json_field(js, "check_similarity");
  GOL_REQUIRE(cs == "true" || cs == "false", "checkpoint '" + dir + "': bad check_similarity");
  m.check_similarity = cs == "true";
  const std::string lay = json_field(js, "layout");
  if (!lay.empty()) m.layout = lay;
  const std::string grid = json_field(js, "grid");
  if (!grid.empty()) {
    GOL_REQUIRE(checkpoint_grid_name_ok(grid), "checkpoint '" + dir + "': bad grid file name '" + grid +
                                                   "' (expected grid-<generation>[b].txt)");
    m.grid = grid;
  }
  GOL_REQUIRE(m.W > 0 && m.H > 0 && m.sim_freq > 0 && m.generation >= 0,
              "checkpoint '" + dir + "': inconsistent metadata");
  return m;
}

}  // namespace gol
