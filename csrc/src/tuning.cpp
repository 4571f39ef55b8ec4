// The tuning table and its one environment reader (gol/tuning.hpp).
#include "gol/tuning.hpp"

#include <cstdlib>

#include "gol/common.hpp"

namespace gol {

const std::vector<TuningKey>& tuning_keys() {
  static const std::vector<TuningKey> keys = {
      // --- tune: the default build's performance knobs -------------------
      {"xlane", "GOL_XLANE", "-1", 'i', "tune",
       "cross-lane window of the bit kernels: -1 auto (adder where the frame may drift, else DPP), 0 DPP, 3 adder"},
      {"group", "GOL_GROUP", "8", 'i', "tune",
       "waves per workgroup of the grouped schedule: 8 or 4; 0 the classic (ungrouped) schedule; -1 the model's "
       "choice"},
      {"group_small", "GOL_GROUP_SMALL", "4", 'i', "tune",
       "waves per group of bit-layout blocks with T <= 8 (follows group when only group is set)"},
      {"target_waves", "GOL_TARGET_WAVES", "0", 'i', "tune",
       "waves per launch the segment planner aims at (0: its makespan model decides)"},
      {"min_seg_rows", "GOL_MIN_SEG_ROWS", "16", 'i', "tune",
       "shortest row segment a wave of the classic schedule is given"},
      {"chain", "GOL_CHAIN", "-1", 'i', "tune",
       "chained groups: -1 timed per launch shape, 0 off, 1 on"},
      {"chain_spin", "GOL_CHAIN_SPIN", "16", 'i', "tune", "log2 of a chained wave's spin budget"},
      {"link", "GOL_LINK", "-1", 'i', "tune",
       "linked launches: -1 where the engine asks (small ring tiles, rank tiles), 0 never, 1 every eligible launch"},
      {"link_queue", "GOL_LINK_QUEUE", "-1", 'i', "tune",
       "the second linked stream on a hardware queue of its own (CU-masked to the whole device): -1 when another "
       "backend already lives on the device in this process, 1 always, 2 both linked streams, 0 never (HIP's pool)"},
      {"wrap", "GOL_WRAP", "1", 'i', "tune", "full-width tiles wrap column reads (no halo columns)"},
      {"fold", "GOL_FOLD", "1", 'i', "tune", "fold a narrow last column strip into the others' waves"},
      {"row_ring", "GOL_ROW_RING", "1", 'i', "tune", "single-rank tiles on a row ring (aliased halo rows)"},
      {"u8_kernel", "GOL_U8_KERNEL", "auto", 's', "tune", "byte kernel on the bytes themselves: auto | lds"},
      {"lds_rows", "GOL_LDS_ROWS", "32", 'i', "tune", "rows per LDS tile of the byte LDS kernel"},
      {"lds_t", "GOL_LDS_T", "0", 'i', "tune", "generations per LDS pass (0: 32 packed, 8 unpacked)"},
      {"lds_pack", "GOL_LDS_PACK", "1", 'i', "tune", "LDS kernel packs its tile to bits"},
      {"lds_xcd", "GOL_LDS_XCD", "0", 'i', "tune", "XCD-aware tile order of the LDS kernel"},
      {"lds_waves", "GOL_LDS_WAVES", "0", 'i', "tune", "LDS kernel waves per block: 0 auto, 8 or 16"},
      {"u8_via_bits", "GOL_U8_VIA_BITS", "-1", 'i', "tune",
       "byte layout computes on bit words: -1 auto, 0 bytes, 1 bits (EngineConfig::u8_compute wins when set)"},
      {"side_poll", "GOL_SIDE_POLL", "-1", 'i', "tune",
       "multi-rank polls reduce on a side stream through a flags communicator: -1 timed on the ranks after the "
       "overlap trial, 0 off, 1 on"},
      {"poll_copy_side", "GOL_POLL_COPY_SIDE", "-1", 'i', "tune",
       "single-rank polls copy their flags on a side stream, linked chains continuing across them: -1 where "
       "blocks are deeper than 8 generations, 1 always, 0 never (join the compute streams, copy there)"},
      {"watchdog_s", "GOL_WATCHDOG_S", "0", 'f', "tune", "poll watchdog in seconds (0: 900; EngineConfig wins)"},
      {"host_threads", "GOL_HOST_THREADS", "0", 'i', "tune", "host thread pool size (0: min(cores, 16))"},
      {"numa_pin", "GOL_NUMA_PIN", "1", 'i', "tune",
       "device backends pin the process's host threads to their GPU's NUMA node: 1 the node, 2 one L3 cache of it "
       "(per GPU of the node), 0 leave placement alone"},
      {"cu_partition", "GOL_CU_PARTITION", "", 's', "tune",
       "k/n: this process's streams run on the k-th of n CU slices (ranks sharing a GPU)"},
      // --- diag ------------------------------------------------------------
      {"check_device", "GOL_CHECK_DEVICE", "0", 'i', "diag", "assert device affinity of every call and buffer"},
      {"tune_log", "GOL_TUNE_LOG", "0", 'i', "diag", "log per-launch-shape autotuning decisions"},
      {"host_profile", "GOL_HOST_PROFILE", "0", 'i', "diag", "host time per block (printed at exit)"},
      {"wg_trace", "GOL_WG_TRACE", "", 's', "diag", "N:path[:pair]: per-workgroup timestamps of launch N"},
      // --- fault injection ---------------------------------------------------
      {"fault_delay_spins", "GOL_FAULT_DELAY_SPINS", "0", 'i', "fault",
       "seam groups of linked launches publish late (x 127 s_sleep, <= 4096)"},
      {"fault_delay_us", "GOL_FAULT_DELAY_US", "0", 'i', "fault", "thread transport delays messages randomly"},
      {"fault_garble", "GOL_FAULT_GARBLE", "0", 'i', "fault", "thread transport corrupts the N-th message"},
      {"fault_checkpoint_crash", "GOL_FAULT_CHECKPOINT_CRASH", "0", 'i', "fault",
       "bin/gol exits after writing (not committing) the N-th checkpoint"},
      {"overlap_auto", "GOL_OVERLAP_AUTO", "", 's', "fault", "plain | trigger: force the overlap trial's outcome"},
      // --- CPU emulation of device features ----------------------------------
      {"cpu_ring", "GOL_CPU_RING", "0", 's', "emul", "CPU backend row rings: 0, 1, or fail (mapping fails)"},
      {"cpu_drift", "GOL_CPU_DRIFT", "0", 'i', "emul", "CPU backend's drifting frame (as the adder window)"},
      {"cpu_trigger", "GOL_CPU_TRIGGER", "0", 'i', "emul", "CPU backend accepts the boundary-trigger schedule"},
      {"cpu_side_poll", "GOL_CPU_SIDE_POLL", "0", 'i', "emul",
       "thread transport claims a flags communicator: the poll placement trial runs on CPU ranks"},
  };
  return keys;
}

namespace {

const TuningKey& key_of(const std::string& k) {
  for (const TuningKey& t : tuning_keys())
    if (k == t.key) return t;
  std::string all;
  for (const TuningKey& t : tuning_keys()) all += std::string(all.empty() ? "" : ", ") + t.key;
  fail("unknown tuning key '" + k + "' (known: " + all + ")");
}

bool parse_int(const std::string& s, long* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  const long v = std::strtol(s.c_str(), &end, 10);
  if (*end != '\0') return false;
  *out = v;
  return true;
}

bool parse_float(const std::string& s, double* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  const double v = std::strtod(s.c_str(), &end);
  if (*end != '\0') return false;
  *out = v;
  return true;
}

}  // namespace

Tuning::Tuning() {
  for (const TuningKey& t : tuning_keys()) {
    v_[t.key] = t.dflt;
    src_[t.key] = "default";
  }
}

Tuning Tuning::from_env() {
  Tuning t;
  for (const TuningKey& k : tuning_keys())
    if (const char* e = std::getenv(k.env))
      if (*e) {
        t.set(k.key, e);
        t.src_[k.key] = "env";
      }
  return t;
}

Tuning& Tuning::set(const std::string& key, const std::string& value) {
  const TuningKey& k = key_of(key);
  long v = 0;
  double f = 0;
  if (k.type == 'i' && !parse_int(value, &v))
    fail(std::string("tuning ") + k.key + "=" + value + " (" + k.env + "): expected an integer");
  if (k.type == 'f' && !parse_float(value, &f))
    fail(std::string("tuning ") + k.key + "=" + value + " (" + k.env + "): expected a number");
  v_[k.key] = value;
  src_[k.key] = "set";
  return *this;
}

Tuning& Tuning::set(const std::string& kv) {
  const size_t eq = kv.find('=');
  GOL_REQUIRE(eq != std::string::npos && eq > 0, "tuning setting '" + kv + "': expected key=value");
  return set(kv.substr(0, eq), kv.substr(eq + 1));
}

int Tuning::i(const std::string& key) const {
  const TuningKey& k = key_of(key);
  long v = 0;
  GOL_REQUIRE(k.type == 'i' && parse_int(v_.at(k.key), &v), std::string("tuning key ") + key + " is not an integer");
  return int(v);
}

double Tuning::f(const std::string& key) const {
  const TuningKey& k = key_of(key);
  double v = 0;
  GOL_REQUIRE(k.type == 'f' && parse_float(v_.at(k.key), &v), std::string("tuning key ") + key + " is not a number");
  return v;
}

const std::string& Tuning::s(const std::string& key) const { return v_.at(key_of(key).key); }

bool Tuning::is_default(const std::string& key) const {
  const TuningKey& k = key_of(key);
  if (k.type == 'i') {
    long a = 0, b = 0;
    parse_int(v_.at(k.key), &a);
    parse_int(k.dflt, &b);
    return a == b;
  }
  if (k.type == 'f') {
    double a = 0, b = 0;
    parse_float(v_.at(k.key), &a);
    parse_float(k.dflt, &b);
    return a == b;
  }
  return v_.at(k.key) == k.dflt;
}

const std::string& Tuning::source(const std::string& key) const { return src_.at(key_of(key).key); }

std::map<std::string, std::string> Tuning::changed() const {
  std::map<std::string, std::string> out;
  for (const TuningKey& k : tuning_keys())
    if (!is_default(k.key)) out[k.key] = v_.at(k.key);
  return out;
}

std::string Tuning::summary() const {
  std::string s;
  for (const auto& kv : changed())
    s += (s.empty() ? "" : " ") + kv.first + "=" + kv.second + "[" + src_.at(kv.first) + "]";
  return s.empty() ? "defaults" : s;
}

}  // namespace gol
